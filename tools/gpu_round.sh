#!/bin/bash
# The GPU sessions of a round, by name (run on the gpurun box: gpurun -- 'bash tools/gpu_round.sh NAME ...').
# Every step runs under its own time limit (tools/gpu_session.sh); an A/B bench line prints the stage times.
#   tests     all GPU tests, then smoke()
#   bench     the default bench line (gpurun_out/bench.json)
#   profile   rocprofv3 kernel trace + PMC passes of the default bench (gpurun_out/prof; tools/prof_summary.py)
#   modes     profiles of the VDICompositor and merged-bricks modes (gpurun_out/prof_comp, prof_merged)
#   timeline  per-ray search timeline of the one-brick share (emulated rank 7 of 8)
#   composite VDICompositor workload statistics and bench lines
#   emu       emulated per-GPU shares of 2, 4 and 8 GPUs, every rank
#   super     super-tile sampling order A/B (N=1, 8- and 4-GPU shares) + the sampling kernel's FETCH_SIZE
#   calib     FETCH_SIZE calibration for scattered 32-B / 8-B reads (tools/fetch_calib.hip) + request-size split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
ab() {   # tag, extra bench args
    local tag=$1; shift
    timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab/$tag.err; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f composite %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel'], s['composite']))" gpurun_out/ab/$tag.json "$tag"
}
abv() {   # tag, library, extra bench args: ab of a variant library (tools/rev_variant.sh, tools/variant_build.sh)
    local tag=$1 lib=$2; shift 2
    INSITU_HIP_LIB=$lib ab "$tag" "$@"
}
pmc() {   # tag, counters, extra bench args: one rocprofv3 PMC pass over a short N=1 bench run -> gpurun_out/pmc/<tag>
    local tag=$1 ctr=$2; shift 2
    mkdir -p gpurun_out/pmc
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex insitu -d gpurun_out/pmc/$tag -o $tag -f csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --update-every 0 "$@" > gpurun_out/pmc/$tag.log 2>&1 || { echo "pmc $tag FAILED"; return 1; }
    python3 tools/pmc_kernel_sum.py gpurun_out/pmc/$tag "$tag"
}
W8="--emulate-world 8 --emulate-rank 7 --update-every 0"
W4="--emulate-world 4 --emulate-rank 3 --update-every 0"
for name in "$@"; do
    case $name in
    tests) tools/gpu_session.sh \
        "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
        "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $? ;;
    bench) tools/gpu_session.sh "bench|300|python bench.py > gpurun_out/bench.json" || exit $? ;;
    profile) tools/gpu_session.sh \
        "prof|600|PROF_OUT=gpurun_out/prof BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline' tools/profile_round.sh" || exit $? ;;
    modes) tools/gpu_session.sh \
        "prof_comp|500|PROF_OUT=gpurun_out/prof_comp BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --compositor vdi --update-every 0' tools/profile_round.sh" \
        "prof_merged|700|PROF_OUT=gpurun_out/prof_merged BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --merge-bricks --update-every 0' tools/profile_round.sh" || exit $? ;;
    timeline) tools/gpu_session.sh \
        "rt_w8|200|python tools/ray_timing.py 8 7 > gpurun_out/rt_w8.json" || exit $? ;;
    composite) tools/gpu_session.sh "comp_stats|300|python tools/composite_stats.py > gpurun_out/composite_stats.json" || exit $?
        ab comp --compositor vdi --update-every 0 && ab merged --merge-bricks --update-every 0 && ab n1 --update-every 0 || exit 1 ;;
    emu)   # per-rank render times of the emulated 2-, 4- and 8-GPU strong-scaling shares (tools/emu_ranks.sh)
        for w in 2 4 8; do EMU_WORLD=$w RAY_RANK=-1 tools/emu_ranks.sh || exit 1; done ;;
    calib) # FETCH_SIZE of known byte counts (tools/fetch_calib.hip, built in-tree) and the read-request size
        # split of the same patterns and of the default bench's kernels
        C=gpurun_out/calib
        mkdir -p $C
        SPLIT="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
        tools/gpu_session.sh \
        "calib_bytes|60|tools/fetch_calib > $C/bytes.json" \
        "calib_trace|90|timeout -s KILL 80 rocprofv3 --kernel-trace --stats -d $C/trace -o trace -f csv -- tools/fetch_calib" \
        "calib_fetch|90|timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $C/fetch -o fetch -f csv -- tools/fetch_calib" \
        "calib_split|90|timeout -s KILL 80 rocprofv3 --pmc $SPLIT -d $C/split -o split -f csv -- tools/fetch_calib" \
        "bench_split|300|timeout -s KILL 280 rocprofv3 --pmc $SPLIT --kernel-include-regex insitu -d $C/bench_split -o bench_split -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" || exit $? ;;
    super) # longest-first order by super-tiles of 1/2/4 tiles per edge: N=1, the 8- and 4-GPU shares, sampling FETCH
        for s in 1 2 4; do
            ab n1_s$s --option super_tile=$s --update-every 0 && ab w8_s$s --option super_tile=$s $W8 &&
                ab w4_s$s --option super_tile=$s $W4 || exit 1
        done
        for s in 1 4; do pmc fetch_s$s FETCH_SIZE --option super_tile=$s || exit 1; done ;;
    sabl) # sampling-kernel timing ablations (wrong results; only the sampling stage is read): no voxel loads,
        # no cache stores, neither, no state machines (pass 1 and the spine), none of the three
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        U="--update-every 0"
        ab s_base $U && abv s_noload ${L}_abl_noload.so $U && abv s_nostore ${L}_abl_nostore.so $U &&
            abv s_nols ${L}_abl_nols.so $U && abv s_nosm ${L}_abl_nosm.so $U && abv s_all ${L}_abl_all.so $U &&
            ab s_base2 $U || exit 1 ;;
    dtime) # search-loop section cycles (diagnostics variant -DINSITU_DIAG_TIME): N=1, the 8- and 4-GPU shares
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_dtime.so
        abv t_n1 $V --update-every 0 && abv t_w8 $V $W8 && abv t_w4 $V $W4 || exit 1
        for t in t_n1 t_w8 t_w4; do echo "$t $(grep dtime gpurun_out/ab/$t.err | tail -n 1)"; done ;;
    sel) # select-form search replay (default) against the branching form (variant sel0): N=1 and the 8- and 4-GPU shares
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_sel0.so
        U="--update-every 0"
        ab sel1 $U && abv sel0 $V $U && ab sel1b $U && abv sel0b $V $U &&
            ab w8_sel1 $W8 && abv w8_sel0 $V $W8 && ab w4_sel1 $W4 && abv w4_sel0 $V $W4 || exit 1 ;;
    selp) # select-form pass 1 and spine counters (default) against the branching form (variant selp0)
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_selp0.so
        U="--update-every 0"
        ab p1 $U && abv p0 $V $U && ab p1b $U && abv p0b $V $U &&
            ab w8_p1 $W8 && abv w8_p0 $V $W8 && ab m_p1 --merge-bricks $U && abv m_p0 $V --merge-bricks $U || exit 1 ;;
    ipc) # instruction counts of the search kernel: select-form replay (default) against the branching form (sel0)
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_sel0.so
        SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
        LN="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
        pmc sq_sel1 "$SQ" && INSITU_HIP_LIB=$V pmc sq_sel0 "$SQ" && pmc ln_sel1 "$LN" && INSITU_HIP_LIB=$V pmc ln_sel0 "$LN" || exit 1 ;;
    fetch) # footprint fetch without the x-face branch + wave-uniform brick descriptor (default) against HEAD's
        # library (variant head), and the sampling kernel at 4 waves per SIMD (variant s4w)
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        U="--update-every 0"
        ab f_new $U && abv f_head $H $U && abv f_s4w scenery-insitu_amd/lib/variants/libinsitu_hip_s4w.so $U &&
            ab f_new2 $U && abv f_head2 $H $U && ab w8_fnew $W8 && abv w8_fhead $H $W8 &&
            ab pl_new --mode plain $U && abv pl_head $H --mode plain $U || exit 1 ;;
    p1lds) # pass-1 bounds and chunk in LDS (sampling kernel at 125 VGPRs: 4 waves per SIMD) against HEAD's library
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        U="--update-every 0"
        ab q_new $U && abv q_head $H $U && ab q_new2 $U && abv q_head2 $H $U && ab w8_qnew $W8 && abv w8_qhead $H $W8 &&
            ab w4_qnew $W4 && abv w4_qhead $H $W4 && ab m_qnew --merge-bricks $U && abv m_qhead $H --merge-bricks $U || exit 1 ;;
    cw) # VDICompositor merge cache without world positions (32-byte entries, default) against 64-byte entries (cw1)
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_cw1.so
        C="--compositor vdi --update-every 0"
        tools/gpu_session.sh "gt_comp|400|python -u -m pytest tests -m gpu -x -q -k \"composit\" --timeout 200 --timeout-method thread" || exit $?
        ab c_new $C && abv c_cw1 $V $C && ab c_new2 $C && abv c_cw12 $V $C || exit 1
        pmc c_fetch "FETCH_SIZE" $C && pmc c_write "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" $C || exit 1 ;;
    msel) # merged search with the select-form replay (default) against HEAD's library
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        M="--merge-bricks --update-every 0"
        tools/gpu_session.sh "gt_merged|400|python -u -m pytest tests -m gpu -x -q -k merged --timeout 200 --timeout-method thread" || exit $?
        ab ms_new $M && abv ms_head $H $M && ab ms_new2 $M && abv ms_head2 $H $M || exit 1 ;;
    knobs5) # round batch and search oversubscription after the select-form replay (N=1; 8-GPU share)
        U="--update-every 0"
        for rep in a b; do
            ab kb28$rep $U && ab kb36$rep $U --option round_batch=36 && ab kb20$rep $U --option round_batch=20 &&
                ab ko8$rep $U --option search_oversub=8 || exit 1
        done
        ab w8_ko6 $W8 && ab w8_ko8 $W8 --option search_oversub=8 && ab w8_ko4 $W8 --option search_oversub=4 || exit 1 ;;
    rgd) # deepest regroup tree 4 (default) against 5 and 6: the 8- and 4-GPU shares, N=1
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        for rep in a b; do
            ab w8_rg4$rep $W8 && abv w8_rg5$rep ${L}_rg5.so $W8 && abv w8_rg6$rep ${L}_rg6.so $W8 &&
                ab w4_rg4$rep $W4 && abv w4_rg5$rep ${L}_rg5.so $W4 && abv w4_rg6$rep ${L}_rg6.so $W4 || exit 1
        done
        ab n1_rg4 --update-every 0 && abv n1_rg6 ${L}_rg6.so --update-every 0 || exit 1 ;;
    ab2) # the working tree's library against HEAD's (variant head): N=1 twice, plain, the 8-GPU share
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        U="--update-every 0"
        ab x_new $U && abv x_head $H $U && ab x_new2 $U && abv x_head2 $H $U && ab xp_new --mode plain $U &&
            abv xp_head $H --mode plain $U && ab xw8_new $W8 && abv xw8_head $H $W8 || exit 1 ;;
    cf) # VDICompositor pass 1 fused with the cache-filling walk (default) against HEAD's library
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        C="--compositor vdi --update-every 0"
        tools/gpu_session.sh "gt_comp|400|python -u -m pytest tests -m gpu -x -q -k \"composit\" --timeout 200 --timeout-method thread" || exit $?
        ab cf_new $C && abv cf_head $H $C && ab cf_new2 $C && abv cf_head2 $H $C || exit 1
        pmc cf_fetch "FETCH_SIZE" $C || exit 1 ;;
    cz) # composited VDI without zero-filled slots (per-pixel counts; default) against HEAD's library
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        C="--compositor vdi --update-every 0"
        tools/gpu_session.sh "gt_cz|600|python -u -m pytest tests -m gpu -x -q -k \"composit or rccl or harness or group\" --timeout 200 --timeout-method thread" || exit $?
        ab cz_new $C && abv cz_head $H $C && ab cz_new2 $C && abv cz_head2 $H $C || exit 1 ;;
    tko) # tile-order knobs at 4 waves per SIMD: XCD chunk 8 / 32 (default 16), length classes of 8 / 32 samples (16)
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        U="--update-every 0"
        for rep in a b; do
            ab t_def$rep $U && abv t_xc8$rep ${L}_xc8.so $U && abv t_xc32$rep ${L}_xc32.so $U &&
                abv t_cs3$rep ${L}_cs3.so $U && abv t_cs5$rep ${L}_cs5.so $U || exit 1
        done
        ab w8_tdef $W8 && abv w8_tcs3 ${L}_cs3.so $W8 && abv w8_txc8 ${L}_xc8.so $W8 || exit 1 ;;
    xc) # XCD chunk 8 (default) against 16 (HEAD's library) and 4 (variant xc4): N=1, merged, the 4-GPU share
        H=scenery-insitu_amd/lib/variants/libinsitu_hip_head.so
        X=scenery-insitu_amd/lib/variants/libinsitu_hip_xc4.so
        U="--update-every 0"
        ab x8a $U && abv x16a $H $U && abv x4a $X $U && ab x8b $U && abv x16b $H $U && abv x4b $X $U &&
            ab m_x8 --merge-bricks $U && abv m_x16 $H --merge-bricks $U && abv m_x4 $X --merge-bricks $U &&
            ab w4_x8 $W4 && abv w4_x16 $H $W4 && abv w4_x4 $X $W4 || exit 1 ;;
    xc2) # XCD chunk 4 (default) against 2 and 1 (hardware order): N=1 twice, merged
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        U="--update-every 0"
        ab y4a $U && abv y2a ${L}_xc2.so $U && abv y1a ${L}_xc1.so $U && ab y4b $U && abv y2b ${L}_xc2.so $U &&
            abv y1b ${L}_xc1.so $U && ab m_y4 --merge-bricks $U && abv m_y2 ${L}_xc2.so --merge-bricks $U &&
            abv m_y1 ${L}_xc1.so --merge-bricks $U || exit 1 ;;
    sl) # speculative spine levels 4 (default) against 3 and 5, at 4 waves per SIMD: N=1 twice, the 8-GPU share
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        U="--update-every 0"
        ab s4a $U && abv s3a ${L}_sl3.so $U && abv s5a ${L}_sl5.so $U && ab s4b $U && abv s3b ${L}_sl3.so $U &&
            abv s5b ${L}_sl5.so $U && ab w8_s4 $W8 && abv w8_s3 ${L}_sl3.so $W8 && abv w8_s5 ${L}_sl5.so $W8 || exit 1 ;;
    promo) # promotion of long searches to 3-lane groups: from pass 12 (pr1) and 9 (pr9) against none (default build)
        L=scenery-insitu_amd/lib/variants/libinsitu_hip
        U="--update-every 0"
        tools/gpu_session.sh "gt_promo|700|INSITU_HIP_LIB=${L}_pr1.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" || exit $?
        abv p_12 ${L}_pr1.so $U && ab p_off $U && abv p_9 ${L}_pr9.so $U && abv p_122 ${L}_pr1.so $U && ab p_off2 $U &&
            abv p_92 ${L}_pr9.so $U && abv w4_p12 ${L}_pr1.so $W4 && ab w4_poff $W4 && abv w4_p9 ${L}_pr9.so $W4 &&
            abv w8_p12 ${L}_pr1.so $W8 && ab w8_poff $W8 && abv m_p12 ${L}_pr1.so --merge-bricks $U && ab m_poff --merge-bricks $U &&
            abv m_p9 ${L}_pr9.so --merge-bricks $U || exit 1 ;;
    mil) # merged slots interleaved in pairs (variant mil2) against single slots (default), and the merged search's HBM
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_mil2.so
        M="--merge-bricks --update-every 0"
        tools/gpu_session.sh "gt_mil2|400|INSITU_HIP_LIB=$V python -u -m pytest tests -m gpu -x -q -k merged --timeout 200 --timeout-method thread" || exit $?
        ab mi1a $M && abv mi2a $V $M && ab mi1b $M && abv mi2b $V $M || exit 1
        INSITU_HIP_LIB=$V pmc mi2_fetch "FETCH_SIZE" $M || exit 1 ;;
    ci) # brick cache chunks interleaved in pairs stored from an LDS pair stage (variant ci2) against single chunks
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_ci2.so
        U="--update-every 0"
        tools/gpu_session.sh "gt_ci2|700|INSITU_HIP_LIB=$V python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" || exit $?
        ab ci1a $U && abv ci2a $V $U && ab ci1b $U && abv ci2b $V $U && ab w8_ci1 $W8 && abv w8_ci2 $V $W8 &&
            ab w4_ci1 $W4 && abv w4_ci2 $V $W4 || exit 1
        INSITU_HIP_LIB=$V pmc ci2_fetch "FETCH_SIZE" $U || exit 1 ;;
    cpair) # VDICompositor merge-cache entries in per-lane pairs (variant cp1) against single entries (default)
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_cp1.so
        C="--compositor vdi --update-every 0"
        tools/gpu_session.sh "gt_cp1|500|INSITU_HIP_LIB=$V python -u -m pytest tests -m gpu -x -q -k \"composit or rccl or harness\" --timeout 200 --timeout-method thread" || exit $?
        ab cp0a $C && abv cp1a $V $C && ab cp0b $C && abv cp1b $V $C || exit 1
        INSITU_HIP_LIB=$V pmc cp1_fetch "FETCH_SIZE" $C || exit 1 ;;
    ns) # the replay body without store branches for trips without stores (variant ns1) against one body
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_ns1.so
        U="--update-every 0"
        tools/gpu_session.sh "gt_ns1|400|INSITU_HIP_LIB=$V python -u -m pytest tests -m gpu -x -q -k \"parity or config2\" --timeout 200 --timeout-method thread" || exit $?
        ab ns0a $U && abv ns1a $V $U && ab ns0b $U && abv ns1b $V $U && ab w8_ns0 $W8 && abv w8_ns1 $V $W8 &&
            ab w4_ns0 $W4 && abv w4_ns1 $V $W4 || exit 1 ;;
    pad) # paired merged slots without (default) and with (variant pad1) their padding stores
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_pad1.so
        M="--merge-bricks --update-every 0"
        tools/gpu_session.sh "gt_pad|400|python -u -m pytest tests -m gpu -x -q -k merged --timeout 200 --timeout-method thread" || exit $?
        ab pd0a $M && abv pd1a $V $M && ab pd0b $M && abv pd1b $V $M || exit 1 ;;
    mknobs) # merged mode: round batch 20 / 36 and search oversubscription 4 / 8 against the defaults (28, 6)
        M="--merge-bricks --update-every 0"
        ab mk_def $M && ab mk_rb20 $M --option round_batch=20 && ab mk_rb36 $M --option round_batch=36 &&
            ab mk_os4 $M --option search_oversub=4 && ab mk_os8 $M --option search_oversub=8 && ab mk_def2 $M || exit 1 ;;
    merged) # merged-bricks mode: its GPU tests, A/B against the r5base variant, the merged search kernel's HBM bytes
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_r5base.so
        tools/gpu_session.sh "gt_merged|400|python -u -m pytest tests -m gpu -x -q -k merged --timeout 200 --timeout-method thread" || exit $?
        abv m_base $V --merge-bricks --update-every 0 && ab m_new --merge-bricks --update-every 0 &&
            abv m_base2 $V --merge-bricks --update-every 0 && ab m_new2 --merge-bricks --update-every 0 || exit 1
        pmc m_fetch FETCH_SIZE --merge-bricks && pmc m_write "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" --merge-bricks || exit 1 ;;
    merged2) # merged mode: slot interleave 2 (variant mil2, its tests too) and the tree-group knobs
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_mil2.so
        tools/gpu_session.sh "gt_mil2|400|INSITU_HIP_LIB=$V python -u -m pytest tests -m gpu -x -q -k merged --timeout 200 --timeout-method thread" || exit $?
        M="--merge-bricks --update-every 0"
        ab m_il1 $M && abv m_il2 $V $M && ab m_d2 $M --option search_depth=2 && ab m_d3 $M --option search_depth=3 &&
            ab m_os12 $M --option search_oversub=12 && abv m_il2_d2 $V $M --option search_depth=2 && ab m_il1b $M || exit 1 ;;
    comp) # VDICompositor: its GPU tests, A/B against the r5base variant, the composite kernel's HBM bytes and lanes
        V=scenery-insitu_amd/lib/variants/libinsitu_hip_r5base.so
        tools/gpu_session.sh "gt_comp|500|python -u -m pytest tests -m gpu -x -q -k 'ompositor or composite or config2_full' --timeout 300 --timeout-method thread" || exit $?
        C="--compositor vdi --update-every 0"
        abv c_base $V $C && ab c_new $C && abv c_base2 $V $C && ab c_new2 $C || exit 1
        pmc c_fetch FETCH_SIZE $C && pmc c_write "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" $C &&
            pmc c_lane "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" $C || exit 1 ;;
    regroup) # tail regrouping: the search GPU tests, A/B regroup=0/1 at N=1 and on the 8- and 4-GPU shares, timelines
        tools/gpu_session.sh "gt_search|600|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread" || exit $?
        for r in 0 1; do
            ab n1_rg$r --option regroup=$r --update-every 0 && ab w8_rg$r --option regroup=$r $W8 && ab w4_rg$r --option regroup=$r $W4 || exit 1
        done
        ab n1_rg0b --option regroup=0 --update-every 0 && ab n1_rg1b --option regroup=1 --update-every 0 || exit 1
        mkdir -p gpurun_out/rt
        timeout -k 10 150 python tools/ray_timing.py 4 3 > gpurun_out/rt/w4r3_rg1.json &&
            timeout -k 10 150 python tools/ray_timing.py 8 7 > gpurun_out/rt/w8r7_rg1.json || exit 1 ;;
    *) echo "unknown session $name"; exit 2 ;;
    esac
done
