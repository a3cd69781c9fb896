#!/bin/bash
# round 4: fused generator modes -- parity first, then A/B against the two-launch generator
# (N=1 and the emulated per-GPU shares of 4 and 8 GPUs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
L=scenery-insitu_amd/lib
ab() {   # tag, library, extra bench args
    local tag=$1 lib=$2; shift 2
    INSITU_HIP_LIB=$lib timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab/$tag.err; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/ab/$tag.json "$tag"
}
tools/gpu_session.sh \
 "fusedtests|300|python -u -m pytest tests/test_gpu_parity.py -k 'fused' -x -q --timeout 120 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/fusedtests.log && ! grep -q "failed" gpurun_out/fusedtests.log || { echo "fused tests failed: no benches"; exit 1; }
W8="--emulate-world 8 --emulate-rank 7 --update-every 0"
W4="--emulate-world 4 --emulate-rank 3 --update-every 0"
ab w8_classic $L/libinsitu_hip.so --option fused=0 $W8 && ab w8_early $L/libinsitu_hip.so --option fused=2 $W8 && \
ab w8_early2 $L/libinsitu_hip.so --option fused=2 --option gen_searchers=2 $W8 && \

ab w4_classic $L/libinsitu_hip.so --option fused=0 $W4 && ab w4_early $L/libinsitu_hip.so --option fused=2 $W4 && \
ab n1_classic $L/libinsitu_hip.so --option fused=0 && ab n1_early $L/libinsitu_hip.so --option fused=2 || exit 1
tools/gpu_session.sh \
 "rt_w8_early|200|python tools/ray_timing.py 8 7 --option fused=2 > gpurun_out/rt_w8_early.json" \
 "rt_w8_classic|200|python tools/ray_timing.py 8 7 --option fused=0 > gpurun_out/rt_w8_classic.json"
