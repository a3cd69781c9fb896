#!/bin/bash
# round 4: fused generator -- parity first, then A/B against the two-launch generator (N=1 and
# emulated per-GPU shares), then the full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
ab() {   # tag, extra bench args
    local tag=$1; shift
    timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab/$tag.err; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/ab/$tag.json "$tag"
}
tools/gpu_session.sh \
 "fusedtests|300|python -u -m pytest tests/test_gpu_parity.py -k 'fused or merged or grows' -x -q --timeout 120 --timeout-method thread" || exit $?
ab n1_classic --option fused=0 && ab n1_fused --option fused=1 && \
ab w8r7_classic --option fused=0 --emulate-world 8 --emulate-rank 7 --update-every 0 && \
ab w8r7_fused --option fused=1 --emulate-world 8 --emulate-rank 7 --update-every 0 && \
ab w8r5_classic --option fused=0 --emulate-world 8 --emulate-rank 5 --update-every 0 && \
ab w8r5_fused --option fused=1 --emulate-world 8 --emulate-rank 5 --update-every 0 && \
ab w4r3_classic --option fused=0 --emulate-world 4 --emulate-rank 3 --update-every 0 && \
ab w4r3_fused --option fused=1 --emulate-world 4 --emulate-rank 3 --update-every 0 && \
ab w8r7_fused_s1 --option fused=1 --option gen_searchers=1 --emulate-world 8 --emulate-rank 7 --update-every 0 && \
ab n1_fused_s1 --option fused=1 --option gen_searchers=1 && \
ab n1_fused2 --option fused=1 && ab n1_classic2 --option fused=0 || exit 1
tools/gpu_session.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "counters|60|rocprofv3 -L > gpurun_out/counters.txt 2>&1; grep -c . gpurun_out/counters.txt"
