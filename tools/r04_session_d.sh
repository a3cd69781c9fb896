#!/bin/bash
# round 4: queued VDICompositor search + merged-volume interval tracking -- parity, then A/B, then all GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
ab() {   # tag, extra bench args
    local tag=$1; shift
    timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab/$tag.err; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f composite %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel'], s['composite']))" gpurun_out/ab/$tag.json "$tag"
}
tools/gpu_session.sh \
 "comptests|400|python -u -m pytest tests/test_gpu_parity.py -k 'compositor or merged or option' -x -q --timeout 120 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/comptests.log && ! grep -q "failed" gpurun_out/comptests.log || { echo "tests failed: no benches"; exit 1; }
U="--update-every 0"
ab comp_q0 --compositor vdi --option comp_queue=0 $U && ab comp_q1 --compositor vdi $U && \
ab comp_b4 --compositor vdi --option comp_batch=4 $U && ab comp_b32 --compositor vdi --option comp_batch=32 $U && \
ab merged --merge-bricks $U && ab n1 $U || exit 1
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
