#!/bin/bash
# round 4: queued VDICompositor search, per-pixel merge-cache layout -- parity, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
ab() {   # tag, extra bench args
    local tag=$1; shift
    timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab/$tag.err; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f composite %.2f' % (d['ms_per_step'], s['render'], s['composite']))" gpurun_out/ab/$tag.json "$tag"
}
tools/gpu_session.sh \
 "comptests|400|python -u -m pytest tests/test_gpu_parity.py -k 'compositor' -x -q --timeout 120 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/comptests.log && ! grep -q "failed" gpurun_out/comptests.log || { echo "tests failed: no benches"; exit 1; }
U="--compositor vdi --update-every 0"
ab comp_q0 --option comp_queue=0 $U && ab comp_q1 $U && ab comp_b8 --option comp_batch=8 $U && \
ab comp_b32 --option comp_batch=32 $U && ab comp_b1 --option comp_batch=1 $U || exit 1
