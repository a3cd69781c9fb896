#!/bin/bash
# Sweep the search-kernel scheduling knobs through bench.py --option (results are identical by
# construction; only time moves).  Each run: config-2 bench, no CPU baseline; N=1 unless
# EMU="--emulate-world 8 --emulate-rank 7" (the one-brick share).
# usage: tools/knob_sweep.sh "round_batch=4" "long_samples=512" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/sweep
one() {
    local tag=$1; shift
    timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --update-every 0 $EMU "$@" > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/sweep/$tag.json "$tag"
}
one base || exit 1
for o in "$@"; do one "${o//=/_}" --option "$o" || exit 1; done
