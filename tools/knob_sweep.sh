#!/bin/bash
# Sweep the search-kernel scheduling knobs (results are identical by construction; only time moves).
# Each run: N=1 config-2 bench, no CPU baseline; prints render.search_kernel / render ms per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/sweep
one() {
    local tag=$1; shift
    env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/sweep/$tag.json "$tag"
}
one base INSITU_NOP=1 &&
for v in ${LS:-192 256 512 768}; do one ls$v INSITU_LONG_SAMPLES=$v || exit 1; done
for v in ${OS:-1 3 4}; do one os$v INSITU_SEARCH_OVERSUB=$v || exit 1; done
for v in ${RB:-4 16 32}; do one rb$v INSITU_ROUND_BATCH=$v || exit 1; done
