#!/bin/bash
# The search knobs on the emulated N=8 share of the slowest brick (bench.py --emulate-world 8 --emulate-rank 7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/sweep
one() {
    local tag=$1; shift
    env "$@" timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --emulate-world 8 --emulate-rank 7 > gpurun_out/sweep/e_$tag.json 2> gpurun_out/sweep/e_$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('emu8r7', sys.argv[2], 'render %.2f sample %.2f search %.2f' % (s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/sweep/e_$tag.json "$tag"
}
one base INSITU_NOP=1 &&
for v in ${OS:-3 4 8 12}; do one os$v INSITU_SEARCH_OVERSUB=$v || exit 1; done
for v in ${LS:-256 512}; do one ls$v INSITU_LONG_SAMPLES=$v || exit 1; done
