#!/bin/bash
# Render-stage ms of knob settings (results identical by construction; only time moves), at N=1 and
# on emulated per-GPU shares.  usage: tools/knob_grid.sh "tag:VAR=v VAR2=v" ...   (EMU="8:7 4:3")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/grid
for spec in "$@"; do
    tag=${spec%%:*}; kv=${spec#*:}
    for e in 1:0 ${EMU:-8:7}; do
        w=${e%%:*}; r=${e#*:}
        extra=""; [ "$w" != 1 ] && extra="--emulate-world $w --emulate-rank $r"
        env $kv timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline $extra > gpurun_out/grid/$tag.w$w.json 2> gpurun_out/grid/$tag.w$w.err || { echo "$tag w$w FAILED"; exit 1; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'render %.2f sample %.2f search %.2f x %d' % (s['render'], s['render.sample_kernel'], s['render.search_kernel'], 0))" gpurun_out/grid/$tag.w$w.json "$tag w$w r$r"
    done
done
