#!/bin/bash
# Per-GPU render time of an N-GPU run emulated on one GPU (bench.py --emulate-world N), with knob
# settings given as "tag:VAR=val" arguments.  Results are identical by construction; only time moves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/emu
W=${EMU_WORLD:-8}
for spec in base:INSITU_NOP=1 "$@"; do
    tag=${spec%%:*}; kv=${spec#*:}
    env $kv timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --emulate-world $W --emulate-rank ${EMU_RANK:-0} > gpurun_out/emu/w$W.r${EMU_RANK:-0}.$tag.json 2> gpurun_out/emu/w$W.r${EMU_RANK:-0}.$tag.err || { echo "$tag FAILED"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'render %.2f sample %.2f search %.2f' % (s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/emu/w$W.r${EMU_RANK:-0}.$tag.json "w$W r${EMU_RANK:-0} $tag"
done
