#!/bin/bash
# Per-rank render times of an emulated N-GPU run (bench.py --emulate-world N --emulate-rank r on one
# GPU, every r), then the per-ray search timing of one rank (tools/ray_timing.py).
# usage: EMU_WORLD=8 RAY_RANK=7 tools/emu_ranks.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
W=${EMU_WORLD:-8}; RR=${RAY_RANK:-7}
mkdir -p gpurun_out/emu_ranks
for r in $(seq 0 $((W - 1))); do
    timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --update-every 0 --emulate-world $W \
        --emulate-rank $r > gpurun_out/emu_ranks/w${W}_r$r.json 2> gpurun_out/emu_ranks/w${W}_r$r.err || { echo "rank $r FAILED"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; c=d['config']; print('w%s r%s render %.2f sample %.2f search %.2f searched %d' % (sys.argv[2], sys.argv[3], s['render'], s['render.sample_kernel'], s['render.search_kernel'], c['rays_searched_per_frame']))" gpurun_out/emu_ranks/w${W}_r$r.json $W $r
done
if [ "$RR" -ge 0 ]; then
    timeout -k 10 120 python tools/ray_timing.py $W $RR > gpurun_out/emu_ranks/rays_w${W}_r$RR.json || exit 1
    cat gpurun_out/emu_ranks/rays_w${W}_r$RR.json
fi
