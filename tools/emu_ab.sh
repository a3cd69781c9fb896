#!/bin/bash
# Variant libraries (tools/variant_build.sh) on the emulated per-GPU share of an N-GPU run
# (bench.py --emulate-world N --emulate-rank R, one GPU): render / sample / search ms per variant.
# usage: EMU_WORLD=8 EMU_RANK=7 tools/emu_ab.sh variant...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/emu_ab
W=${EMU_WORLD:-8}; R=${EMU_RANK:-7}
one() {
    local tag=$1 lib=$2
    INSITU_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --emulate-world $W --emulate-rank $R > gpurun_out/emu_ab/$tag.json 2> gpurun_out/emu_ab/$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'w$W r$R render %.2f sample %.2f search %.2f x %d' % (s['render'], s['render.sample_kernel'], s['render.search_kernel'], 0))" gpurun_out/emu_ab/$tag.json "$tag"
}
L=scenery-insitu_amd/lib
one base $L/libinsitu_hip.so || exit 1
for v in "$@"; do one $v $L/variants/libinsitu_hip_$v.so || exit 1; done
