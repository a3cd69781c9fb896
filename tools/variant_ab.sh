#!/bin/bash
# A/B of variant libraries (tools/variant_build.sh) against the in-tree build: N=1 config-2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
one() {
    local tag=$1 lib=$2
    INSITU_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/ab/$tag.json "$tag"
}
L=scenery-insitu_amd/lib
one base $L/libinsitu_hip.so || exit 1
for v in "$@"; do one $v $L/variants/libinsitu_hip_$v.so || exit 1; done
one base2 $L/libinsitu_hip.so
