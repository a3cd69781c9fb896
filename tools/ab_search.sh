#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/sweep
one() {
    local tag=$1; shift
    env "$@" timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || { echo "$tag FAILED"; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f sample %.2f search %.2f handed %d' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel'], d['config']['search_rounds_handed_on_per_frame']))" gpurun_out/sweep/$tag.json "$tag"
}
one base INSITU_NOP=1 &&
one l1 INSITU_SEARCH_LAUNCHES=1 &&
one l1os6 INSITU_SEARCH_LAUNCHES=1 INSITU_SEARCH_OVERSUB=6 &&
one l1d1 INSITU_SEARCH_LAUNCHES=1 INSITU_SEARCH_DEPTH=1 &&
one exact INSITU_EXACT_SEARCH=1 INSITU_SEARCH_LAUNCHES=1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o ab -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ab.log 2>&1
grep -h "vdi_" gpurun_out/prof_ab/*/*kernel_stats.csv 2>/dev/null | head; find gpurun_out/prof_ab -name "*kernel_stats*"
