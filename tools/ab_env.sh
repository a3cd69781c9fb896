#!/bin/bash
# A/B of runtime options through the environment (INSITU_* seeds of insitu_set_option): N=1 config-2
# bench, or the emulated per-GPU share of an 8-GPU run with EMU=1.  usage: tools/ab_env.sh "TAG|VAR=V ..." ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab_env
EXTRA=""
[ -n "$EMU" ] && EXTRA="--emulate-world ${EMU_W:-8} --emulate-rank ${EMU_RANK:-7}"
for spec in "$@"; do
    tag=${spec%%|*}; vars=${spec#*|}
    env $vars timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $EXTRA > gpurun_out/ab_env/$tag.json 2> gpurun_out/ab_env/$tag.err || { echo "$tag FAILED"; tail -5 gpurun_out/ab_env/$tag.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print(sys.argv[2], 'ms/step %.2f render %.2f split %.2f + %.2f' % (d['ms_per_step'], s['render'], s['render.sample_kernel'], s['render.search_kernel']))" gpurun_out/ab_env/$tag.json "$tag"
done
