#!/bin/bash
# Kernel-trace statistics (rocprofv3 --kernel-trace --stats) of a short bench run, insitu kernels only.
# usage: tools/ktrace.sh NAME "<bench args>"   -> gpurun_out/ktrace_NAME/..._kernel_stats.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
NAME=$1; BARGS=${2:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/ktrace_$NAME
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o kt -f csv -- python3 bench.py $BARGS > "$OUT.log" 2>&1
rc=$?
for f in $(find "$OUT" -name '*.csv'); do
    { head -n 1 "$f"; grep -E 'insitu' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"
done
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('%-60s calls %4s avg %.3f ms' % (r['Name'].split('(')[0].replace('void ','')[:60], r['Calls'], float(r['AverageNs'])/1e6))"
exit $rc
