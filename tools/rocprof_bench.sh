#!/bin/bash
# One rocprofv3 run over bench.py, CSVs filtered to the insitu kernels (torch's synthetic-input
# kernels would otherwise push gpurun_out past its copy-back limit).
# usage: tools/rocprof_bench.sh OUTDIR NAME "<bench args>" <rocprofv3 args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=$1; NAME=$2; BARGS=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$NAME" -o "$NAME" -f csv -- python3 bench.py $BARGS > "$OUT/$NAME.log" 2>&1
rc=$?
for f in $(find "$OUT/$NAME" -name '*.csv'); do
    { head -n 1 "$f"; grep -E 'insitu|vdi_|plain_|brick_|assemble' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"
done
grep -v '^[EW]2026' "$OUT/$NAME.log" | tail -n 3
exit $rc
