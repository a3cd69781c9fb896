#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC passes (each its own run).
# Trace/counter CSVs are filtered to the insitu kernels (torch's synthetic-input kernels flood them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
P="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline}"
# the PMC passes run the frames unpipelined: rocprofv3's counter collection serialises the dispatches and a
# pipelined run stalled in it (round 6: no progress after the bricks were generated); the kernels and their
# per-launch counters are the same, the trace pass runs the command as given
PP="${PMC_BENCH_ARGS:-$P --pipeline 0}"
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 tools/src_hash.py > "$OUT/csrc_sha16.txt"   # the sources these kernels were built from
filter() {  # keep header + insitu rows of every CSV in $1, drop the rest
    for f in $(find "$1" -name '*.csv'); do
        { head -n 1 "$f"; grep -E 'insitu' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"
    done
}
run() {
    local name=$1; shift; echo "== $name"
    local args="$PP"
    [ "$name" = trace ] && args="$P"
    timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" -f csv -- python3 bench.py $args > "$OUT/$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
    filter "$OUT/$name"
    return $rc
}
run trace --kernel-trace --stats &&
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-include-regex insitu &&
run pmc_fetch --pmc FETCH_SIZE --kernel-include-regex insitu &&
run pmc_write --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex insitu &&
run pmc_misc --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex insitu &&
run pmc_lane --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --kernel-include-regex insitu
du -sh "$OUT"
