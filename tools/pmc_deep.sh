#!/bin/bash
# Extra rocprofv3 PMC passes on the generator kernels (address/data path and LDS), one pass per run:
# usage: PROF_OUT=gpurun_out/deep tools/pmc_deep.sh   (then python tools/pmc_deep_summary.py $PROF_OUT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
P="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline}"
OUT=${PROF_OUT:-gpurun_out/deep}
mkdir -p "$OUT"
export TMPDIR=/tmp
filter() { for f in $(find "$1" -name '*.csv'); do { head -n 1 "$f"; grep -E 'vdi_s' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"; done; }
run() {
    local name=$1; shift; echo "== $name"
    timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" -f csv -- python3 bench.py $P > "$OUT/$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; filter "$OUT/$name"; return $rc
}
run ta --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --kernel-include-regex vdi_s &&
run tcp --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex vdi_s &&
run sqmem --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex vdi_s &&
run sqlds --pmc SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU --kernel-include-regex vdi_s
