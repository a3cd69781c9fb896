#!/bin/bash
# A/B counter profile of the VDI generator variants (INSITU_VDI_KERNEL=tile|pool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/ab; mkdir -p $OUT; export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
filter() { for f in $(find "$1" -name '*.csv'); do { head -n 1 "$f"; grep -E 'insitu' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"; done; }
for v in tile pool; do
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    INSITU_VDI_KERNEL=$v timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex insitu -d $OUT/${v}_$tag -o p -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${v}_$tag.log 2>&1
    rc=$?; echo "$v $tag rc=$rc"; filter $OUT/${v}_$tag
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done
