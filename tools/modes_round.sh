#!/bin/bash
# Every bench line DESIGN.md quotes, on the build in the tree (one GPU): config 2 in VDI / plain /
# VDICompositor / merged-brick modes, host-sourced re-ingest, configs 1 (VDI + plain, CPU baselines),
# 3 and 4, two self-launched ranks sharing the GPU (RCCL), the in-process 8-rank frame.
# usage: OUT=gpurun_out/modes tools/modes_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=${OUT:-gpurun_out/modes}; mkdir -p $O
run() { local tag=$1 secs=$2; shift 2; timeout -k 10 $secs python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; cb=d.get('cpu_baseline') or {}; print(sys.argv[2], 'n_gpus', d['n_gpus'], round(d['value'],2), d['unit'], 'ms/step', round(d['ms_per_step'],2), c.get('stage_ms'), 'xbytes', c.get('exchange_bytes_per_rank'), 'cpu', cb.get('value'), cb.get('cores'))" $O/$tag.json $tag; }
run c2_plain 300 --mode plain --steps 20 --no-cpu-baseline
run c2_cvdi 300 --compositor vdi --steps 10 --no-cpu-baseline
run c2_merge 300 --merge-bricks --steps 10 --warmup 2 --no-cpu-baseline
run c2_host 300 --update-source host --steps 20 --no-cpu-baseline
run c1_vdi 300 --config 1 --steps 20
run c1_plain 300 --config 1 --mode plain --steps 20
run c3 300 --config 3 --steps 10 --warmup 2 --no-cpu-baseline
run c4 400 --config 4 --steps 10 --warmup 2 --no-cpu-baseline
run c2_gpus2 400 --gpus 2 --steps 10 --no-cpu-baseline
timeout -k 10 300 python tools/local_group_frame.py --ranks 8 --sim-n 512 --out $O/local_group_w8.json > $O/local_group_w8.log 2>&1 || { echo "local group FAILED"; tail -5 $O/local_group_w8.log; exit 1; }
tail -3 $O/local_group_w8.log
