#!/bin/bash
# Bench lines of the other BASELINE configs and bench variants for DESIGN.md (one GPU):
# config 3 and 4 at N=1, config 2 with host-sourced re-ingest (PCIe GPU-send), emulated N=2/4 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/configs; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(sys.argv[2], round(d['value'],2), d['unit'], 'ms/step', round(d['ms_per_step'],2), c['stage_ms'], 'send/update', c.get('gpu_send_ms_per_update'))" $O/$tag.json $tag; }
run c3 --config 3 --steps 10 --warmup 2 --no-cpu-baseline
run c4 --config 4 --steps 10 --warmup 2 --no-cpu-baseline
run c2_host --steps 20 --warmup 3 --no-cpu-baseline --update-source host
for r in 0 1; do run emu2_r$r --steps 8 --warmup 2 --no-cpu-baseline --emulate-world 2 --emulate-rank $r; done
for r in 0 1 2 3; do run emu4_r$r --steps 8 --warmup 2 --no-cpu-baseline --emulate-world 4 --emulate-rank $r; done
