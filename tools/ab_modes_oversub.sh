#!/bin/bash
# A/B of INSITU_PIPE_OVERSUB (pipelined frames' search oversubscription) on the other configs and modes, one box:
# config 2 (calibration), VDICompositor, merged bricks, configs 1, 3 and 4.  usage: tools/ab_modes_oversub.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ab_modes_oversub; mkdir -p $O
one() { local tag=$1 v=$2 secs=$3; shift 3
    INSITU_PIPE_OVERSUB=$v timeout -k 10 $secs python bench.py --no-cpu-baseline "$@" > $O/${tag}_os$v.json 2> $O/${tag}_os$v.err || { echo "$tag FAILED"; tail -3 $O/${tag}_os$v.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'oversub', sys.argv[3], round(d['value'],2), 'frames/s', round(d['ms_per_step'],3), 'ms')" $O/${tag}_os$v.json $tag $v; }
for v in 6 3 6 3; do one c2 $v 200 --steps 30 || exit 1; done
for v in 6 3; do one cvdi $v 200 --compositor vdi --steps 20 || exit 1; done
for v in 6 3; do one merge $v 200 --merge-bricks --steps 20 || exit 1; done
for v in 6 3; do one c3 $v 200 --config 3 --steps 20 || exit 1; done
for v in 6 3; do one c4 $v 300 --config 4 --steps 10 || exit 1; done
