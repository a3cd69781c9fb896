#!/bin/bash
# A/B of the pipelined search grid (INSITU_PIPE_SEARCH_RAYS=0 + trigger 1: round 6's first pipelined build;
# default: the adaptive grid + trigger 2) on the other configs and modes, one box.  usage: tools/ab_modes_grid.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ab_modes_grid; mkdir -p $O
one() { local tag=$1 vars=$2 secs=$3; shift 3
    env $vars timeout -k 10 $secs python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -3 $O/$tag.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value'],2), 'frames/s', round(d['ms_per_step'],3), 'ms')" $O/$tag.json $tag; }
OLD="INSITU_PIPE_SEARCH_RAYS=0 INSITU_PIPE_TRIGGER=1"
NEW="X=1"
for m in "c2|--steps 30" "cvdi|--compositor vdi --steps 20" "merge|--merge-bricks --steps 20" "c1|--config 1 --steps 60" "c3|--config 3 --steps 20" "c4|--config 4 --steps 10"; do
    tag=${m%%|*}; args=${m#*|}
    one ${tag}_old "$OLD" 300 $args || exit 1
    one ${tag}_new "$NEW" 300 $args || exit 1
done
