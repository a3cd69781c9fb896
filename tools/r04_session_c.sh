#!/bin/bash
# round 4: compositor workload statistics + profile, merged-bricks profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
 "comp_stats|300|python tools/composite_stats.py > gpurun_out/composite_stats.json" \
 "prof_comp|500|PROF_OUT=gpurun_out/prof_comp BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --compositor vdi --update-every 0' tools/profile_round.sh" \
 "prof_merged|700|PROF_OUT=gpurun_out/prof_merged BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --merge-bricks --update-every 0' tools/profile_round.sh"
