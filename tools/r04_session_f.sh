#!/bin/bash
# round 4: profile of the VDICompositor mode with the queued search
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
 "prof_compq|500|PROF_OUT=gpurun_out/prof_compq BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --compositor vdi --update-every 0' tools/profile_round.sh"
