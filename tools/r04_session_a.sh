#!/bin/bash
# round-4 first GPU session: tests, default bench, merged-mode profile, counter list
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_session.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "bench|240|python bench.py > gpurun_out/bench_a.json" \
 "counters|60|rocprofv3 -L > gpurun_out/counters.txt 2>&1; grep -c . gpurun_out/counters.txt" \
 "prof_merged|700|PROF_OUT=gpurun_out/prof_merged BENCH_ARGS='--steps 2 --warmup 1 --no-cpu-baseline --merge-bricks' tools/profile_round.sh"
