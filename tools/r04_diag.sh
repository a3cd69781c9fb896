#!/bin/bash
# round 4: per-ray timeline of the fused generator (N=1 and the one-brick share) against the two launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_session.sh \
 "rt_n1_fused|200|python tools/ray_timing.py 1 0 --option fused=1 > gpurun_out/rt_n1_fused.json" \
 "rt_w8r7_fused|200|python tools/ray_timing.py 8 7 --option fused=1 > gpurun_out/rt_w8r7_fused.json" \
 "rt_w8r7_classic|200|python tools/ray_timing.py 8 7 --option fused=0 > gpurun_out/rt_w8r7_classic.json"
