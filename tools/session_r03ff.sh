#!/bin/bash
# Round 3: per-ray search rounds (INSITU_DEBUG_REPLAYS build) on the one-brick share and at N=1
V=scenery-insitu_amd/lib/variants
tools/gpu_session.sh \
 "rt8|300|INSITU_HIP_LIB=$V/libinsitu_hip_dbgrep.so python tools/ray_timing.py 8 7 > gpurun_out/rt8.json" \
 "rt1|300|INSITU_HIP_LIB=$V/libinsitu_hip_dbgrep.so python tools/ray_timing.py 1 > gpurun_out/rt1.json"
