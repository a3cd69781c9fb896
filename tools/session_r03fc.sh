#!/bin/bash
# Round 3: fast pass restart -- without the stale-children trigger (frns), and lane diagnostics of both builds
V=scenery-insitu_amd/lib/variants
tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh fr0 frns" \
 "emu|300|tools/emu_ab.sh fr0 frns" \
 "diagfr|200|INSITU_HIP_LIB=$V/libinsitu_hip_frdiag.so python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/diagfr.json 2> gpurun_out/diagfr.err; grep diag gpurun_out/diagfr.err | tail -6" \
 "diagfr0|200|INSITU_HIP_LIB=$V/libinsitu_hip_fr0diag.so python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/diagfr0.json 2> gpurun_out/diagfr0.err; grep diag gpurun_out/diagfr0.err | tail -6"
