#!/bin/bash
# Round 3: build with group-dependent speculation: tests, bench, profile, 8-GPU emulated shares
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py > gpurun_out/bench_t.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03t tools/profile_round.sh" \
 "w8|400|EMU_WORLD=8 RAY_RANK=7 tools/emu_ranks.sh"
