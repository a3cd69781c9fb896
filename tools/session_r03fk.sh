#!/bin/bash
# Round 3: the speculative-store build (8075dae): tests, bench, profiles, modes, emulated shares
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py > gpurun_out/bench_s.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03s tools/profile_round.sh" \
 "deep|600|PROF_OUT=gpurun_out/deep_r03s tools/pmc_deep.sh" \
 "modes|900|OUT=gpurun_out/modes_s tools/modes_round.sh" \
 "w8|400|EMU_WORLD=8 RAY_RANK=7 tools/emu_ranks.sh" \
 "w4|300|EMU_WORLD=4 RAY_RANK=3 tools/emu_ranks.sh" \
 "w2|300|EMU_WORLD=2 RAY_RANK=1 tools/emu_ranks.sh"
