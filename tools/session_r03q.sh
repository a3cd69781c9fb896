tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py > gpurun_out/bench_q.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03q tools/profile_round.sh" \
 "deep|600|PROF_OUT=gpurun_out/deep_r03q tools/pmc_deep.sh" \
 "modes|900|OUT=gpurun_out/modes_q tools/modes_round.sh"
