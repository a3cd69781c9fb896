tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py > gpurun_out/bench_head.json" \
 "emu|300|python bench.py --emulate-world 8 --emulate-rank 7 --steps 10 --no-cpu-baseline > gpurun_out/bench_w8r7.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03h tools/profile_round.sh"
