tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "modes|600|python bench.py --mode plain --steps 20 --no-cpu-baseline > gpurun_out/bench_plain.json && python bench.py --compositor vdi --steps 10 --no-cpu-baseline > gpurun_out/bench_cvdi.json && python bench.py --merge-bricks --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_merge.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03f tools/profile_round.sh" \
 "deep|600|PROF_OUT=gpurun_out/deep_r03f tools/pmc_deep.sh" \
 "rays|300|python tools/ray_timing.py 1 > gpurun_out/rays1_r03f.json && python tools/ray_timing.py 8 7 > gpurun_out/rays8_r03f.json"
