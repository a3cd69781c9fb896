tools/gpu_session.sh \
 "merged|300|python -u -m pytest tests/test_gpu_parity.py -k merged -x -q --timeout 200 --timeout-method thread" \
 "merge|300|python bench.py --merge-bricks --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_merge.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03e tools/profile_round.sh" \
 "deep|600|PROF_OUT=gpurun_out/deep_r03e tools/pmc_deep.sh" \
 "rays1|200|python tools/ray_timing.py 1 > gpurun_out/rays1_r03e.json" \
 "rays8|200|python tools/ray_timing.py 8 7 > gpurun_out/rays8_r03e.json"
