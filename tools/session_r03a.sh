tools/gpu_session.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --steps 20 --warmup 3 > gpurun_out/bench_r03a.json" \
 "ab|400|tools/variant_ab.sh lut0 lut1" \
 "lgroup|300|python tools/local_group_frame.py --ranks 8 --frames 2 --out gpurun_out/local_group_w8.json" \
 "trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03a -o trace -f csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
