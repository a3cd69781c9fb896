tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py > gpurun_out/bench_main.json" \
 "plain|200|python bench.py --mode plain --steps 20 --no-cpu-baseline > gpurun_out/bench_plain.json" \
 "cvdi|200|python bench.py --compositor vdi --steps 10 --no-cpu-baseline > gpurun_out/bench_cvdi.json" \
 "merge|300|python bench.py --merge-bricks --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_merge.json" \
 "emu8|200|python bench.py --emulate-world 8 --emulate-rank 7 --steps 10 --no-cpu-baseline > gpurun_out/bench_w8r7.json"
