#!/bin/bash
# Round 3 close: GPU tests, smoke and the default bench line at HEAD
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|400|python bench.py > gpurun_out/bench_final.json"
