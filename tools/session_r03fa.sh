#!/bin/bash
# Round 3: fast pass restart (INSITU_FAST_RESTART, in-tree) vs without (fr0): parity tests, N=1 and
# one-brick-share A/B; smoke and the self-launched two-rank bench
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "ab|400|tools/variant_ab.sh fr0" \
 "emu|300|tools/emu_ab.sh fr0" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "gpus2|400|python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/gpus2.json"
