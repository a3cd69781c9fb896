#!/bin/bash
# Round 3: speculative stores in the root's search passes (in-tree) against sw0 (write passes only); parity
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "ab|400|tools/variant_ab.sh sw0" \
 "emu|300|tools/emu_ab.sh sw0" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh sw0"
