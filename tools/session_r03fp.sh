#!/bin/bash
# Round 3: tree-group children stage their speculative passes (in-tree) against ss0 (root only); parity
tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "emu|300|tools/emu_ab.sh ss0" \
 "emu8b|300|EMU_WORLD=8 EMU_RANK=5 tools/emu_ab.sh ss0" \
 "ab|400|tools/variant_ab.sh ss0"
