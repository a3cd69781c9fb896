#!/bin/bash
# Round 3: whole-chunk replay trips without per-sample tests (in-tree) against pc0 (without); parity
tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh pc0" \
 "emu|300|tools/emu_ab.sh pc0" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh pc0" \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
