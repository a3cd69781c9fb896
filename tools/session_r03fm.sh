#!/bin/bash
# Round 3: speculative stores from pass 7 (g7) or 6 (g6) with tree groups, 8 without, against 8 everywhere (in-tree)
tools/gpu_session.sh \
 "emu|300|tools/emu_ab.sh g7 g6" \
 "emu8b|300|EMU_WORLD=8 EMU_RANK=5 tools/emu_ab.sh g7 g6" \
 "ab|400|tools/variant_ab.sh g7"
