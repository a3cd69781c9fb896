#!/bin/bash
# Round 3: speculation rules: pass >= 8 (in-tree), >= 7 (sf7), >= 8 or 7 after a fewer step (sr1), >= 9 or 8 after a fewer step (sr1f9)
tools/gpu_session.sh \
 "ab|500|tools/variant_ab.sh sf7 sr1 sr1f9" \
 "emu|300|tools/emu_ab.sh sf7 sr1 sr1f9" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh sf7 sr1 sr1f9"
