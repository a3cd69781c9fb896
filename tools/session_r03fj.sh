#!/bin/bash
# Round 3: speculative stores from pass 7 / 8 / 9 on (sf7..9) against every search pass (in-tree) and none (sw0)
tools/gpu_session.sh \
 "ab|500|tools/variant_ab.sh sw0 sf7 sf8 sf9" \
 "emu|300|tools/emu_ab.sh sw0 sf7 sf8 sf9" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh sw0 sf7 sf8 sf9"
