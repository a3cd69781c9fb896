#!/bin/bash
# Round 3: speculative spine levels of pass 1 (2 / 3 against the in-tree 4) on the emulated 8- and 4-GPU shares
tools/gpu_session.sh \
 "emu|300|tools/emu_ab.sh sl2 sl3" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh sl2 sl3" \
 "emu2|300|EMU_WORLD=2 EMU_RANK=1 tools/emu_ab.sh sl3"
