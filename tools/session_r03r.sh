tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh wd" \
 "emuwd|300|tools/emu_ab.sh wd" \
 "w2|300|EMU_WORLD=2 RAY_RANK=-1 tools/emu_ranks.sh" \
 "w4|300|EMU_WORLD=4 RAY_RANK=-1 tools/emu_ranks.sh" \
 "w8|400|EMU_WORLD=8 RAY_RANK=7 tools/emu_ranks.sh"
