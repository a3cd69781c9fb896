#!/bin/bash
# Round 3: search kernel classifying two samples ahead at 4 waves per SIMD (a2w4) and 3 (a2w3), against the
# in-tree build (cold per-ray state out of VGPRs); parity of a2w4
V=scenery-insitu_amd/lib/variants
tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh a2w4 a2w3" \
 "emu|300|tools/emu_ab.sh a2w4 a2w3" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=3 tools/emu_ab.sh a2w4" \
 "gputests|700|INSITU_HIP_LIB=$V/libinsitu_hip_a2w4.so python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
