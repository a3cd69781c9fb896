tools/gpu_session.sh \
 "par|600|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_lc.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "ab|400|tools/variant_ab.sh trim lc" \
 "emu|300|tools/emu_ab.sh trim lc" \
 "emu4|300|EMU_WORLD=4 EMU_RANK=2 tools/emu_ab.sh lc"
