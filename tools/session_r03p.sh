tools/gpu_session.sh \
 "par|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_pk4.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "ab|600|tools/variant_ab.sh pk2 pk4" \
 "emu|400|tools/emu_ab.sh pk2 pk4"
