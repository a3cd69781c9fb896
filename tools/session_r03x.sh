tools/gpu_session.sh \
 "par|600|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_share.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "ab|400|tools/variant_ab.sh share" \
 "ab2|400|tools/variant_ab.sh share" \
 "emu|300|tools/emu_ab.sh share"
