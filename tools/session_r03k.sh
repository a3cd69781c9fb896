tools/gpu_session.sh \
 "ab|600|tools/variant_ab.sh cls2 cls2b cls2v lut0 lut3" \
 "lut3par|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_lut3.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bit_exact'"
