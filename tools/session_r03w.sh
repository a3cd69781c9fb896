tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh fb8 fb12 fb20" \
 "par|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_fb8.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bit_exact or config1'" \
 "kt|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_fb8.so timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_fb8 -o kt -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_fb8.log 2>&1"
