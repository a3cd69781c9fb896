tools/gpu_session.sh \
 "par|600|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_stg.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "ab|400|tools/variant_ab.sh stg" \
 "emu|300|tools/emu_ab.sh stg" \
 "merge|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_stg.so python bench.py --merge-bricks --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/stg_merge.json" \
 "pmcf|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_stg.so timeout -k 10 250 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex vdi_s -d gpurun_out/prof_stg/pmc_fetch -o pmc_fetch -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_stg.log 2>&1" \
 "pmcw|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_stg.so timeout -k 10 250 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex vdi_s -d gpurun_out/prof_stg/pmc_write -o pmc_write -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_stgw.log 2>&1"
