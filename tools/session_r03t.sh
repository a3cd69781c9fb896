tools/gpu_session.sh \
 "ab|400|tools/variant_ab.sh il2 il4" \
 "emu|300|tools/emu_ab.sh il4" \
 "pmc4|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_il4.so PROF_OUT=gpurun_out/prof_il4 timeout -k 10 250 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex vdi_s -d gpurun_out/prof_il4/pmc_fetch -o pmc_fetch -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_il4.log 2>&1" \
 "pmc4w|300|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_il4.so timeout -k 10 250 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex vdi_s -d gpurun_out/prof_il4/pmc_write -o pmc_write -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_il4w.log 2>&1"
