tools/gpu_session.sh \
 "diag|200|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_diag.so python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/diag1.json 2> gpurun_out/diag1.err; grep diag gpurun_out/diag1.err | tail -6" \
 "diag8|200|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_diag.so python bench.py --steps 1 --warmup 1 --no-cpu-baseline --emulate-world 8 --emulate-rank 7 > gpurun_out/diag8.json 2> gpurun_out/diag8.err; grep diag gpurun_out/diag8.err | tail -6"
