tools/gpu_session.sh \
 "probe|300|python tools/concurrency_probe.py --iters 4" \
 "diag|200|INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_diag.so python bench.py --steps 1 --warmup 1 --no-cpu-baseline" \
 "rays1|200|python tools/ray_timing.py 1" \
 "rays8|200|python tools/ray_timing.py 8 7" \
 "lgroup|300|python tools/local_group_frame.py --ranks 8 --frames 2 --out gpurun_out/local_group_w8.json" \
 "prof|900|PROF_OUT=gpurun_out/prof_r03b tools/profile_round.sh"
