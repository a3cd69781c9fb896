tools/gpu_session.sh \
 "d8|400|EMU=1 STEPS=8 tools/ab_env.sh 'base|X=0' 'd1|INSITU_SEARCH_DEPTH=1' 'd2|INSITU_SEARCH_DEPTH=2' 'd3|INSITU_SEARCH_DEPTH=3' 'ov3|INSITU_SEARCH_OVERSUB=3' 'ov12|INSITU_SEARCH_OVERSUB=12'" \
 "d4r3|400|EMU=1 EMU_W=4 EMU_RANK=3 STEPS=8 tools/ab_env.sh 'base|X=0' 'd1|INSITU_SEARCH_DEPTH=1' 'd2|INSITU_SEARCH_DEPTH=2'" \
 "rays|300|python tools/ray_timing.py 8 7 > gpurun_out/rays8_r03o.json && python tools/ray_timing.py 1 > gpurun_out/rays1_r03o.json"
