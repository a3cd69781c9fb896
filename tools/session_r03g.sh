tools/gpu_session.sh \
 "ab1|500|STEPS=10 tools/ab_env.sh 'base|X=0' 'ov12|INSITU_SEARCH_OVERSUB=12' 'rb12|INSITU_ROUND_BATCH=12' 'rb28|INSITU_ROUND_BATCH=28' 'base2|X=0'" \
 "ab8|500|EMU=1 STEPS=10 tools/ab_env.sh 'base|X=0' 'd3|INSITU_SEARCH_DEPTH=3' 'd4|INSITU_SEARCH_DEPTH=4' 'ov12|INSITU_SEARCH_OVERSUB=12' 'ov24|INSITU_SEARCH_OVERSUB=24' 'base2|X=0'" \
 "rays|300|python tools/ray_timing.py 1 > gpurun_out/rays1_r03g.json && python tools/ray_timing.py 8 7 > gpurun_out/rays8_r03g.json"
