tools/gpu_session.sh \
 "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "knobs|500|STEPS=10 tools/ab_env.sh 'base|X=0' 'rb24|INSITU_ROUND_BATCH=24' 'rb28|INSITU_ROUND_BATCH=28' 'ov5|INSITU_SEARCH_OVERSUB=5' 'ov8|INSITU_SEARCH_OVERSUB=8' 'base2|X=0'" \
 "knobs8|400|EMU=1 STEPS=8 tools/ab_env.sh 'base|X=0' 'rb24|INSITU_ROUND_BATCH=24' 'rb28|INSITU_ROUND_BATCH=28' 'ov5|INSITU_SEARCH_OVERSUB=5' 'ov8|INSITU_SEARCH_OVERSUB=8'" \
 "bench|300|python bench.py > gpurun_out/bench_y.json"
