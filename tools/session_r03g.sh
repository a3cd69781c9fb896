tools/gpu_session.sh \
 "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "ab1|500|STEPS=10 tools/ab_env.sh 'base|X=0' 'ov12|INSITU_SEARCH_OVERSUB=12' 'rb12|INSITU_ROUND_BATCH=12' 'rb28|INSITU_ROUND_BATCH=28' 'base2|X=0'" \
 "ab8|500|EMU=1 STEPS=10 tools/ab_env.sh 'base|X=0' 'd3|INSITU_SEARCH_DEPTH=3' 'd4|INSITU_SEARCH_DEPTH=4' 'ov12|INSITU_SEARCH_OVERSUB=12' 'ov24|INSITU_SEARCH_OVERSUB=24' 'base2|X=0'"
