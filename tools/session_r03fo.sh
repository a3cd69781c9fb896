#!/bin/bash
# Round 3: round batch / oversubscription re-sweep after the speculative stores
tools/gpu_session.sh \
 "knobs|500|STEPS=10 tools/ab_env.sh 'base|X=0' 'rb16|INSITU_ROUND_BATCH=16' 'rb24|INSITU_ROUND_BATCH=24' 'rb28|INSITU_ROUND_BATCH=28' 'base2|X=0'" \
 "knobs8|400|EMU=1 STEPS=8 tools/ab_env.sh 'base|X=0' 'rb16|INSITU_ROUND_BATCH=16' 'rb24|INSITU_ROUND_BATCH=24' 'ov4|INSITU_SEARCH_OVERSUB=4' 'ov8|INSITU_SEARCH_OVERSUB=8' 'base2|X=0'"
