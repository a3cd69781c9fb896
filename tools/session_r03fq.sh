#!/bin/bash
# Round 3: round batch 28 / 32 against 20 at N=1, repeated
tools/gpu_session.sh \
 "knobs|500|STEPS=12 tools/ab_env.sh 'base|X=0' 'rb28|INSITU_ROUND_BATCH=28' 'rb32|INSITU_ROUND_BATCH=32' 'base2|X=0' 'rb28b|INSITU_ROUND_BATCH=28' 'base3|X=0'"
