tools/gpu_session.sh \
 "ab|600|tools/variant_ab.sh cls2 est2 lut0 lut1" \
 "rb|400|STEPS=10 tools/ab_env.sh 'base|X=0' 'rb8|INSITU_ROUND_BATCH=8' 'rb12|INSITU_ROUND_BATCH=12' 'rb28|INSITU_ROUND_BATCH=28' 'rb40|INSITU_ROUND_BATCH=40'" \
 "emu|400|tools/emu_ab.sh cls2 est2 lut0"
