tools/gpu_session.sh \
 "par|300|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'deep or depths or option or group_widths'" \
 "ab|500|STEPS=10 tools/ab_env.sh 'base|X=0' 'dp10|INSITU_DEEP_ITER=10' 'dp12|INSITU_DEEP_ITER=12' 'dp14|INSITU_DEEP_ITER=14' 'dp16|INSITU_DEEP_ITER=16' 'base2|X=0'" \
 "emu|500|EMU=1 STEPS=8 tools/ab_env.sh 'base|X=0' 'dp8|INSITU_DEEP_ITER=8' 'dp10|INSITU_DEEP_ITER=10' 'dp12|INSITU_DEEP_ITER=12' 'dp14|INSITU_DEEP_ITER=14' 'dp16|INSITU_DEEP_ITER=16'" \
 "emu4|400|EMU=1 EMU_W=4 EMU_RANK=2 STEPS=8 tools/ab_env.sh 'base|X=0' 'dp10|INSITU_DEEP_ITER=10' 'dp12|INSITU_DEEP_ITER=12' 'dp14|INSITU_DEEP_ITER=14'"
