tools/gpu_session.sh \
 "ab|600|tools/variant_ab.sh len2 logexp2 cls2v" \
 "emu|400|tools/emu_ab.sh len2 logexp2 cls2v"
