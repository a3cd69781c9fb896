#!/bin/bash
# Builds a variant of libinsitu_hip.so with extra compile flags (experiments and diagnostics):
#   tools/variant_build.sh NAME "-DINSITU_DIAG ..."  ->  scenery-insitu_amd/lib/variants/libinsitu_hip_NAME.so
# Run it with INSITU_HIP_LIB=scenery-insitu_amd/lib/variants/libinsitu_hip_NAME.so (insitu_amd/native.py).
set -e
cd "$(dirname "$0")/../scenery-insitu_amd"
NAME=$1; EXTRA=$2
make -s OBJ=build/variant_$NAME OUT=lib/variants ARCH=gfx950 CXXFLAGS_EXTRA="$EXTRA" lib/variants/libinsitu_hip.so
mv lib/variants/libinsitu_hip.so lib/variants/libinsitu_hip_$NAME.so
echo "built lib/variants/libinsitu_hip_$NAME.so"
