#!/bin/bash
# Builds libinsitu_hip.so of a git revision as an A/B variant (tools/variant_ab.sh):
#   tools/rev_variant.sh REV NAME [EXTRA_FLAGS]  ->  scenery-insitu_amd/lib/variants/libinsitu_hip_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2; EXTRA=$3
WT=$(mktemp -d /tmp/insitu_rev_XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
make -s -C "$WT/scenery-insitu_amd" ARCH=gfx950 CXXFLAGS_EXTRA="$EXTRA" -j8
mkdir -p "$ROOT/scenery-insitu_amd/lib/variants"
cp "$WT/scenery-insitu_amd/lib/libinsitu_hip.so" "$ROOT/scenery-insitu_amd/lib/variants/libinsitu_hip_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built lib/variants/libinsitu_hip_$NAME.so from $(git -C "$ROOT" rev-parse --short "$REV")"
