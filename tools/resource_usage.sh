#!/bin/bash
# Registers, spills and occupancy of the kernels of one source file (compiler remarks, no GPU):
#   tools/resource_usage.sh [csrc/vdi_generate.hip] [extra hipcc flags...]
# A static check before an A/B goes to the GPU box (the search kernel must stay at <= 168 VGPRs, 3 waves).
cd "$(dirname "$0")/../scenery-insitu_amd" || exit 2
src=${1:-csrc/vdi_generate.hip}; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
    --cuda-device-only -c "$src" -o /tmp/resource_usage.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
python3 -c '
import re, sys
cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: ([\w /\[\]]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
keys = [("VGPRs", "VGPR"), ("AGPRs", "AGPR"), ("VGPRs Spill", "spillV"), ("SGPRs Spill", "spillS"),
        ("Occupancy [waves/SIMD]", "waves"), ("ScratchSize [bytes/lane]", "scratch")]
for k, v in rows.items():
    if "kernel" in k:
        print("%-58s " % k[:58] + " ".join("%s %4s" % (short, v.get(key, "?")) for key, short in keys))
'
