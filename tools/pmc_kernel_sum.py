#!/usr/bin/env python3
"""Per-kernel mean of every counter in one rocprofv3 --pmc output directory (one line per kernel):
usage: tools/pmc_kernel_sum.py gpurun_out/pmc/<tag> [label]"""
import collections
import csv
import sys
from pathlib import Path

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in Path(sys.argv[1]).rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("insitu::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
label = sys.argv[2] if len(sys.argv) > 2 else ""
for k in sorted(tot):
    vals = {c: v / max(1, len(disp[(k, c)])) for c, v in tot[k].items()}
    # FETCH_SIZE / WRITE_SIZE are KiB; the gfx950 x2 for reads (profiles/r04_calib)
    s = " ".join(f"{c}={v / 1048576:.3f}GiB" if c in ("FETCH_SIZE", "WRITE_SIZE") else f"{c}={v:.4g}"
                 for c, v in sorted(vals.items()))
    print(label, k, s)
