#!/usr/bin/env python3
"""Summarise tools/pmc_deep.sh output: per kernel, the mean per dispatch of every counter collected.
usage: tools/pmc_deep_summary.py gpurun_out/deep profiles/<tag>/deep_summary.json"""
import collections
import csv
import json
import sys
from pathlib import Path


def main(src: str, dst: str) -> None:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in Path(src).rglob("*_counter_collection.csv"):
        per = collections.defaultdict(float)   # (kernel, dispatch, counter) summed over dimensions
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("insitu::", "")
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    out = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in sorted(acc.items())}
    for k, cs in out.items():
        if "TA_TA_BUSY_sum" in cs and "GRBM_GUI_ACTIVE" in cs and cs["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; one TA per CU (256)
            cs["ta_busy_frac_per_ta"] = cs["TA_TA_BUSY_sum"] / (cs["GRBM_GUI_ACTIVE"] / 8.0) / 256.0
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            cs["lds_bank_conflict_frac"] = cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / cs["SQ_LDS_IDX_ACTIVE"]
        if cs.get("TCP_TCC_READ_REQ_sum"):
            cs["tcp_tcc_read_latency_cycles"] = cs.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / cs["TCP_TCC_READ_REQ_sum"]
    Path(dst).parent.mkdir(parents=True, exist_ok=True)
    Path(dst).write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
