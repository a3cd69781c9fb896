#!/usr/bin/env python3
"""Cross-frame overlap in a rocprofv3 kernel trace of pipelined frames (insitu_frame_pipelined).

For every frame's threshold search (vdi_search_kernel) it reports when the NEXT frame's first pass
(vdi_sample_kernel / vdi_merge_kernel) started relative to the search's start and end, how long the two
ran together, and the period between consecutive searches.  usage:
  tools/overlap.py <dir with *kernel_trace.csv> [> profiles/<tag>/overlap.txt]"""
import csv
import statistics
import sys
from pathlib import Path


def main(d):
    f = next(Path(d).rglob("*kernel_trace.csv"))
    rows = [r for r in csv.DictReader(open(f))]
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda t: t[0])
    first = [k for k in ks if "vdi_sample_kernel" in k[2] or "vdi_merge_kernel" in k[2]]
    search = [k for k in ks if "vdi_search_kernel" in k[2]]
    t0 = ks[0][0]
    print(f"{f.name}: {len(first)} first-pass launches, {len(search)} search launches")
    print("frame  search start..end (ms)  next first pass start  overlap with search (ms)  search period (ms)")
    ov, per = [], []
    for i, (s0, s1, _) in enumerate(search):
        nxt = [k for k in first if k[0] > s0]
        if not nxt:
            continue
        n0, n1, _ = nxt[0]
        o = max(0, min(s1, n1) - max(s0, n0)) / 1e6
        p = (search[i + 1][0] - s0) / 1e6 if i + 1 < len(search) else float("nan")
        ov.append(o)
        if p == p:
            per.append(p)
        print(f"{i:5d}  {(s0 - t0) / 1e6:9.3f}..{(s1 - t0) / 1e6:9.3f}   {(n0 - s0) / 1e6:+9.3f} from start "
              f"({(n0 - s1) / 1e6:+7.3f} from end)  {o:8.3f}  {p:8.3f}")
    if ov:
        print(f"mean overlap {statistics.mean(ov):.3f} ms" + (f", median search period {statistics.median(per):.3f} ms" if per else ""))


if __name__ == "__main__":
    main(sys.argv[1])
