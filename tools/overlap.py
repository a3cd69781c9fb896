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
    # how much of the steady state has any kernel running (union of the kernel intervals between the second
    # and the last search start): 1 - busy = the GPU's idle share
    if len(search) >= 3:
        a, b = search[1][0], search[-1][0]
        iv = sorted((max(k[0], a), min(k[1], b)) for k in ks if k[1] > a and k[0] < b)
        busy, cur0, cur1 = 0, None, None
        for s0, s1 in iv:
            if cur1 is None or s0 > cur1:
                if cur1 is not None:
                    busy += cur1 - cur0
                cur0, cur1 = s0, s1
            else:
                cur1 = max(cur1, s1)
        if cur1 is not None:
            busy += cur1 - cur0
        print(f"steady state {(b - a) / 1e6:.3f} ms over {len(search) - 2} frames: some kernel running "
              f"{busy / (b - a):.3f} of the time (idle {(b - a - busy) / 1e6 / (len(search) - 2):.3f} ms per frame)")


if __name__ == "__main__":
    main(sys.argv[1])
