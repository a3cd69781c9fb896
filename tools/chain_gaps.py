#!/usr/bin/env python3
"""Gaps in the chain of first passes (and of searches) of pipelined frames in a rocprofv3 kernel trace: with
the first pass of frame k+1 started at once beside frame k's search (trigger 2), the GPU's work per frame is
bounded by the slower of the two chains, and a gap between consecutive first passes is time that chain waited
(for the host's next call, or for a slot's completion).  usage: tools/chain_gaps.py <dir with *kernel_trace.csv>"""
import csv
import statistics
import sys
from pathlib import Path


def main(d):
    f = next(Path(d).rglob("*kernel_trace.csv"))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
    for name in ("vdi_sample_kernel", "vdi_search_kernel"):
        ev = [(s, e) for s, e, n in ks if name in n]
        gaps = [(ev[i + 1][0] - ev[i][1]) / 1e6 for i in range(len(ev) - 1)]
        durs = [(e - s) / 1e6 for s, e in ev]
        per = [(ev[i + 1][0] - ev[i][0]) / 1e6 for i in range(len(ev) - 1)]
        print(f"{name}: {len(ev)} launches; durations " + " ".join("%.2f" % x for x in durs))
        print("   gap to the next launch " + " ".join("%.2f" % x for x in gaps))
        if len(per) > 4:
            print(f"   median period {statistics.median(per[2:]):.3f} ms, median gap {statistics.median(gaps[2:]):.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
