#!/usr/bin/env python3
"""Launch durations of the frame's short kernels in a rocprofv3 kernel trace of pipelined frames.

A kernel launched while a persistent search kernel holds every CU's wave slots waits until that search's
queue drains, so its traced duration jumps from tenths of a millisecond to milliseconds.
Prints each kernel's per-launch durations (the first `skip` launches dropped: the warmup frames) and how
many exceed `slow_ms`.  usage: tools/starved.py <dir with *kernel_trace.csv> [skip=4] [slow_ms=1.0]"""
import csv
import sys
from pathlib import Path

SHORT = ("vdi_finish", "vdi_flatten", "assemble_columns", "copyBuffer", "vdi_tile_len", "vdi_compact", "vdi_composite")
LONG = ("vdi_sample", "vdi_merge", "vdi_search")


def main(d, skip=4, slow_ms=1.0):
    f = next(Path(d).rglob("*kernel_trace.csv"))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                for r in csv.DictReader(open(f)))
    print(f"{f.name}: per-launch durations in ms (first {skip} launches of each kernel dropped)")
    for name in SHORT + LONG:
        ds = [(e - s) / 1e6 for s, e, n in ks if name in n][skip:]
        if not ds:
            continue
        slow = "" if name in LONG else f"   (> {slow_ms:g} ms: {sum(x > slow_ms for x in ds)} of {len(ds)})"
        print(f"  {name:17s} " + " ".join("%.2f" % x for x in ds) + slow)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4, float(sys.argv[3]) if len(sys.argv) > 3 else 1.0)
