#!/usr/bin/env python3
"""Summarise the `calib` session of tools/gpu_round.sh into profiles/<tag>/fetch_calib.json.

For the known-byte kernels of tools/fetch_calib.hip: FETCH_SIZE per launch (KiB in the CSV) against the
requested bytes and against the 128-byte lines they touch, and the read-request size split
(TCC_EA0_RDREQ_{32B,64B,128B}); for the bench's kernels the same split, so the search kernel's measured
FETCH_SIZE can be corrected with the factor its own access pattern calibrates.
usage: tools/fetch_calib.py gpurun_out/calib profiles/<tag>"""
import collections
import csv
import json
import sys
from pathlib import Path


def per_kernel(path_glob, src):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in src.glob(path_glob):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("insitu::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main(src, dst):
    src, dst = Path(src), Path(dst)
    dst.mkdir(parents=True, exist_ok=True)
    known = json.loads((src / "bytes.json").read_text())
    fetch = per_kernel("fetch/**/*counter_collection.csv", src)
    split = per_kernel("split/**/*counter_collection.csv", src)
    bench = per_kernel("bench_split/**/*counter_collection.csv", src)
    out = {"patterns": {}, "bench_kernels": {}}
    for k, kb in known.items():
        f = fetch.get(k, {}).get("FETCH_SIZE")
        s = split.get(k, {})
        rq = {w: s.get(f"TCC_EA0_RDREQ_{w}B_sum") for w in (32, 64, 128)}
        out["patterns"][k] = {
            "requested_bytes": kb["bytes"], "line_bytes": kb["lines_bytes"],
            "fetch_size_bytes": f * 1024 if f is not None else None,
            "fetch_over_requested": f * 1024 / kb["bytes"] if f else None,
            "fetch_over_lines": f * 1024 / kb["lines_bytes"] if f else None,
            "rdreq": s.get("TCC_EA0_RDREQ_sum"), "rdreq_by_size": rq,
            "rdreq_bytes_by_size": sum((w * n) for w, n in rq.items() if n) if any(rq.values()) else None}
    for k, s in bench.items():
        rq = {w: s.get(f"TCC_EA0_RDREQ_{w}B_sum") for w in (32, 64, 128)}
        out["bench_kernels"][k] = {"rdreq": s.get("TCC_EA0_RDREQ_sum"), "rdreq_by_size": rq,
                                   "rdreq_bytes_by_size": sum((w * n) for w, n in rq.items() if n) if any(rq.values()) else None}
    (dst / "fetch_calib.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
