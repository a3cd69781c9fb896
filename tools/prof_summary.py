#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/<tag>/.

Per insitu kernel: calls, mean duration (kernel trace), and from the PMC passes (one run each):
HBM traffic per launch = FETCH_SIZE*2 + WRITE_SIZE (KiB units; FETCH_SIZE doubled for the gfx950
wide-read halving, MI355X_MICROARCH.md "HBM"), L2 hit rate, VALU issue utilisation
(SQ_INSTS_VALU / (CUs * SIMDs * clock/2 * duration)), lane utilisation
(SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)), wave-cycle split (SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES).
usage: tools/prof_summary.py gpurun_out/prof profiles/r01_<tag>
"""
from __future__ import annotations

import collections
import csv
import json
import shutil
import sys
from pathlib import Path


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("insitu::", "")
    return n


def main(src: str, dst: str) -> None:
    src_p, dst_p = Path(src), Path(dst)
    dst_p.mkdir(parents=True, exist_ok=True)
    kern = {}
    # a gpurun_out/prof run directory (trace/, pmc_*/), or a committed profiles/<tag> directory
    # (kernel_stats.csv, pmc_*.csv: re-summarised in place, its _config kept)
    committed = not (src_p / "trace").exists() and (src_p / "kernel_stats.csv").exists()
    for f in (src_p.glob("kernel_stats.csv") if committed else src_p.glob("trace/*kernel_stats.csv")):
        if f.resolve() != (dst_p / "kernel_stats.csv").resolve():
            shutil.copy(f, dst_p / "kernel_stats.csv")
        for r in csv.DictReader(open(f)):
            kern[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                      "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in (src_p.glob("pmc_*.csv") if committed else src_p.glob("pmc_*/*counter_collection.csv")):
        if not committed:
            shutil.copy(f, dst_p / (f.parent.name + ".csv"))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, c in cnt.items():
        def per(name):
            n = len(disp.get((k, name), ())) or 1
            return c.get(name, 0.0) / n
        d = dict(kern.get(k, {}))
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes_per_launch"] = (2.0 * per("FETCH_SIZE") + per("WRITE_SIZE")) * 1024.0
            d["fetch_bytes_per_launch_raw"] = per("FETCH_SIZE") * 1024.0
            d["write_bytes_per_launch"] = per("WRITE_SIZE") * 1024.0
        if "TCC_HIT_sum" in c:
            d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
            # x2: on gfx950 (SIMD32, a wave64 VALU op spans 2 cycles) a divergence-free kernel
            # (brick_ingest, assemble_columns) reads 0.5 with the plain ratio
            d["lane_utilisation"] = 2.0 * c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    d[n.lower() + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in c and d.get("avg_ms"):
            d["valu_wave_insts_per_launch"] = per("SQ_INSTS_VALU")
            # 256 CUs x 4 SIMD32, one wave64 VALU op per 2 cycles per SIMD at ~2.4 GHz
            d["valu_issue_utilisation"] = per("SQ_INSTS_VALU") / (256 * 4 * 2.4e9 / 2 * d["avg_ms"] * 1e-3)
        if "SQ_INSTS_SALU" in c:
            d["salu_wave_insts_per_launch"] = per("SQ_INSTS_SALU")
        if "SQ_INSTS_VMEM_RD" in c:
            d["vmem_rd_wave_insts_per_launch"] = per("SQ_INSTS_VMEM_RD")
        # effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall time: within 3 % of the in-kernel clock for
        # dispatches of >= 10 ms, high on short ones (MI355X_MICROARCH.md, DVFS give-back): >= 5 ms only
        if "GRBM_GUI_ACTIVE" in c and d.get("avg_ms", 0.0) >= 5.0:
            d["clock_ghz"] = per("GRBM_GUI_ACTIVE") / 8.0 / (d["avg_ms"] * 1e-3) / 1e9
        out[k] = d
    for k, v in kern.items():
        out.setdefault(k, v)
    if committed and (dst_p / "summary.json").exists():
        prev = json.loads((dst_p / "summary.json").read_text()).get("_config")
        if prev:
            out["_config"] = prev
    if len(sys.argv) > 3:   # the bench arguments the profile ran (bench.py's pmc_traffic picks N=1 summaries)
        out["_config"] = {"bench_args_n1": sys.argv[3]}
    # the sources the profiled kernels were built from: the hash profile_round.sh took on the box, else the
    # tree's (bench.py withholds the profile's figures when it differs from the tree it runs from)
    hf = src_p / "csrc_sha16.txt"
    sha = hf.read_text().strip() if hf.exists() else None
    if sha is None and not committed:
        sys.path.insert(0, str(Path(__file__).resolve().parent))
        from src_hash import csrc_hash
        sha = csrc_hash()
    if sha:
        out.setdefault("_config", {})["csrc_sha16"] = sha
        if hf.exists() and hf.resolve() != (dst_p / "csrc_sha16.txt").resolve():
            shutil.copy(hf, dst_p / "csrc_sha16.txt")
    (dst_p / "summary.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])  # optional argv[3]: bench args of an N=1 config-2 run
