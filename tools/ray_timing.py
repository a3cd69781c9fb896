"""Diagnostic: per-ray timing of the search launches for one brick of the bench scene (the per-GPU
work of an 8-GPU run) or all 8 (argument 1).  Runs bench.py's scene with INSITU_DEBUG_RAYS: the
library then records, per search round segment (a ray's stay in one search launch), {start, end,
passes | samples << 8 | group << 24 | launch << 32 | handed-on << 40, pixel | brick << 32}."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
emu = sys.argv[1] if len(sys.argv) > 1 else "8"
path = "/tmp/insitu_rays.bin"
env = dict(os.environ, INSITU_DEBUG_RAYS=path)
args = [sys.executable, str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
if emu != "1":
    args += ["--emulate-world", emu]
subprocess.run(args, env=env, check=True, stdout=subprocess.DEVNULL)
raw = open(path, "rb").read()
HDR = 64   # sizeof(GenCounters)
u32 = np.frombuffer(raw[8:HDR], dtype=np.uint32)
qcount, qhead, fault, qshort = (int(v) for v in u32[:4])
tail_count = [int(v) for v in u32[4:8]]
march = int(u32[12])
e = np.frombuffer(raw[HDR:], dtype=np.uint64).reshape(-1, 4)
t0, t1, meta, key = e[:, 0].astype(np.int64), e[:, 1].astype(np.int64), e[:, 2], e[:, 3]
passes, n, G = meta & 0xFF, (meta >> 8) & 0xFFFF, (meta >> 24) & 0xFF
launch, handed = (meta >> 32) & 0xFF, (meta >> 40) & 1
start = t0.min()
seg_lat = (t1 - t0) / 100.0          # wall_clock64 = 100 MHz -> microseconds
# per ray: first start .. last end over its launches
order = np.lexsort((t0, key))
k_sorted = key[order]
first = np.r_[True, k_sorted[1:] != k_sorted[:-1]]
idx = np.cumsum(first) - 1
nray = int(idx.max()) + 1 if len(idx) else 0
r_start = np.full(nray, np.iinfo(np.int64).max)
r_end = np.zeros(nray, np.int64)
np.minimum.at(r_start, idx, t0[order])
np.maximum.at(r_end, idx, t1[order])
r_pass = np.zeros(nray, np.int64)
np.maximum.at(r_pass, idx, passes[order].astype(np.int64))
r_n = np.zeros(nray, np.int64)
np.maximum.at(r_n, idx, n[order].astype(np.int64))
lat = (r_end - r_start) / 100.0
end = (r_end - start) / 100.0
pop = (r_start - start) / 100.0
span = float(end.max()) if nray else 0.0
out = {"queued": qcount + qshort, "handed_on": tail_count[1:], "uncached_rays": march, "rays_recorded": nray,
       "span_us": span,
       "launch_spans_us": {int(L): [float((t0[launch == L].min() - start) / 100.0), float((t1[launch == L].max() - start) / 100.0)]
                           for L in np.unique(launch)},
       "group_by_launch": {int(L): int(np.median(G[launch == L])) for L in np.unique(launch)},
       "latency_us_pct": {p: float(np.percentile(lat, p)) for p in (50, 90, 99, 99.9, 100)},
       "passes_pct": {p: float(np.percentile(r_pass, p)) for p in (50, 90, 99, 100)},
       "n_pct": {p: float(np.percentile(r_n, p)) for p in (50, 90, 99, 100)},
       "us_per_sample_pass_median": float(np.median(seg_lat / np.maximum(1, n))),
       "slowest": [{"lat_us": float(lat[i]), "pop_us": float(pop[i]), "passes": int(r_pass[i]), "n": int(r_n[i])}
                   for i in np.argsort(-lat)[:5]]}
out["in_flight_at_tenths"] = [int(((pop <= f * span) & (end > f * span)).sum()) for f in np.arange(0.0, 1.0, 0.1)]
out["done_frac_at_tenths"] = [float((end <= f * span).mean()) for f in np.arange(0.1, 1.01, 0.1)]
print(json.dumps(out))
