"""Diagnostic: per-ray timing of the search kernel for one brick of the bench scene (the per-GPU
work of an 8-GPU run) or all 8 (--bricks 8).  Runs bench.py's scene with INSITU_DEBUG_RAYS."""
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
cursor, qcount, qhead = np.frombuffer(raw[:16], dtype=np.uint64)[0], *np.frombuffer(raw[8:16], dtype=np.uint32)
e = np.frombuffer(raw[16:], dtype=np.uint64).reshape(-1, 4)
t0, t1 = e[:, 0].astype(np.int64), e[:, 1].astype(np.int64)
ok = t1 > 0
t0, t1, meta = t0[ok], t1[ok], e[ok, 2]
passes, n, G = meta & 0xFF, (meta >> 8) & 0xFFFF, meta >> 24
start = t0.min()
lat = (t1 - t0) / 100.0          # wall_clock64 = 100 MHz -> microseconds
end = (t1 - start) / 100.0
pop = (t0 - start) / 100.0
out = {"queued": int(qcount), "recorded": int(ok.sum()), "group": int(np.median(G)),
       "span_us": float(end.max()),
       "latency_us_pct": {p: float(np.percentile(lat, p)) for p in (50, 90, 99, 99.9, 100)},
       "pop_us_pct": {p: float(np.percentile(pop, p)) for p in (50, 90, 99, 100)},
       "passes_pct": {p: float(np.percentile(passes, p)) for p in (50, 90, 99, 100)},
       "n_pct": {p: float(np.percentile(n, p)) for p in (50, 90, 99, 100)},
       "us_per_sample_pass_median": float(np.median(lat / np.maximum(1, (passes - 1) * n))),
       "slowest": [{"lat_us": float(lat[i]), "pop_us": float(pop[i]), "passes": int(passes[i]), "n": int(n[i])}
                   for i in np.argsort(-lat)[:5]]}
span = end.max()
# concurrency profile: rays in flight and popped-so-far at tenths of the span
out["in_flight_at_tenths"] = [int(((pop <= f * span) & (end > f * span)).sum()) for f in np.arange(0.0, 1.0, 0.1)]
out["done_frac_at_tenths"] = [float((end <= f * span).mean()) for f in np.arange(0.1, 1.01, 0.1)]
out["queue_drained_us"] = float(pop.max())
late = end > 0.7 * span
out["late_rays"] = {"count": int(late.sum()), "pop_us_pct": {p: float(np.percentile(pop[late], p)) for p in (0, 50, 100)},
                    "passes_pct": {p: float(np.percentile(passes[late], p)) for p in (0, 50, 100)},
                    "n_pct": {p: float(np.percentile(n[late], p)) for p in (0, 50, 100)},
                    "group_hist": np.bincount(G[late].astype(np.int64)).tolist()} if late.any() else {}
print(json.dumps(out))
