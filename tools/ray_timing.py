"""Diagnostic: per-ray timing of the search kernel for one brick of the bench scene (the per-GPU
work of an 8-GPU run, argument 1 = N, argument 2 = the emulated rank) or all 8 (argument 1 = 1);
further arguments go to bench.py.
Runs bench.py's scene with INSITU_DEBUG_RAYS: the library then records, per queued ray,
{pop, done, passes | samples << 8 | group << 24, pixel | brick << 32} in wall_clock64 ticks
(written at the next insitu_synchronize)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
emu = sys.argv[1] if len(sys.argv) > 1 else "8"
emu_rank = sys.argv[2] if len(sys.argv) > 2 else "0"
path = "/tmp/insitu_rays.bin"
env = dict(os.environ, INSITU_DEBUG_RAYS=path)
args = [sys.executable, str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
if emu != "1":
    args += ["--emulate-world", emu, "--emulate-rank", emu_rank]
args += sys.argv[3:]   # extra bench.py arguments (e.g. --option round_batch=28)
subprocess.run(args, env=env, check=True, stdout=subprocess.DEVNULL)
raw = open(path, "rb").read()
HDR = 4 + int(np.frombuffer(raw[:4], dtype=np.uint32)[0])   # u32 sizeof(GenCounters), then GenCounters
u32 = np.frombuffer(raw[12:HDR], dtype=np.uint32)
qcount, qhead, fault, qshort, march = (int(v) for v in u32[:5])
regroups = int(u32[8]) if len(u32) > 8 else 0   # GenCounters.regroups (after cache_need)
e = np.frombuffer(raw[HDR:], dtype=np.uint64).reshape(-1, 4)
t0, t1, meta = e[:, 0].astype(np.int64), e[:, 1].astype(np.int64), e[:, 2]
passes, n, G = meta & 0xFF, (meta >> 8) & 0xFFFF, (meta >> 24) & 0xFF
rounds = (meta >> 32) & 0xFFFF   # INSITU_DEBUG_REPLAYS builds (else 0)
start = t0.min()
lat = (t1 - t0) / 100.0          # wall_clock64 = 100 MHz -> microseconds
end = (t1 - start) / 100.0
pop = (t0 - start) / 100.0
span = float(end.max())
out = {"queued": qcount + qshort, "uncached_rays": march, "regroups": regroups, "recorded": int(len(e)), "group": int(np.median(G)),
       "span_us": span,
       "latency_us_pct": {p: float(np.percentile(lat, p)) for p in (50, 90, 99, 99.9, 100)},
       "pop_us_pct": {p: float(np.percentile(pop, p)) for p in (50, 90, 99, 100)},
       "passes_pct": {p: float(np.percentile(passes, p)) for p in (50, 90, 99, 100)},
       "n_pct": {p: float(np.percentile(n, p)) for p in (50, 90, 99, 100)},
       "us_per_sample_pass_median": float(np.median(lat / np.maximum(1, (passes - 1) * n))),
       "slowest": [{"lat_us": float(lat[i]), "pop_us": float(pop[i]), "passes": int(passes[i]), "rounds": int(rounds[i]),
                 "n": int(n[i]), "G_end": int(G[i])} for i in np.argsort(-lat)[:8]]}
if rounds.any():
    out["rounds_by_passes"] = {int(p): {"rays": int((passes == p).sum()), "mean_rounds": float(rounds[passes == p].mean()),
                                       "mean_lat_us": float(lat[passes == p].mean()), "mean_n": float(n[passes == p].mean()),
                                       "us_per_round_sample": float((lat[passes == p] / np.maximum(1, rounds[passes == p] * n[passes == p])).mean())}
                               for p in np.unique(passes)}
out["in_flight_at_tenths"] = [int(((pop <= f * span) & (end > f * span)).sum()) for f in np.arange(0.0, 1.0, 0.1)]
out["done_frac_at_tenths"] = [float((end <= f * span).mean()) for f in np.arange(0.1, 1.01, 0.1)]
out["queue_drained_us"] = float(pop.max())
print(json.dumps(out))
