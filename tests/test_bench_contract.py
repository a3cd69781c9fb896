"""bench.py's launch contract on the CPU (no GPU is touched): --gpus must equal the world size."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=e, capture_output=True,
                          text=True, timeout=120)


def test_gpus_must_equal_world_size():
    p = _bench(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "must equal the world size" in p.stderr, p.stderr[-2000:]
    p = _bench(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "must equal the world size" in p.stderr, p.stderr[-2000:]


def test_gpus_zero_rejected():
    p = _bench(["--gpus", "0"])
    assert p.returncode != 0 and "at least one GPU" in p.stderr, p.stderr[-2000:]


def test_steps_zero_rejected():
    p = _bench(["--steps", "0"])
    assert p.returncode != 0 and "at least one timed step" in p.stderr, p.stderr[-2000:]


def test_roofline_blocks_reproduce_from_the_committed_profile():
    """The bench line's roofline.valu and traffic come from profiles/CURRENT's summary: recomputing
    them from the summary's raw counters gives the same numbers (no GPU needed)."""
    import json
    sys.path.insert(0, str(ROOT))
    import bench
    prof = bench.pmc_profile()
    assert prof is not None, "profiles/CURRENT must name an N=1 config-2 profile"
    v = bench.valu_roofline(prof)
    t = bench.pmc_traffic(prof)
    summary = json.loads((ROOT / "profiles" / prof[0] / "summary.json").read_text())
    gen = bench.generator_kernels(summary)
    assert gen and v and t
    for name, k in gen.items():
        got = v["kernels"][name.split("<")[0]]
        issue = k["valu_wave_insts_per_launch"] / (256 * 4 * 1.2e9 * k["avg_ms"] * 1e-3)
        assert abs(got["issue_frac"] - issue) < 1e-3
        assert abs(got["issue_frac"] - k["valu_issue_utilisation"]) < 1e-3   # prof_summary's own figure
        assert got["salu_insts"] == k.get("salu_wave_insts_per_launch")
    assert abs(t["hbm"] - sum(k["hbm_bytes_per_launch"] for k in gen.values())) < 1.0
    assert abs(t["hbm"] - (2 * t["fetch_raw"] + t["write"])) < 1e3
