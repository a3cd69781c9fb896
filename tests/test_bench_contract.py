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
