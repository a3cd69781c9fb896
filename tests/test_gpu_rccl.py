"""The RCCL data path of libinsitu_hip.so in separate processes (one rank per process): exchange,
composite and gather over RCCL, bit-identical to one rank rendering every brick
(tests/rccl_worker.py has the cases).  On a one-GPU box the ranks share the GPU and RCCL connects
them over its socket transport (distinct NCCL host ids); on a multi-GPU node each rank has its own
GPU and RCCL uses xGMI.  Also runs bench.py's multi-rank frame loop (torchrun, gloo bootstrap,
ncclCommInitRank, barrier + max-over-ranks timing)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, args: list[str], timeout: int):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", NCCL_DEBUG="WARN")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_exchange_composite_gather(world):
    """world 8 = config 2's decomposition (8 bricks, one per rank); rank 0's image is also checked against
    the CPU oracle's flatten of all 8 sub-VDIs."""
    p = _run(world, [str(ROOT / "tests" / "rccl_worker.py")], timeout=280)
    out = p.stdout + p.stderr
    # (the ranks' own lines first: a failing rank's traceback is in stderr before torchrun's summary)
    assert p.returncode == 0 and "RCCL_OK" in p.stdout, p.stdout[-6000:] + "\n--- stderr ---\n" + p.stderr[:6000]
    assert out.count("== 1-rank result: True") == 5, out[-4000:]
    assert out.count("pipelined frames == 1-rank frames: True") == 2, out[-4000:]
    nb = 8 if world == 8 else 4
    assert f"image == oracle ({nb} bricks): True" in out, out[-4000:]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("launch", ["torchrun", "self"])
def test_bench_two_ranks(launch):
    """bench.py --gpus 2 (reduced bricks): the multi-rank path runs, launched by torch.distributed.run
    (the driver's form) or by bench.py itself (`python bench.py --gpus 2`, no WORLD_SIZE), and prints
    one JSON line with the whole-job value."""
    args = [str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--brick", "64",
            "--no-cpu-baseline"]
    if launch == "torchrun":
        p = _run(2, args, timeout=280)
    else:
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", NCCL_DEBUG="WARN")
        p = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    assert rec["config"]["exchange_bytes_per_rank"] > 0
    assert rec["config"]["pipeline_depth"] == 2   # the default bench runs pipelined frames
