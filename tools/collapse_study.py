"""Driver of tools/collapse_study.c (design study, CPU): spine counts of rays by the length of their search.
usage: python tools/collapse_study.py [--brick 7] [--ystep 16] [--threads 8]"""
from __future__ import annotations

import argparse
import ctypes
import json
import subprocess
import sys
import threading
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests"), str(ROOT)]

import numpy as np  # noqa: E402

import oracle_binding as orc  # noqa: E402


class CRay(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("c", ctypes.c_int * 5), ("passes", ctypes.c_int), ("l1_implied", ctypes.c_int)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--brick", type=int, default=7)
    ap.add_argument("--ystep", type=int, default=16)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    so = Path("/tmp/libcstudy.so")
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-std=gnu99", "-fPIC", "-ffp-contract=off", "-shared", "-o",
                    str(so), str(ROOT / "tools" / "collapse_study.c"), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    import torch

    import bench
    from insitu_amd import native, scene
    W, H, S, n = 1920, 1080, 20, 512
    units = scene.grid_bricks(2 * n, 2)
    origin, vw, _ = units[args.brick]
    vol = bench.make_brick(args.brick, n, torch.device("cpu"), sim_n=128).numpy()
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    inp = orc.Inputs(vol, scene.inverse_model(scene.brick_model(origin, vw)), scene.transfer_function(),
                     scene.colormap_hot(), scene.folded_conv_scale(2.0, native.F32), 0.0, cam)
    bands = np.linspace(0, W, args.threads + 1).astype(int)
    cap = 200000
    bufs = [(CRay * cap)() for _ in range(args.threads)]
    counts = [0] * args.threads

    def run(i):
        counts[i] = lib.study_collapse(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                                       int(bands[i]), int(bands[i + 1]), 0, H, args.ystep, bufs[i], cap)
    th = [threading.Thread(target=run, args=(i,)) for i in range(args.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    rays = [(r.n, tuple(r.c), r.passes) for i in range(args.threads) for r in bufs[i][:counts[i]]]
    P = np.array([r[2] for r in rays])
    C = np.array([r[1] for r in rays])
    N = np.array([r[0] for r in rays])
    L1 = np.array([r.l1_implied for i in range(args.threads) for r in bufs[i][:counts[i]]])
    res = {"searched": len(rays), "level1_implied_by_level2_interval": float(L1.mean()), "passes_hist": {int(k): int(v) for k, v in zip(*np.unique(P, return_counts=True))}}
    for name, m in (("collapse (>= 20 passes)", P >= 20), ("others", P < 20)):
        res[name] = {"rays": int(m.sum()), "n_mean": float(N[m].mean()) if m.any() else None,
                     "spine_counts_mean": C[m].mean(axis=0).round(2).tolist() if m.any() else None,
                     "examples": [list(map(int, C[i])) + [int(P[i])] for i in np.flatnonzero(m)[:12]]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
