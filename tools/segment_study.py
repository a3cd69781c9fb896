"""Driver of tools/segment_study.c (design study, CPU): segment-parallel replay of the search passes on
one config-2 brick (512^3 fp32 Gray-Scott, 1920x1080, S = 20, the bench camera of frame 0), every
`--ystep`-th row: latency and work of a pass split into K = 1..8 lanes, against n.

usage: python tools/segment_study.py [--brick 7] [--ystep 16] [--threads 8] [--M 4]
"""
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

MAXK = 8


class SegOut(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_double), ("passes", ctypes.c_double), ("samples", ctypes.c_double),
                ("lat", ctypes.c_double * (MAXK + 1)), ("work", ctypes.c_double * (MAXK + 1)),
                ("unsynced", ctypes.c_double * (MAXK + 1)), ("mismatch", ctypes.c_double * (MAXK + 1)),
                ("overlap_hist", ctypes.c_double * ((MAXK + 1) * 8))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--brick", type=int, default=7)
    ap.add_argument("--ystep", type=int, default=16)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--M", type=int, default=4)
    args = ap.parse_args()
    so = Path("/tmp/libsegstudy.so")
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-std=gnu99", "-fPIC", "-ffp-contract=off", "-shared", "-o",
                    str(so), str(ROOT / "tools" / "segment_study.c"), "-lm"], check=True)
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
    outs = [SegOut() for _ in range(args.threads)]

    def run(i):
        lib.study_seg(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                      int(bands[i]), int(bands[i + 1]), 0, H, args.ystep, args.M, ctypes.byref(outs[i]))
    th = [threading.Thread(target=run, args=(i,)) for i in range(args.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    tot = {k: sum(getattr(o, k) for o in outs) for k in ("rays", "passes", "samples")}
    res = {"brick": args.brick, "ystep": args.ystep, "M": args.M, **tot}
    for K in range(1, MAXK + 1):
        lat = sum(o.lat[K] for o in outs)
        work = sum(o.work[K] for o in outs)
        hist = np.sum([np.array(o.overlap_hist[K * 8:(K + 1) * 8]) for o in outs], axis=0)
        res[f"K={K}"] = {"latency_frac": round(lat / tot["samples"], 4), "work_frac": round(work / tot["samples"], 4),
                         "unsynced_per_pass": round(sum(o.unsynced[K] for o in outs) / tot["passes"], 4),
                         "mismatch": int(sum(o.mismatch[K] for o in outs)),
                         "resync_dist_hist(0,4,16,32,64,128,256,more)": [int(v) for v in hist]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
