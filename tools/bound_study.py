"""Driver of tools/bound_study.c (design study, CPU): share of supersegment decisions a cheap upper
bound on diff settles, on one config-2 brick (bench camera of frame 0), every `--ystep`-th row.
usage: python tools/bound_study.py [--brick 7] [--ystep 16] [--threads 8]"""
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


class Out(ctypes.Structure):
    _fields_ = [("dec", ctypes.c_double * 2), ("nocl_bound", ctypes.c_double * 2), ("close", ctypes.c_double * 2),
                ("hist", ctypes.c_double * 32), ("rays", ctypes.c_double),
                ("steps_hist", ctypes.c_double * 16), ("max_relerr", ctypes.c_double * 8),
                ("spine_dec", ctypes.c_double * 4), ("spine_bound", ctypes.c_double * 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--brick", type=int, default=7)
    ap.add_argument("--ystep", type=int, default=16)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    so = Path("/tmp/libbstudy.so")
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-std=gnu99", "-fPIC", "-ffp-contract=off", "-shared", "-o",
                    str(so), str(ROOT / "tools" / "bound_study.c"), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    import torch

    import bench
    from insitu_amd import native, scene
    W, H, S, n = 1920, 1080, 20, 512
    units = scene.grid_bricks(2 * n, 2)
    origin, vw, _ = units[args.brick]
    vol = bench.make_brick(args.brick, n, torch.device("cpu"), sim_n=128).numpy()
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    cmap = scene.colormap_hot()
    C = float(np.abs(cmap[:, :3]).max())
    inp = orc.Inputs(vol, scene.inverse_model(scene.brick_model(origin, vw)), scene.transfer_function(),
                     cmap, scene.folded_conv_scale(2.0, native.F32), 0.0, cam)
    bands = np.linspace(0, W, args.threads + 1).astype(int)
    outs = [Out() for _ in range(args.threads)]

    def run(i):
        lib.study_bound(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                        int(bands[i]), int(bands[i + 1]), 0, H, args.ystep, ctypes.c_float(C), ctypes.byref(outs[i]))
    th = [threading.Thread(target=run, args=(i,)) for i in range(args.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dec = np.sum([np.array(o.dec[:]) for o in outs], axis=0)
    nb = np.sum([np.array(o.nocl_bound[:]) for o in outs], axis=0)
    cl = np.sum([np.array(o.close[:]) for o in outs], axis=0)
    hist = np.sum([np.array(o.hist[:]) for o in outs], axis=0).reshape(2, 16)
    res = {"brick": args.brick, "ystep": args.ystep, "rays": sum(o.rays for o in outs),
           "decisions": {"pass1": dec[0], "later": dec[1]},
           "no_close_by_cheap_bound": {"pass1": nb[0] / dec[0], "later": nb[1] / dec[1]},
           "close_frac": {"pass1": cl[0] / dec[0], "later": cl[1] / dec[1]},
           "log10_diff_over_t_hist_later": {int(i) - 8: round(float(v / dec[1]), 4) for i, v in enumerate(hist[1]) if v}}
    sh = np.sum([np.array(o.steps_hist[:]) for o in outs], axis=0).reshape(2, 8)
    cls = ["1", "2-4", "5-8", "9-16", "17-32", "33-64", "65-128", ">128"]
    res["steps_share_later"] = {c: round(float(v / dec[1]), 4) for c, v in zip(cls, sh[1])}
    res["crude_L_max_relerr"] = {c: float(max(o.max_relerr[i] for o in outs)) for i, c in enumerate(cls)}
    sd = np.sum([np.array(o.spine_dec[:]) for o in outs], axis=0)
    sb = np.sum([np.array(o.spine_bound[:]) for o in outs], axis=0)
    res["spine_levels_settled_by_cheap_bound"] = [round(float(b / d), 4) if d else None for b, d in zip(sb, sd)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
