"""Driver of tools/checkpoint_study.c (design study, CPU): replayed cache samples of the threshold
search with and without resuming passes from saved states of the low/high passes, on one config-2
brick (512^3 fp32 Gray-Scott, 1920x1080, S = 20, the bench camera of frame 0), every `--ystep`-th row.

usage: python tools/checkpoint_study.py [--brick 7] [--ystep 16] [--threads 8]
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

KS = (1, 16, 32, 64)


class StudyOut(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_double), ("passes_hist", ctypes.c_double * 65), ("base", ctypes.c_double),
                ("ck", ctypes.c_double * 4), ("search_passes", ctypes.c_double), ("skipped_base", ctypes.c_double),
                ("samples", ctypes.c_double), ("real_by_passes", ctypes.c_double * 65),
                ("left_run", ctypes.c_double * 65), ("dec", ctypes.c_double * 48),
                ("base_by_passes", ctypes.c_double * 65), ("ck1_by_passes", ctypes.c_double * 65),
                ("ck16_by_passes", ctypes.c_double * 65), ("write_samples", ctypes.c_double),
                ("write_samples_rec", ctypes.c_double)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--brick", type=int, default=7)
    ap.add_argument("--ystep", type=int, default=16)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    so = Path("/tmp/libckstudy.so")
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-std=gnu99", "-fPIC", "-ffp-contract=off", "-shared", "-o",
                    str(so), str(ROOT / "tools" / "checkpoint_study.c"), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    import torch

    import bench
    from insitu_amd import native, scene
    W, H, S, n = 1920, 1080, 20, 512
    units = scene.grid_bricks(2 * n, 2)
    origin, vw, _ = units[args.brick]
    vol = bench.make_brick(args.brick, n, torch.device("cpu")).numpy()
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    inp = orc.Inputs(vol, scene.inverse_model(scene.brick_model(origin, vw)), scene.transfer_function(),
                     scene.colormap_hot(), scene.folded_conv_scale(2.0, native.F32), 0.0, cam)
    bands = np.linspace(0, W, args.threads + 1).astype(int)
    outs = [StudyOut() for _ in range(args.threads)]

    def run(i):
        lib.study_vdi(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                      int(bands[i]), int(bands[i + 1]), 0, H, args.ystep, ctypes.byref(outs[i]))
    th = [threading.Thread(target=run, args=(i,)) for i in range(args.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    tot = {k: sum(getattr(o, k) for o in outs) for k in ("rays", "base", "search_passes", "skipped_base", "samples")}
    ck = [sum(o.ck[k] for o in outs) for k in range(4)]
    hist = np.sum([np.array(o.passes_hist[:]) for o in outs], axis=0)
    res = {"brick": args.brick, "ystep": args.ystep, **tot,
           "replayed_with_checkpoints": {f"K={k}": c for k, c in zip(KS, ck)},
           "saving_vs_base": {f"K={k}": 1.0 - c / tot["base"] for k, c in zip(KS, ck)},
           "passes_hist": {int(i): int(v) for i, v in enumerate(hist) if v},
           "mean_replayed_search_passes_by_passes": {int(i): round(float(r) / float(v), 2) for i, (r, v) in enumerate(
               zip(np.sum([np.array(o.real_by_passes[:]) for o in outs], axis=0), hist)) if v}}
    lr = np.sum([np.array(o.left_run[:]) for o in outs], axis=0)
    res["searched_rays_by_initial_left_run"] = {int(i): int(v) for i, v in enumerate(lr) if v}
    dec = np.sum([np.array(o.dec[:]) for o in outs], axis=0).reshape(4, 4, 3)
    names = "LRF-"
    res["decisions_after_spine"] = {f"{names[a]}{names[b]}": {names[c]: int(dec[a, b, c]) for c in range(3)}
                                    for a in range(4) for b in range(4) if dec[a, b].sum()}
    res["write_samples"] = sum(o.write_samples for o in outs)
    res["write_samples_recorded"] = sum(o.write_samples_rec for o in outs)
    bb = np.sum([np.array(o.base_by_passes[:]) for o in outs], axis=0)
    c1 = np.sum([np.array(o.ck1_by_passes[:]) for o in outs], axis=0)
    c16 = np.sum([np.array(o.ck16_by_passes[:]) for o in outs], axis=0)
    res["saving_by_passes(K=1,K=16)"] = {int(i): [round(1.0 - c1[i] / bb[i], 3), round(1.0 - c16[i] / bb[i], 3)]
                                         for i in range(65) if bb[i] > 0}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
