#!/usr/bin/env python3
"""Probe: does running the generator kernels of different bricks CONCURRENTLY (separate contexts on
separate HIP streams, one GPU) beat running them back to back?  K contexts each render 8/K of the
config-2 bricks; the time for all 8 bricks is measured (a) one context after the other with a sync
in between and (b) all contexts submitted before one sync.  A gain in (b) means the sampling and
search kernels leave units idle that the other kernel could use -- the case for overlapping them
inside one frame.  A measurement tool, not the bench.

    python tools/concurrency_probe.py [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT)]

import torch  # noqa: E402

from insitu_amd import native, scene  # noqa: E402
from insitu_amd.renderer import InSituContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    W, H, S, NB, n = 1920, 1080, 20, 8, 512
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from bench import make_brick
    bricks = scene.grid_bricks(2 * n, 2)
    vols = [make_brick(b, n, dev) for b in range(NB)]
    models = [scene.brick_model(bricks[b][0], bricks[b][1]) for b in range(NB)]
    torch.cuda.synchronize()
    tf, cm = scene.transfer_function(), scene.colormap_hot()
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=bricks[0][1])
    out = {}
    for K in (1, 2, 4):
        B = NB // K
        ctxs = []
        for k in range(K):
            c = InSituContext(W, H, max_supersegments=S, bricks_per_rank=B, device=0)
            c.set_transfer(tf, cm, conv_scale=2.0)
            for s in range(B):
                c.set_brick(s, vols[k * B + s], models[k * B + s], dtype=native.F32)
            ctxs.append(c)
        for c in ctxs:   # warm-up (sizes the sample caches)
            c.render(cam)
            c.synchronize()
            c.render(cam)
            c.synchronize()
        seq, conc = [], []
        for _ in range(args.iters):
            t = time.perf_counter()
            for c in ctxs:
                c.render(cam)
                c.synchronize()
            seq.append(1e3 * (time.perf_counter() - t))
            t = time.perf_counter()
            for c in ctxs:
                c.render(cam)
            for c in ctxs:
                c.synchronize()
            conc.append(1e3 * (time.perf_counter() - t))
        out[f"K{K}"] = {"bricks_per_context": B, "sequential_ms": round(min(seq), 3), "concurrent_ms": round(min(conc), 3)}
        print(json.dumps({f"K{K}": out[f"K{K}"]}), flush=True)
        for c in ctxs:
            c.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
