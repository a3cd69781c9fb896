#!/usr/bin/env python3
"""Design study (no GPU): how large is the set of brick blocks a sampling wave reads -- the working set an
LDS-staged brick (north_star: "software trilinear sampling from LDS-staged volume bricks") would have to hold?

The sampling kernel runs one wave per 8x8 pixel tile; lane l marches its ray from its own tnear with step nw
(VDIGenerator.comp:372-447) and reads a 2x2x2 trilinear footprint that lies in ONE 9^3 halo block of the
brick (insitu_sampling.h): so at march step i the wave needs the distinct blocks of its active lanes' samples.
This restates the kernel's ray setup in float64 (positions differ from the float32 kernel by far less than a
voxel: the statistics, not the bits, are the point) for the config-2 frame (8 x 512^3 bricks, 1920x1080,
the bench's first camera) and reports per brick, over every `stride`-th tile row and column:
  * distinct blocks per wave and step (the per-step working set), and over windows of 8 steps;
  * the same for 2x2-tile quads (a 4-wave workgroup sharing one stage);
  * bytes a perfect stage would load (each distinct block of a tile's march once, 9^3 x 4 B) against the
    bytes the per-lane gathers request (4 x 8 B per sample) -- the L1/TA traffic the stage would replace.
usage: tools/lds_stage_study.py [--stride 4] [--bricks 0,7]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scenery-insitu_amd"))
from insitu_amd import scene  # noqa: E402

W, H, N = 1920, 1080, 512
BLOCK_BYTES = 9 * 9 * 9 * 4


def rays(cam, gx, gy):
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    uvx = gx / W * 2.0 - 1.0
    uvy = gy / H * 2.0 - 1.0
    def unproject(z):
        p = np.stack([uvx, uvy, np.full_like(uvx, z), np.ones_like(uvx)], axis=-1) @ ipv.T
        return p[..., :3] / p[..., 3:4]
    return unproject(-1.0), unproject(1.0)


def tile_blocks(cam, im, gx, gy, nw):
    """(steps, 64) block ids of a tile's rays (-1: lane inactive at that step)."""
    wf, wb = rays(cam, gx, gy)
    mf = wf @ im[:3, :3].T + im[:3, 3]
    mb = wb @ im[:3, :3].T + im[:3, 3]
    rd = mb - mf
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / rd
        t0 = inv * (0.0 - mf)
        t1 = inv * (N - mf)
    tn = np.max(np.minimum(t0, t1), axis=1)
    tf = np.minimum(np.min(np.maximum(t0, t1), axis=1), 1.0)
    hit = tn < tf
    tnear = np.where(hit, np.maximum(tn, 0.0), 1.0)
    nsteps = np.where(hit, np.trunc((tf - tnear) / nw), 0).astype(np.int64)
    S = int(nsteps.max()) if hit.any() else 0
    if S == 0:
        return None, 0
    i = np.arange(S)[:, None]
    t = tnear[None, :] + i * nw
    p = mf[None] + t[..., None] * rd[None]                              # (S, 64, 3) voxel space
    v = np.clip(np.floor(p), 0, N - 1).astype(np.int64) >> 3            # block coordinates
    ids = (v[..., 2] * 64 + v[..., 1]) * 64 + v[..., 0]
    active = (i < nsteps[None, :]) & hit[None, :]
    return np.where(active, ids, -1), int(active.sum())


def distinct_per_row(ids):
    """Distinct non-negative ids per row of a 2-D array."""
    s = np.sort(ids, axis=1)
    new = np.ones_like(s, dtype=bool)
    new[:, 1:] = s[:, 1:] != s[:, :-1]
    return np.sum(new & (s >= 0), axis=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=4)
    ap.add_argument("--bricks", default="0,7")
    a = ap.parse_args()
    units = scene.grid_bricks(2 * N, 2)
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    nw = float(cam.nw)
    for b in (int(x) for x in a.bricks.split(",")):
        origin, vw, _ = units[b]
        im = np.linalg.inv(np.asarray(scene.brick_model(origin, vw), np.float64).reshape(4, 4).T)
        per_step, per_win, quad_step, staged, gathered, samples = [], [], [], 0, 0, 0
        for ty in range(0, H // 8 - 1, a.stride):
            for tx in range(0, W // 8 - 1, a.stride):
                quad = []
                for qy in range(2):
                    for qx in range(2):
                        gy, gx = np.mgrid[0:8, 0:8]
                        ids, ns = tile_blocks(cam, im, (gx + 8 * (tx + qx)).ravel().astype(np.float64),
                                              (gy + 8 * (ty + qy)).ravel().astype(np.float64), nw)
                        if ids is None:
                            continue
                        if qx == 0 and qy == 0:
                            d = distinct_per_row(ids)
                            act = d > 0
                            per_step.append(d[act])
                            w = (ids.shape[0] // 8) * 8
                            if w:
                                per_win.append(distinct_per_row(ids[:w].reshape(-1, 8 * 64)))
                            staged += len(np.unique(ids[ids >= 0])) * BLOCK_BYTES
                            gathered += ns * 32
                            samples += ns
                        quad.append(ids)
                if len(quad) == 4:
                    S = max(q.shape[0] for q in quad)
                    qa = np.concatenate([np.pad(q, ((0, S - q.shape[0]), (0, 0)), constant_values=-1) for q in quad], 1)
                    d = distinct_per_row(qa)
                    quad_step.append(d[d > 0])
        ps = np.concatenate(per_step)
        pw = np.concatenate(per_win) if per_win else np.zeros(1)
        qs = np.concatenate(quad_step) if quad_step else np.zeros(1)
        q = lambda x: f"mean {x.mean():.2f}  p50 {np.percentile(x, 50):.0f}  p90 {np.percentile(x, 90):.0f}  max {x.max():.0f}"
        print(f"brick {b}: {len(per_step)} tiles (every {a.stride}th row/column), {samples} samples, nw {nw:.3g}")
        print(f"  distinct blocks per wave-step          {q(ps)}  -> {ps.mean() * BLOCK_BYTES / 1024:.1f} KiB per wave")
        print(f"  distinct blocks per wave, 8-step window {q(pw)}  -> {pw.mean() * BLOCK_BYTES / 1024:.1f} KiB per wave")
        print(f"  distinct blocks per 2x2-tile quad-step  {q(qs)}  -> {qs.mean() * BLOCK_BYTES / 1024:.1f} KiB per workgroup")
        print(f"  bytes: perfect stage {staged / 1e6:.1f} MB, per-lane gathers {gathered / 1e6:.1f} MB "
              f"(stage / gathers = {staged / max(1, gathered):.3f}), samples per staged block "
              f"{samples / max(1, staged / BLOCK_BYTES):.0f}")


if __name__ == "__main__":
    main()
