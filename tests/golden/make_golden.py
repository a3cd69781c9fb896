#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ with the pure-Python restatement
(tests/pyref.py) -- independent of the C oracle and of the HIP library.

The reference (Kotlin/Vulkan, scenery) cannot run here and ships no fixtures,
so these vectors pin behaviour across the two CPU restatements and the GPU path; they are not
outputs of the reference itself.  Inputs are stored alongside the expected outputs.

usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(HERE.parent)]

import pyref  # noqa: E402
from scenes import make_scene  # noqa: E402


def _inputs(sc):
    vol = sc["vol"]
    V = pyref.Volume(vol.ravel().tolist(), (vol.shape[2], vol.shape[1], vol.shape[0]), sc["im"].tolist(),
                     sc["tf"].tolist(), sc["cmap"].tolist(), float(sc["conv_k"]), float(sc["conv_offset"]))
    c = sc["cam"]
    cam = dict(view=c.view.tolist(), proj=c.proj.tolist(), inv_view=c.inv_view.tolist(),
               inv_proj=c.inv_proj.tolist(), nw=float(c.nw), fwnw=float(c.fwnw), tmax=float(c.tmax))
    return V, cam


def _common(sc):
    c = sc["cam"]
    return dict(vol=sc["vol"], im=sc["im"], tf=sc["tf"], cmap=sc["cmap"], conv_k=np.float32(sc["conv_k"]),
                conv_off=np.float32(sc["conv_offset"]), view=c.view, proj=c.proj, inv_view=c.inv_view,
                inv_proj=c.inv_proj, nw=np.float32(c.nw), fwnw=np.float32(c.fwnw), tmax=np.float32(c.tmax),
                model=sc["model"])


def main():
    # VDI: 16^3 uint16 Gray-Scott brick, 24x16 window, S = 6
    W, H, S = 24, 16, 6
    sc = make_scene(n=16, W=W, H=H, yaw=30.0)
    V, cam = _inputs(sc)
    color, depth, octree, passes = pyref.vdi_image(V, cam, W, H, S)
    color = np.asarray(color, np.float32)
    depth = np.asarray(depth, np.float32)
    ipv = pyref.matmul(cam["inv_view"], cam["inv_proj"])
    image = np.zeros((H, W, 4), np.uint8)
    for x in range(W):
        for y in range(H):
            lst = [(float(depth[x, y, 2 * i]), float(depth[x, y, 2 * i + 1]), tuple(map(float, color[x, y, i])))
                   for i in range(S)]
            image[y, x] = pyref.flatten_pixel([lst], ipv, x, y, W, H)
    np.savez_compressed(HERE / "vdi_small.npz", **_common(sc), whs=np.array([W, H, S]), color=color, depth=depth,
                        octree=np.asarray(octree, np.uint32), passes=np.asarray(passes, np.int32), image=image)

    # plain: 16^3 uint16 brick, 20x20 texture
    dim = 20
    sc = make_scene(n=16, W=dim, H=dim, yaw=60.0)
    V, cam = _inputs(sc)
    pc = np.zeros((dim, dim, 4), np.uint8)
    pd = np.zeros((dim, dim, 4), np.uint8)
    for gy in range(dim):
        for gx in range(dim):
            c, d = pyref.plain_pixel(V, cam, gx, gy, dim, dim)
            pc[gy, gx], pd[gy, gx] = c, d
    np.savez_compressed(HERE / "plain_small.npz", **_common(sc), dims=np.array([dim, dim]), color=pc, depth=pd)
    print("wrote", sorted(p.name for p in HERE.glob("*.npz")))


if __name__ == "__main__":
    main()
