"""Diagnostic: distribution of raymarch passes per ray (and supersegments per pixel) for one brick
of the bench scene -- the per-GPU work of an 8-GPU run.  Prints one JSON line."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from insitu_amd import native, scene  # noqa: E402
from insitu_amd.renderer import InSituContext  # noqa: E402

W, H, S = bench.W_IMG, bench.H_IMG, bench.S
n = 512
bricks = scene.grid_bricks(n * 2, 2)
out = {}
for bid, yaw in ((0, 30.0), (0, 85.0), (5, 85.0)):
    origin, vw, _ = bricks[bid]
    vol = bench.make_brick(bid, n, torch.device("cuda", 0))
    ctx = InSituContext(W, H, max_supersegments=S, keep_passes=True)
    ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=2.0)
    ctx.set_brick(0, vol, scene.brick_model(origin, vw), dtype=native.F32)
    cam = scene.orbit_camera(W, H, yaw_deg=yaw, pitch_deg=20.0, voxel_world=vw)
    ctx.render(cam)
    passes = ctx.read(native.BUF_PASSES).astype(np.int64)
    dep = ctx.read(native.BUF_VDI_DEPTH)
    nseg = np.count_nonzero(dep[..., 0::2] != 0, axis=2).T
    hit = passes > 0
    hist = np.bincount(passes[hit], minlength=30)
    out[f"brick{bid}_yaw{yaw}"] = {"vol": [float(vol.min()), float(vol.mean()), float(vol.max())], "rays_hit": int(hit.sum()), "passes_hist": hist.tolist(),
                          "segs_hist": np.bincount(nseg[hit], minlength=S + 1).tolist(),
                          "ms_render": ctx.stats()["ms_render"]}
    ctx.close()
print(json.dumps(out))
