#!/usr/bin/env python3
"""Diagnostic: the VDICompositor (composite_vdi) workload of the bench scene (config 2, N=1): per-pixel
search passes of the compositor (INSITU_BUF_COMPOSITE_PASSES), merged entries per pixel (the sum of the
bricks' supersegment counts), composite time, as JSON.  usage: tools/composite_stats.py [sim_n]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests"), str(ROOT)]
import bench  # noqa: E402
from insitu_amd import native, scene  # noqa: E402
from insitu_amd.renderer import InSituContext  # noqa: E402

sim_n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
n, W, H, S = 512, 1920, 1080, 20
units = scene.grid_bricks(2 * n, 2)
vols = [bench.make_brick(b, n, dev, sim_n=sim_n) for b in range(8)]
models = [scene.brick_model(o, vw) for (o, vw, _) in units]
cam = scene.orbit_camera(W, H, yaw_deg=30.0 + 5.0 * 3, pitch_deg=20.0, voxel_world=units[0][1])
ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=8, keep_passes=True, composite_vdi=True,
                    max_output_supersegments=S)
ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=1.0 / 0.5, conv_offset=0.0)
for b, v in enumerate(vols):
    ctx.set_brick(b, v, models[b], dtype=native.F32)
ms = []
for _ in range(4):
    ctx.frame(cam)
    ms.append(ctx.stats()["ms_composite"])
cp = ctx.read(native.BUF_COMPOSITE_PASSES).astype(np.int64)
ent = np.zeros((H, W), np.int64)
for b in range(8):   # supersegments per pixel and brick: the non-empty slots of the reference-layout depth
    for x0 in range(0, W, 240):
        d = ctx.read_columns(native.BUF_VDI_DEPTH, x0, x0 + 240, slot=b).reshape(240, H, 2 * S)
        ent[:, x0:x0 + 240] += np.count_nonzero(d[..., 0::2], axis=2).T
hit = ent > 0
tiles = ent.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
ptile = cp.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
out = {"ms_composite": ms, "pixels_with_entries": int(hit.sum()),
       "entries_mean_hit": float(ent[hit].mean()), "entries_pct": {p: float(np.percentile(ent[hit], p)) for p in (50, 90, 99, 100)},
       "passes_mean_hit": float(cp[hit].mean()), "passes_pct": {p: float(np.percentile(cp[hit], p)) for p in (50, 90, 99, 100)},
       "entry_passes_total": int((ent * cp).sum()),
       "wave_max_entry_passes_total": int(((ent * cp).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).max(axis=1) * 64).sum()),
       "tile_max_passes_mean": float(ptile.max(axis=1).mean())}
print(json.dumps(out))
ctx.close()
