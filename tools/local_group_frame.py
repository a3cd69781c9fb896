#!/usr/bin/env python3
"""One config-2 frame of an N-rank run on ONE GPU through the in-process rank group
(insitu_local_group): N contexts, one brick set each, driven stage by stage and synchronised after
every rank's stage so each stage time is that rank's alone.  Reports per rank the render time, the
compaction of the variable-length exchange (ms_compact), the bytes and entries it sends to its peers,
the exchange and the flatten of its strip's N*B lists; checks rank 0's image against a 1-rank context
rendering every brick (bit for bit).  A measurement tool, not the bench.

    python tools/local_group_frame.py [--ranks 8] [--brick 512] [--out profiles/r03_local_group.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from insitu_amd import native, scene  # noqa: E402
from insitu_amd.renderer import InSituContext, LocalGroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--brick", type=int, default=512)
    ap.add_argument("--sim-n", type=int, default=128)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    W, H, S, NB = 1920, 1080, 20, 8
    N = args.ranks
    B = NB // N
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.brick
    bricks = scene.grid_bricks(2 * n, 2)
    from bench import make_brick
    vols = [make_brick(b, n, dev, sim_n=min(args.sim_n, n)) for b in range(NB)]
    models = [scene.brick_model(bricks[b][0], bricks[b][1]) for b in range(NB)]
    torch.cuda.synchronize()
    tf, cm = scene.transfer_function(), scene.colormap_hot()
    g = LocalGroup(N)
    ctxs = []
    for r in range(N):
        c = InSituContext(W, H, max_supersegments=S, bricks_per_rank=B, rank=r, nranks=N, device=0, local_group=g)
        c.set_transfer(tf, cm, conv_scale=2.0)
        for s in range(B):
            c.set_brick(s, vols[r * B + s], models[r * B + s], dtype=native.F32)
        ctxs.append(c)
    ref = InSituContext(W, H, max_supersegments=S, bricks_per_rank=NB, device=0)
    ref.set_transfer(tf, cm, conv_scale=2.0)
    for s in range(NB):
        ref.set_brick(s, vols[s], models[s], dtype=native.F32)
    rows = []
    same = True
    for f in range(args.frames):
        cam = scene.orbit_camera(W, H, yaw_deg=30.0 + 5.0 * f, pitch_deg=20.0, voxel_world=bricks[0][1])
        st = [dict() for _ in range(N)]
        for r, c in enumerate(ctxs):
            c.render(cam)
            c.synchronize()
        for r, c in enumerate(ctxs):
            t = time.perf_counter()
            c.exchange()
            c.synchronize()
            st[r]["exchange_wall_ms"] = 1e3 * (time.perf_counter() - t)
        for r, c in enumerate(ctxs):   # wall time: the stage events of one rank span the others' stages
            t = time.perf_counter()
            c.composite()
            c.synchronize()
            st[r]["composite_wall_ms"] = 1e3 * (time.perf_counter() - t)
        img = None
        for r, c in reversed(list(enumerate(ctxs))):   # the root pulls the strips last
            out = c.gather(want_image=(r == 0))
            if r == 0:
                img = out
        for r, c in enumerate(ctxs):
            s = c.stats()
            st[r].update(rank=r, ms_render=round(s["ms_render"], 3), ms_compact=round(s["ms_compact"], 3),
                         ms_exchange_sync=round(s["ms_exchange_sync"], 3),
                         exchange_bytes=int(s["exchange_bytes"]), exchange_entries=int(s["exchange_entries"]))
        want = ref.frame(cam, want_image=True)
        eq = bool(np.array_equal(img, want))
        same = same and eq
        rows.append({"frame": f, "image_equals_1rank": eq, "ranks": st})
        print(json.dumps(rows[-1]), flush=True)
    last = rows[-1]["ranks"]
    summary = {
        "config": f"config 2 frame split over {N} in-process ranks on one GPU ({B} brick(s) of {n}^3 each), "
                  f"{W}x{H}, S={S}; stages serialised per rank",
        "image_equals_1rank_all_frames": same,
        "exchange_bytes_per_rank": [r["exchange_bytes"] for r in last],
        "exchange_bytes_mean": float(np.mean([r["exchange_bytes"] for r in last])),
        "exchange_entries_per_rank": [r["exchange_entries"] for r in last],
        "slotted_alltoall_bytes_per_rank": (N - 1) * B * H * (W // N) * S * 24,
        "ms_compact_per_rank": [r["ms_compact"] for r in last],
        "ms_render_per_rank": [r["ms_render"] for r in last],
        "ms_flatten_wall_per_rank": [round(r["composite_wall_ms"], 3) for r in last],
        "ms_exchange_wall_per_rank": [round(r["exchange_wall_ms"], 3) for r in last],
        "frames": rows,
    }
    print(json.dumps({k: v for k, v in summary.items() if k != "frames"}), flush=True)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(summary, indent=1))
    for c in ctxs:
        c.close()
    ref.close()
    g.close()
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
