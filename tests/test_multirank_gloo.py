"""N > 1 decomposition on CPU (gloo, world_size 2 and 4): each rank renders its bricks' sub-VDIs
(oracle), the screen-strip blocks are exchanged with an all-to-all, each rank flattens its
strip, rank 0 gathers the strips -- and the image equals the single-rank composite of all
bricks.  This is the decomposition libinsitu_hip.so runs with RCCL on device (insitu_exchange,
insitu_composite, insitu_gather); here the transport is gloo and the compute the oracle."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent

W, H, S, N_BRICKS = 32, 24, 4, 4
S_OUT = 3


def _scene():
    sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests")]
    from insitu_amd import scene
    from scenes import gray_scott_u16
    vol = gray_scott_u16(16)
    cam = scene.orbit_camera(W, H, yaw_deg=40.0, pitch_deg=25.0, voxel_world=1.0 / 16)
    bricks = []
    for i in range(N_BRICKS):    # 4 bricks of a 2x2x1 arrangement, each 16^3 with its own data
        origin = (-1.0 + (i % 2), -1.0 + (i // 2), -0.5)
        model = scene.brick_model(origin, 1.0 / 16)
        bricks.append((np.roll(vol, 3 * i, axis=0).copy(), scene.inverse_model(model)))
    return cam, bricks, scene.transfer_function(), scene.colormap_hot()


def _sub_vdi(brick, cam, tf, cmap):
    import oracle_binding as orc
    from insitu_amd import native, scene
    vol, im = brick
    inp = orc.Inputs(vol, im, tf, cmap, scene.folded_conv_scale(1.0, native.U16), 0.0, cam)
    c, d, _, _ = orc.vdi_generate(inp, W, H, S)
    return c, d


def _worker(rank, world, port, q, sc, composite_vdi=False):
    import torch
    import torch.distributed as dist
    torch.set_num_threads(1)
    sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_binding as orc
        from insitu_amd import partition
        cam, bricks, tf, cmap = sc
        mine = partition.bricks_of_rank(rank, world, N_BRICKS)
        B = len(mine)
        subs = [_sub_vdi(bricks[i], cam, tf, cmap) for i in mine]
        x0, sw = partition.strip_of_rank(rank, world, W)
        # send blocks [d][b]: strip d of my brick b (reference layout: x slowest -> contiguous)
        send_c = [torch.from_numpy(np.ascontiguousarray(np.stack([c[d * sw:(d + 1) * sw] for c, _ in subs])))
                  for d in range(world)]
        send_d = [torch.from_numpy(np.ascontiguousarray(np.stack([dd[d * sw:(d + 1) * sw] for _, dd in subs])))
                  for d in range(world)]
        recv_c = [torch.empty_like(send_c[0]) for _ in range(world)]
        recv_d = [torch.empty_like(send_d[0]) for _ in range(world)]
        # the all-to-all as pairwise send/recv (gloo has no alltoall; the device path uses
        # grouped ncclSend/ncclRecv the same way, insitu_exchange)
        recv_c[rank], recv_d[rank] = send_c[rank], send_d[rank]
        reqs = []
        for p in range(world):
            if p != rank:
                reqs += [dist.isend(send_c[p], p), dist.isend(send_d[p], p),
                         dist.irecv(recv_c[p], p), dist.irecv(recv_d[p], p)]
        for r in reqs:
            r.wait()
        colors, depths = [], []
        for s, b in partition.list_order(world, B):
            # pad back to full-width arrays so the oracle flatten sees global x indexing
            cfull = np.zeros((W, H, S, 4), np.float32)
            dfull = np.zeros((W, H, 2 * S), np.float32)
            cfull[x0:x0 + sw] = recv_c[s][b].numpy()
            dfull[x0:x0 + sw] = recv_d[s][b].numpy()
            colors.append(cfull)
            depths.append(dfull)
        if composite_vdi:   # VDICompositor.comp on the strip, composited VDIs gathered (DistributedVolumes.kt:903)
            oc, od, _ = orc.vdi_composite(colors, depths, W, H, x0, sw, orc.ipv_of(cam), S_OUT)
            parts = [torch.from_numpy(oc), torch.from_numpy(od)]
            out = []
            for t in parts:
                gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
                dist.gather(t, gathered, dst=0)
                if rank == 0:
                    out.append(np.concatenate([g.numpy() for g in gathered], axis=0))
            if rank == 0:
                q.put(tuple(out))
        else:
            strip = torch.from_numpy(orc.vdi_flatten(colors, depths, W, H, x0, sw, orc.ipv_of(cam)))
            gathered = [torch.empty_like(strip) for _ in range(world)] if rank == 0 else None
            dist.gather(strip, gathered, dst=0)
            if rank == 0:
                q.put(np.concatenate([g.numpy() for g in gathered], axis=1))
    except Exception as e:  # report instead of leaving the parent waiting
        q.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,composite_vdi", [(2, False), (4, False), (2, True)])
def test_distributed_frame_matches_single_rank(world, composite_vdi):
    sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests")]
    import oracle_binding as orc
    sc = _scene()      # simulated once here; workers get the inputs (as ranks get their bricks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, sc, composite_vdi)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=300)
    assert not isinstance(img, str), img
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    cam, bricks, tf, cmap = sc
    subs = [_sub_vdi(b, cam, tf, cmap) for b in bricks]
    if composite_vdi:
        oc, od, _ = orc.vdi_composite([c for c, _ in subs], [d for _, d in subs], W, H, 0, W, orc.ipv_of(cam), S_OUT)
        assert np.count_nonzero(od) > 0
        assert np.array_equal(img[0].view(np.uint32), oc.view(np.uint32))
        assert np.array_equal(img[1].view(np.uint32), od.view(np.uint32))
        return
    ref = orc.vdi_flatten([c for c, _ in subs], [d for _, d in subs], W, H, 0, W, orc.ipv_of(cam))
    assert np.count_nonzero(ref[..., 3]) > 0
    assert np.array_equal(img, ref)
