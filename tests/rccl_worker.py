"""One rank of the multi-process RCCL check (launched by tests/test_gpu_rccl.py through
torch.distributed.run; test infrastructure).

Every case runs the N-rank data path of libinsitu_hip.so with RCCL as the transport -- grouped
ncclSend/ncclRecv of screen-strip blocks (insitu_exchange, the MPI_Alltoall behind
DistributedVolumes.kt:860-861), the composite of this rank's strip, and the gather to rank 0
(insitu_gather, the MPI_Gather behind DistributedVolumes.kt:903-904) -- and rank 0 compares the
result with a single-rank context that renders every brick itself (bit for bit):
  vdi      : VDI mode, RGBA flatten, bricks split over the ranks
  cvdi     : VDI mode, VDICompositor output gathered as a composited VDI
  plain    : plain mode (VolumeRaycaster + PlainImageCompositor)
  host     : the reference-shaped host-buffer entry points distributeVDIs -> composite ->
             gatherCompositedVDIs (insitu_distribute_vdis / insitu_gather_composited_vdis)
  host_cvdi: distributeVDIs -> VDICompositor -> gatherCompositedVDIs(colour, depth) (the set)
  pipe     : pipelined frames (insitu_frame_pipelined, three cameras + the flush): each completed frame's
             image equals the single-rank frame of its camera (the exchange runs in the next frame's call)
  pipe_cvdi: the same through the VDICompositor (gathered composited VDI of every frame)
When the ranks outnumber the GPUs (a one-GPU box), each rank announces a distinct NCCL host id so
that RCCL accepts two ranks on one device and connects them through its socket transport on the
loopback interface: the same library code paths, a slower wire.
"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests")]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])

import torch  # noqa: E402

if torch.cuda.device_count() < world:   # before any RCCL call (RCCL reads these at its first init)
    os.environ["NCCL_HOSTID"] = f"insitu-rank-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from insitu_amd import native, scene  # noqa: E402
from insitu_amd.renderer import InSituContext  # noqa: E402
from scenes import gray_scott_u16  # noqa: E402

dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group("gloo")
W, H, S = 64, 48, 6
NB = 8 if world == 8 else 4   # bricks (virtual ranks): 2x2x1, or 2x2x2 for the 8-way decomposition
vol = gray_scott_u16(32)
bricks = [(np.roll(vol, 5 * i, axis=1).copy(),
           scene.brick_model((-1.0 + (i % 2), -1.0 + ((i // 2) % 2), -0.5 + (i // 4) - (0.5 if NB == 8 else 0.0)),
                             1.0 / 32))
          for i in range(NB)]
tf, cm = scene.transfer_function(), scene.colormap_hot()


def comm_id() -> bytes:
    """A fresh ncclUniqueId for every communicator (an id serves one ncclCommInitRank)."""
    buf = torch.zeros(native.COMM_ID_BYTES, dtype=torch.uint8)
    if rank == 0:
        raw = ctypes.create_string_buffer(native.COMM_ID_BYTES)
        native.check(native.load().insitu_comm_id(raw, native.COMM_ID_BYTES))
        buf = torch.frombuffer(bytearray(raw.raw), dtype=torch.uint8).clone()
    dist.broadcast(buf, 0)
    return bytes(buf.numpy().tobytes())


def single_rank(mode, hm, cam, cvdi, mine):
    ref = InSituContext(W, hm, mode=mode, max_supersegments=S, bricks_per_rank=len(mine), device=dev,
                        composite_vdi=cvdi, max_output_supersegments=5 if cvdi else 0)
    ref.set_transfer(tf, cm)
    for s, i in enumerate(mine):
        ref.set_brick(s, *bricks[i])
    img = ref.frame(cam, want_image=True)
    gv = (ref.read(native.BUF_GATHERED_COLOR), ref.read(native.BUF_GATHERED_DEPTH)) if cvdi else None
    sub = None
    if len(mine) == 1 and mode == native.MODE_VDI:
        sub = (ref.read(native.BUF_VDI_COLOR), ref.read(native.BUF_VDI_DEPTH))
    elif len(mine) == 1:
        sub = (ref.read(native.BUF_PLAIN_COLOR), ref.read(native.BUF_PLAIN_DEPTH))
    ref.close()
    return img, gv, sub


def oracle_image(cam):
    """The CPU oracle's frame: every brick's sub-VDI (VDIGenerator.comp + AccumulateVDI.comp) merged in
    brick order and flattened (accumulateSupseg), the image the N-rank RCCL path must reproduce."""
    import oracle_binding as orc
    cols, deps = [], []
    for data, model in bricks:
        inp = orc.Inputs(data, scene.inverse_model(model), tf, cm, scene.folded_conv_scale(1.0, native.U16), 0.0, cam)
        c, d, _, _ = orc.vdi_generate(inp, W, H, S)
        cols.append(c)
        deps.append(d)
    return orc.vdi_flatten(cols, deps, W, H, 0, W, orc.ipv_of(cam))


def bits_equal(a, b):
    return a is not None and b is not None and np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                                                                np.ascontiguousarray(b).view(np.uint8))


def pipelined_case(cvdi):
    """Three pipelined frames and the flush on `world` ranks; rank 0 checks every completed frame."""
    B = NB // world
    mine = list(range(rank * B, rank * B + B))
    cams = [scene.orbit_camera(W, H, yaw_deg=35.0 + 50.0 * k, pitch_deg=20.0, voxel_world=1.0 / 32) for k in range(3)]
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=B, rank=rank, nranks=world, device=dev,
                        comm_id=comm_id(), composite_vdi=cvdi, max_output_supersegments=5 if cvdi else 0)
    ctx.set_transfer(tf, cm)
    for s_, i in enumerate(mine):
        ctx.set_brick(s_, *bricks[i])
    got = {}
    for k, cam in enumerate(cams + [None]):
        done, img = ctx.frame_pipelined(cam, want_image=True) if cam is not None else ctx.pipeline_flush(want_image=True)
        assert done == k - 1, (k, done)
        if done >= 0 and rank == 0:
            gv = (ctx.read(native.BUF_GATHERED_COLOR), ctx.read(native.BUF_GATHERED_DEPTH)) if cvdi else None
            got[done] = (img.copy(), gv)
    st = ctx.stats()
    ctx.close()
    ok = True
    if rank == 0:
        for k, cam in enumerate(cams):
            want, want_gv, _ = single_rank(native.MODE_VDI, H, cam, cvdi, list(range(NB)))
            ok = ok and bits_equal(got[k][0], want) and np.count_nonzero(want[..., 3]) > 0
            if cvdi:
                ok = ok and bits_equal(got[k][1][0], want_gv[0]) and bits_equal(got[k][1][1], want_gv[1])
        ok = ok and st["pipelined"] == 1
    return ok, st


failures = []
for case in ("pipe", "pipe_cvdi"):
    ok, st = pipelined_case(case == "pipe_cvdi")
    if rank == 0:
        print(f"[rccl] case {case}: {world}-rank pipelined frames == 1-rank frames: {ok}; exchange bytes sent by "
              f"rank 0: {st['exchange_bytes']}", flush=True)
        if not ok:
            failures.append(case)
for case in ("vdi", "cvdi", "plain", "host", "host_cvdi"):
    mode = native.MODE_PLAIN if case == "plain" else native.MODE_VDI
    cvdi = case in ("cvdi", "host_cvdi")
    hm = W if mode == native.MODE_PLAIN else H
    cam = scene.orbit_camera(W, hm, yaw_deg=35.0, pitch_deg=20.0, voxel_world=1.0 / 32)
    host = case.startswith("host")
    B = 1 if host else NB // world
    mine = [rank] if host else list(range(rank * B, rank * B + B))
    everyone = list(range(world)) if host else list(range(NB))
    ctx = InSituContext(W, hm, mode=mode, max_supersegments=S, bricks_per_rank=B, rank=rank, nranks=world,
                        device=dev, comm_id=comm_id(), composite_vdi=cvdi, max_output_supersegments=5 if cvdi else 0)
    ctx.set_transfer(tf, cm)
    img = gv = None
    if host:
        # the sub-VDI this rank's Vulkan renderer would have read back (DistributedVolumes.kt:742-744)
        _, _, (col, dep) = single_rank(mode, hm, cam, False, mine)
        ctx.set_camera(cam)
        ctx.distributeVDIs(col, dep, hm * W * S * 4 // world, world, recv=False)
        if cvdi:
            gv = ctx.gatherCompositedVDISet(H * W * 5 * 4 // world, 0, rank, world)
        else:
            img = ctx.gatherCompositedVDIs(0, hm * W * 4 // world, rank, world)
    else:
        for s, i in enumerate(mine):
            ctx.set_brick(s, *bricks[i])
        img = ctx.frame(cam, want_image=True)
        if cvdi and rank == 0:
            gv = (ctx.read(native.BUF_GATHERED_COLOR), ctx.read(native.BUF_GATHERED_DEPTH))
    st = ctx.stats()
    ctx.close()
    if rank == 0:
        want, want_gv, _ = single_rank(mode, hm, cam, cvdi, everyone)
        ok = True
        if img is not None:
            ok = ok and bits_equal(img, want) and np.count_nonzero(want[..., 3]) > 0
        if case == "vdi":   # and the N-rank image against the oracle, not only against one HIP rank
            ora = bits_equal(img, oracle_image(cam))
            print(f"[rccl] case vdi: {world}-rank image == oracle ({NB} bricks): {ora}", flush=True)
            ok = ok and ora
        if cvdi:
            ok = ok and bits_equal(gv[0], want_gv[0]) and bits_equal(gv[1], want_gv[1])
        print(f"[rccl] case {case}: {world}-rank result == 1-rank result: {ok}; exchange bytes sent by rank 0: "
              f"{st['exchange_bytes']}", flush=True)
        if not ok:
            failures.append(case)
dist.barrier()
if rank == 0:
    print("RCCL_OK" if not failures else f"RCCL_FAILED {failures}", flush=True)
dist.destroy_process_group()
sys.exit(1 if failures else 0)
