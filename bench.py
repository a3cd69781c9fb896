#!/usr/bin/env python3
"""Benchmark of the distributed VDI hot path (BASELINE.json metric, config 2).

One "step" = one in-situ frame of an 8 x 512^3 fp32 Gray-Scott volume (2x2x2 bricks of a
1024^3 global grid) at 1920x1080, S = 20 supersegments:
    render (VDI generation of every local brick) -> screen-strip all-to-all (RCCL)
    -> sort-last composite of the strip -> gather of the RGBA strips on rank 0
    -> the final image copied to a (pinned) host buffer on rank 0, as streamImage receives it.
The 8 bricks are the units of work: with N GPUs each rank owns 8/N of them (virtual ranks),
so the image is identical for every N and the total work is fixed ("strong" scaling).
Bricks are resident in HBM before the timed region (in-situ: the simulation's device array).

Other BASELINE.json configs (reported in DESIGN.md, not the headline line): --config 1 (one 128^3
Gray-Scott volume at 1280x720 on one rank, VDI or --mode plain, with its own CPU baseline),
--config 3 (vortex-in-cell |w| on a 1024^3 global grid, one z-slab per GPU), --config 4 (8 x 768^3
bricks at 3840x2160).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4]
  N > 1 is launched by torch.distributed.run (one process per GPU, RCCL for the data path;
  a gloo group is used only to bootstrap the RCCL id and for the timing barrier).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT / "scenery-insitu_amd", ROOT / "tests", ROOT):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

W_IMG, H_IMG, S = 1920, 1080, 20          # config 2 (and 3); config 4 renders 3840x2160
N_GLOBAL, BRICKS_PER_AXIS = 1024, 2
N_BRICKS = BRICKS_PER_AXIS ** 3
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_brick(brick_id: int, n: int, device, sim_n: int = 128) -> torch.Tensor:
    """One Gray-Scott brick: simulated on a sim_n^3 grid (default 128^3, trilinearly upsampled to n^3;
    --sim-n n simulates at full resolution: finer structure, more supersegments)."""
    from insitu_amd import scene
    v = scene.gray_scott(n, steps=1500, seed=1000 + brick_id, device=device, sim_n=sim_n)
    return v.contiguous()


def cpu_baseline(camera, vols, models, ctx_tf, n: int, threads: int, budget_s: float = 20.0,
                 W_IMG: int = W_IMG, H_IMG: int = H_IMG, n_total: int = N_BRICKS, plain: bool = False):
    """Oracle on this host's cores: whole-frame generation of the bricks one after another until the
    time budget is used, scaled to all n_total bricks if the budget ran out first.  VDI mode: the C
    restatement of VDIGenerator.comp + AccumulateVDI.comp (OpenMP over columns); plain mode: of
    VolumeRaycaster.comp + AccumulatePlainImage.comp (row blocks on a thread pool)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    import oracle_binding as orc
    from insitu_amd import native, scene
    tf, cmap = ctx_tf
    lib = orc.load()
    if plain:
        color = np.zeros((H_IMG, W_IMG, 4), np.uint8)
        depth = np.zeros((H_IMG, W_IMG, 4), np.uint8)
    else:
        color = np.zeros((W_IMG, H_IMG, S, 4), np.float32)
        depth = np.zeros((W_IMG, H_IMG, 2 * S), np.float32)
        octree = np.zeros((S, H_IMG // 8, W_IMG // 8), np.uint32)
        passes = np.zeros((H_IMG, W_IMG), np.int32)
    done, t_total = 0, 0.0
    hosts = {}
    # bricks in turn until the budget is spent, and for at least 3 s (a small config repeats its frame)
    while t_total < budget_s and (done < len(vols) or t_total < min(3.0, budget_s)):
        b = done % len(vols)
        vol = vols[b]
        if b not in hosts:
            hosts[b] = vol.detach().cpu().numpy()
        host = hosts[b]
        inp = orc.Inputs(host, scene.inverse_model(models[b]), tf, cmap,
                         scene.folded_conv_scale(1.0 / 0.5, native.F32), 0.0, camera)
        t0 = time.perf_counter()
        if plain:
            step = (H_IMG + 4 * threads - 1) // (4 * threads)

            def rows(y0):
                return lib.orc_plain_raycast(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam),
                                             W_IMG, H_IMG, color.ctypes.data, depth.ctypes.data, y0,
                                             min(H_IMG, y0 + step))
            with ThreadPoolExecutor(threads) as ex:
                assert all(r == 0 for r in ex.map(rows, range(0, H_IMG, step)))
        else:
            octree[:] = 0
            rc = lib.orc_vdi_generate_mt(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam),
                                         W_IMG, H_IMG, S, color.ctypes.data, depth.ctypes.data, octree.ctypes.data,
                                         passes.ctypes.data, threads)
            assert rc == 0
        t_total += time.perf_counter() - t0
        done += 1
    sec_per_frame = t_total / done * n_total
    what = ("VolumeRaycaster.comp+AccumulatePlainImage.comp), thread pool" if plain else
            "VDIGenerator.comp+AccumulateVDI.comp), OpenMP")
    return {"value": 1.0 / sec_per_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": (f"C oracle (restatement of {what} {threads} threads, "
                       f"{done} brick renders of a {n_total}-brick frame, full-frame ({W_IMG}x{H_IMG}"
                       + ("" if plain else f", S={S}") + f") in {t_total:.1f} s"
                       + ("" if done % n_total == 0 else f", scaled to whole frames")
                       + "; compositing (<1% of the GPU frame) not included")}


VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2   # 256 CUs x 4 SIMD32, one wave64 VALU op per 2 cycles at 2.4 GHz


def pmc_profile():
    """(tag, summary) of the committed rocprofv3 summary of this configuration (profiles/CURRENT names
    the profile of the build in the tree; an N=1 config-2 run), or None."""
    cur = ROOT / "profiles" / "CURRENT"
    files = ([ROOT / "profiles" / cur.read_text().strip() / "summary.json"] if cur.exists()
             else sorted((ROOT / "profiles").glob("*/summary.json")))
    best = None
    for f in files:
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if d.get("_config", {}).get("bench_args_n1") is not None:
            best = (f.parent.name, d)
    return best


def profile_matches_head(prof) -> bool:
    """The profile was taken of the kernels this tree builds (tools/src_hash.py over csrc/, the Makefile and the
    header, recorded by tools/prof_summary.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("src_hash", ROOT / "tools" / "src_hash.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return bool(prof) and prof[1].get("_config", {}).get("csrc_sha16") == mod.csrc_hash(ROOT)


def generator_kernels(summary):
    """The VDI generator kernels of a profile summary (the render stage's sampling and search work)."""
    return {name: v for name, v in summary.items()
            if name.startswith(("vdi_sample_kernel", "vdi_search_kernel"))}


def pmc_traffic(prof):
    """HBM bytes per frame of the generator kernels (FETCH_SIZE x2 + WRITE_SIZE per launch), with the
    raw FETCH_SIZE bytes (the x2 gfx950 correction: every read request is a 128-B line of which FETCH_SIZE
    counts 64 B, for streaming 16-B and scattered 32-B / 8-B reads alike, profiles/r04_calib), or None."""
    if not prof:
        return None
    k = [v for v in generator_kernels(prof[1]).values() if "hbm_bytes_per_launch" in v]
    if not k:
        return None
    return {"tag": prof[0], "hbm": sum(v["hbm_bytes_per_launch"] for v in k),
            "fetch_raw": sum(v["fetch_bytes_per_launch_raw"] for v in k),
            "write": sum(v["write_bytes_per_launch"] for v in k)}


def valu_roofline(prof, frame_ms=None):
    """The VALU bound of the generator kernels from the profile's SQ counters, per kernel and for the
    render stage: wave-level VALU / SALU instructions per frame, VALU issue fraction against
    256 CU x 4 SIMD x 1.2 G wave-insts/s over the kernel's profiled duration, lane utilisation
    (active lanes per VALU instruction), and their product (the fraction of the chip's VALU lanes doing
    work).  frame_ms (pipelined frames, whose kernels overlap): the render stage's fractions over the frame
    period instead of the sum of the kernels' durations."""
    if not prof:
        return None
    out, tot_v, tot_t, tot_lane = {}, 0.0, 0.0, 0.0
    for name, v in sorted(generator_kernels(prof[1]).items()):
        if "valu_wave_insts_per_launch" not in v or not v.get("avg_ms"):
            continue
        t = v["avg_ms"] * 1e-3
        issue = v["valu_wave_insts_per_launch"] / (VALU_PEAK_WAVE_INSTS * t)
        lane = v.get("lane_utilisation")
        out[name.split("<")[0]] = {
            "ms": round(v["avg_ms"], 3), "valu_insts": v["valu_wave_insts_per_launch"],
            "salu_insts": v.get("salu_wave_insts_per_launch"), "issue_frac": round(issue, 4),
            "lane_util": round(lane, 4) if lane else None,
            "effective_frac": round(issue * lane, 4) if lane else None}
        tot_v += v["valu_wave_insts_per_launch"]
        tot_t += t
        tot_lane += v["valu_wave_insts_per_launch"] * (lane or 0.0)
    if not out:
        return None
    if frame_ms:
        tot_t = frame_ms * 1e-3
    issue = tot_v / (VALU_PEAK_WAVE_INSTS * tot_t)
    return {"source": f"profiles/{prof[0]}/summary.json (rocprofv3 SQ_INSTS_VALU, SQ_INSTS_SALU, "
                      "SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU)",
            "peak_wave_insts_per_s": VALU_PEAK_WAVE_INSTS, "kernels": out,
            "render_issue_frac": round(issue, 4), "render_effective_frac": round(tot_lane / tot_v * issue, 4)}


def self_launch(n: int) -> int:
    """Run this script on n ranks (one per GPU) with torch.distributed.run as a child process;
    stdout/stderr are inherited, so rank 0's JSON line is this process's output."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *sys.argv[1:]]
    log(f"[bench] --gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--brick", type=int, default=0, help="brick edge (config 2/4; default 512/768)")
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4))
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="tuning aid: on one GPU, render only the bricks rank --emulate-rank would own in an "
                         "N-GPU run (no exchange); the JSON line is marked 'emulated'")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=V",
                    help="tuning option for insitu_set_option (experiments; results are identical by construction): "
                         "search_depth, long_samples, round_batch, search_oversub")
    ap.add_argument("--update-every", type=int, default=20,
                    help="re-ingest every local brick every K frames, timed as the reference's 'GPU-send' "
                         "(DistributedVolumeRenderer.kt:521-527, updateVolumes :656-681); 0 = never")
    ap.add_argument("--sim-n", type=int, default=512,
                    help="config 2/4: grid the Gray-Scott bricks are simulated on (default 512: the brick edge, "
                         "full resolution, ~1 s per brick on the GPU; smaller grids are upsampled)")
    ap.add_argument("--mode", choices=("vdi", "plain"), default="vdi",
                    help="vdi: VDIGenerator+AccumulateVDI -> exchange -> composite (DistributedVolumes.kt); "
                         "plain: VolumeRaycaster+AccumulatePlainImage -> PlainImageCompositor "
                         "(DistributedVolumeRenderer.kt:182-188)")
    ap.add_argument("--compositor", choices=("flatten", "vdi"), default="flatten",
                    help="VDI mode: flatten the merged lists to RGBA (default) or VDICompositor.comp "
                         "(re-supersegmented composited VDI, S_out = S, gathered on rank 0; DistributedVolumes.kt:423-439)")
    ap.add_argument("--merge-bricks", action="store_true",
                    help="VDI mode: each rank's bricks are the volumes of ONE sub-VDI ($repeat, VDIGenerator.comp:333-347) "
                         "instead of one sub-VDI (virtual rank) per brick")
    ap.add_argument("--pipeline", type=int, default=1, choices=(0, 1),
                    help="VDI mode: 1 = pipelined frames (insitu_frame_pipelined: frame k+1's render overlaps frame k's "
                         "search tail, exchange, composite and gather -- the reference's one-frame-stale loop, "
                         "DistributedVolumeRenderer.kt:530-542); 0 = each frame completes before the next starts")
    ap.add_argument("--update-source", choices=("device", "host"), default="device",
                    help="where the simulation's brick lives: device (GPU simulation, read in place) or "
                         "host (pinned host copy uploaded over PCIe, as the reference's shared-memory grids)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least one GPU")
    if args.steps < 1 or args.warmup < 0:
        raise SystemExit(f"--steps {args.steps} --warmup {args.warmup}: need at least one timed step")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start one process per GPU under
        # torch.distributed.run as a CHILD (nothing here has touched the GPU yet), relay its output
        # (rank 0 prints the JSON line) and exit with its status
        sys.exit(self_launch(args.gpus))

    from insitu_amd import native, scene
    from insitu_amd.renderer import InSituContext

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    N = max(world, 1)
    if args.gpus != N:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: the GPU count must equal the world size")
    cfg = args.config
    W_IMG, H_IMG = {1: (1280, 720), 4: (3840, 2160)}.get(cfg, (1920, 1080))
    if cfg == 1 and N != 1:
        raise SystemExit("--config 1 is the reference's one-rank case: --gpus 1")
    # config 3: one slab per GPU; config 1: one volume; else 8 bricks (virtual ranks)
    n_units = N if cfg == 3 else (1 if cfg == 1 else N_BRICKS)
    if n_units % N:
        raise SystemExit(f"{n_units} bricks do not split over {N} GPUs")
    B = n_units // N
    emu = args.emulate_world > 1 and N == 1 and cfg == 2
    if emu:
        B = N_BRICKS // args.emulate_world
    ndev = torch.cuda.device_count()   # (does not initialise the GPU)
    if N > ndev:
        # more ranks than GPUs (rehearsal on a small box): ranks share GPUs, and distinct NCCL host
        # ids make RCCL accept that and connect them through its socket transport on loopback
        os.environ["NCCL_HOSTID"] = f"insitu-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    dev = torch.device("cuda", local_rank % max(1, ndev))
    torch.cuda.set_device(dev)
    pg = None
    if N > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=N)
        pg = dist
    comm_id = None
    if N > 1:
        buf = torch.zeros(native.COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            import ctypes
            raw = ctypes.create_string_buffer(native.COMM_ID_BYTES)
            native.check(native.load().insitu_comm_id(raw, native.COMM_ID_BYTES), None, "insitu_comm_id")
            buf = torch.frombuffer(bytearray(raw.raw), dtype=torch.uint8).clone()
        pg.broadcast(buf, 0)
        comm_id = bytes(buf.numpy().tobytes())

    # ---- scene: bricks of a [-1,1]^3 cube, this rank's bricks generated on its GPU
    #   config 2/4: 2x2x2 Gray-Scott bricks; config 3: z-slabs of one 1024^3 vortex-ring grid
    n = args.brick or {1: 128, 4: 768}.get(cfg, N_GLOBAL // BRICKS_PER_AXIS)
    first = (args.emulate_rank if emu else rank) * B
    my_ids = list(range(first, first + B))
    t0 = time.perf_counter()
    vols, models = [], []
    if cfg == 3:
        ng = args.brick or N_GLOBAL
        bricks = scene.slab_bricks(ng, N)
        for bid in my_ids:
            origin, vw, (z0, nz) = bricks[bid]
            vols.append(scene.vortex_ring(ng, z0, nz, device=dev))
            models.append(scene.brick_model(origin, vw))
        vb = ng * ng * (ng // N) * 4
        what = f"vortex-ring |w| slab(s) of {ng}^2 x {ng // N}"
    else:
        bricks = scene.grid_bricks(n, 1) if cfg == 1 else scene.grid_bricks(n * BRICKS_PER_AXIS, BRICKS_PER_AXIS)
        for bid in my_ids:
            origin, vw, _ = bricks[bid]
            vols.append(make_brick(bid, n, dev, sim_n=min(args.sim_n, n)))
            models.append(scene.brick_model(origin, vw))
        vb = n ** 3 * 4
        what = f"Gray-Scott bricks of {n}^3"
    torch.cuda.synchronize()
    log(f"[rank {rank}] generated {B} {what} fp32 in {time.perf_counter() - t0:.1f} s")

    tf, cmap = scene.transfer_function(), scene.colormap_hot()
    vdi = args.mode == "vdi"
    ctx = InSituContext(W_IMG, H_IMG, mode=native.MODE_VDI if vdi else native.MODE_PLAIN, max_supersegments=S,
                        bricks_per_rank=B, rank=rank, nranks=N, device=dev.index, comm_id=comm_id, keep_passes=vdi,
                        composite_vdi=vdi and args.compositor == "vdi", max_output_supersegments=S if vdi else 0,
                        merge_bricks=vdi and args.merge_bricks)
    # display range: Gray-Scott v in [0, 0.5], vortex |w| in [0, 1]
    ctx.set_transfer(tf, cmap, conv_scale=1.0 if cfg == 3 else 1.0 / 0.5, conv_offset=0.0)
    for opt in args.option:
        name, val = opt.split("=")
        ctx.set_option(getattr(native, "OPT_" + name.upper()), int(val))
    for slot, v in enumerate(vols):
        ctx.set_brick(slot, v, models[slot], dtype=native.F32)
    vw = bricks[0][1]
    # the simulation's arrays the periodic update re-ingests (host: pinned copies, DMA-able)
    sources = [v.cpu().pin_memory() for v in vols] if args.update_source == "host" else vols

    def update_volumes(g):
        """DistributedVolumeRenderer.kt:521-527: every K-th frame (counting from 0) re-ingest the grids.  Returns
        the host seconds it took, or None when no update was due.  Unpipelined frames wait for the re-ingest (its
        wall time is the reference's "GPU-send"); pipelined frames do not: the library orders it after the search
        of the frame in flight and before the next first pass, and its GPU time is insitu_stats.ms_ingest."""
        if args.update_every <= 0 or g % args.update_every:
            return None
        t = time.perf_counter()
        for slot, v in enumerate(sources):
            ctx.set_brick(slot, v, models[slot], dtype=native.F32)
        if not (vdi and args.pipeline == 1):
            ctx.synchronize()
        return time.perf_counter() - t

    def cam_at(i):
        return scene.orbit_camera(W_IMG, H_IMG, yaw_deg=30.0 + 5.0 * i, pitch_deg=20.0, voxel_world=vw)

    cams = [cam_at(i) for i in range(args.warmup + args.steps)]

    def barrier():
        if pg is not None:
            pg.barrier()

    # the root's final image lands in a host buffer every frame, as streamImage receives it
    # (DistributedVolumeRenderer.kt:726; the gather buffer is native-owned memory in the reference: pinned here)
    img_host = torch.empty((H_IMG, W_IMG, 4), dtype=torch.uint8, pin_memory=True) if rank == 0 else None

    pipelined = vdi and args.pipeline == 1

    def frame(cam):
        """One frame call; returns the index of the frame it completed (pipelined: the one before, or -1)."""
        if pipelined:   # (the library counts frames from the context's first: the warmup frames come first)
            done = ctx.frame_pipelined(cam, want_image=rank == 0, out=img_host)[0]
            return done - args.warmup if done >= 0 else -1
        ctx.frame(cam, want_image=rank == 0, out=img_host)
        return 0

    def flush():
        done = ctx.pipeline_flush(want_image=rank == 0, out=img_host)[0] if pipelined else -1
        return done - args.warmup if done >= 0 else -1

    for i in range(args.warmup):
        update_volumes(i)
        frame(cams[i])
    flush()
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    stage = np.zeros(8)
    render_ms, latency_ms, host_latency_ms = [], [], []
    counters = np.zeros(3)
    gpu_send, n_updates = 0.0, 0
    last_stats = ctx.stats()
    t_call = {}

    def account(done):
        """Per-stage HIP-event times and counters of the frame just completed (already synchronised)."""
        nonlocal stage, counters, last_stats
        if done < 0:
            return
        host_latency_ms.append(1e3 * (time.perf_counter() - t_call[done]))
        st = ctx.stats()
        stage += [st["ms_render"], st["ms_exchange"], st["ms_composite"], st["ms_gather"], st["ms_sample"],
                  st["ms_search"], st["ms_exchange_sync"], st["ms_image_d2h"]]
        counters += [st["rays_searched"], st["rays_uncached"], st["exchange_bytes"]]
        render_ms.append(st["ms_render"])
        latency_ms.append(st["ms_latency"])
        last_stats = st

    for i in range(args.steps):
        dt = update_volumes(args.warmup + i)
        if dt is not None:
            gpu_send += dt
            n_updates += 1
        t_call[i] = time.perf_counter()
        done = frame(cams[args.warmup + i])
        account(done if pipelined else i)
    account(flush())   # (pipelined: the last frame completes here, in the timed region)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if pg is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        elapsed = float(t.item())
    mean_passes, rays_hit = ctx.pass_stats() if vdi else (1.0, 0)
    if pipelined and n_updates:   # the re-ingests' GPU time (the last batch, complete after the flush)
        gpu_send = n_updates * 1e-3 * ctx.stats()["ms_ingest"]

    if rank == 0:
        fps = args.steps / elapsed
        assert len(render_ms) == args.steps, (len(render_ms), args.steps)
        # the render stage's time per frame: its HIP-event span; pipelined, consecutive renders overlap (frame
        # k+1's first pass runs in frame k's search tail), so the spans add up to more than the frames take and
        # the frame period (wall time per frame, everything included) is the render's share -- conservative
        ms_render = float(np.mean(render_ms))
        if pipelined:
            ms_render = min(ms_render, 1000.0 * elapsed / args.steps)
        # algorithmic bytes of the dominant kernel:
        #   VDI mode, per brick Vb * P_mean (one brick read per raymarch pass), per sub-VDI H*W*S*24 (VDI out)
        #   + octree (one sub-VDI per brick, or one per rank with merged bricks)
        #   plain mode, per brick Vb (one pass) + 8*H*W (rgba8 colour + encoded depth)
        if vdi:
            sub_vdis = 1 if args.merge_bricks else B
            alg_bytes = vb * mean_passes * B + (W_IMG * H_IMG * S * 24 + (W_IMG // 8) * (H_IMG // 8) * S * 4) * sub_vdis
        else:
            alg_bytes = (vb + 8 * W_IMG * H_IMG) * B
        achieved = alg_bytes / (ms_render * 1e-3) / 1e9
        cpu = None
        default_run = vdi and args.compositor == "flatten" and not args.merge_bricks
        if not args.no_cpu_baseline and N == 1 and not emu and (cfg == 2 and default_run or cfg == 1):
            threads = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(cams[args.warmup], vols, models, (tf, cmap), n, threads, args.cpu_budget,
                               W_IMG=W_IMG, H_IMG=H_IMG, n_total=n_units, plain=not vdi)
        prof = pmc_profile() if (N == 1 and not emu and cfg == 2 and n == N_GLOBAL // BRICKS_PER_AXIS and
                                 default_run) else None
        prof_ok = profile_matches_head(prof)
        # the profile's traffic and VALU figures describe this build only if its kernels are this tree's
        traffic = pmc_traffic(prof) if prof_ok else None
        valu = valu_roofline(prof, ms_render if pipelined else None) if prof_ok else None
        traffic_frac = traffic["hbm"] / 1e9 / (ms_render * 1e-3) / HBM_PEAK_GBS if traffic else None
        valu_frac = valu["render_effective_frac"] if valu else None
        # the bound that governs: the larger of the measured HBM traffic's and the effective VALU's share of
        # their peaks over the render stage, when it is near that peak (> 0.6); with both below it neither
        # unit is saturated and the kernels wait on per-ray latency ("latency").  (BASELINE.md quotes HBM GB/s,
        # so `frac` stays the HBM figure.)
        governing = None
        if traffic_frac is not None and valu_frac is not None:
            top = max(traffic_frac, valu_frac)
            governing = "latency" if top <= 0.6 else ("valu" if valu_frac >= traffic_frac else "hbm")
        workload = {1: f"config 1: one {n}^3 fp32 Gray-Scott volume, 1 rank",
                    2: f"config 2: 8 bricks x {n}^3 fp32 Gray-Scott",
                    3: f"config 3: vortex-in-cell |w| {args.brick or N_GLOBAL}^3 global grid fp32, {N} z-slab(s)",
                    4: f"config 4: 8 bricks x {n}^3 fp32 Gray-Scott"}[cfg]
        metric = {1: "frames/sec @1280x720 (128^3 volume, 1 rank)",
                  2: "frames/sec @1920x1080 (8x512^3 volume)",
                  3: "frames/sec @1920x1080 (1024^3 vortex-in-cell, slab per GPU)",
                  4: "frames/sec @3840x2160 (8x768^3 volume)"}[cfg]
        if not default_run:
            metric += (", plain mode" if not vdi else "") + (", VDICompositor" if vdi and args.compositor == "vdi"
                                                              else "") + (", merged bricks" if vdi and args.merge_bricks else "")
        pipeline = ("VDI generate + strip all-to-all + " + ("VDICompositor composite + composited-VDI gather"
                                                            if args.compositor == "vdi" else "flatten composite + gather")
                    + (" (bricks merged into one sub-VDI per rank)" if args.merge_bricks else "")) if vdi else \
            "plain raymarch (ERT) + all-to-all + PlainImageCompositor + gather"
        kernels = ("render stage = vdi_sample_kernel + vdi_search_kernel" if not args.merge_bricks else
                   "render stage = vdi_merge_kernel") if vdi else "render stage = plain_generate_kernel"
        out = {
            "metric": metric,
            "value": fps, "unit": "frames/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (vortex ring, seed 1000)" if cfg == 3 else
            f"synthetic (Gray-Scott simulated on {min(args.sim_n, n)}^3, seed 1000+brick)",
            "config": {"workload": f"{workload}, {W_IMG}x{H_IMG}, S={S}, {pipeline}", "mode": args.mode,
                       "bricks_per_gpu": B, "mean_raymarch_passes": round(mean_passes, 3),
                       "rays_hit_per_frame": int(rays_hit),
                       "rays_searched_per_frame": int(counters[0] / args.steps),
                       "rays_without_cache_space": int(counters[1] / args.steps),
                       "sample_cache_gb": round(last_stats["cache_bytes"] / 1e9, 3),
                       "sample_cache_demand_gb": round(last_stats["cache_demand_bytes"] / 1e9, 3),
                       "exchange_bytes_per_rank": int(counters[2] / args.steps),
                       "update_every": args.update_every, "update_source": args.update_source,
                       "gpu_send_ms_per_update": round(1e3 * gpu_send / n_updates, 3) if n_updates else None,
                       "pipeline_depth": 2 if pipelined else 1,
                       "frame_latency_ms": round(float(np.mean(latency_ms)), 3),
                       "frame_latency_host_ms": round(float(np.mean(host_latency_ms)), 3),
                       "stage_ms": dict(zip(["render", "exchange", "composite", "gather", "render.sample_kernel",
                                             "render.search_kernel", "exchange.host_sync_idle", "image_d2h"],
                                            [round(x / args.steps, 3) for x in stage]))
                       | {"gpu_send": round(1e3 * gpu_send / args.steps, 3)}},
            "roofline": {"kernel": kernels, "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["hbm"] if traffic else None,
                         "traffic_gbs": (traffic["hbm"] / 1e9 / (ms_render * 1e-3)) if traffic else None,
                         "traffic_fetch_raw": traffic["fetch_raw"] if traffic else None,
                         "traffic_fetch_x2": 2 * traffic["fetch_raw"] if traffic else None,
                         "traffic_write": traffic["write"] if traffic else None,
                         "traffic_source": (f"profiles/{traffic['tag']}/summary.json (rocprofv3 FETCH_SIZE*2+WRITE_SIZE; "
                                            "the x2 is calibrated for 16-B/lane streaming reads and for scattered "
                                            "32-B and 8-B reads alike: every read request is one 128-B line, "
                                            "FETCH_SIZE counts 64 B of it, profiles/r04_calib)") if traffic else None,
                         "traffic_frac": traffic_frac,
                         "valu": valu,
                         "render_effective_frac": valu_frac,
                         "governing": governing,
                         "profile": prof[0] if prof else None,
                         "profile_matches_head": prof_ok if prof else None,
                         "algorithmic_bytes_per_frame": alg_bytes,
                         "note": ("achieved = algorithmic bytes (Vb*P_mean + H*W*S*24 + octree per brick, SURVEY.md "
                                  "8d) / render-stage HIP-event time; traffic = measured HBM bytes per frame (traffic_frac = traffic / "
                                  "render time / peak); render_effective_frac = VALU issue x lane utilisation over the "
                                  "generator kernels; governing = the larger of the two when it exceeds 0.6, else "
                                  "'latency': the generator waits on per-ray latency of the threshold re-march (VALU "
                                  "issue and memory round trips of dependent passes), neither unit is saturated; "
                                  "traffic and valu are withheld unless the profile's csrc hash is this tree's. "
                                  "Pipelined frames: the render time per frame is the frame period") if vdi else
                                 "achieved = algorithmic bytes (Vb + 8*H*W per brick, SURVEY.md 8d) / render-stage "
                                 "HIP-event time"},
            "cpu_baseline": cpu,
        }
        if emu:
            out["emulated"] = f"bricks {my_ids} of an {args.emulate_world}-GPU run on one GPU, no exchange"
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    ctx.synchronize()
    ctx.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
