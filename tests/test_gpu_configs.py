"""GPU parity at the BASELINE.json workloads (configs 2, 3 and 4), through libinsitu_hip.so.

The whole frame is rendered on the GPU at full size; the CPU oracle (C restatement of
VDIGenerator.comp + AccumulateVDI.comp, OpenMP) recomputes the whole frame of every config (every brick's
sub-VDI and the composited image), which must match BIT FOR BIT (supersegment colours,
depths, raymarch pass counts, octree cells, and the RGBA flatten of all bricks).  On top of that the
frames are checked for size-independent properties: at most S supersegments per pixel, compact lists
(no filled slot after an empty one), end >= start, and no ray without cache space.

  config 2: 8 x 512^3 fp32 Gray-Scott bricks (2x2x2 of a 1024^3 grid), 1920x1080, S = 20 (also with the
            bricks merged into one sub-VDI, whole frame)
  config 3: vortex-ring |w| on a 1024^3 grid as 2 z-slabs (the 2-GPU decomposition), 1920x1080
            (+ the single 1024^3 slab of the 1-GPU run and the 4- and 8-slab decompositions, bit for bit)
  config 4: 8 x 768^3 fp32 Gray-Scott bricks, 3840x2160, S = 20
  config 1: one 128^3 fp32 Gray-Scott volume, 1280x720 -- whole frames bit for bit, VDI mode and the
            DistributedVolumeRenderer plain path (VolumeRaycaster + PlainImageCompositor, also as two
            z-slab virtual ranks with and without the faithful numProcesses of PlainImageCompositor.comp:43)
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import bench
import oracle_binding as orc
from insitu_amd import native, scene
from insitu_amd.renderer import InSituContext

pytestmark = pytest.mark.gpu

S = 20
THREADS = 16   # the GPU box's CPU share


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _scene(cfg: int, slabs: int = 2, sim_n: int = 128):
    """sim_n: grid the Gray-Scott bricks are simulated on (config 2/4); 512 at config 2 is the field bench.py
    times (--sim-n 512, full resolution), 128 the upsampled field of rounds 1-5's tests."""
    dev = torch.device("cuda", 0)
    if cfg == 3:
        W, H, ng = 1920, 1080, 1024
        units = scene.slab_bricks(ng, slabs)
        vols = [scene.vortex_ring(ng, z0, nz, device=dev) for (_, _, (z0, nz)) in units]
        conv = 1.0
    else:
        W, H, n = (3840, 2160, 768) if cfg == 4 else (1920, 1080, 512)
        units = scene.grid_bricks(2 * n, 2)
        vols = [bench.make_brick(b, n, dev, sim_n=min(sim_n, n)) for b in range(len(units))]
        conv = 1.0 / 0.5
    models = [scene.brick_model(origin, vw) for (origin, vw, _) in units]
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    torch.cuda.synchronize()
    return dict(W=W, H=H, vols=vols, models=models, cam=cam, conv=conv)


def _render(sc):
    """Full frame of all bricks on one GPU; returns (context, RGBA image).  Caller closes."""
    print(f"[configs] rendering {len(sc['vols'])} bricks at {sc['W']}x{sc['H']}", flush=True)
    W, H = sc["W"], sc["H"]
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=len(sc["vols"]), keep_passes=True)
    ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=sc["conv"], conv_offset=0.0)
    for b, v in enumerate(sc["vols"]):
        ctx.set_brick(b, v, sc["models"][b], dtype=native.F32)
    img = ctx.frame(sc["cam"], want_image=True)
    return ctx, img


def _properties(dep):
    """Size-independent VDI properties of a (nx, H, 2S) depth block."""
    starts, ends = dep[..., 0::2], dep[..., 1::2]
    filled = starts != 0
    assert filled.sum(axis=2).max() <= S
    assert np.all(ends[filled] >= starts[filled])
    assert np.all(np.diff(filled.astype(np.int8), axis=2) <= 0), "a filled slot follows an empty one"
    assert not np.any(ends[~filled]), "an empty slot has a non-zero end"


def _full_frame(sc, ctx, img, comp=None, band=480):
    """The WHOLE frame bit for bit, band-major (the host holds one band of all bricks at a time): every
    brick's sub-VDI (colours, depths, pass counts, octree cells), the flatten of every pixel, and with
    comp = (colour, depth, passes) of a VDICompositor context the composited VDI and its pass counts."""
    W, H = sc["W"], sc["H"]
    assert ctx.stats()["rays_uncached"] == 0
    B = len(sc["vols"])
    tf, cmap = scene.transfer_function(), scene.colormap_hot()
    k = scene.folded_conv_scale(sc["conv"], native.F32)
    ipv = orc.ipv_of(sc["cam"])
    octs = [ctx.read(native.BUF_OCTREE, b) for b in range(B)]
    inps = [orc.Inputs(sc["vols"][b].detach().cpu().numpy(), scene.inverse_model(sc["models"][b]), tf, cmap, k,
                       0.0, sc["cam"]) for b in range(B)]
    covered = 0
    for x0 in range(0, W, band):
        x1 = min(W, x0 + band)
        print(f"[configs] full frame: columns [{x0},{x1}) of {B} bricks", flush=True)   # progress
        rcs, rds = [], []
        for b in range(B):
            gc, gd, gp = (ctx.read_columns(w, x0, x1, b) for w in (native.BUF_VDI_COLOR, native.BUF_VDI_DEPTH,
                                                                   native.BUF_PASSES))
            _properties(gd)
            rc, rd, ro, rp = orc.vdi_generate_cols(inps[b], W, H, S, x0, x1, THREADS)
            bad = np.count_nonzero(_bits(gc) != _bits(rc)) + np.count_nonzero(_bits(gd) != _bits(rd))
            assert bad == 0, f"brick {b} columns [{x0},{x1}): {bad} mismatching words"
            assert np.array_equal(gp.astype(np.int32), rp), f"brick {b} columns [{x0},{x1}): pass counts differ"
            assert np.array_equal(octs[b][:, :, x0 // 8:x1 // 8], ro[:, :, x0 // 8:x1 // 8]), \
                f"brick {b}: octree cells differ"
            rcs.append(rc)
            rds.append(rd)
        want = orc.vdi_flatten(rcs, rds, W, H, x0, x1 - x0, ipv, arrays_x0=x0)
        assert np.array_equal(img[:, x0:x1], want), f"columns [{x0},{x1}): image differs"
        covered += np.count_nonzero(want[..., 3])
        if comp is not None:
            cc, cd, cp = comp
            oc, od, op = orc.vdi_composite(rcs, rds, W, H, x0, x1 - x0, ipv, S, arrays_x0=x0)
            bad = np.count_nonzero(_bits(cc[x0:x1]) != _bits(oc)) + np.count_nonzero(_bits(cd[x0:x1]) != _bits(od))
            assert bad == 0, f"composited VDI, columns [{x0},{x1}): {bad} mismatching words"
            assert np.array_equal(cp[:, x0:x1].astype(np.int32), op), f"columns [{x0},{x1}): compositor passes differ"
    assert covered > 100000, "the frame misses the volume"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sim_n", [512, 128], ids=["sim512", "sim128"])
def test_config2_full_frame_8_bricks(sim_n):
    """Config 2 (the headline workload) on the WHOLE frame: every brick's sub-VDI (colours, depths, pass
    counts, octree cells), the 8-brick flatten of every pixel, and the VDICompositor's composited VDI
    (VDI mode's product, S_out = S, DistributedVolumes.kt:423-439) with its pass counts, bit for bit, in
    480-column bands (band-major, so the host holds one band of all bricks at a time).  sim512 is the
    field bench.py times (Gray-Scott simulated at full resolution, --sim-n 512); sim128 the upsampled one."""
    import time
    t0 = time.perf_counter()
    sc = _scene(2, sim_n=sim_n)
    ctx, img = _render(sc)
    st = ctx.stats()
    mp, hit = ctx.pass_stats()
    print(f"[configs] sim{sim_n}: rays searched {st['rays_searched']}, search regroups {st.get('regroups')}, "
          f"mean passes {mp:.3f} over {hit} hit rays", flush=True)
    comp = InSituContext(sc["W"], sc["H"], max_supersegments=S, bricks_per_rank=len(sc["vols"]), composite_vdi=True,
                         max_output_supersegments=S)
    try:
        comp.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=sc["conv"], conv_offset=0.0)
        for b, v in enumerate(sc["vols"]):
            comp.set_brick(b, v, sc["models"][b], dtype=native.F32)
        comp.frame(sc["cam"])
        cc, cd = comp.read(native.BUF_COMPOSITED_COLOR), comp.read(native.BUF_COMPOSITED_DEPTH)
        cp = comp.read(native.BUF_COMPOSITE_PASSES)
        comp.close()
        _full_frame(sc, ctx, img, comp=(cc, cd, cp))
        print(f"[configs] sim{sim_n}: whole frame bit-exact in {time.perf_counter() - t0:.1f} s", flush=True)
    finally:
        ctx.close()
        comp.close()


@pytest.mark.timeout(900)
def test_config2_pipelined_frames_sim512():
    """The bench's own loop on its own field: config 2 (sim512 bricks) through insitu_frame_pipelined, two
    cameras with the bench's re-ingest of every brick from its device array between them, then the flush --
    both completed frames' sub-VDIs, pass counts, octree cells and images equal the oracle's on the WHOLE frame."""
    sc = _scene(2, sim_n=512)
    cams = [sc["cam"], scene.orbit_camera(sc["W"], sc["H"], yaw_deg=35.0, pitch_deg=20.0, voxel_world=1.0 / 512)]
    W, H = sc["W"], sc["H"]
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=len(sc["vols"]), keep_passes=True)
    try:
        ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=sc["conv"], conv_offset=0.0)
        for b, v in enumerate(sc["vols"]):
            ctx.set_brick(b, v, sc["models"][b], dtype=native.F32)
        assert ctx.frame_pipelined(cams[0], want_image=True)[0] == -1
        for b, v in enumerate(sc["vols"]):   # bench.py's update_volumes, without a synchronisation
            ctx.set_brick(b, v, sc["models"][b], dtype=native.F32)
        for k, call in enumerate((lambda: ctx.frame_pipelined(cams[1], want_image=True),
                                  lambda: ctx.pipeline_flush(want_image=True))):
            done, img = call()
            assert done == k
            print(f"[configs] pipelined sim512 frame {done}: checking the whole frame", flush=True)
            _full_frame(dict(sc, cam=cams[done]), ctx, img)
    finally:
        ctx.close()


@pytest.mark.timeout(900)
def test_config2_merged_full_frame():
    """Config 2 with the rank's 8 bricks merged into ONE sub-VDI (merge_bricks, VDIGenerator.comp's $repeat
    over the grids a rank owns, DistributedVolumeRenderer.kt:57-63) on the WHOLE frame: colours, depths,
    pass counts, octree cells and the image, bit for bit against the oracle's multi-volume restatement."""
    sc = _scene(2)
    W, H = sc["W"], sc["H"]
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=len(sc["vols"]), keep_passes=True,
                        merge_bricks=True)
    try:
        ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=sc["conv"], conv_offset=0.0)
        for b, v in enumerate(sc["vols"]):
            ctx.set_brick(b, v, sc["models"][b], dtype=native.F32)
        img = ctx.frame(sc["cam"], want_image=True)
        octree = ctx.read(native.BUF_OCTREE)
        tf, cmap = scene.transfer_function(), scene.colormap_hot()
        k = scene.folded_conv_scale(sc["conv"], native.F32)
        ipv = orc.ipv_of(sc["cam"])
        inps = [orc.Inputs(v.detach().cpu().numpy(), scene.inverse_model(m), tf, cmap, k, 0.0, sc["cam"])
                for v, m in zip(sc["vols"], sc["models"])]
        for x0 in range(0, W, 480):
            x1 = min(W, x0 + 480)
            print(f"[configs] merged full frame: columns [{x0},{x1})", flush=True)   # progress
            gc, gd, gp = (ctx.read_columns(w, x0, x1, 0) for w in (native.BUF_VDI_COLOR, native.BUF_VDI_DEPTH,
                                                                   native.BUF_PASSES))
            _properties(gd)
            rc, rd, ro, rp = orc.vdi_generate_multi(inps, W, H, S, x0, x1, THREADS)
            bad = np.count_nonzero(_bits(gc) != _bits(rc)) + np.count_nonzero(_bits(gd) != _bits(rd))
            assert bad == 0, f"merged VDI, columns [{x0},{x1}): {bad} mismatching words"
            assert np.array_equal(gp.astype(np.int32), rp), f"merged VDI, columns [{x0},{x1}): pass counts differ"
            assert np.array_equal(octree[:, :, x0 // 8:x1 // 8], ro[:, :, x0 // 8:x1 // 8]), "octree cells differ"
            want = orc.vdi_flatten([rc], [rd], W, H, x0, x1 - x0, ipv, arrays_x0=x0)
            assert np.array_equal(img[:, x0:x1], want), f"columns [{x0},{x1}): image differs"
    finally:
        ctx.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("slabs", [2, 4, 8])
def test_config3_slabs_full_frame(slabs):
    """Config 3 (vortex-in-cell |w|, 1024^3 grid) as the 2-, 4- and 8-GPU slab decompositions
    (1024x1024x512 / 256 / 128 slabs as virtual ranks on one GPU), whole frame bit for bit."""
    sc = _scene(3, slabs=slabs)
    ctx, img = _render(sc)
    try:
        _full_frame(sc, ctx, img)
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_config3_single_slab_full_frame():
    """Config 3 at 1 GPU: the whole 1024^3 grid as one brick (the longest rays of all configs):
    every ray fits the per-sample cache; the WHOLE frame bit for bit (sub-VDI, passes, octree, image)."""
    sc = _scene(3, slabs=1)
    ctx, img = _render(sc)
    try:
        _full_frame(sc, ctx, img)
    finally:
        ctx.close()


@pytest.mark.timeout(900)
def test_config4_full_frame_8_bricks():
    """Config 4 (8 x 768^3 at 3840x2160) on the WHOLE frame: every brick's sub-VDI and the 8-brick flatten
    of every pixel, bit for bit."""
    sc = _scene(4)
    ctx, img = _render(sc)
    try:
        _full_frame(sc, ctx, img)
    finally:
        ctx.close()


def _config1():
    """Config 1: one 128^3 fp32 Gray-Scott volume (seed 1000), 1280x720."""
    dev = torch.device("cuda", 0)
    n, W, H = 128, 1280, 720
    vol = bench.make_brick(0, n, dev, sim_n=n)
    torch.cuda.synchronize()
    host = vol.detach().cpu().numpy()
    (origin, vw, _), = scene.grid_bricks(n, 1)
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=vw)
    return dict(n=n, W=W, H=H, vol=vol, host=host, origin=origin, vw=vw, cam=cam, conv=1.0 / 0.5)


def _oracle_inputs(c, host, origin):
    k = scene.folded_conv_scale(c["conv"], native.F32)
    im = scene.inverse_model(scene.brick_model(origin, c["vw"]))
    return orc.Inputs(np.ascontiguousarray(host), im, scene.transfer_function(), scene.colormap_hot(), k, 0.0, c["cam"])


@pytest.mark.timeout(300)
def test_config1_vdi_full_frame():
    """Config 1 in VDI mode (S = 20): the whole 1280x720 sub-VDI, octree, pass counts and flattened
    image equal the oracle bit for bit."""
    c = _config1()
    W, H = c["W"], c["H"]
    with InSituContext(W, H, max_supersegments=S, keep_passes=True) as ctx:
        ctx.set_transfer(scene.transfer_function(), scene.colormap_hot(), conv_scale=c["conv"], conv_offset=0.0)
        ctx.set_brick(0, c["vol"], scene.brick_model(c["origin"], c["vw"]), dtype=native.F32)
        img = ctx.frame(c["cam"], want_image=True)
        col, dep = ctx.read(native.BUF_VDI_COLOR), ctx.read(native.BUF_VDI_DEPTH)
        octree, passes = ctx.read(native.BUF_OCTREE), ctx.read(native.BUF_PASSES)
        assert ctx.stats()["rays_uncached"] == 0
    rc, rd, ro, rp = orc.vdi_generate(_oracle_inputs(c, c["host"], c["origin"]), W, H, S, THREADS)
    bad = np.count_nonzero(_bits(col) != _bits(rc)) + np.count_nonzero(_bits(dep) != _bits(rd))
    assert bad == 0, f"{bad} mismatching words"
    assert np.array_equal(octree, ro)
    assert np.array_equal(passes.astype(np.int32), rp)
    want = orc.vdi_flatten([rc], [rd], W, H, 0, W, orc.ipv_of(c["cam"]))
    assert np.array_equal(img, want)
    assert np.count_nonzero(want[..., 3]) > W * H // 20, "config 1 frame barely hits the volume"


@pytest.mark.timeout(300)
def test_config1_plain_full_frame():
    """Config 1 through the DistributedVolumeRenderer shaders (plain mode): the 1280x720 rgba8
    colour/depth textures and the composited image equal the oracle; then the volume as two z-slab
    virtual ranks, composited over both lists (default) or over numProcesses = dim0 / dim1 = 1 list
    (INSITU_FAITHFUL_PLAIN_NUM_PROCESSES, PlainImageCompositor.comp:43 as written)."""
    c = _config1()
    W, H, n = c["W"], c["H"], c["n"]
    tf, cm = scene.transfer_function(), scene.colormap_hot()
    with InSituContext(W, H, mode=native.MODE_PLAIN) as ctx:
        ctx.set_transfer(tf, cm, conv_scale=c["conv"], conv_offset=0.0)
        ctx.set_brick(0, c["vol"], scene.brick_model(c["origin"], c["vw"]), dtype=native.F32)
        img = ctx.frame(c["cam"], want_image=True)
        col, dep = ctx.read(native.BUF_PLAIN_COLOR), ctx.read(native.BUF_PLAIN_DEPTH)
    rc, rd = orc.plain_raycast(_oracle_inputs(c, c["host"], c["origin"]), W, H)
    assert np.array_equal(col, rc) and np.array_equal(dep, rd)
    assert np.array_equal(img, orc.plain_composite([rc], [rd], H))
    assert np.count_nonzero(rc[..., 3]) > W * H // 20
    # two z-slabs of the same volume as two virtual ranks
    slabs = scene.slab_bricks(n, 2, world=2.0)
    subs = []
    for (origin, vw, (z0, nz)) in slabs:
        assert abs(vw - c["vw"]) < 1e-12
        subs.append(orc.plain_raycast(_oracle_inputs(c, c["host"][z0:z0 + nz], origin), W, H))
    for faithful, lists in ((0, subs), (native.FAITHFUL_PLAIN_NUM_PROCESSES, subs[:1])):
        with InSituContext(W, H, mode=native.MODE_PLAIN, bricks_per_rank=2, faithful=faithful) as ctx:
            ctx.set_transfer(tf, cm, conv_scale=c["conv"], conv_offset=0.0)
            for b, (origin, vw, (z0, nz)) in enumerate(slabs):
                ctx.set_brick(b, c["vol"][z0:z0 + nz].contiguous(), scene.brick_model(origin, vw), dtype=native.F32)
            got = ctx.frame(c["cam"], want_image=True)
        assert np.array_equal(got, orc.plain_composite([s[0] for s in lists], [s[1] for s in lists], H)), faithful
