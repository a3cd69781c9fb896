"""GPU parity at the BASELINE.json workloads (configs 2, 3 and 4), through libinsitu_hip.so.

The whole frame is rendered on the GPU at full size; the CPU oracle (C restatement of
VDIGenerator.comp + AccumulateVDI.comp, OpenMP) recomputes full-height column bands of every
brick's sub-VDI and of the composited image, which must match BIT FOR BIT (supersegment colours,
depths, raymarch pass counts, the bands' octree cells, and the RGBA flatten of all bricks).  The
whole frame is checked through size-independent properties: at most S supersegments per pixel,
compact lists (no filled slot after an empty one), end >= start, and no ray without cache space.

  config 2: 8 x 512^3 fp32 Gray-Scott bricks (2x2x2 of a 1024^3 grid), 1920x1080, S = 20
  config 3: vortex-ring |w| on a 1024^3 grid as 2 z-slabs (the 2-GPU decomposition), 1920x1080
            (+ the single 1024^3 slab of the 1-GPU run, through the properties)
  config 4: 8 x 768^3 fp32 Gray-Scott bricks, 3840x2160, S = 20
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


def _scene(cfg: int, slabs: int = 2):
    dev = torch.device("cuda", 0)
    if cfg == 3:
        W, H, ng = 1920, 1080, 1024
        units = scene.slab_bricks(ng, slabs)
        vols = [scene.vortex_ring(ng, z0, nz, device=dev) for (_, _, (z0, nz)) in units]
        conv = 1.0
    else:
        W, H, n = (3840, 2160, 768) if cfg == 4 else (1920, 1080, 512)
        units = scene.grid_bricks(2 * n, 2)
        vols = [bench.make_brick(b, n, dev) for b in range(len(units))]
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


def _check(sc, ctx, img, bands, property_chunk):
    W, H = sc["W"], sc["H"]
    st = ctx.stats()
    assert st["rays_uncached"] == 0, f"{st['rays_uncached']} rays without cache space"
    B = len(sc["vols"])
    tf, cmap = scene.transfer_function(), scene.colormap_hot()
    k = scene.folded_conv_scale(sc["conv"], native.F32)
    ipv = orc.ipv_of(sc["cam"])
    octs = [ctx.read(native.BUF_OCTREE, b) for b in range(B)]
    got = {(b, x0): [ctx.read_columns(w, x0, x1, b) for w in (native.BUF_VDI_COLOR, native.BUF_VDI_DEPTH,
                                                                native.BUF_PASSES)]
           for b in range(B) for (x0, x1) in bands}
    # whole-frame properties, in column chunks
    for b in range(B):
        for x0 in range(0, W, property_chunk):
            _properties(ctx.read_columns(native.BUF_VDI_DEPTH, x0, min(W, x0 + property_chunk), b))
    ref = {}
    for b in range(B):
        print(f"[configs] oracle bands of brick {b}/{B}", flush=True)   # progress (long test)
        host = sc["vols"][b].detach().cpu().numpy()
        inp = orc.Inputs(host, scene.inverse_model(sc["models"][b]), tf, cmap, k, 0.0, sc["cam"])
        for (x0, x1) in bands:
            rc, rd, ro, rp = orc.vdi_generate_cols(inp, W, H, S, x0, x1, THREADS)
            gc, gd, gp = got[(b, x0)]
            bad = np.count_nonzero(_bits(gc) != _bits(rc)) + np.count_nonzero(_bits(gd) != _bits(rd))
            assert bad == 0, (f"brick {b} band [{x0},{x1}): {bad} mismatching words; count-match rate "
                              f"{np.mean(np.count_nonzero(gd[..., 0::2], axis=2) == np.count_nonzero(rd[..., 0::2], axis=2)):.6f}")
            assert np.array_equal(gp.astype(np.int32), rp), f"brick {b} band [{x0},{x1}): pass counts differ"
            c0, c1 = x0 // 8, x1 // 8
            assert np.array_equal(octs[b][:, :, c0:c1], ro[:, :, c0:c1]), f"brick {b}: octree cells differ"
            ref[(b, x0)] = (rc, rd)
        del host, inp
    hit = 0
    for (x0, x1) in bands:
        want = orc.vdi_flatten([ref[(b, x0)][0] for b in range(B)], [ref[(b, x0)][1] for b in range(B)], W, H, x0,
                               x1 - x0, ipv, arrays_x0=x0)
        assert np.array_equal(img[:, x0:x1], want), \
            f"band [{x0},{x1}): max |dRGBA| {np.max(np.abs(img[:, x0:x1].astype(int) - want.astype(int)))}"
        hit += np.count_nonzero(want[..., 3])
    assert hit > 0, "bands miss the volume"


@pytest.mark.timeout(600)
def test_config2_bands_8_bricks():
    """Config 2 (the headline workload): every brick's sub-VDI on three 64-column bands + the
    8-brick flatten of those bands, bit for bit; whole-frame properties of all 8 bricks."""
    sc = _scene(2)
    ctx, img = _render(sc)
    try:
        _check(sc, ctx, img, [(600, 664), (928, 992), (1280, 1344)], property_chunk=480)
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_config3_bands_two_slabs():
    """Config 3 (vortex-in-cell |w|, 1024^3 grid) as the 2-GPU slab decomposition on one GPU."""
    sc = _scene(3, slabs=2)
    ctx, img = _render(sc)
    try:
        _check(sc, ctx, img, [(640, 704), (928, 992), (1216, 1280)], property_chunk=480)
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_config3_single_slab_properties():
    """Config 3 at 1 GPU: the whole 1024^3 grid as one brick (the longest rays of all configs):
    every ray fits the per-sample cache, one band bit for bit, whole-frame properties."""
    sc = _scene(3, slabs=1)
    ctx, img = _render(sc)
    try:
        _check(sc, ctx, img, [(928, 992)], property_chunk=480)
    finally:
        ctx.close()


@pytest.mark.timeout(900)
def test_config4_bands_8_bricks():
    """Config 4 (8 x 768^3 at 3840x2160): two 64-column bands of every brick + their flatten,
    whole-frame properties of all 8 bricks."""
    sc = _scene(4)
    ctx, img = _render(sc)
    try:
        _check(sc, ctx, img, [(1536, 1600), (2240, 2304)], property_chunk=480)
    finally:
        ctx.close()
