"""GPU parity: libinsitu_hip.so (HIP, gfx950) against the CPU oracle on identical inputs.

The numerical contract is shared, so every integer AND floating-point output is
required to match BIT FOR BIT: supersegment colours and depths, octree counts, pass counts,
plain rgba8 images, and the composited RGBA.  (The north-star tolerance -- RGBA within 1/255,
depths within 1e-4 -- is implied; tests report the max deviation as well.)
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import oracle_binding as orc
from insitu_amd import native, scene
from insitu_amd.renderer import InSituContext
from scenes import make_scene

pytestmark = pytest.mark.gpu


def _ctx_for(sc, S=8, mode=native.MODE_VDI, B=1, cache_mb=0):
    ctx = InSituContext(sc["W"], sc["H"], mode=mode, max_supersegments=S, bricks_per_rank=B, keep_passes=True,
                        sample_cache_mb=cache_mb)
    ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
    return ctx


def _oracle_vdi(sc, S, vol=None, im=None):
    inp = orc.Inputs(sc["vol"] if vol is None else vol, sc["im"] if im is None else im, sc["tf"], sc["cmap"],
                     sc["conv_k"], sc["conv_offset"], sc["cam"])
    return orc.vdi_generate(inp, sc["W"], sc["H"], S)


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _assert_vdi_equal(got_c, got_d, ref_c, ref_d):
    mism = np.count_nonzero(_bits(got_c) != _bits(ref_c)) + np.count_nonzero(_bits(got_d) != _bits(ref_d))
    if mism:
        W, H = ref_d.shape[:2]
        cnt_ref = np.count_nonzero(ref_d[..., 0::2] != 0, axis=2)
        cnt_got = np.count_nonzero(got_d[..., 0::2] != 0, axis=2)
        bad = np.argwhere(np.any(_bits(got_d) != _bits(ref_d), axis=2))
        raise AssertionError(
            f"{mism} mismatching words; count-match rate {np.mean(cnt_ref == cnt_got):.6f}; "
            f"max |dDepth| {np.max(np.abs(got_d - ref_d)):.3g}; first bad pixels (x,y) {bad[:5].tolist()}")


@pytest.mark.parametrize("dtype,S,W,H,yaw", [
    ("u16", 8, 64, 48, 30.0),
    ("u16", 20, 64, 48, 120.0),
    ("u8", 4, 40, 24, 200.0),
    ("f32", 8, 48, 40, 300.0),
    ("u16", 5, 50, 37, 75.0),     # ragged: W, H not multiples of 8
])
def test_vdi_generate_bit_exact(dtype, S, W, H, yaw):
    sc = make_scene(n=32, W=W, H=H, yaw=yaw, dtype=dtype)
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        octree = ctx.read(native.BUF_OCTREE)
        passes = ctx.read(native.BUF_PASSES)
    rc, rd, ro, rp = _oracle_vdi(sc, S)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.array_equal(octree, ro)
    assert np.array_equal(passes.astype(np.int32), rp)
    assert np.count_nonzero(rd) > 0, "scene produced no supersegments"


@pytest.mark.parametrize("cache_mb", [-1, 1])
def test_vdi_sample_cache_off_and_overflow(cache_mb):
    """Per-sample cache disabled (-1) and too small to hold every ray (1 MiB: some waves replay
    from the cache, the rest re-sample every pass): both bit-identical to the oracle."""
    sc = make_scene(n=32, W=96, H=80, yaw=30.0)
    S = 8
    with _ctx_for(sc, S=S, cache_mb=cache_mb) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        octree = ctx.read(native.BUF_OCTREE)
    rc, rd, ro, _ = _oracle_vdi(sc, S)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.array_equal(octree, ro)


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6])
def test_vdi_search_tree_depths(depth):
    """The search kernel evaluates `depth` levels of the threshold search tree per replay round
    (groups of 2^depth - 1 lanes per ray, chosen from the queue length unless fixed): every depth
    lands on the same thresholds, supersegments and pass counts as the sequential oracle."""
    sc = make_scene(n=32, W=72, H=56, yaw=120.0)
    S = 12
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_option(native.OPT_SEARCH_DEPTH, depth)
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        octree = ctx.read(native.BUF_OCTREE)
        passes = ctx.read(native.BUF_PASSES)
    rc, rd, ro, rp = _oracle_vdi(sc, S)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.array_equal(octree, ro)
    assert np.array_equal(passes.astype(np.int32), rp)
    assert rp.max() > 8, "scene needs rays with a long search"


def test_vdi_known_answers_on_gpu():
    """KAT 1/2 on the GPU: TF alpha == 0 -> no supersegment opens; missing rays zero-filled."""
    sc = make_scene(n=16, W=32, H=24)
    tf0 = np.zeros_like(sc["tf"])
    with _ctx_for(sc, S=4) as ctx:
        ctx.set_transfer(tf0, sc["cmap"])
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        assert not np.any(ctx.read(native.BUF_VDI_COLOR))
        assert not np.any(ctx.read(native.BUF_VDI_DEPTH))
        assert not np.any(ctx.read(native.BUF_OCTREE))


def test_vdi_flatten_two_bricks_bit_exact():
    """Two bricks on one rank (two virtual ranks): merged front to back in the flatten."""
    sc = make_scene(n=24, W=64, H=48, yaw=45.0)
    sc2 = make_scene(n=24, W=64, H=48, yaw=45.0, seed=7, origin=(0.0, -0.25, -0.75))
    S = 6
    with _ctx_for(sc, S=S, B=2) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.set_brick(1, sc2["vol"], sc2["model"])
        img = ctx.frame(sc["cam"], want_image=True)
        cols = [ctx.read(native.BUF_VDI_COLOR, b) for b in range(2)]
        deps = [ctx.read(native.BUF_VDI_DEPTH, b) for b in range(2)]
    r0 = _oracle_vdi(sc, S)
    r1 = _oracle_vdi(sc, S, vol=sc2["vol"], im=sc2["im"])
    _assert_vdi_equal(cols[0], deps[0], r0[0], r0[1])
    _assert_vdi_equal(cols[1], deps[1], r1[0], r1[1])
    ref = orc.vdi_flatten([r0[0], r1[0]], [r0[1], r1[1]], sc["W"], sc["H"], 0, sc["W"], orc.ipv_of(sc["cam"]))
    assert np.array_equal(img, ref), f"max |dRGBA| = {np.max(np.abs(img.astype(int) - ref.astype(int)))}"
    assert np.count_nonzero(ref[..., 3]) > 0


@pytest.mark.parametrize("dtype,dim,yaw", [("u16", 48, 30.0), ("u8", 40, 150.0), ("f32", 32, 260.0)])
def test_plain_bit_exact(dtype, dim, yaw):
    sc = make_scene(n=32, W=dim, H=dim, yaw=yaw, dtype=dtype)
    with _ctx_for(sc, mode=native.MODE_PLAIN) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        img = ctx.frame(sc["cam"], want_image=True)
        col = ctx.read(native.BUF_PLAIN_COLOR)
        dep = ctx.read(native.BUF_PLAIN_DEPTH)
    inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], sc["cam"])
    rc, rd = orc.plain_raycast(inp, dim, dim)
    assert np.array_equal(col, rc)
    assert np.array_equal(dep, rd)
    ref = orc.plain_composite([rc], [rd], dim)
    assert np.array_equal(img, ref)
    assert np.count_nonzero(rc[..., 3]) > 0


def test_plain_two_bricks_composite():
    sc = make_scene(n=24, W=40, H=40, yaw=45.0)
    sc2 = make_scene(n=24, W=40, H=40, yaw=45.0, seed=7, origin=(0.0, -0.25, -0.75))
    with _ctx_for(sc, mode=native.MODE_PLAIN, B=2) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.set_brick(1, sc2["vol"], sc2["model"])
        img = ctx.frame(sc["cam"], want_image=True)
    i1 = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    i2 = orc.Inputs(sc2["vol"], sc2["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    c1, d1 = orc.plain_raycast(i1, 40, 40)
    c2, d2 = orc.plain_raycast(i2, 40, 40)
    ref = orc.plain_composite([c1, c2], [d1, d2], 40)
    assert np.array_equal(img, ref)


def test_device_pointer_brick_upload():
    """In-situ zero-copy source: a device tensor handed over as a device pointer."""
    import torch
    sc = make_scene(n=16, W=32, H=24)
    t = torch.from_numpy(sc["vol"].astype(np.int16, copy=False).view(np.int16)).cuda()
    with _ctx_for(sc, S=4) as ctx:
        ctx.set_brick(0, t, sc["model"], dtype=native.U16)
        ctx.render(sc["cam"])
        dep = ctx.read(native.BUF_VDI_DEPTH)
    rd = _oracle_vdi(sc, 4)[1]
    assert np.array_equal(_bits(dep), _bits(rd))


@pytest.mark.parametrize("dtype", ["u8", "u16", "f32"])
def test_ragged_brick_ingest(dtype):
    """Bricks whose dims are not multiples of 8 (nor of the ingest's 64-voxel rows): the padded
    blocked layout samples exactly like the oracle's linear array (clamp to edge)."""
    sc = make_scene(n=72, W=56, H=40, yaw=50.0, dtype=dtype)
    vol = np.ascontiguousarray(sc["vol"][:13, 5:25, :69])   # (z, y, x) = 13 x 20 x 69
    S = 6
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_brick(0, vol, sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
    rc, rd, _, _ = _oracle_vdi(sc, S, vol=vol)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.count_nonzero(rd) > 0


def test_periodic_reingest_matches_fresh_context():
    """updateVolumes every N frames (DistributedVolumeRenderer.kt:521-527, 656-681): re-ingesting the
    bricks of a live context -- host sources through the kept staging buffer, which grows when a
    larger grid arrives, and a device source in place -- renders what a fresh context renders."""
    import torch
    sc_small = make_scene(n=16, W=40, H=32)
    sc_big = make_scene(n=24, W=40, H=32, seed=5)
    S = 4
    with _ctx_for(sc_small, S=S) as ctx:
        ctx.set_brick(0, sc_small["vol"], sc_small["model"])
        ctx.render(sc_small["cam"])
        ctx.set_brick(0, sc_big["vol"], sc_big["model"])            # host, larger: staging grows
        ctx.render(sc_big["cam"])
        dep_big = ctx.read(native.BUF_VDI_DEPTH)
        ctx.set_brick(0, sc_small["vol"], sc_small["model"])        # host, smaller: staging reused
        ctx.render(sc_small["cam"])
        dep_small = ctx.read(native.BUF_VDI_DEPTH)
        t = torch.from_numpy(sc_big["vol"].view(np.int16)).cuda()   # device source after host ones
        ctx.set_brick(0, t, sc_big["model"], dtype=native.U16)
        ctx.render(sc_big["cam"])
        dep_dev = ctx.read(native.BUF_VDI_DEPTH)
    assert np.array_equal(_bits(dep_big), _bits(_oracle_vdi(sc_big, S)[1]))
    assert np.array_equal(_bits(dep_small), _bits(_oracle_vdi(sc_small, S)[1]))
    assert np.array_equal(_bits(dep_dev), _bits(dep_big))


@pytest.mark.parametrize("x0,x1", [(0, 64), (600, 664), (1216, 1280)])
def test_config1_column_bands(x0, x1):
    """Config 1 shapes (128^3 Gray-Scott, 1280x720, S=20): full-resolution GPU frame,
    oracle on column bands (the oracle takes minutes on the whole frame)."""
    sc = make_scene(n=128, W=1280, H=720, yaw=35.0, origin=(-1.0, -1.0, -1.0), world=2.0)
    S = 20
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        passes = ctx.read(native.BUF_PASSES)
    lib = orc.load()
    inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    W, H = 1280, 720
    rc = np.zeros((W, H, S, 4), np.float32)
    rd = np.zeros((W, H, 2 * S), np.float32)
    ro = np.zeros((S, H // 8, W // 8), np.uint32)
    rp = np.zeros((H, W), np.int32)
    assert lib.orc_vdi_generate(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                                rc.ctypes.data, rd.ctypes.data, ro.ctypes.data, rp.ctypes.data, x0, x1) == 0
    _assert_vdi_equal(col[x0:x1], dep[x0:x1], rc[x0:x1], rd[x0:x1])
    assert np.array_equal(passes[:, x0:x1].astype(np.int32), rp[:, x0:x1])
    # size-independent properties over the whole GPU frame
    cnt = np.count_nonzero(dep[..., 0::2] != 0, axis=2)
    assert cnt.max() <= S
    starts, ends = dep[..., 0::2], dep[..., 1::2]
    filled = starts != 0
    assert np.all(ends[filled] >= starts[filled])
    # lists are compact: no filled slot after an empty one
    assert np.all(np.diff(filled.astype(np.int8), axis=2) <= 0)


@pytest.mark.parametrize("mode", [native.MODE_VDI, native.MODE_PLAIN])
def test_reference_shaped_host_path(mode):
    """distributeVDIs / gatherCompositedVDIs with host buffers in the reference layouts (the JNI
    drop-in) give the same image as the device-resident frame."""
    W = H = 48
    sc = make_scene(n=32, W=W, H=H, yaw=40.0)
    S = 6
    with _ctx_for(sc, S=S, mode=mode) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        want = ctx.frame(sc["cam"], want_image=True)
        if mode == native.MODE_VDI:
            col = ctx.read(native.BUF_VDI_COLOR)
            dep = ctx.read(native.BUF_VDI_DEPTH)
            size = H * W * S * 4
        else:
            col = ctx.read(native.BUF_PLAIN_COLOR)
            dep = ctx.read(native.BUF_PLAIN_DEPTH)
            size = H * W * 4
    with _ctx_for(sc, S=S, mode=mode) as ctx2:
        ctx2.set_camera(sc["cam"])
        rc_, rd_ = ctx2.distributeVDIs(col, dep, size, 1)
        assert np.array_equal(rc_.view(np.uint8), col.view(np.uint8))
        assert np.array_equal(rd_.view(np.uint8), dep.view(np.uint8))
        img = ctx2.gatherCompositedVDIs(0, H * W * 4, 0, 1)
    assert np.array_equal(img, want)
    assert np.count_nonzero(want[..., 3]) > 0


@pytest.mark.parametrize("S,S_out,W,H", [(6, 6, 64, 48), (8, 4, 50, 37), (5, 12, 40, 24)])
def test_vdi_compositor_bit_exact(S, S_out, W, H):
    """VDICompositor.comp on the GPU (composite_vdi context, two bricks = two lists) against the
    oracle's orc_vdi_composite on the oracle's sub-VDIs: composited colour, depth, pass counts
    bit for bit; the root image is the flatten of the composited VDI."""
    sc = make_scene(n=24, W=W, H=H, yaw=45.0)
    sc2 = make_scene(n=24, W=W, H=H, yaw=45.0, seed=7, origin=(0.0, -0.25, -0.75))
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=2, keep_passes=True, composite_vdi=True,
                        max_output_supersegments=S_out)
    with ctx:
        ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.set_brick(1, sc2["vol"], sc2["model"])
        img = ctx.frame(sc["cam"], want_image=True)
        cc = ctx.read(native.BUF_COMPOSITED_COLOR)
        cd = ctx.read(native.BUF_COMPOSITED_DEPTH)
        cp = ctx.read(native.BUF_COMPOSITE_PASSES)
        gc = ctx.read(native.BUF_GATHERED_COLOR)
        gd = ctx.read(native.BUF_GATHERED_DEPTH)
    r0 = _oracle_vdi(sc, S)
    r1 = _oracle_vdi(sc, S, vol=sc2["vol"], im=sc2["im"])
    ipv = orc.ipv_of(sc["cam"])
    oc, od, op = orc.vdi_composite([r0[0], r1[0]], [r0[1], r1[1]], W, H, 0, W, ipv, S_out)
    _assert_vdi_equal(cc, cd, oc, od)
    _assert_vdi_equal(gc, gd, oc, od)
    assert np.array_equal(cp.astype(np.int32), op)
    assert np.count_nonzero(od) > 0
    ref_img = orc.vdi_flatten([oc], [od], W, H, 0, W, ipv)
    assert np.array_equal(img, ref_img)


def test_reference_shaped_composited_vdi_gather():
    """distributeVDIs (host sub-VDI) -> VDICompositor -> gatherCompositedVDIs(colour, depth, ...)
    (DistributedVolumes.kt:860, :903) returns the composited VDI in the reference layouts."""
    W, H, S, S_out = 48, 40, 6, 5
    sc = make_scene(n=32, W=W, H=H, yaw=40.0)
    rc, rd, _, _ = _oracle_vdi(sc, S)
    with InSituContext(W, H, max_supersegments=S, composite_vdi=True, max_output_supersegments=S_out) as ctx:
        ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
        ctx.set_camera(sc["cam"])
        ctx.distributeVDIs(rc, rd, H * W * S * 4, 1, recv=False)
        col, dep = ctx.gatherCompositedVDISet(H * W * S_out * 4, 0, 0, 1)
    oc, od, _ = orc.vdi_composite([rc], [rd], W, H, 0, W, orc.ipv_of(sc["cam"]), S_out)
    _assert_vdi_equal(col, dep, oc, od)
    assert np.count_nonzero(od) > 0


@pytest.mark.parametrize("world,composite_vdi,mode", [(2, False, native.MODE_VDI), (4, False, native.MODE_VDI),
                                                      (2, True, native.MODE_VDI), (4, True, native.MODE_VDI),
                                                      (2, False, native.MODE_PLAIN)])
def test_multi_rank_data_path_local_group(world, composite_vdi, mode):
    """The N-rank data path of libinsitu_hip.so on one GPU (in-process rank group instead of RCCL,
    which refuses two ranks per device): every rank renders its bricks, the strip blocks are
    exchanged, each rank composites its strip and rank 0 gathers -- the image (and the gathered
    composited VDI) are identical to one rank rendering all bricks."""
    from insitu_amd.renderer import LocalGroup
    W, S, NB = 64, 6, 4
    H = W if mode == native.MODE_PLAIN else 48
    sc = make_scene(n=24, W=W, H=H, yaw=35.0)
    bricks = []
    for i in range(NB):
        s_i = make_scene(n=24, W=W, H=H, yaw=35.0, seed=11 + i, origin=(-1.0 + (i % 2), -1.0 + (i // 2), -0.5))
        bricks.append((s_i["vol"], s_i["model"]))
    kw = dict(mode=mode, max_supersegments=S, composite_vdi=composite_vdi,
              max_output_supersegments=4 if composite_vdi else 0)
    group = LocalGroup(world)
    B = NB // world
    ctxs = [InSituContext(W, H, bricks_per_rank=B, rank=r, nranks=world, local_group=group, **kw) for r in range(world)]
    try:
        for r, ctx in enumerate(ctxs):
            ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
            for b in range(B):
                ctx.set_brick(b, *bricks[r * B + b])
        for ctx in ctxs:
            ctx.render(sc["cam"])
        for ctx in ctxs:
            ctx.exchange()
        for ctx in ctxs:
            ctx.composite()
        for ctx in ctxs[1:]:
            ctx.gather(want_image=False)
        img = ctxs[0].gather(want_image=True)
        if mode == native.MODE_VDI:   # variable-length exchange: only stored supersegments travel
            st = ctxs[0].stats()
            full = (world - 1) * B * ((W // world + 7) // 8) * S * H * 8 * 24
            assert 0 < st["exchange_bytes"] < full, (st["exchange_bytes"], full)
        gv = (ctxs[0].read(native.BUF_GATHERED_COLOR), ctxs[0].read(native.BUF_GATHERED_DEPTH)) if composite_vdi else None
        # the received set each rank composites (SetOfVDI), expanded from the compact messages
        recv = ([(c.read(native.BUF_RECEIVED_COLOR), c.read(native.BUF_RECEIVED_DEPTH)) for c in ctxs]
                if mode == native.MODE_VDI else None)
    finally:
        for ctx in ctxs:
            ctx.close()
        group.close()
    with InSituContext(W, H, bricks_per_rank=NB, **kw) as ref:
        ref.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
        for b in range(NB):
            ref.set_brick(b, *bricks[b])
        want = ref.frame(sc["cam"], want_image=True)
        if composite_vdi:
            _assert_vdi_equal(gv[0], gv[1], ref.read(native.BUF_GATHERED_COLOR), ref.read(native.BUF_GATHERED_DEPTH))
        subs = [(ref.read(native.BUF_VDI_COLOR, b), ref.read(native.BUF_VDI_DEPTH, b)) for b in range(NB)] if recv else None
    if recv:   # rank r received strip r of every brick, source-major (brick order = source rank, slot)
        sw = W // world
        for r, (rc_, rd_) in enumerate(recv):
            assert rc_.shape == (NB, sw, H, S, 4)
            for v in range(NB):
                _assert_vdi_equal(rc_[v], rd_[v], subs[v][0][r * sw:(r + 1) * sw], subs[v][1][r * sw:(r + 1) * sw])
    assert np.count_nonzero(want[..., 3]) > 0
    assert np.array_equal(img, want)


def test_local_group_composited_vdi_falling_counts():
    """Two frames through the 2-rank VDICompositor path (in-process group), the second from another camera, so
    many pixels get fewer output supersegments than in the first: the slots past a pixel's new count keep the
    first frame's data, and the second frame's gathered composited VDI, its counts and the root's
    image must still equal a fresh one-rank context's render of that frame alone."""
    from insitu_amd.renderer import LocalGroup
    W, H, S, S_out, NB, world = 64, 48, 6, 4, 4, 2
    sc = make_scene(n=24, W=W, H=H, yaw=35.0)
    bricks = []
    for i in range(NB):
        s_i = make_scene(n=24, W=W, H=H, yaw=35.0, seed=11 + i, origin=(-1.0 + (i % 2), -1.0 + (i // 2), -0.5))
        bricks.append((s_i["vol"], s_i["model"]))
    cam_b = scene.orbit_camera(W, H, yaw_deg=110.0, pitch_deg=-25.0, voxel_world=1.0 / 24)
    kw = dict(mode=native.MODE_VDI, max_supersegments=S, composite_vdi=True, max_output_supersegments=S_out)
    group = LocalGroup(world)
    B = NB // world
    ctxs = [InSituContext(W, H, bricks_per_rank=B, rank=r, nranks=world, local_group=group, **kw) for r in range(world)]
    counts = []
    try:
        for r, ctx in enumerate(ctxs):
            ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
            for b in range(B):
                ctx.set_brick(b, *bricks[r * B + b])
        for cam in (sc["cam"], cam_b):
            for ctx in ctxs:
                ctx.render(cam)
            for ctx in ctxs:
                ctx.exchange()
            for ctx in ctxs:
                ctx.composite()
            for ctx in ctxs[1:]:
                ctx.gather(want_image=False)
            img = ctxs[0].gather(want_image=True)
            gd = ctxs[0].read(native.BUF_GATHERED_DEPTH)
            counts.append(np.count_nonzero(gd[..., 0::2] != 0, axis=2))
        gv = (ctxs[0].read(native.BUF_GATHERED_COLOR), ctxs[0].read(native.BUF_GATHERED_DEPTH))
    finally:
        for ctx in ctxs:
            ctx.close()
        group.close()
    assert np.count_nonzero(counts[1] < counts[0]) > 0, "the second frame must lower some pixels' counts"
    with InSituContext(W, H, bricks_per_rank=NB, **kw) as ref:
        ref.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
        for b in range(NB):
            ref.set_brick(b, *bricks[b])
        want = ref.frame(cam_b, want_image=True)
        _assert_vdi_equal(gv[0], gv[1], ref.read(native.BUF_GATHERED_COLOR), ref.read(native.BUF_GATHERED_DEPTH))
    assert np.count_nonzero(want[..., 3]) > 0
    assert np.array_equal(img, want)


def test_composite_requires_exchange_local_group():
    """With N > 1 in VDI mode the compositor reads the exchanged compact lists (per-tile counts and
    offsets): composite after a render but before exchange must fail with an error, not read the
    previous frame's (or uninitialised) messages; after the exchange it succeeds."""
    from insitu_amd.renderer import LocalGroup
    W, H, S = 64, 48, 6
    sc = make_scene(n=24, W=W, H=H, yaw=35.0)
    group = LocalGroup(2)
    ctxs = [InSituContext(W, H, max_supersegments=S, bricks_per_rank=1, rank=r, nranks=2, local_group=group)
            for r in range(2)]
    try:
        for ctx in ctxs:
            ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
            ctx.set_brick(0, sc["vol"], sc["model"])
        for frame in range(2):   # the second frame: exchanged lists of frame 0 must not count
            for ctx in ctxs:
                ctx.render(sc["cam"])
            with pytest.raises(RuntimeError, match="exchange"):
                ctxs[0].composite()
            for ctx in ctxs:
                ctx.exchange()
            for ctx in ctxs:
                ctx.composite()
    finally:
        for ctx in ctxs:
            ctx.close()
        group.close()


@pytest.mark.parametrize("case", ["config1", "bench_brick"])
def test_filtered_search_equals_exact(case):
    """The supersegment decisions of the search (hardware-reciprocal estimate + margin, exact
    fallback) give the same bits as the exact contract path on whole frames: config 1 and one
    512^3 brick of the bench scene at 1920x1080 -- billions of decisions."""
    import torch
    if case == "config1":
        sc = make_scene(n=128, W=1280, H=720, yaw=35.0, origin=(-1.0, -1.0, -1.0), world=2.0)
        W, H, vol, model, dt, k = 1280, 720, sc["vol"], sc["model"], None, sc["conv_scale"]
        cam = sc["cam"]
    else:
        import bench
        W, H = bench.W_IMG, bench.H_IMG
        bricks = scene.grid_bricks(1024, 2)
        origin, vw, _ = bricks[0]
        vol = bench.make_brick(0, 512, torch.device("cuda", 0))
        model, dt, k = scene.brick_model(origin, vw), native.F32, 2.0
        cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=vw)
        sc = {"tf": scene.transfer_function(), "cmap": scene.colormap_hot()}
    out = []
    with InSituContext(W, H, max_supersegments=20, keep_passes=True) as ctx:
        ctx.set_transfer(sc["tf"], sc["cmap"], k, 0.0)
        ctx.set_brick(0, vol, model, dtype=dt)
        for exact in (1, 0):
            ctx.set_option(native.OPT_EXACT_SEARCH, exact)
            ctx.render(cam)
            out.append([ctx.read(b) for b in (native.BUF_VDI_COLOR, native.BUF_VDI_DEPTH, native.BUF_OCTREE,
                                              native.BUF_PASSES)])
    for a, b in zip(*out):
        assert np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))
    assert out[0][3].max() > 8


def test_distributed_volumes_mirror_dumps(tmp_path):
    """The Python mirror of DistributedVolumes (addVolume/updateVolume/manageVDIGeneration) with
    benchmarking off writes the reference's raw dumps (sub-VDI, composited VDI, metadata); the dumps
    read back equal the library's buffers and the composited VDI equals the oracle's."""
    from insitu_amd import vdi_io
    from insitu_amd.renderer import DistributedVolumes
    W, H, S = 48, 40, 6
    sc = make_scene(n=32, W=W, H=H, yaw=40.0)
    dv = DistributedVolumes(W, H, maxSupersegments=S, compositeVDIs=True, maxOutputSupersegments=4,
                            basePath=str(tmp_path) + "/", dataset="GS")
    dv.ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
    dv.setVolumeDims((32, 32, 32))
    dv.addVolume(0, (32, 32, 32), (0.0, 0.0, 0.0), True, model=sc["model"])
    dv.updateVolume(0, sc["vol"].tobytes())
    dv.camera = sc["cam"]
    img = dv.manageVDIGeneration(frames=1, benchmarking=False)
    assert img is not None and np.count_nonzero(img[..., 3]) > 0
    c, d = vdi_io.read_vdi(tmp_path / "GSSubVDI0_ndc_col", tmp_path / "GSSubVDI0_ndc_depth", W, H, S)
    rc, rd, ro, _ = _oracle_vdi(sc, S)
    _assert_vdi_equal(c, d, rc, rd)
    # octree grid next to the sub-VDI, and the received set (one rank: its own whole-width block)
    oct_ = vdi_io.read_octree(tmp_path / "GSSubVDI0_ndc_octree", W, H, S)
    assert np.array_equal(oct_, ro.reshape(oct_.shape)) and oct_.sum() > 0
    sc_, sd_ = vdi_io.read_vdi(tmp_path / "GSSetOfVDI0_ndc_col", tmp_path / "GSSetOfVDI0_ndc_depth", W, H, S)
    _assert_vdi_equal(sc_, sd_, rc, rd)
    cc, cd = vdi_io.read_vdi(tmp_path / "GSCompositedVDI0_ndc_col", tmp_path / "GSCompositedVDI0_ndc_depth", W, H, 4)
    oc, od, _ = orc.vdi_composite([rc], [rd], W, H, 0, W, orc.ipv_of(sc["cam"]), 4)
    _assert_vdi_equal(cc, cd, oc, od)
    meta = vdi_io.read_metadata(tmp_path / f"GSvdi_{W}_{H}_{S}_0_dump0")
    assert meta["windowDimensions"] == [W, H]
    dv.ctx.close()


@pytest.mark.parametrize("oversub", [1, 6, 64])
def test_search_group_widths_and_counters(oversub):
    """The search kernel picks its tree-group width from the queue length x oversubscription
    (1: one lane per ray here, 64: the widest groups); every choice lands on the oracle's
    supersegments and pass counts, and the counters report the searched rays and no uncached ray."""
    sc = make_scene(n=32, W=72, H=56, yaw=120.0)
    S = 12
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_option(native.OPT_SEARCH_OVERSUB, oversub)
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        octree = ctx.read(native.BUF_OCTREE)
        passes = ctx.read(native.BUF_PASSES)
        st = ctx.stats()
    rc, rd, ro, rp = _oracle_vdi(sc, S)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.array_equal(octree, ro)
    assert np.array_equal(passes.astype(np.int32), rp)
    assert st["rays_searched"] > 0 and st["rays_uncached"] == 0


@pytest.mark.parametrize("order", [1, 0])
def test_tile_order_bit_exact(order):
    """The sampling kernel's tile order (INSITU_OPT_TILE_ORDER: 1 = longest tiles first, through
    vdi_tile_len_kernel and a radix sort; 0 = plain XCD order) only changes which waves run first:
    three bricks, VDI, octree and pass counts equal the oracle either way."""
    W, H, S = 72, 56, 6
    sc = make_scene(n=32, W=W, H=H, yaw=35.0)
    with _ctx_for(sc, S=S, B=3) as ctx:
        ctx.set_option(native.OPT_TILE_ORDER, order)
        for b in range(3):
            ctx.set_brick(b, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        got = [(ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b), ctx.read(native.BUF_OCTREE, b),
                ctx.read(native.BUF_PASSES, b)) for b in range(3)]
    rc, rd, ro, rp = _oracle_vdi(sc, S)
    for col, dep, octree, passes in got:   # every brick slot holds the same volume: each sub-VDI is the oracle's
        _assert_vdi_equal(col, dep, rc, rd)
        assert np.array_equal(octree, ro)
        assert np.array_equal(passes.astype(np.int32), rp)
    assert np.count_nonzero(rd) > 0


def test_set_option_validation():
    sc = make_scene(n=16, W=32, H=24)
    with _ctx_for(sc, S=4) as ctx:
        for opt, bad in ((native.OPT_SEARCH_DEPTH, 7), (native.OPT_SEARCH_DEPTH, -1), (native.OPT_ROUND_BATCH, 0),
                         (native.OPT_SEARCH_OVERSUB, 0), (native.OPT_EXACT_SEARCH, 2), (native.OPT_TILE_ORDER, 2),
                         (6, 0), (7, 0), (native.OPT_SUPER_TILE, 3), (native.OPT_REGROUP, 2), (native.OPT_EXACT_TILE_KEYS, 2),
                         (native.OPT_PIPE_TRIGGER, 3), (native.OPT_PIPE_OVERSUB, 0), (native.OPT_PIPE_OVERSUB, 65),
                         (native.OPT_PIPE_SEARCH_RAYS, -1), (native.OPT_PIPE_SEARCH_RAYS, (1 << 24) + 1),
                         (99, 1)):   # 6, 7: ABI 6's fused modes
            with pytest.raises(RuntimeError):
                ctx.set_option(opt, bad)
        ctx.set_option(native.OPT_SEARCH_DEPTH, 6)
        ctx.set_option(native.OPT_PIPE_OVERSUB, 64)


def test_lut_sizes_checked_against_lds():
    """LUTs the generator kernels could not stage in one block's LDS are refused by insitu_set_transfer (the
    largest the ABI admits, 8192 + 4096 texels, need more than the 160 KiB of a gfx950 CU), not at the next
    launch; large LUTs that fit still render what the oracle renders."""
    sc = make_scene(n=16, W=32, H=24)
    S = 4
    with _ctx_for(sc, S=S) as ctx:
        with pytest.raises(RuntimeError, match="LDS"):
            ctx.set_transfer(np.linspace(0, 1, 8192, dtype=np.float32), np.ones((4096, 4), np.float32))
        tf = scene.transfer_function(n=4096)
        ctx.set_transfer(tf, sc["cmap"], sc["conv_scale"], sc["conv_offset"])
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        dep = ctx.read(native.BUF_VDI_DEPTH)
    inp = orc.Inputs(sc["vol"], sc["im"], tf, sc["cmap"], sc["conv_k"], sc["conv_offset"], sc["cam"])
    assert np.array_equal(_bits(dep), _bits(orc.vdi_generate(inp, sc["W"], sc["H"], S)[1]))


def test_host_path_on_fresh_context_after_render():
    """The host-buffer path (distributeVDIs -> gatherCompositedVDIs, the Vulkan-rendering caller)
    on a context that never renders, created after another context rendered and was destroyed
    (its freed device memory is reused): no stale fault flag, the image equals the oracle's."""
    W, H, S = 48, 40, 6
    sc = make_scene(n=32, W=W, H=H, yaw=40.0)
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        ctx.frame(sc["cam"])
    rc, rd, _, _ = _oracle_vdi(sc, S)
    with _ctx_for(sc, S=S) as ctx2:
        ctx2.set_camera(sc["cam"])
        ctx2.distributeVDIs(rc, rd, H * W * S * 4, 1, recv=False)
        img = ctx2.gatherCompositedVDIs(0, H * W * 4, 0, 1)
    ref = orc.vdi_flatten([rc], [rd], W, H, 0, W, orc.ipv_of(sc["cam"]))
    assert np.array_equal(img, ref)


def test_faithful_compositor_ndc_x_two_ranks():
    """INSITU_FAITHFUL_COMPOSITOR_NDC_X: VDICompositor.comp:204 as written (ndc_x from the strip-local
    column over the full width) on 2 ranks; equals the oracle's faithful restatement per strip, and
    differs from the default on rank 1's strip."""
    from insitu_amd.renderer import LocalGroup
    W, H, S, S_out = 64, 48, 6, 4
    sc = make_scene(n=24, W=W, H=H, yaw=35.0)
    bricks = [make_scene(n=24, W=W, H=H, yaw=35.0), make_scene(n=24, W=W, H=H, yaw=35.0, seed=7, origin=(0.0, -0.25, -0.75))]
    out = {}
    for faithful in (0, native.FAITHFUL_COMPOSITOR_NDC_X):
        group = LocalGroup(2)
        ctxs = [InSituContext(W, H, max_supersegments=S, rank=r, nranks=2, local_group=group, composite_vdi=True,
                              max_output_supersegments=S_out, faithful=faithful) for r in range(2)]
        try:
            for r, ctx in enumerate(ctxs):
                ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
                ctx.set_brick(0, bricks[r]["vol"], bricks[r]["model"])
            for step in ("render", "exchange", "composite"):
                for ctx in ctxs:
                    getattr(ctx, step)(sc["cam"]) if step == "render" else getattr(ctx, step)()
            ctxs[1].gather(want_image=False)
            ctxs[0].gather(want_image=False)
            out[faithful] = (ctxs[0].read(native.BUF_GATHERED_COLOR), ctxs[0].read(native.BUF_GATHERED_DEPTH))
        finally:
            for ctx in ctxs:
                ctx.close()
            group.close()
    subs = [_oracle_vdi(sc, S, vol=b["vol"], im=b["im"]) for b in bricks]
    ipv = orc.ipv_of(sc["cam"])
    sw = W // 2
    for faithful, (gc, gd) in out.items():
        parts = [orc.vdi_composite([s[0] for s in subs], [s[1] for s in subs], W, H, r * sw, sw, ipv, S_out,
                                   faithful=bool(faithful)) for r in range(2)]
        _assert_vdi_equal(gc, gd, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    assert np.count_nonzero(out[0][1][sw:]) > 0, "rank 1's strip is empty"
    assert not np.array_equal(out[0][0][sw:], out[native.FAITHFUL_COMPOSITOR_NDC_X][0][sw:]), \
        "the faithful mode should change rank 1's composited colours"
    assert np.array_equal(out[0][0][:sw], out[native.FAITHFUL_COMPOSITOR_NDC_X][0][:sw]), \
        "rank 0's strip is the same in both modes"


def test_faithful_plain_num_processes():
    """INSITU_FAITHFUL_PLAIN_NUM_PROCESSES: PlainImageCompositor.comp:43 as written composites
    numProcesses = dim0 / dim1 lists (1 of the 2 here); equals the oracle over the first list."""
    dim0, dim1 = 96, 64
    sc = make_scene(n=24, W=dim0, H=dim1, yaw=45.0)
    sc2 = make_scene(n=24, W=dim0, H=dim1, yaw=45.0, seed=7, origin=(0.0, -0.25, -0.75))
    imgs = {}
    for faithful in (0, native.FAITHFUL_PLAIN_NUM_PROCESSES):
        with InSituContext(dim0, dim1, mode=native.MODE_PLAIN, bricks_per_rank=2, faithful=faithful) as ctx:
            ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
            ctx.set_brick(0, sc["vol"], sc["model"])
            ctx.set_brick(1, sc2["vol"], sc2["model"])
            imgs[faithful] = ctx.frame(sc["cam"], want_image=True)
    i1 = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    i2 = orc.Inputs(sc2["vol"], sc2["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    c1, d1 = orc.plain_raycast(i1, dim0, dim1)
    c2, d2 = orc.plain_raycast(i2, dim0, dim1)
    assert np.array_equal(imgs[0], orc.plain_composite([c1, c2], [d1, d2], dim1))
    assert np.array_equal(imgs[native.FAITHFUL_PLAIN_NUM_PROCESSES], orc.plain_composite([c1], [d1], dim1))


@pytest.mark.parametrize("cache_mb", [0, -1, 1])
def test_merged_volumes_one_vdi_bit_exact(cache_mb):
    """merge_bricks: three bricks of one rank rendered into ONE sub-VDI (VDIGenerator.comp $repeat,
    AccumulateVDI once per volume and step) -- equal to the oracle's multi-volume restatement, and the
    image is the flatten of that single list.  cache_mb: 0 the default sample cache (every ray cached and
    searched by vdi_search_kernel), -1 no cache (every ray searched in place by re-sampling, the
    merge_search_in_place fallback), 1 a fixed 1-MiB cache (the waves that find no room in place)."""
    W, H, S = 64, 48, 8
    scs = [make_scene(n=24, W=W, H=H, yaw=35.0),
           make_scene(n=24, W=W, H=H, yaw=35.0, seed=7, origin=(0.0, -0.25, -0.75)),
           make_scene(n=16, W=W, H=H, yaw=35.0, seed=9, origin=(-0.7, 0.1, 0.2), world=0.6)]
    with InSituContext(W, H, max_supersegments=S, bricks_per_rank=3, keep_passes=True, merge_bricks=True,
                       sample_cache_mb=cache_mb) as ctx:
        ctx.set_transfer(scs[0]["tf"], scs[0]["cmap"], scs[0]["conv_scale"], scs[0]["conv_offset"])
        for b, sc in enumerate(scs):
            ctx.set_brick(b, sc["vol"], sc["model"])
        img = ctx.frame(scs[0]["cam"], want_image=True)
        st = ctx.stats()
        col = ctx.read(native.BUF_VDI_COLOR)
        dep = ctx.read(native.BUF_VDI_DEPTH)
        octree = ctx.read(native.BUF_OCTREE)
        passes = ctx.read(native.BUF_PASSES)
        with pytest.raises(RuntimeError):
            ctx.read(native.BUF_VDI_COLOR, 1)   # one sub-VDI only
    if cache_mb < 0:
        assert st["rays_uncached"] > 0 and st["rays_searched"] == 0
    elif cache_mb == 0:
        assert st["rays_searched"] > 0
    inps = [orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], scs[0]["cam"])
            for sc in scs]
    rc, rd, ro, rp = orc.vdi_generate_multi(inps, W, H, S)
    _assert_vdi_equal(col, dep, rc, rd)
    assert np.array_equal(octree, ro)
    assert np.array_equal(passes.astype(np.int32), rp)
    assert np.array_equal(img, orc.vdi_flatten([rc], [rd], W, H, 0, W, orc.ipv_of(scs[0]["cam"])))
    assert np.count_nonzero(rd) > 0


def test_merged_volumes_two_ranks_local_group():
    """merge_bricks on 2 ranks (2 bricks each): one list per rank exchanged and composited."""
    from insitu_amd.renderer import LocalGroup
    W, H, S = 64, 48, 6
    sc = make_scene(n=24, W=W, H=H, yaw=35.0)
    bricks = [make_scene(n=24, W=W, H=H, yaw=35.0, seed=11 + i, origin=(-1.0 + (i % 2), -1.0 + (i // 2), -0.5))
              for i in range(4)]
    group = LocalGroup(2)
    ctxs = [InSituContext(W, H, max_supersegments=S, bricks_per_rank=2, rank=r, nranks=2, local_group=group,
                          merge_bricks=True) for r in range(2)]
    try:
        for r, ctx in enumerate(ctxs):
            ctx.set_transfer(sc["tf"], sc["cmap"], sc["conv_scale"], sc["conv_offset"])
            for b in range(2):
                ctx.set_brick(b, bricks[2 * r + b]["vol"], bricks[2 * r + b]["model"])
        for ctx in ctxs:
            ctx.render(sc["cam"])
        for ctx in ctxs:
            ctx.exchange()
        for ctx in ctxs:
            ctx.composite()
        ctxs[1].gather(want_image=False)
        img = ctxs[0].gather(want_image=True)
    finally:
        for ctx in ctxs:
            ctx.close()
        group.close()
    subs = []
    for r in range(2):
        inps = [orc.Inputs(b["vol"], b["im"], b["tf"], b["cmap"], b["conv_k"], b["conv_offset"], sc["cam"])
                for b in bricks[2 * r:2 * r + 2]]
        c, d, _, _ = orc.vdi_generate_multi(inps, W, H, S)
        subs.append((c, d))
    ref = orc.vdi_flatten([c for c, _ in subs], [d for _, d in subs], W, H, 0, W, orc.ipv_of(sc["cam"]))
    assert np.count_nonzero(ref[..., 3]) > 0
    assert np.array_equal(img, ref)


def test_default_cache_grows_to_demand(monkeypatch):
    """A default-sized sample cache that starts below the frame's demand (test knob
    INSITU_CACHE_START_CHUNKS: no first-frame sizing): the first frame searches the rays without
    space by re-sampling (counted as uncached), the cache grows to 1.25x the measured demand before
    the second frame, which caches every ray -- both frames bit-identical to the oracle."""
    sc = make_scene(n=32, W=96, H=80, yaw=30.0)
    S = 8
    monkeypatch.setenv("INSITU_CACHE_START_CHUNKS", "2048")
    rc, rd, ro, _ = _oracle_vdi(sc, S)
    with _ctx_for(sc, S=S) as ctx:
        ctx.set_brick(0, sc["vol"], sc["model"])
        stats = []
        for _ in range(2):
            ctx.render(sc["cam"])
            stats.append(ctx.stats())
            _assert_vdi_equal(ctx.read(native.BUF_VDI_COLOR), ctx.read(native.BUF_VDI_DEPTH), rc, rd)
            assert np.array_equal(ctx.read(native.BUF_OCTREE), ro)
    assert stats[0]["rays_uncached"] > 0 and stats[0]["cache_bytes"] == 2048 * 32
    assert stats[1]["rays_uncached"] == 0 and stats[1]["cache_bytes"] > stats[0]["cache_bytes"]
    assert stats[1]["cache_bytes"] >= stats[0]["cache_demand_bytes"]


@pytest.mark.parametrize("case", [
    dict(n=32, W=72, H=56, yaw=120.0, S=12, B=1, depth=0),
    dict(n=32, W=96, H=80, yaw=30.0, S=8, B=3, depth=0),
    dict(n=32, W=72, H=56, yaw=120.0, S=12, B=2, depth=3),
    dict(n=24, W=50, H=37, yaw=75.0, S=5, B=1, depth=1),
    dict(n=32, W=96, H=80, yaw=30.0, S=8, B=2, depth=0),
])
def test_generator_two_renders_bit_exact(case):
    """Two renders in a row on one context (the second reuses the queue, the cache and the tile order)
    for several tree-group depths and bricks per rank: VDI, octree and pass counts of every brick equal
    the oracle's both times."""
    sc = make_scene(n=case["n"], W=case["W"], H=case["H"], yaw=case["yaw"])
    S, B = case["S"], case["B"]
    with _ctx_for(sc, S=S, B=B) as ctx:
        if case["depth"]:
            ctx.set_option(native.OPT_SEARCH_DEPTH, case["depth"])
        for b in range(B):
            ctx.set_brick(b, sc["vol"], sc["model"])
        for _ in range(2):
            ctx.render(sc["cam"])
            st = ctx.stats()
            got = [(ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b),
                    ctx.read(native.BUF_OCTREE, b), ctx.read(native.BUF_PASSES, b)) for b in range(B)]
            rc, rd, ro, rp = _oracle_vdi(sc, S)
            for col, dep, octree, passes in got:
                _assert_vdi_equal(col, dep, rc, rd)
                assert np.array_equal(octree, ro)
                assert np.array_equal(passes.astype(np.int32), rp)
    assert st["rays_searched"] > 0 and st["rays_uncached"] == 0


@pytest.mark.parametrize("regroup", [0, 1])
@pytest.mark.parametrize("case", [
    dict(n=32, W=96, H=80, yaw=30.0, S=8, B=3, depth=1),
    dict(n=32, W=72, H=56, yaw=120.0, S=12, B=2, depth=2),
    dict(n=24, W=50, H=37, yaw=75.0, S=5, B=1, depth=3),
])
def test_regroup_bit_exact(case, regroup):
    """INSITU_OPT_REGROUP: once the search queue is drained, waves re-form their groups with deeper trees
    for the rays left (ray state broadcast from the old leader lanes, LDS slots kept) -- VDI, octree and
    pass counts of every brick equal the oracle's, from a forced first depth of 1, 2 or 3 (small frames get
    the deepest tree automatically, where no regroup is possible).  The regroups happened (insitu_stats
    search_regroups > 0) with the option on, and none with it off."""
    sc = make_scene(n=case["n"], W=case["W"], H=case["H"], yaw=case["yaw"])
    S, B = case["S"], case["B"]
    with _ctx_for(sc, S=S, B=B) as ctx:
        ctx.set_option(native.OPT_REGROUP, regroup)
        if case["depth"]:
            ctx.set_option(native.OPT_SEARCH_DEPTH, case["depth"])
        for b in range(B):
            ctx.set_brick(b, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        st = ctx.stats()
        rc, rd, ro, rp = _oracle_vdi(sc, S)
        for b in range(B):
            _assert_vdi_equal(ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b), rc, rd)
            assert np.array_equal(ctx.read(native.BUF_OCTREE, b), ro)
            assert np.array_equal(ctx.read(native.BUF_PASSES, b).astype(np.int32), rp)
    assert st["rays_searched"] > 0 and st["rays_uncached"] == 0
    assert (st["search_regroups"] > 0) == bool(regroup), st["search_regroups"]


@pytest.mark.parametrize("exact_keys", [0, 1])
def test_tile_key_modes_bit_exact(exact_keys):
    """INSITU_OPT_EXACT_TILE_KEYS: the longest-first sampling order keyed by 16 or by all 64 rays of a tile,
    over three renders (the first sizes the cache with the exact keys) -- VDI, octree and pass counts equal
    the oracle's."""
    sc = make_scene(n=32, W=96, H=80, yaw=30.0)
    S, B = 8, 2
    with _ctx_for(sc, S=S, B=B) as ctx:
        ctx.set_option(native.OPT_EXACT_TILE_KEYS, exact_keys)
        for b in range(B):
            ctx.set_brick(b, sc["vol"], sc["model"])
        rc, rd, ro, rp = _oracle_vdi(sc, S)
        for _ in range(3):
            ctx.render(sc["cam"])
            for b in range(B):
                _assert_vdi_equal(ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b), rc, rd)
                assert np.array_equal(ctx.read(native.BUF_OCTREE, b), ro)
                assert np.array_equal(ctx.read(native.BUF_PASSES, b).astype(np.int32), rp)


@pytest.mark.parametrize("sup", [2, 4])
def test_super_tile_order_bit_exact(sup):
    """INSITU_OPT_SUPER_TILE: the longest-first sampling order by super-tiles of sup x sup tiles (a ragged
    last row and column of super-tiles: 96x80 px = 12 x 10 tiles) -- VDI, octree and pass counts of
    every brick equal the oracle's."""
    sc = make_scene(n=32, W=96, H=80, yaw=30.0)
    S, B = 8, 3
    with _ctx_for(sc, S=S, B=B) as ctx:
        ctx.set_option(native.OPT_SUPER_TILE, sup)
        for b in range(B):
            ctx.set_brick(b, sc["vol"], sc["model"])
        ctx.render(sc["cam"])
        st = ctx.stats()
        rc, rd, ro, rp = _oracle_vdi(sc, S)
        for b in range(B):
            _assert_vdi_equal(ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b), rc, rd)
            assert np.array_equal(ctx.read(native.BUF_OCTREE, b), ro)
            assert np.array_equal(ctx.read(native.BUF_PASSES, b).astype(np.int32), rp)
    assert st["rays_searched"] > 0 and st["rays_uncached"] == 0


@pytest.mark.parametrize("exact", [0, 1])
def test_vdi_compositor_cached_search_bit_exact(exact):
    """VDICompositor with the merge cache grown to the demand (the second frame: every wave replays its
    cached sequence -- 32-byte entries, the world positions recomputed from the depths
    (INSITU_COMP_ENTRY_WORLD 0) -- with filtered decisions and the interval walk; exact = 1: every decision by
    the exact path) -- composited VDI and pass counts equal the oracle's, three lists."""
    W, H, S, S_out = 72, 56, 8, 6
    scs = [make_scene(n=24, W=W, H=H, yaw=120.0),
           make_scene(n=24, W=W, H=H, yaw=120.0, seed=7, origin=(0.0, -0.25, -0.75)),
           make_scene(n=24, W=W, H=H, yaw=120.0, seed=9, origin=(-0.7, 0.1, 0.2))]
    with InSituContext(W, H, max_supersegments=S, bricks_per_rank=3, keep_passes=True, composite_vdi=True,
                       max_output_supersegments=S_out) as ctx:
        ctx.set_option(native.OPT_EXACT_SEARCH, exact)
        ctx.set_transfer(scs[0]["tf"], scs[0]["cmap"], scs[0]["conv_scale"], scs[0]["conv_offset"])
        for b, sc in enumerate(scs):
            ctx.set_brick(b, sc["vol"], sc["model"])
        subs = [_oracle_vdi(scs[0], S, vol=sc["vol"], im=sc["im"]) for sc in scs]
        ipv = orc.ipv_of(scs[0]["cam"])
        oc, od, op = orc.vdi_composite([r[0] for r in subs], [r[1] for r in subs], W, H, 0, W, ipv, S_out)
        for _ in range(2):   # frame 1 sizes the merge cache, frame 2 runs every wave from it
            ctx.frame(scs[0]["cam"])
            _assert_vdi_equal(ctx.read(native.BUF_COMPOSITED_COLOR), ctx.read(native.BUF_COMPOSITED_DEPTH), oc, od)
            assert np.array_equal(ctx.read(native.BUF_COMPOSITE_PASSES).astype(np.int32), op)
    assert np.count_nonzero(od) > 0 and op.max() > 4
