"""Known-answer tests derived by hand from the shader text (SURVEY.md 8c list), checked
against analytic float64 expectations.  They pin what the oracle computes, independently of
its own arithmetic.  CPU only."""
from __future__ import annotations

import math

import numpy as np
import pytest

import oracle_binding as orc
from insitu_amd import native, scene

N = 16           # brick edge (voxels), brick = [-0.5, 0.5]^3 world
W = H = 32


def _setup(vol, tf, cmap, yaw=0.0, pitch=0.0, spv=1.0, target_offset=None):
    model = scene.brick_model((-0.5, -0.5, -0.5), 1.0 / N)
    cam = scene.orbit_camera(W, H, yaw_deg=yaw, pitch_deg=pitch, voxel_world=1.0 / N, samples_per_voxel=spv)
    if target_offset is not None:   # look away from the brick
        eye = np.linalg.inv(cam.view_rm)[:3, 3]
        cam = scene.CameraSpec(scene.look_at(eye, eye + np.asarray(target_offset)), scene.perspective(50.0, 1.0),
                               cam.nw)
    conv_k = scene.folded_conv_scale(1.0, native.U16)
    inp = orc.Inputs(vol, scene.inverse_model(model), tf, cmap, conv_k, 0.0, cam)
    return inp, cam


def _hits(cam):
    """float64 ray/box test per pixel, returns (hit mask [x][y], entry t, exit t, wfront, wback)."""
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    hit = np.zeros((W, H), bool)
    ent = np.zeros((W, H, 3))
    ext = np.zeros((W, H, 3))
    for x in range(W):
        for y in range(H):
            uv = (2.0 * x / W - 1.0, 2.0 * y / H - 1.0)
            f = ipv @ np.array([uv[0], uv[1], -1.0, 1.0]); f = f[:3] / f[3]
            b = ipv @ np.array([uv[0], uv[1], 1.0, 1.0]); b = b[:3] / b[3]
            d = b - f
            with np.errstate(divide="ignore"):
                t0 = (-0.5 - f) / d
                t1 = (0.5 - f) / d
            tn, tf = np.max(np.minimum(t0, t1)), np.min(np.maximum(t0, t1))
            if tn < tf:
                hit[x, y] = True
                ent[x, y], ext[x, y] = f + tn * d, f + tf * d
    return hit, ent, ext


def _ndc_z(cam, p):
    c = cam.proj_rm @ cam.view_rm @ np.array([p[0], p[1], p[2], 1.0])
    return c[2] / c[3]


def _const(value=30000):
    return np.full((N, N, N), value, np.uint16)


def test_kat_miss_rays_zero_filled():
    """KAT 1 (VDIGenerator.comp:570-590): a ray that misses the brick writes zeros in all S slots."""
    inp, cam = _setup(_const(), np.full(64, 0.3, np.float32), scene.colormap_hot(), target_offset=(1.0, 0.0, 0.0))
    c, d, o, p = orc.vdi_generate(inp, W, H, 4)
    assert not c.any() and not d.any() and not o.any() and not p.any()


def test_kat_transparent_tf_no_supersegment():
    """KAT 2 (AccumulateVDI.comp:24-26,185): TF alpha 0 -> w = 0 -> nothing opens; the search
    stops after the first pass (0 terminations) plus the write pass (VDIGenerator.comp:520-525)."""
    inp, cam = _setup(_const(), np.zeros(64, np.float32), scene.colormap_hot(), yaw=20.0, pitch=10.0)
    c, d, o, p = orc.vdi_generate(inp, W, H, 4)
    hit, _, _ = _hits(cam)
    assert not c.any() and not d.any() and not o.any()
    assert set(np.unique(p[hit.T])) <= {2}
    assert hit.sum() > 100


@pytest.mark.parametrize("a0,yaw,pitch", [(0.3, 0.0, 0.0), (0.6, 25.0, 15.0)])
def test_kat_homogeneous_brick_one_supersegment(a0, yaw, pitch):
    """KAT 3: a homogeneous brick gives exactly one supersegment per hit ray, whose colour is the
    (un-premultiplied) sample colour and per-unit-length alpha the TF alpha, spanning the ray's
    entry to exit (AccumulateVDI.comp:214-217, 243-248); the flatten gives 1-(1-a0)^L."""
    rgb = np.array([0.8, 0.4, 0.2], np.float32)
    cmap = np.tile(np.append(rgb, 1.0).astype(np.float32), (16, 1))
    inp, cam = _setup(_const(), np.full(64, a0, np.float32), cmap, yaw=yaw, pitch=pitch)
    S = 4
    c, d, o, p = orc.vdi_generate(inp, W, H, S)
    hit, ent, ext = _hits(cam)
    cnt = np.count_nonzero(d[..., 0::2], axis=2)
    inner = hit.copy()   # skip grazing rays (a few samples only)
    inner &= np.linalg.norm(ext - ent, axis=2) > 0.2
    assert inner.sum() > 50
    assert np.all(cnt[inner] == 1)
    assert np.all(cnt[~hit] == 0)
    step_ndc = []
    for x, y in zip(*np.nonzero(inner)):
        assert np.allclose(c[x, y, 0, :3], rgb, atol=2e-5)
        assert abs(c[x, y, 0, 3] - a0) < 2e-3
        zs, ze = _ndc_z(cam, ent[x, y]), _ndc_z(cam, ext[x, y])
        dz = abs(_ndc_z(cam, ent[x, y] + (ext[x, y] - ent[x, y]) * (1.0 / N) / np.linalg.norm(ext[x, y] - ent[x, y])) - zs)
        step_ndc.append(dz)
        assert abs(d[x, y, 0] - zs) <= 2.5 * dz + 1e-6       # first sample inside the brick
        assert abs(d[x, y, 1] - ze) <= 2.5 * dz + 1e-6       # sample after the last one inside
    img = orc.vdi_flatten([c], [d], W, H, 0, W, orc.ipv_of(cam))
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    for x, y in zip(*np.nonzero(inner)):
        # the segment runs from the first sample strictly inside (one step past the entry) to
        # the sample after the last one inside (at or up to one step past the exit)
        uv = (2.0 * x / W - 1.0, 2.0 * y / H - 1.0)
        f = ipv @ np.array([uv[0], uv[1], -1.0, 1.0])
        b = ipv @ np.array([uv[0], uv[1], 1.0, 1.0])
        step = float(cam.nw) * np.linalg.norm(b[:3] / b[3] - f[:3] / f[3])
        L = float(np.linalg.norm(ext[x, y] - ent[x, y]))
        lo, hi = 1.0 - (1.0 - a0) ** max(L - 2 * step, 0.0), 1.0 - (1.0 - a0) ** L
        got = img[y, x, 3] / 255.0
        assert lo - 2.0 / 255.0 <= got <= hi + 2.0 / 255.0, (x, y, got, lo, hi)


def test_kat_two_slabs_split_at_interface():
    """KAT 4: two slabs of different colour -> the supersegment closes at the interface
    (AccumulateVDI.comp:74,91) and a new one opens there (:185)."""
    vol = _const(10000)
    vol[N // 2:] = 50000            # z >= 8 (front half for a camera on +z)
    cmap = scene.colormap_hot()
    inp, cam = _setup(vol, np.full(64, 0.4, np.float32), cmap)
    S = 8
    c, d, o, p = orc.vdi_generate(inp, W, H, S)
    hit, ent, ext = _hits(cam)
    cnt = np.count_nonzero(d[..., 0::2], axis=2)
    interface_world_z = -0.5 + (N // 2 - 0.5) / N      # halfway between voxel centres 7 and 8
    # rays that cross the interface plane inside the brick with >= 2 voxels on either side
    central = hit & (ent[..., 2] > interface_world_z + 2.0 / N) & (ext[..., 2] < interface_world_z - 2.0 / N)
    assert central.sum() > 50
    assert np.all(cnt[central] >= 2)
    assert np.all(cnt[hit & ~central & (ext[..., 2] > interface_world_z + 2.0 / N)] == 1)
    for x, y in zip(*np.nonzero(central)):
        e, q = ent[x, y], ext[x, y]
        t = (interface_world_z - e[2]) / (q[2] - e[2])
        zi = _ndc_z(cam, e + t * (q - e))
        ends = d[x, y, 1:2 * cnt[x, y]:2]
        dz = abs(_ndc_z(cam, e + (q - e) * 0.125) - _ndc_z(cam, e))   # ~2 voxels of NDC
        assert np.min(np.abs(ends - zi)) <= dz, (x, y)


def test_kat_count_bounded_and_compact():
    """KAT 5: supersegment count <= S on every pixel; lists compact; end >= start."""
    from scenes import make_scene
    sc = make_scene(n=32, W=48, H=40, yaw=70.0)
    for S in (3, 6, 20):
        inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
        c, d, o, p = orc.vdi_generate(inp, 48, 40, S)
        starts, ends = d[..., 0::2], d[..., 1::2]
        filled = starts != 0
        assert filled.sum(axis=2).max() <= S
        assert np.all(np.diff(filled.astype(np.int8), axis=2) <= 0)
        assert np.all(ends[filled] >= starts[filled])
        assert p.max() <= 24


def test_kat_depth_encode_roundtrip():
    """KAT 6: EncodeFloatRGBA (VolumeRaycaster.comp:63-69) -> rgba8 -> DecodeFloatRGBA
    (PlainImageCompositor.comp:25-29) round-trips within 1e-6 on [0,1)."""
    import ctypes
    lib = orc.load()
    rng = np.random.default_rng(3)
    buf = (ctypes.c_uint8 * 4)()
    worst = 0.0
    for v in np.concatenate([rng.uniform(0, 1, 2000), [0.0, 0.5, 0.999]]).astype(np.float32):
        lib.orc_encode_depth_rgba8(float(v), buf)
        worst = max(worst, abs(lib.orc_decode_depth_rgba8(buf) - float(v)))
    assert worst < 1e-6


def test_kat_plain_composite_order_and_empty():
    """KAT 7: the plain compositor blends ranks in ascending decoded depth and skips depth 0
    (PlainImageCompositor.comp:58-86), with colour premultiplied by alpha (:81)."""
    import ctypes
    lib = orc.load()

    def enc(v):
        b = (ctypes.c_uint8 * 4)()
        lib.orc_encode_depth_rgba8(v, b)
        return np.frombuffer(bytes(b), np.uint8)

    A = np.array([200, 100, 50, 128], np.uint8)
    Bc = np.array([10, 20, 250, 200], np.uint8)
    cols = [A.reshape(1, 1, 4), Bc.reshape(1, 1, 4)]
    deps = [enc(0.6).reshape(1, 1, 4), enc(0.3).reshape(1, 1, 4)]
    out = orc.plain_composite(cols, deps, 1)[0, 0]
    a, b = A / 255.0, Bc / 255.0
    C = np.zeros(4)
    for col in (b, a):                      # B (depth 0.3) first, then A
        C[:3] += (1 - C[3]) * col[:3] * col[3]
        C[3] += (1 - C[3]) * col[3]
    assert np.all(np.abs(out.astype(int) - np.round(C * 255)) <= 1)
    deps[0] = np.zeros((1, 1, 4), np.uint8)  # rank 0 empty -> only B
    out = orc.plain_composite(cols, deps, 1)[0, 0]
    C = np.append(b[:3] * b[3], b[3])
    assert np.all(np.abs(out.astype(int) - np.round(C * 255)) <= 1)


def test_kat_plain_constant_opacity():
    """KAT 8: constant opacity a, no opacity correction in plain mode (AccumulatePlainImage.comp:8-9):
    after n samples alpha = 1-(1-a)^n with n = trunc((tfar-tnear)/nw + 1) (VolumeRaycaster.comp:135)."""
    a0 = 0.02
    cmap = np.ones((8, 4), np.float32)
    inp, cam = _setup(_const(), np.full(64, a0, np.float32), cmap)
    col, dep = orc.plain_raycast(inp, W, H)
    hit, ent, ext = _hits(cam)
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    checked = 0
    for x, y in zip(*np.nonzero(hit)):
        uv = (2.0 * x / W - 1.0, 2.0 * y / H - 1.0)
        f = ipv @ np.array([uv[0], uv[1], -1.0, 1.0]); f = f[:3] / f[3]
        b = ipv @ np.array([uv[0], uv[1], 1.0, 1.0]); b = b[:3] / b[3]
        L = np.linalg.norm(b - f)
        tn, tf = np.linalg.norm(ent[x, y] - f) / L, np.linalg.norm(ext[x, y] - f) / L
        n = math.trunc((tf - tn) / float(cam.nw) + 1)
        expect = [round(255 * (1 - (1 - a0) ** k)) for k in (n - 1, n, n + 1)]
        assert min(abs(int(col[y, x, 3]) - e) for e in expect) <= 1, (x, y)
        checked += 1
    assert checked > 100
    assert not col[~hit.T].any() and not dep[~hit.T].any()


def test_kat_octree_counts():
    """KAT 9: octree counts sum to the sum over written supersegments of
    (end_cell - start_cell + 1) (AccumulateVDI.comp:158-177, VDIGenerator.comp:244-254)."""
    from scenes import make_scene
    sc = make_scene(n=32, W=64, H=48, yaw=50.0)
    S = 8
    inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    c, d, o, p = orc.vdi_generate(inp, 64, 48, S)
    cam = sc["cam"]
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    interval = (20.0 - 0.1) / S
    total = 0
    for x in range(64):
        for y in range(48):
            for i in range(S):
                s, e = d[x, y, 2 * i], d[x, y, 2 * i + 1]
                if s == 0:
                    break
                uv = (2.0 * x / 64 - 1.0, 2.0 * y / 48 - 1.0)
                cells = []
                for z in (s, e):
                    w = ipv @ np.array([uv[0], uv[1], z, 1.0])
                    v = cam.view_rm @ (w / w[3])
                    cells.append(min(int(math.floor(abs(v[2] + 0.1) / interval)), S))
                total += max(0, min(cells[1], S - 1) - cells[0] + 1)
    assert total > 0
    assert abs(int(o.sum()) - total) <= max(2, total // 200)
