"""Oracle restatement of several volumes in ONE VDI (VDIGenerator.comp $repeat, :333-347, with
AccumulateVDI spliced once per volume, AV:1) -- pinned against the single-volume restatement on the
cases where the shader text fixes the answer (CPU)."""
from __future__ import annotations

import numpy as np

import oracle_binding as orc
from scenes import make_scene

W, H, S = 64, 48, 8


def _inp(sc):
    return orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], sc["cam"])


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def test_one_volume_equals_single_brick_restatement():
    sc = make_scene(n=32, W=W, H=H, yaw=30.0)
    a = orc.vdi_generate(_inp(sc), W, H, S)
    b = orc.vdi_generate_multi([_inp(sc)], W, H, S)
    for x, y in zip(a, b):
        assert np.array_equal(_bits(x) if x.dtype == np.float32 else x, _bits(y) if y.dtype == np.float32 else y)


def test_volume_outside_every_ray_changes_nothing():
    """A second volume no ray intersects is never `vis`: the VDI is the first volume's."""
    sc = make_scene(n=32, W=W, H=H, yaw=30.0)
    far = make_scene(n=16, W=W, H=H, yaw=30.0, seed=5, origin=(40.0, 40.0, 40.0))
    a = orc.vdi_generate(_inp(sc), W, H, S)
    b = orc.vdi_generate_multi([_inp(sc), _inp(far)], W, H, S)
    assert np.array_equal(_bits(a[0]), _bits(b[0])) and np.array_equal(_bits(a[1]), _bits(b[1]))
    assert np.array_equal(a[3], b[3])


def test_disjoint_volumes_commute_and_merge():
    """Two volumes no step samples both (a gap between them): volume order is irrelevant, and rays
    through both get supersegments from both in one list (more than either alone on some pixels)."""
    s1 = make_scene(n=24, W=W, H=H, yaw=35.0, origin=(-0.9, -0.5, -0.5), world=0.8)
    s2 = make_scene(n=24, W=W, H=H, yaw=35.0, seed=7, origin=(0.1, -0.5, -0.5), world=0.8)
    ab = orc.vdi_generate_multi([_inp(s1), _inp(s2)], W, H, S)
    ba = orc.vdi_generate_multi([_inp(s2), _inp(s1)], W, H, S)
    assert np.array_equal(_bits(ab[0]), _bits(ba[0])) and np.array_equal(_bits(ab[1]), _bits(ba[1]))
    n_ab = np.count_nonzero(ab[1][..., 0::2], axis=2)
    n_1 = np.count_nonzero(orc.vdi_generate(_inp(s1), W, H, S)[1][..., 0::2], axis=2)
    n_2 = np.count_nonzero(orc.vdi_generate(_inp(s2), W, H, S)[1][..., 0::2], axis=2)
    assert np.any((n_1 > 0) & (n_2 > 0)), "no ray crosses both volumes"
    assert n_ab.max() <= S
    assert np.all(n_ab[(n_1 == 0) & (n_2 == 0)] == 0)
