"""VDICompositor.comp restatement (oracle/insitu_oracle.c: orc_vdi_composite) pinned on CPU:
bit-exact agreement with the independent pure-Python restatement (tests/pyref.py
composite_pixel) and known-answer tests derived from the shader text."""
from __future__ import annotations

import numpy as np
import pytest

import oracle_binding as orc
import pyref
from scenes import make_scene


def _sub_vdis(W, H, S, yaw=45.0):
    sc = make_scene(n=16, W=W, H=H, yaw=yaw)
    sc2 = make_scene(n=16, W=W, H=H, yaw=yaw, seed=7, origin=(0.0, -0.25, -0.75))
    outs = []
    for s in (sc, sc2):
        inp = orc.Inputs(s["vol"], s["im"], s["tf"], s["cmap"], s["conv_k"], 0.0, sc["cam"])
        outs.append(orc.vdi_generate(inp, W, H, S))
    return sc, [o[0] for o in outs], [o[1] for o in outs]


def _lists(colors, depths, x, y, S):
    return [[(float(d[x, y, 2 * i]), float(d[x, y, 2 * i + 1]), tuple(float(v) for v in c[x, y, i]))
             for i in range(S)] for c, d in zip(colors, depths)]


@pytest.mark.parametrize("S_out,x0,sw", [(4, 0, 20), (3, 8, 12), (6, 4, 8)])
def test_composite_pyref_equals_oracle(S_out, x0, sw):
    W, H, S = 20, 16, 4
    sc, colors, depths = _sub_vdis(W, H, S)
    ipv = orc.ipv_of(sc["cam"])
    oc, od, op = orc.vdi_composite(colors, depths, W, H, x0, sw, ipv, S_out)
    ipv_l = pyref.matmul(sc["cam"].inv_view.tolist(), sc["cam"].inv_proj.tolist())
    written = 0
    for xl in range(sw):
        for y in range(H):
            slots, passes = pyref.composite_pixel(_lists(colors, depths, x0 + xl, y, S), ipv_l, x0 + xl, y, W, H, S_out)
            assert passes == op[y, xl], (xl, y)
            for i, (s, e, c) in enumerate(slots):
                got = (od[xl, y, 2 * i], od[xl, y, 2 * i + 1], *oc[xl, y, i])
                want = np.array((s, e, *c), np.float32)
                assert np.array_equal(np.array(got, np.float32).view(np.uint32), want.view(np.uint32)), (xl, y, i)
                written += s != 0.0
    assert written > 0


def test_composite_empty_lists_give_zero():
    """No input supersegment -> every output slot zero (VDICompositor.comp:461-468)."""
    W, H, S, S_out = 8, 8, 4, 5
    c = np.zeros((W, H, S, 4), np.float32)
    d = np.zeros((W, H, 2 * S), np.float32)
    sc = make_scene(n=16, W=W, H=H)
    oc, od, op = orc.vdi_composite([c, c], [d, d], W, H, 0, W, orc.ipv_of(sc["cam"]), S_out)
    assert not oc.any() and not od.any()
    assert op.min() > 1   # the search still bisects down to |high - low| < 1e-6, then writes


def test_composite_single_supersegment_round_trips():
    """One input supersegment -> one output supersegment with the same start/end, and its colour
    back within float rounding (opacity corrected to the segment length and back)."""
    W, H, S, S_out = 8, 8, 3, 4
    sc = make_scene(n=16, W=W, H=H)
    c = np.zeros((W, H, S, 4), np.float32)
    d = np.zeros((W, H, 2 * S), np.float32)
    c[:, :, 0] = (0.8, 0.4, 0.2, 0.3)
    d[:, :, 0] = 0.95
    d[:, :, 1] = 0.97
    oc, od, _ = orc.vdi_composite([c], [d], W, H, 0, W, orc.ipv_of(sc["cam"]), S_out)
    assert np.array_equal(od[..., 0], d[..., 0]) and np.array_equal(od[..., 1], d[..., 1])
    assert not od[..., 2:].any() and not oc[:, :, 1:].any()
    np.testing.assert_allclose(oc[:, :, 0], c[:, :, 0], rtol=0, atol=2e-5)


def test_composite_merges_in_depth_order():
    """Interleaved lists merge front to back: every output list is sorted, compact, count <= S_out,
    and the first start is the smallest input start (determineNextSupseg, VDICompositor.comp:58-91)."""
    W, H, S = 20, 16, 4
    sc, colors, depths = _sub_vdis(W, H, S)
    S_out = 3
    oc, od, _ = orc.vdi_composite(colors, depths, W, H, 0, W, orc.ipv_of(sc["cam"]), S_out)
    starts, ends = od[..., 0::2], od[..., 1::2]
    filled = starts != 0
    assert filled.any()
    assert np.all(np.diff(filled.astype(np.int8), axis=2) <= 0)
    nxt = filled[..., 1:]
    assert np.all(starts[..., 1:][nxt] > starts[..., :-1][nxt])
    assert np.all(ends[filled] >= starts[filled])
    in_starts = np.concatenate([d[..., 0::2] for d in depths], axis=2)
    in_min = np.where(in_starts != 0, in_starts, np.inf).min(axis=2)
    has = np.isfinite(in_min)
    assert np.array_equal(starts[..., 0][has], in_min[has].astype(np.float32))
