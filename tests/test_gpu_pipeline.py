"""GPU parity of pipelined frames (insitu_frame_pipelined): the reference's own frame loop composites the
previous render frame while it distributes the current one (DistributedVolumeRenderer.kt:530-542, 577,
602-603; SURVEY.md 3.2 "the composite is one frame stale").  Here frame k's render (its first pass on a
second stream, started in frame k-1's search tail) overlaps frame k-1's exchange, composite and gather.

Every completed frame -- consecutive frames with different cameras, and a brick re-ingest between two of
them -- must equal the CPU oracle bit for bit: each brick's sub-VDI, octree cells and pass counts, the
flattened image (or, with the VDICompositor, the composited VDI, its pass counts and the root's image of
it), under each trigger mode of INSITU_OPT_PIPE_TRIGGER.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle_binding as orc
from insitu_amd import native, scene
from insitu_amd.renderer import InSituContext
from scenes import make_scene

pytestmark = pytest.mark.gpu

S = 8
W, H = 96, 80


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _scenes():
    """Two bricks side by side, and the volumes the re-ingest swaps in."""
    a = make_scene(n=32, W=W, H=H, origin=(-0.5, -0.5, -0.5))
    b = make_scene(n=32, W=W, H=H, seed=7, origin=(0.0, -0.25, -0.75))
    a2 = make_scene(n=32, W=W, H=H, seed=11, origin=(-0.5, -0.5, -0.5))
    return a, b, a2


def _cams(n):
    vw = 1.0 / 32
    return [scene.orbit_camera(W, H, yaw_deg=30.0 + 37.0 * i, pitch_deg=20.0 - 9.0 * i, voxel_world=vw)
            for i in range(n)]


def _oracle_frame(vols, scs, cam):
    """Per brick (colour, depth, octree, passes) of the oracle, for one frame's camera and volumes."""
    out = []
    for vol, sc in zip(vols, scs):
        inp = orc.Inputs(vol, sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], cam)
        out.append(orc.vdi_generate(inp, W, H, S))
    return out


def _ctx(composite_vdi=False, S_out=0, cache_mb=0):
    a = _scenes()[0]
    ctx = InSituContext(W, H, max_supersegments=S, bricks_per_rank=2, keep_passes=True,
                        composite_vdi=composite_vdi, max_output_supersegments=S_out, sample_cache_mb=cache_mb)
    ctx.set_transfer(a["tf"], a["cmap"], a["conv_scale"], a["conv_offset"])
    return ctx


def _check_frame(ctx, ref, cam, img, composite=False, S_out=0, all_cached=True):
    for b, (rc, rd, ro, rp) in enumerate(ref):
        col, dep = ctx.read(native.BUF_VDI_COLOR, b), ctx.read(native.BUF_VDI_DEPTH, b)
        bad = np.count_nonzero(_bits(col) != _bits(rc)) + np.count_nonzero(_bits(dep) != _bits(rd))
        assert bad == 0, f"brick {b}: {bad} mismatching sub-VDI words"
        assert np.array_equal(ctx.read(native.BUF_OCTREE, b), ro), f"brick {b}: octree cells differ"
        assert np.array_equal(ctx.read(native.BUF_PASSES, b).astype(np.int32), rp), f"brick {b}: passes differ"
    ipv = orc.ipv_of(cam)
    cols, deps = [r[0] for r in ref], [r[1] for r in ref]
    if composite:
        oc, od, op = orc.vdi_composite(cols, deps, W, H, 0, W, ipv, S_out)
        for which_c, which_d in ((native.BUF_COMPOSITED_COLOR, native.BUF_COMPOSITED_DEPTH),
                                 (native.BUF_GATHERED_COLOR, native.BUF_GATHERED_DEPTH)):
            cc, cd = ctx.read(which_c), ctx.read(which_d)
            bad = np.count_nonzero(_bits(cc) != _bits(oc)) + np.count_nonzero(_bits(cd) != _bits(od))
            assert bad == 0, f"composited VDI ({which_c}): {bad} mismatching words"
        assert np.array_equal(ctx.read(native.BUF_COMPOSITE_PASSES).astype(np.int32), op)
        want = orc.vdi_flatten([oc], [od], W, H, 0, W, ipv)
    else:
        want = orc.vdi_flatten(cols, deps, W, H, 0, W, ipv)
    assert np.array_equal(img, want), f"image differs: max |dRGBA| {np.max(np.abs(img.astype(int) - want.astype(int)))}"
    assert np.count_nonzero(want[..., 3]) > 0
    st = ctx.stats()
    assert st["pipelined"] == 1 and (st["rays_uncached"] == 0 or not all_cached)
    return st


def _run(ctx, trigger, composite=False, S_out=0, nframes=5, reingest_after=2, all_cached=True):
    """nframes pipelined frames, cameras differing every frame, brick 0 re-ingested (from a device tensor)
    after frame `reingest_after` was enqueued; every completed frame checked against the oracle."""
    a, b, a2 = _scenes()
    ctx.set_option(native.OPT_PIPE_TRIGGER, trigger)
    dev_a2 = torch.from_numpy(a2["vol"].view(np.int16)).cuda()
    ctx.set_brick(0, a["vol"], a["model"])
    ctx.set_brick(1, b["vol"], b["model"])
    cams = _cams(nframes)
    vols_of = [[a["vol"], b["vol"]] if k <= reingest_after else [a2["vol"], b["vol"]] for k in range(nframes)]
    seen, stats = [], []
    for k, cam in enumerate(cams):
        done, img = ctx.frame_pipelined(cam, want_image=True)
        assert done == k - 1, f"call {k} completed frame {done}"
        if done >= 0:
            stats.append(_check_frame(ctx, _oracle_frame(vols_of[done], [a, b], cams[done]), cams[done], img, composite,
                                      S_out, all_cached))
            seen.append(done)
        if k == reingest_after:   # enqueued behind frame k's search, before frame k+1's first pass
            ctx.set_brick(0, dev_a2, a2["model"], dtype=native.U16)
    done, img = ctx.pipeline_flush(want_image=True)
    assert done == nframes - 1
    stats.append(_check_frame(ctx, _oracle_frame(vols_of[done], [a, b], cams[done]), cams[done], img, composite, S_out,
                              all_cached))
    seen.append(done)
    assert seen == list(range(nframes))
    assert ctx.pipeline_flush()[0] == -1   # nothing in flight
    assert ctx.stats()["ms_ingest"] > 0    # the re-ingest's GPU time (insitu_stats.ms_ingest)
    return stats


@pytest.mark.parametrize("trigger", [1, 0, 2])
def test_pipelined_frames_bit_exact(trigger):
    """Five pipelined frames (different cameras, a re-ingest between frames 2 and 3) under each trigger of
    the next frame's first pass: at the previous search's queue drain (1, default), after it (0), at once (2)
    -- every frame's sub-VDIs, octree cells, pass counts and flattened image bit for bit."""
    with _ctx() as ctx:
        _run(ctx, trigger)


@pytest.mark.parametrize("oversub,depth", [(1, 0), (64, 0), (3, 1)])
def test_pipelined_search_groups_bit_exact(oversub, depth):
    """Pipelined frames under their own oversubscription (INSITU_OPT_PIPE_OVERSUB: the tree-group size the
    search picks from its queue length) and under a fixed depth of 1 (one lane per ray, deeper groups only
    from the regroup at the queue's tail): the results do not depend on how the lanes are grouped."""
    with _ctx() as ctx:
        ctx.set_option(native.OPT_PIPE_OVERSUB, oversub)
        if depth:
            ctx.set_option(native.OPT_SEARCH_DEPTH, depth)
        _run(ctx, 1, nframes=3, reingest_after=0)


@pytest.mark.parametrize("rays,trigger", [(0, 1), (1, 2), (2048, 2), (1 << 24, 1)])
def test_pipelined_search_grid_bit_exact(rays, trigger):
    """INSITU_OPT_PIPE_SEARCH_RAYS: the pipelined search keeps clamp(queue / rays, one block per CU, two) of its
    blocks (0: the full persistent grid) and the next frame's first pass takes the other wave slots, at once
    (trigger 2) or at the drain (1) -- the frames are the same bit for bit."""
    with _ctx() as ctx:
        ctx.set_option(native.OPT_PIPE_SEARCH_RAYS, rays)
        _run(ctx, trigger, nframes=3, reingest_after=0)


def test_pipelined_vdi_compositor_bit_exact():
    """Pipelined frames through the VDICompositor (composite_vdi, S_out = 6 < S): each frame's composited VDI
    (strip and gathered copy, count-bounded readback), compositor passes and root image equal the oracle's.
    The cameras change every frame, so a pixel's slot count falls below the previous frame's and the slots
    past it keep stale data that every reader must stop before."""
    with _ctx(composite_vdi=True, S_out=6) as ctx:
        _run(ctx, 1, composite=True, S_out=6)


@pytest.mark.parametrize("cache", ["grow", "off"])
def test_pipelined_cache_paths(cache, monkeypatch):
    """Pipelined frames through the sample cache's other paths, each frame bit for bit: grow -- a default cache
    that starts below the demand (INSITU_CACHE_START_CHUNKS): the first frame of each slot runs the rays without
    space through their whole search in the sampling kernel, re-sampling the brick that the re-ingest after
    frame 1 replaces (it must wait for them), then each slot's cache is re-allocated larger while the other
    slot's frame is in flight; off -- refused (no search queue to pipeline)."""
    if cache == "off":
        with _ctx(cache_mb=-1) as ctx:
            a, b, _ = _scenes()
            ctx.set_brick(0, a["vol"], a["model"])
            ctx.set_brick(1, b["vol"], b["model"])
            with pytest.raises(RuntimeError, match="sample cache"):
                ctx.frame_pipelined(_cams(1)[0])
        return
    monkeypatch.setenv("INSITU_CACHE_START_CHUNKS", "2048")
    with _ctx() as ctx:
        stats = _run(ctx, 1, reingest_after=1, all_cached=False)
    assert stats[0]["rays_uncached"] > 0 and stats[1]["rays_uncached"] > 0   # the first frame of each slot
    assert stats[-1]["rays_uncached"] == 0 and stats[-1]["cache_bytes"] > 2048 * 32   # both slots grew


def test_pipelined_merged_bricks_bit_exact():
    """Pipelined frames with the rank's bricks merged into one sub-VDI (merge_bricks, VDIGenerator.comp's
    $repeat): the merge kernel and the merged search on the pipeline's streams, three frames with different
    cameras -- each frame's merged VDI, pass counts and image equal the oracle's multi-volume restatement."""
    a, b, _ = _scenes()
    cams = _cams(3)
    with InSituContext(W, H, max_supersegments=S, bricks_per_rank=2, keep_passes=True, merge_bricks=True) as ctx:
        ctx.set_transfer(a["tf"], a["cmap"], a["conv_scale"], a["conv_offset"])
        ctx.set_brick(0, a["vol"], a["model"])
        ctx.set_brick(1, b["vol"], b["model"])
        got = []
        for call in [lambda c=c: ctx.frame_pipelined(c, want_image=True) for c in cams] + \
                    [lambda: ctx.pipeline_flush(want_image=True)]:
            done, img = call()
            if done >= 0:
                got.append((done, img, ctx.read(native.BUF_VDI_COLOR), ctx.read(native.BUF_VDI_DEPTH),
                            ctx.read(native.BUF_PASSES), ctx.stats()))
    assert [g[0] for g in got] == [0, 1, 2]
    for done, img, col, dep, passes, st in got:
        cam = cams[done]
        inps = [orc.Inputs(s_["vol"], s_["im"], s_["tf"], s_["cmap"], s_["conv_k"], s_["conv_offset"], cam) for s_ in (a, b)]
        rc, rd, ro, rp = orc.vdi_generate_multi(inps, W, H, S)
        assert np.array_equal(_bits(col), _bits(rc)) and np.array_equal(_bits(dep), _bits(rd)), f"frame {done}"
        assert np.array_equal(passes.astype(np.int32), rp)
        assert np.array_equal(img, orc.vdi_flatten([rc], [rd], W, H, 0, W, orc.ipv_of(cam)))
        assert st["pipelined"] == 1 and st["rays_searched"] > 0


def test_pipelined_then_unpipelined_frames():
    """A context can go back to unpipelined frames after a flush (and the stage calls refuse while a frame is
    in flight); the unpipelined frame renders what the oracle renders."""
    a, b, _ = _scenes()
    cams = _cams(3)
    with _ctx() as ctx:
        ctx.set_brick(0, a["vol"], a["model"])
        ctx.set_brick(1, b["vol"], b["model"])
        assert ctx.frame_pipelined(cams[0])[0] == -1
        with pytest.raises(RuntimeError, match="in flight"):
            ctx.render(cams[1])
        with pytest.raises(RuntimeError, match="in flight"):
            ctx.gather()
        assert ctx.pipeline_flush()[0] == 0
        img = ctx.frame(cams[2], want_image=True)
        assert ctx.stats()["pipelined"] == 0
        ref = _oracle_frame([a["vol"], b["vol"]], [a, b], cams[2])
        _check_frame_unpipelined(ctx, ref, cams[2], img)


def test_destroy_with_frames_in_flight():
    """insitu_destroy while a pipelined frame is in flight (no flush; its first pass waits on the previous
    search's trigger, its search and the completion streams still busy): the context synchronises every stream
    before it frees what they read, and a new context then renders what the oracle renders."""
    a, b, _ = _scenes()
    cams = _cams(3)
    for _ in range(2):
        ctx = _ctx()
        ctx.set_brick(0, a["vol"], a["model"])
        ctx.set_brick(1, b["vol"], b["model"])
        ctx.frame_pipelined(cams[0])
        ctx.frame_pipelined(cams[1])   # frame 1 in flight behind frame 0's completion
        ctx.close()
    with _ctx() as ctx:
        ctx.set_brick(0, a["vol"], a["model"])
        ctx.set_brick(1, b["vol"], b["model"])
        img = ctx.frame(cams[2], want_image=True)
        _check_frame_unpipelined(ctx, _oracle_frame([a["vol"], b["vol"]], [a, b], cams[2]), cams[2], img)


def _check_frame_unpipelined(ctx, ref, cam, img):
    for b, (rc, rd, ro, rp) in enumerate(ref):
        assert np.array_equal(_bits(ctx.read(native.BUF_VDI_DEPTH, b)), _bits(rd))
        assert np.array_equal(_bits(ctx.read(native.BUF_VDI_COLOR, b)), _bits(rc))
    want = orc.vdi_flatten([r[0] for r in ref], [r[1] for r in ref], W, H, 0, W, orc.ipv_of(cam))
    assert np.array_equal(img, want)


def test_pipelined_rejects_plain_mode():
    a = _scenes()[0]
    with InSituContext(W, H, mode=native.MODE_PLAIN) as ctx:
        ctx.set_transfer(a["tf"], a["cmap"])
        ctx.set_brick(0, a["vol"], a["model"])
        with pytest.raises(RuntimeError, match="VDI mode"):
            ctx.frame_pipelined(_cams(1)[0])
