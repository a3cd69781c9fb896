"""The reference-shaped C entry points driven from C with the Kotlin argument units.

tests/c_harness/kotlin_units_harness.c is a plain C program (one process per rank) that calls
insitu_distribute_vdis / insitu_gather_composited_vdis / insitu_gather_composited_vdi_set with the
sizes scenery-insitu_amd/jni/kotlin_units.h computes -- the header the JNI adaptor
(scenery-insitu_amd/jni/insitu_jni.cpp) takes its sizes from:
  DistributedVolumes.distributeVDIs        sizePerProcess = H*W*S*4/commSize floats   (DistributedVolumes.kt:860)
  DistributedVolumes.gatherCompositedVDIs  compositedVDILen = H*W*S_out*4/commSize    (DistributedVolumes.kt:903)
  DistributedVolumeRenderer.distributeVDIs sizePerProcess = H*W*4/commSize bytes      (DistributedVolumeRenderer.kt:577)
  DistributedVolumeRenderer.gatherCompositedVDIs subVDILen = H*W*4/commSize bytes     (DistributedVolumeRenderer.kt:602)
The inputs are the oracle's sub-VDIs / sub-images; the outputs are checked bit for bit against the
oracle's flatten, VDICompositor and PlainImageCompositor restatements, and the received sets
against the source-major blocks of the senders' buffers.  Two ranks run RCCL (on a one-GPU box
through its socket transport, as tests/test_gpu_rccl.py)."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_binding as orc
from insitu_amd import native
from scenes import make_scene

ROOT = Path(__file__).resolve().parent.parent
HARNESS = ROOT / "tests" / "c_harness" / "build" / "kotlin_units_harness"


def _need_harness():
    if not HARNESS.exists():
        pytest.fail(f"{HARNESS} not built (run __graft_entry__.build() or make -C tests/c_harness)")


def test_harness_links_and_reports_abi():
    """CPU: the C program links libinsitu_hip.so and agrees on the ABI version (no GPU call)."""
    _need_harness()
    p = subprocess.run([str(HARNESS), "--abi"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and f"insitu_abi_version {native.ABI_VERSION}" in p.stdout, p.stdout + p.stderr


def _write_common(d: Path, sc, W, H, S, S_out, dims=(0, 0, 0)):
    (d / "case.txt").write_text(f"{W} {H} {S} {S_out} {dims[0]} {dims[1]} {dims[2]}\n")
    (d / "camera.bin").write_bytes(bytes(sc["cam"].native()))
    (d / "tf.bin").write_bytes(np.ascontiguousarray(sc["tf"], np.float32).tobytes())
    (d / "cmap.bin").write_bytes(np.ascontiguousarray(sc["cmap"], np.float32).reshape(-1, 4).tobytes())
    (d / "conv.bin").write_bytes(np.array([sc["conv_scale"], sc["conv_offset"]], np.float32).tobytes())


def _run(kind: str, d: Path, nranks: int):
    import torch
    ndev = torch.cuda.device_count()   # does not initialise the GPU
    procs = []
    for r in range(nranks):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", NCCL_DEBUG="WARN")
        if ndev < nranks:   # ranks share a GPU: distinct host ids, RCCL socket transport on loopback
            env.update(NCCL_HOSTID=f"harness-rank-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([str(HARNESS), kind, str(d), str(r), str(nranks), str(r % max(1, ndev))],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for r, (rc, out) in enumerate(outs):
        assert rc == 0 and "HARNESS_OK" in out, f"rank {r}: rc {rc}\n{out[-3000:]}"


def _scenes(W, H, nranks):
    sc = make_scene(n=24, W=W, H=H, yaw=40.0)
    scs = [sc, make_scene(n=24, W=W, H=H, yaw=40.0, seed=7, origin=(0.0, -0.25, -0.75))][:nranks]
    return sc, scs


def _oracle_sub(sc_r, cam_sc, S):
    inp = orc.Inputs(sc_r["vol"], sc_r["im"], cam_sc["tf"], cam_sc["cmap"], cam_sc["conv_k"], cam_sc["conv_offset"],
                     cam_sc["cam"])
    c, d, _, _ = orc.vdi_generate(inp, cam_sc["W"], cam_sc["H"], S)
    return c, d


def _check_recv(d: Path, subs, nranks):
    """rank r received block r of every sender's buffer, source-major (allToAllColorPointer)."""
    for r in range(nranks):
        for which, k in (("col", 0), ("dep", 1)):
            got = np.fromfile(d / f"recv_{which}_{r}.bin", np.uint8)
            want = np.concatenate([np.array_split(np.ascontiguousarray(s[k]).view(np.uint8).ravel(), nranks)[r]
                                   for s in subs])
            assert np.array_equal(got, want), (which, r)


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("nranks", [1, 2])
def test_harness_vdi_flatten(tmp_path, nranks):
    _need_harness()
    W, H, S = 48, 40, 6
    sc, scs = _scenes(W, H, nranks)
    subs = [_oracle_sub(s, sc, S) for s in scs]
    _write_common(tmp_path, sc, W, H, S, 0)
    for r, (c, dd) in enumerate(subs):
        (tmp_path / f"sub_col_{r}.bin").write_bytes(c.tobytes())
        (tmp_path / f"sub_dep_{r}.bin").write_bytes(dd.tobytes())
    _run("vdi", tmp_path, nranks)
    _check_recv(tmp_path, subs, nranks)
    img = np.fromfile(tmp_path / "image.bin", np.uint8).reshape(H, W, 4)
    want = orc.vdi_flatten([c for c, _ in subs], [dd for _, dd in subs], W, H, 0, W, orc.ipv_of(sc["cam"]))
    assert np.array_equal(img, want)
    assert np.count_nonzero(want[..., 3]) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_harness_composited_vdi_set_two_ranks(tmp_path):
    _need_harness()
    W, H, S, S_out = 48, 40, 6, 5
    sc, scs = _scenes(W, H, 2)
    subs = [_oracle_sub(s, sc, S) for s in scs]
    _write_common(tmp_path, sc, W, H, S, S_out)
    for r, (c, dd) in enumerate(subs):
        (tmp_path / f"sub_col_{r}.bin").write_bytes(c.tobytes())
        (tmp_path / f"sub_dep_{r}.bin").write_bytes(dd.tobytes())
    _run("cvdi", tmp_path, 2)
    _check_recv(tmp_path, subs, 2)
    oc, od, _ = orc.vdi_composite([c for c, _ in subs], [dd for _, dd in subs], W, H, 0, W, orc.ipv_of(sc["cam"]), S_out)
    gc = np.fromfile(tmp_path / "gcol.bin", np.float32).reshape(oc.shape)
    gd = np.fromfile(tmp_path / "gdep.bin", np.float32).reshape(od.shape)
    assert np.array_equal(gc.view(np.uint32), oc.view(np.uint32))
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    assert np.count_nonzero(od) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_harness_plain_two_ranks(tmp_path):
    _need_harness()
    W = H = 40
    sc, scs = _scenes(W, H, 2)
    subs = []
    for s in scs:
        inp = orc.Inputs(s["vol"], s["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], sc["cam"])
        subs.append(orc.plain_raycast(inp, W, H))
    _write_common(tmp_path, sc, W, H, 1, 0)
    for r, (c, dd) in enumerate(subs):
        (tmp_path / f"sub_col_{r}.bin").write_bytes(c.tobytes())
        (tmp_path / f"sub_dep_{r}.bin").write_bytes(dd.tobytes())
    _run("plain", tmp_path, 2)
    _check_recv(tmp_path, subs, 2)
    img = np.fromfile(tmp_path / "image.bin", np.uint8).reshape(H, W, 4)
    rows = H // 2
    want = np.concatenate([orc.plain_composite([c[r * rows:(r + 1) * rows] for c, _ in subs],
                                               [dd[r * rows:(r + 1) * rows] for _, dd in subs], rows)
                           for r in range(2)], axis=0)
    assert np.array_equal(img, want)
    assert np.count_nonzero(want[..., 3]) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_harness_device_frame(tmp_path):
    """The device-resident path from C: insitu_set_brick (host u16 grid) + insitu_frame."""
    _need_harness()
    W, H, S = 48, 40, 6
    sc = make_scene(n=24, W=W, H=H, yaw=40.0)
    nz, ny, nx = sc["vol"].shape
    _write_common(tmp_path, sc, W, H, S, 0, dims=(nx, ny, nz))
    (tmp_path / "brick_0.bin").write_bytes(np.ascontiguousarray(sc["vol"], np.uint16).tobytes())
    (tmp_path / "model_0.bin").write_bytes(np.asarray(sc["model"], np.float32).tobytes())
    _run("frame", tmp_path, 1)
    img = np.fromfile(tmp_path / "image.bin", np.uint8).reshape(H, W, 4)
    c, dd = _oracle_sub(sc, sc, S)
    want = orc.vdi_flatten([c], [dd], W, H, 0, W, orc.ipv_of(sc["cam"]))
    assert np.array_equal(img, want)


def _write_kt_grid(d: Path, r: int, s, p2w: float):
    """Rank r's grid as the Kotlin host hands it over: u16 voxels, its voxel origin (the world origin
    over pixelToWorld: integers in these scenes) and inclusive extent -- updateData's arrays."""
    nz, ny, nx = s["vol"].shape
    m = np.asarray(s["model"], np.float32)
    org = np.rint(m[12:15].astype(np.float64) / p2w).astype(np.int32)
    assert np.allclose(org * p2w, m[12:15], atol=1e-7), "scene origin is not a whole number of voxels"
    (d / f"grid_{r}.bin").write_bytes(np.ascontiguousarray(s["vol"], np.uint16).tobytes())
    (d / f"origins_{r}.bin").write_bytes(org.tobytes())
    (d / f"griddims_{r}.bin").write_bytes(np.array([0, 0, 0, nx - 1, ny - 1, nz - 1], np.int32).tobytes())
    (d / f"pos_{r}.bin").write_bytes(m[12:15].tobytes())


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind,nranks", [("ktgrids", 1), ("ktgrids", 2), ("ktplain", 2), ("ktvolume", 2), ("ktpipe", 2)])
def test_harness_kotlin_device_frame(tmp_path, kind, nranks):
    """The device-resident frame with the Kotlin arguments (jni/kotlin_device_path.h: the bodies of the
    JNI externals insituUpdateData / insituUpdateVolume + insituFrame that replace the Vulkan dispatch):
    the grids go in as updateData's ByteBuffers with origins / gridDims / pixelToWorld, one call per frame
    renders, exchanges, composites and gathers; the root's image (streamImage) or gathered composited VDI
    (gatherColorPointer / gatherDepthPointer) equals the oracle's.  ktpipe: the pipelined loop
    (insituFramePipelined twice + insituFrameFlush, one frame stale): both completed frames' images."""
    _need_harness()
    W, H, S, S_out = 48, 40, 6, 5
    sc, scs = _scenes(W, H, nranks)
    p2w = float(np.float32(1.0 / 24.0))   # the scenes' voxel size (world 1, n = 24)
    nz, ny, nx = sc["vol"].shape
    plain = kind == "ktplain"
    _write_common(tmp_path, sc, W, H, 1 if plain else S, S_out if kind == "ktvolume" else 0, dims=(nx, ny, nz))
    (tmp_path / "p2w.bin").write_bytes(np.array([p2w], np.float32).tobytes())
    for r, s in enumerate(scs):
        _write_kt_grid(tmp_path, r, s, p2w)
    _run(kind, tmp_path, nranks)
    ipv = orc.ipv_of(sc["cam"])
    if kind == "ktvolume":
        subs = [_oracle_sub(s, sc, S) for s in scs]
        oc, od, _ = orc.vdi_composite([c for c, _ in subs], [dd for _, dd in subs], W, H, 0, W, ipv, S_out)
        gc = np.fromfile(tmp_path / "gcol.bin", np.float32).reshape(oc.shape)
        gd = np.fromfile(tmp_path / "gdep.bin", np.float32).reshape(od.shape)
        assert np.array_equal(gc.view(np.uint32), oc.view(np.uint32))
        assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
        assert np.count_nonzero(od) > 0
        return
    img = np.fromfile(tmp_path / "image.bin", np.uint8).reshape(H, W, 4)
    if plain:
        subs = []
        for s in scs:
            inp = orc.Inputs(s["vol"], s["im"], sc["tf"], sc["cmap"], sc["conv_k"], sc["conv_offset"], sc["cam"])
            subs.append(orc.plain_raycast(inp, W, H))
        rows = H // nranks
        want = np.concatenate([orc.plain_composite([c[r * rows:(r + 1) * rows] for c, _ in subs],
                                                   [dd[r * rows:(r + 1) * rows] for _, dd in subs], rows)
                               for r in range(nranks)], axis=0)
    else:
        subs = [_oracle_sub(s, sc, S) for s in scs]
        want = orc.vdi_flatten([c for c, _ in subs], [dd for _, dd in subs], W, H, 0, W, ipv)
    assert np.array_equal(img, want)
    assert np.count_nonzero(want[..., 3]) > 0
    if kind == "ktpipe":
        assert np.array_equal(np.fromfile(tmp_path / "image0.bin", np.uint8).reshape(H, W, 4), want)
