"""VDI dump files (insitu_amd/vdi_io.py): names and byte layout of the
reference's SystemHelpers.dumpToFile dumps, metadata round trip."""
from __future__ import annotations

import numpy as np

from insitu_amd import scene, vdi_io


def test_dump_names_and_round_trip(tmp_path):
    W, H, S = 6, 5, 3
    rng = np.random.default_rng(2)
    col = rng.random((W, H, S, 4), dtype=np.float32)
    dep = rng.random((W, H, 2 * S), dtype=np.float32)
    base = str(tmp_path) + "/"
    cp, dp = vdi_io.write_vdi(base, "Kingsnake", "SubVDI", 7, col, dep)
    assert cp.name == "KingsnakeSubVDI7_ndc_col" and dp.name == "KingsnakeSubVDI7_ndc_depth"
    assert cp.stat().st_size == W * H * S * 16 and dp.stat().st_size == W * H * S * 8
    c2, d2 = vdi_io.read_vdi(cp, dp, W, H, S)
    assert np.array_equal(c2, col) and np.array_equal(d2, dep)
    # byte layout of the reference image3D (S, H, W): supersegment fastest, then y, then x
    raw = np.fromfile(cp, dtype=np.float32)
    x, y, i = 4, 2, 1
    assert np.array_equal(raw[((x * H + y) * S + i) * 4:((x * H + y) * S + i) * 4 + 4], col[x, y, i])
    rawd = np.fromfile(dp, dtype=np.float32)
    assert rawd[(x * H + y) * 2 * S + 2 * i + 1] == dep[x, y, 2 * i + 1]


def test_read_rejects_wrong_size(tmp_path):
    col = np.zeros((2, 2, 2, 4), np.float32)
    dep = np.zeros((2, 2, 4), np.float32)
    cp, dp = vdi_io.write_vdi(str(tmp_path) + "/", "", "CompositedVDI", 0, col, dep)
    try:
        vdi_io.read_vdi(cp, dp, 2, 2, 3)
    except ValueError:
        return
    raise AssertionError("size mismatch not detected")


def test_metadata_round_trip(tmp_path):
    W, H, S = 64, 48, 20
    cam = scene.orbit_camera(W, H, yaw_deg=30.0)
    model = scene.brick_model((-0.5, -0.5, -0.5), 1.0 / 32)
    p = vdi_io.write_metadata(str(tmp_path) + "/", "ds", W, H, S, 3, cam, model, (32, 32, 32))
    assert p.name == "dsvdi_64_48_20_0_dump3"
    m = vdi_io.read_metadata(p)
    assert m["windowDimensions"] == [W, H] and m["maxSupersegments"] == S
    assert np.allclose(m["view"], cam.view) and np.allclose(m["projection_vulkan"], cam.proj)
    # projection is stored without the Vulkan fix (the consumer applies it, DistributedVolumes.kt:721)
    fixed = scene.VULKAN_FIX @ np.asarray(m["projection"], np.float64).reshape(4, 4).T
    assert np.allclose(scene.col_major(fixed), cam.proj, atol=1e-6)
    assert np.isclose(m["nw"], float(cam.nw))
