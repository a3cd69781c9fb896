"""On-disk VDI dumps in the reference's formats.

The reference dumps raw texture bytes with `SystemHelpers.dumpToFile(buffer, path)`:
  sub-VDIs       `{basePath}{dataset}SubVDI{n}_ndc_col` / `_ndc_depth`         DistributedVolumes.kt:848-849
  received sets  `{basePath}{dataset}SetOfVDI{n}_ndc_col` / `_ndc_depth`       DistributedVolumes.kt:974-975
  composited     `{basePath}{dataset}CompositedVDI{n}_ndc_col` / `_ndc_depth`  DistributedVolumes.kt:894-895
Colour is the rgba32f image3D (S, H, W) -- supersegment fastest, then y, then x -- and depth the r32f
image3D (2S, H, W) (DistributedVolumes.kt:349-368), which is exactly the byte order of the
(W, H, S, 4) / (W, H, 2S) float32 arrays `InSituContext.read` returns.

The octree grid (OctreeCells, r32ui (W/8, H/8, S), x fastest) is dumped next to a VDI as
`{fileName}_octree` (VolumeFromFileExample.kt:1061-1071, fileName
`{dataset}VDI_{W}_{H}_{S}_{vo}_{cnt}_ndc` or `..._world_new`): `volume_file_paths` / `write_octree`.

The frame metadata (`VDIDataIO.write(VDIData(VDIBufferSizes(), VDIMetadata(index, projection, view,
volumeDimensions, model, nw, windowDimensions)))`, DistributedVolumes.kt:706-716, 910-915;
VDIConverter.kt:243-257) is written by scenery's serializer, which is a dependency outside the
reference tree and absent here, so its byte format cannot be reproduced or checked (parity unpinned).
The constructor arguments are written instead, under the reference's file name
`{basePath}{dataset}vdi_{W}_{H}_{S}_0_dump{n}`, as JSON with the VDIMetadata parameter names;
INTEGRATION.md shows the few Kotlin lines that turn it into a VDIDataIO file with scenery on the
classpath.  Matrices are column-major float lists (JOML order); `projection` is the OpenGL projection
as the reference stores it (the Vulkan fix is applied by the consumer, DistributedVolumes.kt:721),
`projection_vulkan` the corrected one the kernels use.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

KINDS = ("SubVDI", "SetOfVDI", "CompositedVDI")


def vdi_paths(base_path: str | Path, dataset: str, kind: str, counter: int) -> tuple[Path, Path]:
    if kind not in KINDS:
        raise ValueError(f"kind must be one of {KINDS}")
    stem = f"{base_path}{dataset}{kind}{counter}_ndc"
    return Path(stem + "_col"), Path(stem + "_depth")


def dump_to_file(array: np.ndarray, path: str | Path) -> None:
    """SystemHelpers.dumpToFile: the buffer's bytes, nothing else."""
    with open(path, "wb") as f:
        f.write(np.ascontiguousarray(array).tobytes())


def write_vdi(base_path: str | Path, dataset: str, kind: str, counter: int, colour: np.ndarray,
              depth: np.ndarray) -> tuple[Path, Path]:
    colour = np.asarray(colour, dtype=np.float32)
    depth = np.asarray(depth, dtype=np.float32)
    if colour.ndim != 4 or colour.shape[3] != 4 or depth.shape != colour.shape[:2] + (2 * colour.shape[2],):
        raise ValueError("expected colour (W, H, S, 4) and depth (W, H, 2S) float32")
    cp, dp = vdi_paths(base_path, dataset, kind, counter)
    dump_to_file(colour, cp)
    dump_to_file(depth, dp)
    return cp, dp


def read_vdi(colour_path: str | Path, depth_path: str | Path, width: int, height: int,
             supersegments: int) -> tuple[np.ndarray, np.ndarray]:
    """Raw dump -> ((W, H, S, 4), (W, H, 2S)) float32; the file sizes must match exactly."""
    n = width * height * supersegments
    c = np.fromfile(colour_path, dtype=np.float32)
    d = np.fromfile(depth_path, dtype=np.float32)
    if c.size != 4 * n or d.size != 2 * n:
        raise ValueError(f"dump sizes {c.size}, {d.size} floats do not match {width}x{height}x{supersegments}")
    return c.reshape(width, height, supersegments, 4), d.reshape(width, height, 2 * supersegments)


def volume_file_paths(dataset: str, width: int, height: int, supersegments: int, vo: int, counter: int,
                      world_abs: bool = False, base_path: str | Path = "") -> tuple[Path, Path, Path]:
    """VolumeFromFileExample.kt:1056-1071: (colour, depth, octree) dump paths of a stored VDI."""
    suffix = "world_new" if world_abs else "ndc"
    stem = f"{base_path}{dataset}VDI_{width}_{height}_{supersegments}_{vo}_{counter}_{suffix}"
    return Path(stem + "_col"), Path(stem + "_depth"), Path(stem + "_octree")


def write_octree(path: str | Path, octree: np.ndarray) -> Path:
    """gridCellsBuff: the (S, H/8, W/8) uint32 cell counts (x fastest), raw."""
    octree = np.asarray(octree)
    if octree.dtype != np.uint32 or octree.ndim != 3:
        raise ValueError("expected a (S, H/8, W/8) uint32 octree grid")
    dump_to_file(octree, path)
    return Path(path)


def read_octree(path: str | Path, width: int, height: int, supersegments: int) -> np.ndarray:
    o = np.fromfile(path, dtype=np.uint32)
    if o.size != supersegments * (height // 8) * (width // 8):
        raise ValueError(f"octree dump has {o.size} cells, expected {supersegments}x{height // 8}x{width // 8}")
    return o.reshape(supersegments, height // 8, width // 8)


def write_received_set(base_path: str | Path, dataset: str, counter: int, colour: np.ndarray,
                       depth: np.ndarray) -> tuple[Path, Path]:
    """SetOfVDI{n}_ndc_col / _ndc_depth (DistributedVolumes.kt:974-975): the received blocks,
    source-major, each (W/P, H, S) -- (V, W/P, H, S, 4) / (V, W/P, H, 2S) float32."""
    colour = np.asarray(colour, dtype=np.float32)
    depth = np.asarray(depth, dtype=np.float32)
    if colour.ndim != 5 or depth.shape != colour.shape[:3] + (2 * colour.shape[3],):
        raise ValueError("expected colour (V, W/P, H, S, 4) and depth (V, W/P, H, 2S) float32")
    cp, dp = vdi_paths(base_path, dataset, "SetOfVDI", counter)
    dump_to_file(colour, cp)
    dump_to_file(depth, dp)
    return cp, dp


def metadata_path(base_path: str | Path, dataset: str, width: int, height: int, supersegments: int,
                  counter: int) -> Path:
    return Path(f"{base_path}{dataset}vdi_{width}_{height}_{supersegments}_0_dump{counter}")


def write_metadata(base_path: str | Path, dataset: str, width: int, height: int, supersegments: int, counter: int,
                   cam, model: np.ndarray, volume_dims, nw: float | None = None) -> Path:
    """VDIMetadata fields of one frame (DistributedVolumes.kt:706-716) as JSON."""
    from .scene import VULKAN_FIX, col_major
    proj_gl = np.linalg.inv(VULKAN_FIX) @ cam.proj_rm
    meta = {
        "format": "scenery-insitu_amd VDIMetadata v2 (constructor arguments of graphics.scenery.volumes.vdi."
                  "VDIData(VDIBufferSizes(), VDIMetadata(...)))",
        "index": int(counter),
        "projection": col_major(proj_gl).tolist(),
        "projection_vulkan": np.asarray(cam.proj, np.float32).tolist(),
        "view": np.asarray(cam.view, np.float32).tolist(),
        "model": np.asarray(model, np.float32).reshape(16).tolist(),
        "volumeDimensions": [float(v) for v in volume_dims],
        "nw": float(cam.nw if nw is None else nw),
        "windowDimensions": [int(width), int(height)],
        "maxSupersegments": int(supersegments),
        "layout": {"colour": "rgba32f image3D (S, H, W), x = supersegment fastest",
                   "depth": "r32f image3D (2S, H, W): start, end per supersegment (NDC z)"},
    }
    p = metadata_path(base_path, dataset, width, height, supersegments, counter)
    p.write_text(json.dumps(meta, indent=1))
    return p


def read_metadata(path: str | Path) -> dict:
    return json.loads(Path(path).read_text())
