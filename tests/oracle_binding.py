"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) -- TEST INFRASTRUCTURE.

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  Arrays returned are in the reference texture layouts (see oracle/insitu_oracle.h).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
LIB = ORACLE_DIR / "_build" / "liboracle.so"

F16 = ctypes.c_float * 16
FP = ctypes.POINTER(ctypes.c_float)


class OrcBrick(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("dtype", ctypes.c_int), ("dims", ctypes.c_int * 3), ("im", F16)]


class OrcTransfer(ctypes.Structure):
    _fields_ = [("tf", FP), ("n_tf", ctypes.c_int), ("cmap", FP), ("n_cm", ctypes.c_int),
                ("conv_scale", ctypes.c_float), ("conv_offset", ctypes.c_float)]


class OrcCamera(ctypes.Structure):
    _fields_ = [("view", F16), ("proj", F16), ("inv_view", F16), ("inv_proj", F16),
                ("nw", ctypes.c_float), ("fwnw", ctypes.c_float), ("tmax", ctypes.c_float)]


_lib = None
_variants: dict = {}
VARIANTS = ("nofma", "libm_pow", "fixed_weights", "lut_edge")   # oracle/Makefile `variants`


def _bind(lib):
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.orc_vdi_generate.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp, vp, i, i]
    lib.orc_vdi_generate_mt.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp, vp, i]
    lib.orc_vdi_generate_cols.argtypes = [vp, vp, vp, i, i, i, i, i, vp, vp, vp, vp, i]
    lib.orc_vdi_generate_multi.argtypes = [vp, i, vp, vp, i, i, i, i, i, vp, vp, vp, vp, i]
    lib.orc_plain_raycast.argtypes = [vp, vp, vp, i, i, vp, vp, i, i]
    lib.orc_plain_composite.argtypes = [vp, vp, i, i, i, vp]
    lib.orc_vdi_flatten.argtypes = [vp, vp, i, i, i, i, i, i, vp, vp]
    lib.orc_vdi_composite.argtypes = [vp, vp, i, i, i, i, i, i, i, vp, vp, vp, vp, i]
    lib.orc_mat4_mul.argtypes = [vp, vp, vp]
    for f in ("orc_log2", "orc_exp2"):
        getattr(lib, f).restype = ctypes.c_float
        getattr(lib, f).argtypes = [ctypes.c_float]
    lib.orc_pow.restype = ctypes.c_float
    lib.orc_pow.argtypes = [ctypes.c_float, ctypes.c_float]
    lib.orc_encode_depth_rgba8.argtypes = [ctypes.c_float, vp]
    lib.orc_decode_depth_rgba8.restype = ctypes.c_float
    lib.orc_decode_depth_rgba8.argtypes = [vp]
    return lib


def _stale(path: Path) -> bool:
    deps = [ORACLE_DIR / "insitu_oracle.c", ORACLE_DIR / "insitu_oracle.h", ORACLE_DIR / "Makefile"]
    return not path.exists() or any(path.stat().st_mtime < d.stat().st_mtime for d in deps)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if _stale(LIB):
        subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    _lib = _bind(ctypes.CDLL(str(LIB)))
    return _lib


def load_variant(name: str):
    """A robustness variant of the oracle (one part of the numerical contract replaced)."""
    if name not in VARIANTS:
        raise ValueError(name)
    if name not in _variants:
        path = ORACLE_DIR / "_build" / f"liboracle_{name}.so"
        if _stale(path):
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), f"_build/liboracle_{name}.so"], check=True)
        _variants[name] = _bind(ctypes.CDLL(str(path)))
    return _variants[name]


class Inputs:
    """Keeps numpy buffers alive for the structs that point into them."""

    def __init__(self, vol: np.ndarray, im_cm: np.ndarray, tf: np.ndarray, cmap: np.ndarray, conv_k: float,
                 conv_off: float, cam):
        self.vol = np.ascontiguousarray(vol)
        dt = {np.dtype(np.uint8): 0, np.dtype(np.uint16): 1, np.dtype(np.float32): 2}[self.vol.dtype]
        self.tf = np.ascontiguousarray(tf, dtype=np.float32)
        self.cmap = np.ascontiguousarray(cmap, dtype=np.float32).reshape(-1)
        self.brick = OrcBrick(self.vol.ctypes.data, dt, (ctypes.c_int * 3)(vol.shape[2], vol.shape[1], vol.shape[0]),
                              F16(*np.asarray(im_cm, np.float32).tolist()))
        self.xfer = OrcTransfer(self.tf.ctypes.data_as(FP), self.tf.size, self.cmap.ctypes.data_as(FP),
                                self.cmap.size // 4, ctypes.c_float(conv_k), ctypes.c_float(conv_off))
        self.cam = OrcCamera(F16(*cam.view.tolist()), F16(*cam.proj.tolist()), F16(*cam.inv_view.tolist()),
                             F16(*cam.inv_proj.tolist()), ctypes.c_float(cam.nw), ctypes.c_float(cam.fwnw),
                             ctypes.c_float(cam.tmax))


def vdi_generate(inp: Inputs, W: int, H: int, S: int, threads: int = 0, lib=None):
    lib = lib or load()
    color = np.zeros((W, H, S, 4), np.float32)
    depth = np.zeros((W, H, 2 * S), np.float32)
    octree = np.zeros((S, H // 8, W // 8), np.uint32)
    passes = np.zeros((H, W), np.int32)
    rc = lib.orc_vdi_generate_mt(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                                 color.ctypes.data, depth.ctypes.data, octree.ctypes.data, passes.ctypes.data, threads)
    assert rc == 0, rc
    return color, depth, octree, passes


def vdi_generate_cols(inp: Inputs, W: int, H: int, S: int, x0: int, x1: int, threads: int = 0, lib=None):
    """Columns [x0, x1): colour (nx, H, S, 4), depth (nx, H, 2S), octree (S, H/8, W/8) with only the
    band's cells added to, passes (H, nx)."""
    lib = lib or load()
    nx = x1 - x0
    color = np.zeros((nx, H, S, 4), np.float32)
    depth = np.zeros((nx, H, 2 * S), np.float32)
    octree = np.zeros((S, H // 8, W // 8), np.uint32)
    passes = np.zeros((H, nx), np.int32)
    rc = lib.orc_vdi_generate_cols(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), W, H, S,
                                   x0, x1, color.ctypes.data, depth.ctypes.data, octree.ctypes.data,
                                   passes.ctypes.data, threads)
    assert rc == 0, rc
    return color, depth, octree, passes


def vdi_generate_multi(inps: list, W: int, H: int, S: int, x0: int = 0, x1: int | None = None, threads: int = 0,
                       lib=None):
    """All volumes of `inps` (same transfer function and camera) in ONE VDI ($repeat), columns [x0, x1):
    colour (nx, H, S, 4), depth (nx, H, 2S), octree (S, H/8, W/8), passes (H, nx)."""
    lib = lib or load()
    x1 = W if x1 is None else x1
    nx = x1 - x0
    color = np.zeros((nx, H, S, 4), np.float32)
    depth = np.zeros((nx, H, 2 * S), np.float32)
    octree = np.zeros((S, H // 8, W // 8), np.uint32)
    passes = np.zeros((H, nx), np.int32)
    bricks = (ctypes.c_void_p * len(inps))(*[ctypes.addressof(i.brick) for i in inps])
    rc = lib.orc_vdi_generate_multi(bricks, len(inps), ctypes.byref(inps[0].xfer), ctypes.byref(inps[0].cam), W, H, S,
                                    x0, x1, color.ctypes.data, depth.ctypes.data, octree.ctypes.data,
                                    passes.ctypes.data, threads)
    assert rc == 0, rc
    return color, depth, octree, passes


def plain_raycast(inp: Inputs, dim0: int, dim1: int, lib=None):
    lib = lib or load()
    color = np.zeros((dim1, dim0, 4), np.uint8)
    depth = np.zeros((dim1, dim0, 4), np.uint8)
    rc = lib.orc_plain_raycast(ctypes.byref(inp.brick), ctypes.byref(inp.xfer), ctypes.byref(inp.cam), dim0, dim1,
                               color.ctypes.data, depth.ctypes.data, 0, dim1)
    assert rc == 0, rc
    return color, depth


def plain_composite(colors: list[np.ndarray], depths: list[np.ndarray], rows: int):
    """colors/depths: per process a (dim1, dim0, 4) uint8 image; composites strip rows block `rows` of
    the stacked per-process strip blocks (the receive layout)."""
    lib = load()
    c = np.ascontiguousarray(np.concatenate(colors, axis=0))
    d = np.ascontiguousarray(np.concatenate(depths, axis=0))
    dim0 = c.shape[1]
    out = np.zeros((rows, dim0, 4), np.uint8)
    rc = lib.orc_plain_composite(c.ctypes.data, d.ctypes.data, dim0, rows, len(colors), out.ctypes.data)
    assert rc == 0, rc
    return out


def vdi_flatten(colors: list[np.ndarray], depths: list[np.ndarray], W: int, H: int, x_offset: int, strip_w: int,
                ipv: np.ndarray, arrays_x0: int = 0, lib=None):
    """colors[j]: (W_any, H, S, 4) reference layout whose row 0 is column arrays_x0, sliced to the strip
    columns [x_offset, x_offset + strip_w); returns (H, strip_w, 4)."""
    lib = lib or load()
    V = len(colors)
    S = colors[0].shape[2]
    a = x_offset - arrays_x0
    cs = [np.ascontiguousarray(c[a:a + strip_w], dtype=np.float32) for c in colors]
    ds = [np.ascontiguousarray(d[a:a + strip_w], dtype=np.float32) for d in depths]
    cptr = (ctypes.c_void_p * V)(*[c.ctypes.data for c in cs])
    dptr = (ctypes.c_void_p * V)(*[d.ctypes.data for d in ds])
    out = np.zeros((H, strip_w, 4), np.uint8)
    ipv32 = np.ascontiguousarray(ipv, dtype=np.float32)
    rc = lib.orc_vdi_flatten(cptr, dptr, V, S, H, W, strip_w, x_offset, ipv32.ctypes.data, out.ctypes.data)
    assert rc == 0, rc
    return out


def vdi_composite(colors: list[np.ndarray], depths: list[np.ndarray], W: int, H: int, x_offset: int, strip_w: int,
                  ipv: np.ndarray, S_out: int, faithful: bool = False, arrays_x0: int = 0):
    """VDICompositor.comp over the strip; inputs as vdi_flatten (row 0 of the arrays is column arrays_x0).
    Returns (colour (strip_w, H, S_out, 4), depth (strip_w, H, 2*S_out), passes (H, strip_w)) in the
    reference layout."""
    lib = load()
    V = len(colors)
    S = colors[0].shape[2]
    a = x_offset - arrays_x0
    cs = [np.ascontiguousarray(c[a:a + strip_w], dtype=np.float32) for c in colors]
    ds = [np.ascontiguousarray(d[a:a + strip_w], dtype=np.float32) for d in depths]
    cptr = (ctypes.c_void_p * V)(*[c.ctypes.data for c in cs])
    dptr = (ctypes.c_void_p * V)(*[d.ctypes.data for d in ds])
    oc = np.zeros((strip_w, H, S_out, 4), np.float32)
    od = np.zeros((strip_w, H, 2 * S_out), np.float32)
    op = np.zeros((H, strip_w), np.int32)
    ipv32 = np.ascontiguousarray(ipv, dtype=np.float32)
    rc = lib.orc_vdi_composite(cptr, dptr, V, S, S_out, H, W, strip_w, x_offset, ipv32.ctypes.data, oc.ctypes.data,
                               od.ctypes.data, op.ctypes.data, 1 if faithful else 0)
    assert rc == 0, rc
    return oc, od, op


def mat4_mul(a: np.ndarray, b: np.ndarray, lib=None) -> np.ndarray:
    lib = lib or load()
    a32, b32 = np.ascontiguousarray(a, np.float32), np.ascontiguousarray(b, np.float32)
    out = np.zeros(16, np.float32)
    lib.orc_mat4_mul(a32.ctypes.data, b32.ctypes.data, out.ctypes.data)
    return out


def ipv_of(cam, lib=None) -> np.ndarray:
    return mat4_mul(cam.inv_view, cam.inv_proj, lib)
