"""ctypes binding of libinsitu_hip.so (include/insitu_hip.h).

The library is the product: HIP kernels for gfx950 + RCCL.  This module only declares the
C signatures.  It never falls back to anything else: if the shared object is missing or a
call fails, a RuntimeError is raised.

torch is imported before the library is loaded on purpose: torch ships its own
libamdhip64.so.7 / librccl.so.1, and loading those first makes libinsitu_hip.so bind to the
same HIP runtime (same SONAMEs), so device pointers and streams are shared with torch.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

try:  # noqa: SIM105 - ordering matters, see module docstring
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("INSITU_HIP_LIB", PKG_ROOT / "lib" / "libinsitu_hip.so"))

ABI_VERSION = 8
COMM_ID_BYTES = 128

MODE_PLAIN, MODE_VDI = 0, 1
FAITHFUL_COMPOSITOR_NDC_X, FAITHFUL_PLAIN_NUM_PROCESSES = 1, 2   # enum insitu_faithful
U8, U16, F32 = 0, 1, 2
BUF_VDI_COLOR, BUF_VDI_DEPTH, BUF_OCTREE, BUF_PASSES = 0, 1, 2, 3
BUF_PLAIN_COLOR, BUF_PLAIN_DEPTH, BUF_STRIP, BUF_IMAGE = 4, 5, 6, 7
BUF_COMPOSITED_COLOR, BUF_COMPOSITED_DEPTH, BUF_GATHERED_COLOR, BUF_GATHERED_DEPTH, BUF_COMPOSITE_PASSES = 8, 9, 10, 11, 12
BUF_RECEIVED_COLOR, BUF_RECEIVED_DEPTH = 13, 14

# every symbol include/insitu_hip.h declares (tests check the .so exports all of them)
EXPORTED_SYMBOLS = (
    "insitu_abi_version", "insitu_comm_id", "insitu_create", "insitu_destroy", "insitu_last_error",
    "insitu_set_brick", "insitu_set_transfer", "insitu_set_camera", "insitu_render", "insitu_exchange", "insitu_composite",
    "insitu_gather", "insitu_frame", "insitu_synchronize", "insitu_read", "insitu_buffer_bytes",
    "insitu_get_stats", "insitu_pass_stats", "insitu_stream", "insitu_distribute_vdis", "insitu_gather_composited_vdis",
    "insitu_gather_composited_vdi_set", "insitu_local_group_create", "insitu_local_group_destroy",
    "insitu_set_option", "insitu_read_region", "insitu_frame_pipelined", "insitu_pipeline_flush",
)

# enum insitu_option
OPT_EXACT_SEARCH, OPT_SEARCH_DEPTH, OPT_LONG_SAMPLES, OPT_ROUND_BATCH, OPT_SEARCH_OVERSUB, OPT_TILE_ORDER = range(6)
OPT_SUPER_TILE, OPT_REGROUP, OPT_EXACT_TILE_KEYS, OPT_PIPE_TRIGGER, OPT_PIPE_OVERSUB, OPT_PIPE_SEARCH_RAYS = 8, 9, 10, 11, 12, 13

F16 = ctypes.c_float * 16


class Config(ctypes.Structure):
    _fields_ = [
        ("rank", ctypes.c_int), ("nranks", ctypes.c_int), ("device", ctypes.c_int),
        ("width", ctypes.c_int), ("height", ctypes.c_int), ("max_supersegments", ctypes.c_int),
        ("mode", ctypes.c_int), ("bricks_per_rank", ctypes.c_int), ("comm_id", ctypes.c_void_p),
        ("stream", ctypes.c_void_p), ("keep_passes", ctypes.c_int), ("sample_cache_mb", ctypes.c_int),
        ("composite_vdi", ctypes.c_int), ("max_output_supersegments", ctypes.c_int),
        ("local_group", ctypes.c_void_p), ("faithful", ctypes.c_int), ("merge_bricks", ctypes.c_int),
    ]


class Camera(ctypes.Structure):
    _fields_ = [
        ("view", F16), ("proj", F16), ("inv_view", F16), ("inv_proj", F16),
        ("has_inverses", ctypes.c_int), ("nw", ctypes.c_float), ("fwnw", ctypes.c_float),
        ("tmax", ctypes.c_float),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("ms_render", ctypes.c_float), ("ms_exchange", ctypes.c_float),
        ("ms_composite", ctypes.c_float), ("ms_gather", ctypes.c_float),
        ("ms_sample", ctypes.c_float), ("ms_search", ctypes.c_float),
        ("rays_searched", ctypes.c_longlong),
        ("rays_uncached", ctypes.c_longlong), ("cache_bytes", ctypes.c_longlong),
        ("exchange_bytes", ctypes.c_longlong), ("exchange_entries", ctypes.c_longlong),
        ("ms_compact", ctypes.c_float), ("ms_exchange_sync", ctypes.c_float),
        ("cache_demand_bytes", ctypes.c_longlong), ("search_regroups", ctypes.c_int),
        ("ms_image_d2h", ctypes.c_float), ("ms_latency", ctypes.c_float), ("pipelined", ctypes.c_int),
        ("ms_ingest", ctypes.c_float),
    ]


_lib = None


def load() -> ctypes.CDLL:
    """Load libinsitu_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} not found: build it with `make -C scenery-insitu_amd` "
                           "(or __graft_entry__.build())")
    lib = ctypes.CDLL(str(LIB_PATH))
    vp, i, sz, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_longlong
    sig = {
        "insitu_abi_version": (i, []),
        "insitu_comm_id": (i, [vp, sz]),
        "insitu_create": (i, [ctypes.POINTER(Config), ctypes.POINTER(vp)]),
        "insitu_destroy": (None, [vp]),
        "insitu_last_error": (ctypes.c_char_p, [vp]),
        "insitu_set_brick": (i, [vp, i, vp, i, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float), i]),
        "insitu_set_transfer": (i, [vp, ctypes.POINTER(ctypes.c_float), i, ctypes.POINTER(ctypes.c_float), i,
                                    ctypes.c_float, ctypes.c_float]),
        "insitu_set_camera": (i, [vp, ctypes.POINTER(Camera)]),
        "insitu_render": (i, [vp, ctypes.POINTER(Camera)]),
        "insitu_exchange": (i, [vp]),
        "insitu_composite": (i, [vp]),
        "insitu_gather": (i, [vp, vp, sz]),
        "insitu_frame": (i, [vp, ctypes.POINTER(Camera), vp, sz]),
        "insitu_synchronize": (i, [vp]),
        "insitu_read": (i, [vp, i, i, vp, sz]),
        "insitu_buffer_bytes": (sz, [vp, i]),
        "insitu_get_stats": (i, [vp, ctypes.POINTER(Stats)]),
        "insitu_pass_stats": (i, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)]),
        "insitu_stream": (vp, [vp]),
        "insitu_distribute_vdis": (i, [vp, vp, vp, ll, i, vp, vp]),
        "insitu_gather_composited_vdis": (i, [vp, i, ll, i, i, vp, sz]),
        "insitu_gather_composited_vdi_set": (i, [vp, ll, i, i, i, vp, vp]),
        "insitu_local_group_create": (i, [i, ctypes.POINTER(vp)]),
        "insitu_local_group_destroy": (None, [vp]),
        "insitu_set_option": (i, [vp, i, ll]),
        "insitu_read_region": (i, [vp, i, i, i, i, vp, sz]),
        "insitu_frame_pipelined": (i, [vp, ctypes.POINTER(Camera), vp, sz, ctypes.POINTER(ll)]),
        "insitu_pipeline_flush": (i, [vp, vp, sz, ctypes.POINTER(ll)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.insitu_abi_version() != ABI_VERSION:
        raise RuntimeError("libinsitu_hip.so ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int, ctx=None, what: str = "insitu call") -> None:
    if rc != 0:
        msg = load().insitu_last_error(ctx)
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else '?'}")
