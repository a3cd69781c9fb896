"""C-ABI checks that need no GPU: the library loads, exports every symbol include/insitu_hip.h
declares, the ctypes structs match the C layouts, and creation fails cleanly (no crash, a
message) when no device is present."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from insitu_amd import native

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "insitu_hip.h"


def _declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(insitu_\w+)\s*\(", text, re.M)))


def test_header_declarations_match_binding():
    assert sorted(native.EXPORTED_SYMBOLS) == _declared()


def test_library_exports_every_declared_symbol():
    lib = native.load()
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing
    out = subprocess.run(["nm", "-D", "--defined-only", str(native.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (insitu_\w+)", out))
    assert set(_declared()) <= exported
    assert lib.insitu_abi_version() == native.ABI_VERSION


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "insitu_hip.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(insitu_config), offsetof(insitu_config, comm_id),
         offsetof(insitu_config, keep_passes), offsetof(insitu_config, sample_cache_mb), sizeof(insitu_camera),
         offsetof(insitu_camera, nw), sizeof(insitu_stats));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(native.Config), native.Config.comm_id.offset, native.Config.keep_passes.offset,
            native.Config.sample_cache_mb.offset, ctypes.sizeof(native.Camera), native.Camera.nw.offset,
            ctypes.sizeof(native.Stats)]
    assert got == want


def test_enum_values_match_binding():
    """Every INSITU_OPT_* / INSITU_BUF_* / INSITU_MODE_* / voxel-type value of the header has its native.py
    constant with the same value (a binding constant that drifted would set or read the wrong thing without an
    error)."""
    text = HEADER.read_text()
    pairs = re.findall(r"\bINSITU_((?:OPT|BUF|MODE)_\w+|U8|U16|F32)\s*=\s*(\d+)", text)
    assert len(pairs) >= 31
    for name, value in pairs:
        assert getattr(native, name) == int(value), name


def test_header_compiles_as_c_and_cpp(tmp_path):
    for comp, ext in (("gcc", "c"), ("g++", "cpp")):
        src = tmp_path / f"t.{ext}"
        src.write_text('#include "insitu_hip.h"\nint main(void){return INSITU_ABI_VERSION - 1;}\n')
        subprocess.run([comp, "-Wall", "-Werror", "-I", str(ROOT / "include"), str(src), "-o", str(tmp_path / "t")],
                       check=True)


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = native.load()
    cfg = native.Config(rank=0, nranks=1, device=0, width=64, height=48, max_supersegments=8,
                        mode=native.MODE_VDI, bricks_per_rank=1)
    h = ctypes.c_void_p()
    rc = lib.insitu_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc < 0 and not h.value
    assert b"device" in lib.insitu_last_error(None).lower()


@pytest.mark.parametrize("field,value,msg", [
    ("nranks", 0, b"rank"), ("width", 0, b"window"), ("mode", 7, b"mode"),
    ("max_supersegments", 0, b"max_supersegments"), ("bricks_per_rank", 0, b"bricks_per_rank"),
])
def test_create_rejects_bad_config(field, value, msg):
    lib = native.load()
    cfg = native.Config(rank=0, nranks=1, device=0, width=64, height=48, max_supersegments=8,
                        mode=native.MODE_VDI, bricks_per_rank=1)
    setattr(cfg, field, value)
    h = ctypes.c_void_p()
    assert lib.insitu_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    assert msg in lib.insitu_last_error(None)


def test_create_rejects_uneven_strips_and_missing_comm_id():
    lib = native.load()
    cfg = native.Config(rank=0, nranks=3, device=0, width=64, height=48, max_supersegments=8,
                        mode=native.MODE_VDI, bricks_per_rank=1)
    h = ctypes.c_void_p()
    assert lib.insitu_create(ctypes.byref(cfg), ctypes.byref(h)) == -1   # 64 % 3 != 0
    cfg.nranks = 2
    assert lib.insitu_create(ctypes.byref(cfg), ctypes.byref(h)) == -1   # no comm_id
    assert b"comm_id" in lib.insitu_last_error(None)


def test_null_context_calls_fail():
    lib = native.load()
    assert lib.insitu_render(None, None) == -1
    assert lib.insitu_exchange(None) == -1
    assert lib.insitu_composite(None) == -1
    assert lib.insitu_gather(None, None, 0) == -1
    assert lib.insitu_buffer_bytes(None, 0) == 0
    done = ctypes.c_longlong(7)
    assert lib.insitu_frame_pipelined(None, None, None, 0, ctypes.byref(done)) == -1
    assert lib.insitu_pipeline_flush(None, None, 0, ctypes.byref(done)) == -1


def test_gather_out_validation():
    """gather(out=...) writes raw rgba8 through a host copy: only a C-contiguous uint8 (H, W, 4) CPU
    array or tensor is accepted."""
    import torch
    from insitu_amd.renderer import _check_image_out
    H, W = 6, 10
    _check_image_out(np.zeros((H, W, 4), np.uint8), H, W)
    _check_image_out(torch.zeros((H, W, 4), dtype=torch.uint8), H, W)
    bad = [np.zeros((H, W, 4), np.float32), np.zeros((W, H, 4), np.uint8), np.zeros((H, 2 * W, 4), np.uint8)[:, ::2],
           np.zeros(H * W * 4, np.uint8), torch.zeros((H, W, 4), dtype=torch.int32),
           torch.zeros((H, 2 * W, 4), dtype=torch.uint8)[:, ::2]]
    for b in bad:
        with pytest.raises(ValueError):
            _check_image_out(b, H, W)
