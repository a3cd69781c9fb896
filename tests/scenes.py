"""Small deterministic scenes shared by the CPU and GPU tests (test infrastructure)."""
from __future__ import annotations

import numpy as np

from insitu_amd import native, scene


_CACHE: dict = {}


def gray_scott_u16(n: int = 32, steps: int = 1500, seed: int = 1000) -> np.ndarray:
    key = (n, steps, seed)
    if key not in _CACHE:
        _CACHE[key] = scene.to_uint16(scene.gray_scott(n, steps=steps, seed=seed), vmax=0.5)
    return _CACHE[key]


def make_scene(n=32, W=64, H=48, yaw=30.0, pitch=20.0, samples_per_voxel=1.0, dtype="u16", seed=1000,
               origin=(-0.5, -0.5, -0.5), world=1.0, steps=1500, conv_scale=1.0, conv_offset=0.0):
    """One brick of edge `world` centred at the origin, camera orbiting at radius 3.5."""
    vol16 = gray_scott_u16(n, steps=steps, seed=seed)
    if dtype == "u16":
        vol, dt = vol16, native.U16
    elif dtype == "u8":
        vol, dt = (vol16 >> 8).astype(np.uint8), native.U8
    else:
        vol, dt = (vol16.astype(np.float32) / np.float32(65535.0) * np.float32(0.5)), native.F32
    vw = world / n
    model = scene.brick_model(origin, vw)
    im = scene.inverse_model(model)
    cam = scene.orbit_camera(W, H, yaw_deg=yaw, pitch_deg=pitch, voxel_world=vw,
                             samples_per_voxel=samples_per_voxel)
    tf = scene.transfer_function()
    cmap = scene.colormap_hot()
    conv_k = scene.folded_conv_scale(conv_scale, dt)
    return dict(vol=vol, dtype=dt, model=model, im=im, cam=cam, tf=tf, cmap=cmap, conv_scale=conv_scale,
                conv_offset=conv_offset, conv_k=conv_k, W=W, H=H)
