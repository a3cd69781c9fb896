"""Parity robustness study (CPU only): how far do the outputs move when one part of the numerical
contract is replaced by another plausible implementation of the same GLSL?

The reference runs its shaders through Vulkan drivers whose fma contraction, pow() and texture-unit
filtering are implementation-defined; the build's contract fixes one choice for each.  Every
variant of oracle/Makefile `variants` replaces one choice (oracle/insitu_oracle.c header):
  nofma          no contraction (every * and + of the shader expressions rounded apart)
  libm_pow       pow() from the C library instead of exp2(y*log2(x)) with fixed polynomials
  fixed_weights  texture-unit filtering: trilinear and LUT weights rounded to 8 fraction bits
  lut_edge       LUT lookups without the texel-centre shift
and the study compares its sub-VDIs and flattened image with the contract's:
  count-match rate (pixels hit by the volume whose supersegment count agrees), depth deviation on
  count-matching pixels, and the flattened RGBA image: max |dRGBA| (8-bit units), the share of
  pixels within 1/255, and PSNR over the pixels the volume covers.
Workloads: config 1 (128^3 Gray-Scott u16, 1280x720, S = 20, whole frame) and a config-2 band
(8 x 512^3 fp32 bricks, 1920x1080, S = 20, columns [928, 992), all bricks + their flatten).

usage: python tools/parity_robustness.py [--threads N] [--out profiles/r02_parity_robustness.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "scenery-insitu_amd"), str(ROOT / "tests"), str(ROOT)]

import numpy as np  # noqa: E402

import oracle_binding as orc  # noqa: E402


def compare(ref_subs, var_subs, ref_img, var_img):
    """ref_subs/var_subs: list of (colour, depth) per brick in the reference layout (nx, H, S, 4)/(nx, H, 2S)."""
    hit = match = 0
    dmax = 0.0
    depth_ok = 0
    for (rc, rd), (vc, vd) in zip(ref_subs, var_subs):
        nr = np.count_nonzero(rd[..., 0::2], axis=2)
        nv = np.count_nonzero(vd[..., 0::2], axis=2)
        h = (nr > 0) | (nv > 0)
        m = h & (nr == nv)
        hit += int(h.sum())
        match += int(m.sum())
        if m.any():
            dd = np.abs(rd[m].astype(np.float64) - vd[m].astype(np.float64)).max(axis=1)
            dmax = max(dmax, float(dd.max()))
            depth_ok += int((dd <= 1e-4).sum())
    a = ref_img.astype(np.int32)
    b = var_img.astype(np.int32)
    diff = np.abs(a - b).max(axis=2)
    cover = (a[..., 3] > 0) | (b[..., 3] > 0)
    mse = float(np.mean(((a[cover] - b[cover]) / 255.0) ** 2)) if cover.any() else 0.0
    return {
        "pixels_hit": hit,
        "count_match_rate": match / hit if hit else 1.0,
        "depth_max_abs_on_matching": dmax,
        "depth_within_1e-4_rate": depth_ok / match if match else 1.0,
        "rgba_max_abs_8bit": int(diff.max()),
        "rgba_within_1_rate": float((diff[cover] <= 1).mean()) if cover.any() else 1.0,
        "psnr_db_covered": (float("inf") if mse == 0.0 else 10.0 * np.log10(1.0 / mse)),
        "pixels_covered": int(cover.sum()),
    }


def config1(threads):
    from scenes import make_scene
    sc = make_scene(n=128, W=1280, H=720, yaw=35.0, origin=(-1.0, -1.0, -1.0), world=2.0)
    W, H, S = 1280, 720, 20
    inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])

    def run(lib):
        c, d, _, _ = orc.vdi_generate_cols(inp, W, H, S, 0, W, threads, lib=lib)
        img = orc.vdi_flatten([c], [d], W, H, 0, W, orc.ipv_of(sc["cam"], lib), lib=lib)
        return [(c, d)], img
    return run


def config2_band(threads, x0=928, x1=992):
    import torch

    import bench
    from insitu_amd import native, scene
    W, H, S, n = 1920, 1080, 20, 512
    units = scene.grid_bricks(2 * n, 2)
    vols = [bench.make_brick(b, n, torch.device("cpu")).numpy() for b in range(len(units))]
    cam = scene.orbit_camera(W, H, yaw_deg=30.0, pitch_deg=20.0, voxel_world=units[0][1])
    tf, cmap = scene.transfer_function(), scene.colormap_hot()
    k = scene.folded_conv_scale(2.0, native.F32)
    inps = [orc.Inputs(v, scene.inverse_model(scene.brick_model(o, vw)), tf, cmap, k, 0.0, cam)
            for v, (o, vw, _) in zip(vols, units)]

    def run(lib):
        subs = []
        for inp in inps:
            c, d, _, _ = orc.vdi_generate_cols(inp, W, H, S, x0, x1, threads, lib=lib)
            subs.append((c, d))
        img = orc.vdi_flatten([c for c, _ in subs], [d for _, d in subs], W, H, x0, x1 - x0,
                              orc.ipv_of(cam, lib), arrays_x0=x0, lib=lib)
        return subs, img
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r02_parity_robustness.json"))
    ap.add_argument("--skip-config2", action="store_true")
    args = ap.parse_args()
    result = {}
    workloads = [("config1_1280x720_full", config1(args.threads))]
    if not args.skip_config2:
        workloads.append(("config2_band_928_992_8_bricks", config2_band(args.threads)))
    for name, run in workloads:
        t = time.time()
        ref_subs, ref_img = run(orc.load())
        result[name] = {}
        for v in orc.VARIANTS:
            subs, img = run(orc.load_variant(v))
            result[name][v] = compare(ref_subs, subs, ref_img, img)
            print(name, v, json.dumps(result[name][v]), flush=True)
        result[name]["_seconds"] = round(time.time() - t, 1)
    Path(args.out).write_text(json.dumps(result, indent=1) + "\n")
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
