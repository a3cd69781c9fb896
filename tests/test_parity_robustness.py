"""How robust is parity to the parts of GLSL the reference leaves to the driver? (CPU only)

The oracle and the HIP kernels share one numerical contract: fma contraction
as written, pow = exp2(y*log2(x)) with fixed polynomials, software trilinear with exact weights,
LUT lookups at texel centres.  A Vulkan driver may choose differently on each point.  The oracle
variants of oracle/Makefile `variants` each replace one choice; this test renders the same scene
with the contract and with each variant and checks the north-star tolerances on the difference:

* HOLDS for the library pow, 8-bit filter weights and edge-aligned LUTs: the flattened RGBA image
  within 1/255 per channel on every covered pixel, PSNR >= 50 dB.
* HOLDS ALMOST EVERYWHERE without contraction: PSNR >= 50 dB, but a few pixels exceed 1/255 (here
  0.1 % of the covered pixels, up to 3/255; config 1 at full size: 1 pixel in 3e5 at 2/255).
* DOES NOT HOLD: identical supersegment lists.  The threshold search is discontinuous (SURVEY.md
  7.3): a 1-ulp change can flip a termination, so supersegment counts differ on up to ~13 % of the
  pixels (LUT without the texel-centre shift) and, where counts agree, depth boundaries can move by
  more than 1e-4.  The test records the rates and only bounds them loosely.
Full-size numbers (config 1 whole frame, config-2 band): tools/parity_robustness.py ->
profiles/r02_parity_robustness.json, tabulated in DESIGN.md section 2.1.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_binding as orc
from scenes import make_scene

W, H, S = 160, 120, 20


@pytest.fixture(scope="module")
def contract():
    sc = make_scene(n=48, W=W, H=H, yaw=35.0, pitch=25.0)
    inp = orc.Inputs(sc["vol"], sc["im"], sc["tf"], sc["cmap"], sc["conv_k"], 0.0, sc["cam"])
    c, d, _, _ = orc.vdi_generate(inp, W, H, S)
    img = orc.vdi_flatten([c], [d], W, H, 0, W, orc.ipv_of(sc["cam"]))
    return sc, inp, c, d, img


@pytest.mark.parametrize("variant", orc.VARIANTS)
def test_variant_within_north_star_rgba_tolerance(contract, variant):
    sc, inp, c0, d0, img0 = contract
    lib = orc.load_variant(variant)
    c1, d1, _, _ = orc.vdi_generate(inp, W, H, S, lib=lib)
    img1 = orc.vdi_flatten([c1], [d1], W, H, 0, W, orc.ipv_of(sc["cam"], lib), lib=lib)
    a, b = img0.astype(np.int32), img1.astype(np.int32)
    cover = (a[..., 3] > 0) | (b[..., 3] > 0)
    assert cover.sum() > 1000, "scene too empty"
    diff = np.abs(a - b).max(axis=2)[cover]
    mse = np.mean(((a[cover] - b[cover]) / 255.0) ** 2)
    psnr = np.inf if mse == 0 else 10 * np.log10(1.0 / mse)
    # the north-star image tolerance: exact for three variants, almost everywhere without contraction
    max_diff, within = (3, 0.998) if variant == "nofma" else (1, 1.0)
    assert diff.max() <= max_diff and np.mean(diff <= 1) >= within, (variant, int(diff.max()), float(np.mean(diff <= 1)))
    assert psnr >= 50.0, (variant, psnr)
    # the supersegment structure is not invariant (recorded, loosely bounded)
    n0 = np.count_nonzero(d0[..., 0::2], axis=2)
    n1 = np.count_nonzero(d1[..., 0::2], axis=2)
    hit = (n0 > 0) | (n1 > 0)
    match = float(np.mean(n0[hit] == n1[hit]))
    assert match >= 0.75, (variant, match)
    print(f"{variant}: RGBA max {int(diff.max())}/255, PSNR {psnr:.1f} dB, count-match {match:.4f}")


def test_contract_build_differs_from_every_variant(contract):
    """Each variant really changes the arithmetic (the study measures something)."""
    sc, inp, c0, d0, _ = contract
    for v in orc.VARIANTS:
        c1, d1, _, _ = orc.vdi_generate(inp, W, H, S, lib=orc.load_variant(v))
        assert not np.array_equal(c0.view(np.uint32), c1.view(np.uint32)), v
