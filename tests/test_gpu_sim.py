"""The synthetic Gray-Scott simulation on the GPU (libinsitu_sim.so, the bench's input generator)
follows the torch formulation of scene.gray_scott: same fields up to float rounding."""
from __future__ import annotations

import numpy as np
import pytest

from insitu_amd import scene

pytestmark = pytest.mark.gpu


def test_device_gray_scott_matches_cpu():
    import torch
    a = scene.gray_scott(64, steps=300, seed=1000, device="cpu", sim_n=64).numpy()
    b = scene.gray_scott(64, steps=300, seed=1000, device="cuda", sim_n=64).cpu().numpy()
    assert a.shape == b.shape == (64, 64, 64)
    assert float(a.max()) > 0.05          # the seeds survived
    assert np.max(np.abs(a - b)) < 1e-3, np.max(np.abs(a - b))
    torch.cuda.synchronize()
