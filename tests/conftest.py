"""Shared pytest setup.

* ``gpu`` marks tests that need a real MI355X (run with ``-m gpu``); everything else runs
  on the CPU-only container.
* Never import torch at module level here or in any test module: torch bundles its own
  HIP runtime (same soname as /opt/rocm's), and libtic.so must bind to the system one.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libtic.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture
def rng():
    return np.random.default_rng(np.random.PCG64(20240229))


def structured_patches(n, P, seed=0):
    """Smooth gradients + sinusoid texture + Gaussian noise (sigma 8), uint8."""
    r = np.random.default_rng(np.random.PCG64(1234 + seed))
    yy, xx = np.meshgrid(np.arange(P), np.arange(P), indexing="ij")
    out = np.empty((n, P, P, 3), np.uint8)
    for i in range(n):
        base = np.zeros((P, P, 3))
        for c in range(3):
            a, b, f1, f2 = r.uniform(-1, 1), r.uniform(-1, 1), r.uniform(0.02, 0.3), r.uniform(0.02, 0.3)
            base[..., c] = (128 + 60 * (a * xx + b * yy) / P + 40 * np.sin(f1 * xx + r.uniform(0, 6))
                            * np.cos(f2 * yy + r.uniform(0, 6)))
        base += r.normal(0, 8, size=base.shape)
        out[i] = np.clip(np.rint(base), 0, 255).astype(np.uint8)
    return out
