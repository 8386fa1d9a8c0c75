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


from tf_image_compression_amd.synthetic import structured_patches  # noqa: E402,F401
