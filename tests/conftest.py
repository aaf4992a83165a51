"""pytest configuration.

Markers:
  gpu -- needs a HIP device (MI355X) and libmcodec.so; run with ``-m gpu``.
         These are the parity tests proper: every codec call goes through the
         C ABI into the gfx950 kernels, and results are checked against the
         oracle (oracle/) and the golden vectors (tests/golden/).
Everything else runs on CPU (``-m "not gpu"``).
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device and libmcodec.so (MI355X)")


@pytest.fixture(scope="session")
def device():
    """The HIP device; GPU tests fail (not skip) when it is missing."""
    import torch

    import numcodecs_amd._native as nat

    nat.require_device()
    return torch.device("cuda", 0)
