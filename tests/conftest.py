import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def sweep_fixtures():
    return sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "sweep_*.npz")))


def model_fixtures():
    return sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "model_*.npz"))
                  if not os.path.basename(f).startswith("model_int_"))


def int_model_fixtures():
    return sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "model_int_*.npz")))


@pytest.fixture(scope="session")
def gpu():
    """Select cuda:0 and make sure the native library is the thing that runs."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a GPU")
    torch.cuda.set_device(0)
    from itrails_amd import _lib

    _lib.lib()  # raises if libitrails_hip.so is missing: no fallback
    return torch.device("cuda:0")
