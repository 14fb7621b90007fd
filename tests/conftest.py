import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "smartphone-based-rti_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs on the GPU box")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json) cases")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def coef_close(got, ref, rtol=1e-4):
    """SURVEY §8(c) criterion: |c - c_ref| <= rtol * max(|c_ref|, max_k |c_ref,k|) per pixel."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.max(np.abs(ref), axis=-1, keepdims=True)
    err = np.abs(got - ref) / np.maximum(scale, 1e-30)
    return float(err.max()), bool((err <= rtol).all())


def relight_close(got, ref, rtol=1e-4):
    """|L - L_ref| <= rtol * max(|L_ref|, 255)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 255.0)
    return float(err.max()), bool((err <= rtol).all())


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import rti

    rti.load()
    return torch.device("cuda", 0)
