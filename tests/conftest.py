import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "async-rl_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def load_checkpoint():
    """trained_model/breakout_ff/80000000_finish.h5 converted to npz
    (tests/golden/gen_golden.py); keys are the Chainer HDF5 paths."""
    with np.load(os.path.join(GOLDEN, "breakout_ff.npz")) as z:
        return {k.replace("|", "/"): z[k] for k in z.files}


def close_normscaled(a, b, rtol=1e-5):
    """|a - b| <= rtol * max(|b|, ||b||_inf) elementwise: fp32
    parity for long reductions, tolerance stated in the test."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.maximum(np.abs(b), np.abs(b).max() if b.size else 0.0)
    err = np.abs(a - b) - rtol * scale
    return bool((err <= 0).all()), float((np.abs(a - b) / np.maximum(scale, 1e-30)).max()) if b.size else 0.0


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
