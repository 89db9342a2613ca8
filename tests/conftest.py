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
    parity for long reductions, tolerance stated in the test.  Returns (ok,
    max error in units of the scale).  ARL_TOL_STATS=<file>: also append the
    error in units of max(|b|, rms(b)) per call (tolerance calibration)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if not b.size:
        return True, 0.0
    d = np.abs(a - b)
    scale = np.maximum(np.abs(b), np.abs(b).max())
    err = float((d / np.maximum(scale, 1e-30)).max())
    if os.environ.get("ARL_TOL_STATS"):
        import json
        rms = float(np.sqrt((b * b).mean()))
        e_rms = float((d / np.maximum(np.maximum(np.abs(b), rms), 1e-30)).max())
        with open(os.environ["ARL_TOL_STATS"], "a") as f:
            f.write(json.dumps({"n": int(b.size), "err_inf": err, "err_rms": e_rms,
                                "test": os.environ.get("PYTEST_CURRENT_TEST", "")}) + "\n")
    return bool((d - rtol * scale <= 0).all()), err


def close_grad(a, b, scale, rtol=1e-5):
    """Componentwise parity of a reduction result (a weight / bias gradient):
    |a - b| <= rtol * scale per element, scale = the element's own error
    scale from the oracle (grad_mag: its summands' operand uncertainties in
    quadrature, oracle._mag_mm).  Every element -- small ones included -- is
    held to a bound built from its own summands instead of the tensor's
    largest value.  Returns (ok, max |a - b| / scale)."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    m = np.asarray(scale, np.float64).reshape(-1)
    if not b.size:
        return True, 0.0
    m = np.maximum(m, 1e-30)
    err = np.abs(a - b) / m
    if os.environ.get("ARL_TOL_STATS"):
        import json
        with open(os.environ["ARL_TOL_STATS"], "a") as f:
            f.write(json.dumps({"n": int(b.size), "err_elem": float(err.max()),
                                "tight": float(np.median(m / np.maximum(np.abs(b).max(), 1e-30))),
                                "test": os.environ.get("PYTEST_CURRENT_TEST", "")}) + "\n")
    return bool((err <= rtol).all()), float(err.max())


def grads_match(got, g_oracle, mag=None, rtol=1e-5, rtol_elem=1e-5):
    """Every gradient tensor: norm-scaled at rtol (close_normscaled, SURVEY
    H5) AND, where the oracle gave summand norms, componentwise at
    rtol_elem (close_grad) -- the per-element bound keeps small entries of a
    tensor checked against their own scale, not the tensor's largest."""
    bad = []
    for k, want in g_oracle.items():
        ok, err = close_normscaled(got[k], want, rtol)
        if not ok:
            bad.append((k, "normscaled", err))
        if mag is not None and k in mag:
            ok, err = close_grad(got[k], want, mag[k], rtol_elem)
            if not ok:
                bad.append((k, "componentwise", err))
    assert not bad, bad


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
