"""Shared test setup.

* ``gpu`` marker: tests that need a gfx950 device (run on the MI355X box with ``-m gpu``).
* sys.path: the repo root (for ``oracle``) and the package root (for ``dhcos``).
* golden fixtures produced from the reference by tests/golden/make_golden.py.
"""
import json
import os
import sys

import numpy as np
import pytest
# torch before the first libdhcos call: both then bind one HIP runtime (dhcos/_native.py), in
# whatever order the GPU tests run
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def calib_golden():
    with open(os.path.join(GOLDEN, "calib.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def gen_golden():
    with open(os.path.join(GOLDEN, "generator.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def cf_complex_golden():
    with open(os.path.join(GOLDEN, "cf_complex.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def calib_noise():
    with open(os.path.join(GOLDEN, "calib_noise.json")) as fh:
        return json.load(fh)


ENSEMBLE_MARGIN = 0.25      # of the members' log-spread, on each side (ensemble_band)
LOSS_TOL = 1e-9             # the loss bar (relative)


def ensemble_band(values, margin=ENSEMBLE_MARGIN, tol=LOSS_TOL):
    """The band a GPU calibration outcome must fall in: the noise ensemble members' range
    [lo, hi], widened on each side by `margin` x its own width in log space, W = log(hi / lo),
    and by the loss bar.  The members sample a chaotic map (tests/test_calibration_sensitivity.py):
    a further draw lands outside the range of n members with probability 2 / (n + 1), so the band
    reaches past the sampled extremes by a fixed share of the spread the members themselves show
    (a quarter: x/ 2.1 for the test market's winners, which span 20x; nothing past the loss bar
    where every member agrees)."""
    import numpy as np
    lo, hi = float(np.min(values)), float(np.max(values))
    w = np.log(hi / lo) if lo > 0 else 0.0
    f = np.exp(margin * w)
    return lo / f * (1 - tol), hi * f * (1 + tol)


def assert_in_noise_ensemble(res, runs, ens, reference_starts, label):
    """calibrate(300, 3) on the reference's test market (np.random.seed(0) starts) against the
    reference algorithm's outcomes under the GPU's measured price noise (tests/golden/
    calib_noise.json, member 0 = the reference's own run): the winner CONVERGED inside the
    ensemble's band of final losses (ensemble_band), start 0 exactly as every member (nit 0,
    'ABNORMAL: ', the Feller kink), starts 1 and 2 with a message some member ends with and a
    loss inside the band of that start's members.  Prints per-start (nit, message, fun) beside
    the reference's."""
    import numpy as np
    lo, hi = ensemble_band([m["final_loss"] for m in ens["members"]])
    assert res.message.startswith("CONVERGENCE") and res.success, (label, res.message)
    assert lo <= res.final_loss <= hi, (label, res.final_loss, lo, hi)
    for s, ((r, _), ref) in enumerate(zip(runs, reference_starts)):
        members = [m["starts"][s] for m in ens["members"]]
        print(f"{label} start {s}: nit {r.nit:3d} {r.message!r:58} fun {r.fun:.6e}   reference: "
              f"nit {ref['nit']:3d} {ref['message']!r:58} fun {ref['fun']:.6e}")
        assert r.message in {m["message"] for m in members}, (label, s, r.message)
        if s == 0:
            assert r.nit == 0 and r.message == "ABNORMAL: "
        f_lo, f_hi = ensemble_band([m["fun"] for m in members])
        assert f_lo <= r.fun <= f_hi, (label, s, r.fun, f_lo, f_hi)
    assert res.final_loss == min(r.fun for r, _ in runs)
    assert np.isfinite(res.final_loss)


@pytest.fixture(scope="session")
def grid():
    with np.load(os.path.join(GOLDEN, "pricing_grid.npz")) as z:   # allow_pickle=False default
        return {k: z[k] for k in z.files}


def rel_close(got, want, rtol=1e-6, atol=1e-10):
    """The parity bar of SURVEY 8(d): |got - want| <= rtol*|want| + atol (elementwise)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    return np.abs(got - want) <= rtol * np.abs(want) + atol


def fd_grad_tol(g, f0, dx, eps_price, rtol=1e-6):
    """Bar for a forward-difference gradient whose losses carry relative price noise eps_price:
    loss = mean(rel^2) moves by ~2 sqrt(f0) eps_price per evaluation, two evaluations per
    component, divided by the step dx."""
    return rtol * np.abs(np.asarray(g)) + 4.0 * np.sqrt(abs(f0)) * eps_price / np.asarray(dx)
