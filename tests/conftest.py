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
