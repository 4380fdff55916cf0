"""The host side of the generator's device draw: glibc's log restated (csrc/dh_legacy_gauss.h,
constants from tools/gen_glibc_log_table.py) against libm's log -- the function NumPy's legacy
gauss calls (numpy/random/src/legacy/legacy-distributions.c, f = sqrt(-2 log(r2) / r2)) -- bit for
bit, over the polar method's r2 values, uniform doubles, the near-1 branch and random bit
patterns (tests/native/log_check.cpp; CPU only)."""
import ctypes
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "liblogcheck.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("tests/native/liblogcheck.so not built (make -C option-pricing-ffn-lbfgs_amd/csrc)")
    L = ctypes.CDLL(LIB)
    L.dh_log_mismatches.restype = ctypes.c_int64
    L.dh_log_mismatches.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)]
    return L


def test_restated_log_equals_libm(lib):
    bad = ctypes.c_double(0.0)
    for seed in (1, 2, 3):
        n = lib.dh_log_mismatches(seed, 2_000_000, ctypes.byref(bad))
        assert n == 0, (seed, n, bad.value)


def test_restated_log_equals_python_math_log(lib):
    """Also against Python's math.log (libm's log through another caller) on a small sample."""
    rs = np.random.RandomState(5)
    x = np.concatenate([rs.random_sample(2000), 1.0 + rs.uniform(-0.0625, 0.0645, 2000),
                        np.exp(rs.uniform(-700, 700, 2000))])
    got = np.empty_like(x)
    lib.dh_restated_log(x.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size),
                        got.ctypes.data_as(ctypes.c_void_p))
    want = np.array([math.log(v) for v in x])
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
