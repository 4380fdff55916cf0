"""The generator's batch path on the device (dh_gen_device) against the host
pipeline, bit for bit.

Reference: src/data/synthetic_generator.py:98-157.  The host pipeline (dh_gen_draw: NumPy's
legacy RandomState restated on the host, held to NumPy's own per-sample loop by
tests/test_generator_rng.py; price_grid's chunks; dh_gen_assemble, held to np.mean) is the
checker here: every output array of the device path -- blended params, spots, model prices,
market prices, losses, strikes, dates -- and np.random's continuation must equal it exactly, for
sizes around the chunk and AR(1)-segment boundaries, with and without a gauss value cached at
entry, and at the 1M-sample size the bench times.  The device's glibc-log restatement is held to
libm's log (the values NumPy's legacy gauss takes) bit for bit on the GPU."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def G():
    from dhcos import _native, generator
    if _native.device_count() == 0:
        pytest.skip("no GPU")
    return generator


def host_pipeline(G, n):
    """The host path from np.random's current state: (outputs, np.random's next 5 doubles)."""
    p, s, nz = G.draw_paths(n)
    model = G.price_grid(p, s, chunk=1 << 16)
    out = G.assemble(p, s, nz, model, None, as_arrays=True, verbose=False)
    return out, np.random.random(5)


def check_equal(got, want):
    for k in ("params", "spot", "market_prices", "model_prices", "strikes", "final_loss",
              "dates", "maturities"):
        assert got[k].shape == want[k].shape, k
        assert np.array_equal(got[k], want[k]), (k, np.flatnonzero(got[k] != want[k])[:5])


@pytest.mark.parametrize("n, seed, cached", [(1, 3, False), (2, 4, True), (15, 5, False),
                                             (4096, 6, True), (65_536, 7, False),
                                             (70_001, 8, True), (300_000, 9, False)])
def test_device_generator_equals_host_pipeline(G, n, seed, cached):
    np.random.seed(seed)
    if cached:
        np.random.normal()            # leaves has_gauss = 1: the first sample's first normal is it
    st = np.random.get_state()
    want, after_want = host_pipeline(G, n)
    np.random.set_state(st)
    got = G.generate_synthetic_calibrations(n, None, as_arrays=True, verbose=False)
    after_got = np.random.random(5)
    check_equal(got, want)
    assert np.array_equal(after_got, after_want)
    assert G.last_device_stats["ar1_segments_rerun"] == 0


def test_device_generator_full_size(G):
    """The bench's call, generate_synthetic_calibrations(1_000_000, as_arrays=True) under
    np.random.seed(0): every array equals the host pipeline's, np.random continues identically,
    and the host's share ends with the walk."""
    n = 1_000_000
    np.random.seed(0)
    want, after_want = host_pipeline(G, n)
    np.random.seed(0)
    got = G.generate_synthetic_calibrations(n, None, as_arrays=True, verbose=False)
    after_got = np.random.random(5)
    check_equal(got, want)
    assert np.array_equal(after_got, after_want)
    st = G.last_device_stats
    print(f"device generator 1M: twister {st['twister_s'] * 1e3:.1f} ms, walk "
          f"{st['walk_s'] * 1e3:.1f} ms, first chunk {st['first_chunk_s'] * 1e3:.1f} ms, total "
          f"{st['total_s'] * 1e3:.1f} ms, AR(1) segments re-run {st['ar1_segments_rerun']}")
    assert st["ar1_segments_rerun"] == 0 and st["chunks"] == 16


def test_device_generator_pickle_output_matches_reference(G, gen_golden, tmp_path):
    """The list[CalibrationResult] path of the device draw against the reference's own samples
    (tests/golden/generator.json): parameters, spots, dates and strikes exactly."""
    np.random.seed(0)
    res = G.generate_synthetic_calibrations(len(gen_golden), str(tmp_path / "g.pkl"),
                                            verbose=False)
    for r, w in zip(res, gen_golden):
        assert r.date == w["date"] and r.spot == w["spot"]
        assert [r.parameters[k] for k in w["parameters"]] == list(w["parameters"].values())
        assert [o["strike"] for o in r.market_options] == w["strikes"]


def test_device_log_equals_libm(G):
    """dh_gen_log (glibc's log restated, dh_legacy_gauss.h) against libm's log of the host, bit
    for bit: the polar method's r2 values, uniform doubles, values near 1 (the polynomial branch)
    and random positive finite bit patterns."""
    from dhcos import _native
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "liblogcheck.so"))
    rs = np.random.RandomState(11)
    d = rs.random_sample((2, 400_000))
    x1, x2 = 2 * d[0] - 1, 2 * d[1] - 1
    r2 = x1 * x1 + x2 * x2
    r2 = r2[(r2 < 1) & (r2 > 0)]
    near1 = 1.0 + rs.uniform(-0.0625, float.fromhex("0x1.09p-4"), 100_000)
    bits = rs.randint(1, 0x7FEFFFFFFFFFFFFF, size=200_000, dtype=np.int64).view(np.float64)
    x = np.concatenate([r2, rs.random_sample(100_000) + 1e-300, near1, bits,
                        [1.0, 0.9375, 2.0 ** -1074, 2.0 ** -1022, 0.5]])
    want = np.empty_like(x)
    lib.dh_libm_log(x.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size),
                    want.ctypes.data_as(ctypes.c_void_p))
    got = _native.gen_log(x)
    bad = np.flatnonzero(got.view(np.int64) != want.view(np.int64))
    assert bad.size == 0, (bad.size, x[bad[:3]], got[bad[:3]], want[bad[:3]])
