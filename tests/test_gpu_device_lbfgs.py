"""GPU tests of the device-resident L-BFGS-B (dh_calibrate_lbfgs, csrc/dh_lbfgs.h): the whole
multi-start calibration loop runs as loss launches + step launches on the device.

What is asserted, and why (trajectory bits are not a well-posed target: see
test_gpu_parity.test_calibrate_seed0):
  * the reference's robust start (guess 0) reproduces its result exactly in kind:
    ABNORMAL, nit 0, 21 requests (294 loss evaluations), x = x0, fun = the last trial's loss
    (loss tolerance 1e-9 relative);
  * calibrate(300, 3, driver="device") under np.random.seed(0) converges below 1e-6 (the
    reference reaches 1.02e-7), like the SciPy-driven path;
  * the host loop is an implementation detail: results are bitwise identical for every chunk
    size (compaction of finished starts and re-emission of their requests) and for every way of
    batching starts (a start's values depend only on its own x);
  * the device state machine computes the bits of its CPU build (tests/native/liblbhost.so):
    replaying the device's own request trace (f, g per request) through the CPU build asks for
    the same points, bit for bit, and ends with the same x, fun, nit, nfev and stop;
    (driven instead with losses the host forms itself -- records by NumPy exp / tanh, not the
    device's ocml ones -- the runs agree only to ~1e-7 after two iterations and separate
    further: the records' last-bit differences reach the FD gradient amplified by 1 / h = 1e8).
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT, rel_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dh():
    import dhcos
    from dhcos import _native
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return dhcos


def _cal(dh, g):
    return dh.DoubleHestonJumpCalibrator(100.0, 0.05, g["test_market"])


def test_device_driver_robust_start(dh, calib_golden):
    from dhcos.calibrator import run_starts_device
    want = calib_golden["calibrate_seed0_starts"][0]
    cal = _cal(dh, calib_golden)
    x0 = np.array(want["x0"])
    (res, _), = run_starts_device(cal, [x0], 300)
    assert res.nit == 0 and res.message == want["message"] == "ABNORMAL: "
    assert res.nfev * 14 == want["nfev"] == 294 and cal.n_calls == want["n_calls"]
    assert np.array_equal(res.x, x0)
    assert rel_close(res.fun, want["fun"], 1e-9, 0)
    assert rel_close(cal.best_loss, want["best_loss"], 1e-6, 0)
    assert not res.success


def test_device_driver_calibrate_seed0(dh, calib_golden, calib_noise):
    """As test_gpu_parity.test_calibrate_seed0, on the device-resident L-BFGS-B: the winner and
    every start inside the reference algorithm's noise ensemble (tests/golden/calib_noise.json)."""
    from conftest import assert_in_noise_ensemble
    from dhcos.calibrator import run_starts_device
    np.random.seed(0)
    cal = _cal(dh, calib_golden)
    r = cal.calibrate(maxiter=300, multi_start=3, driver="device")
    x0s = [np.array(s["x0"]) for s in calib_golden["calibrate_seed0_starts"]]
    runs = run_starts_device(_cal(dh, calib_golden), x0s, 300)
    assert_in_noise_ensemble(r, runs, calib_noise, calib_golden["calibrate_seed0_starts"],
                             "device")
    assert rel_close(r.model_prices, cal.market_prices, 5e-3, 0).all()
    assert 0 < r.calibration_time < 5.0
    assert cal.lockstep_launches > 0


def _starts(g, n, seed=3):
    rs = np.random.RandomState(seed)
    base = [np.array(s["x0"]) for s in g["calibrate_seed0_starts"]]
    return np.stack([base[i % 3] + (0.0 if i < 3 else 0.05) * rs.randn(13) for i in range(n)])


def _same(a, b):
    for ra, rb in zip(a, b):
        assert np.array_equal(np.array(ra.x[:]), np.array(rb.x[:]))
        assert ra.fun == rb.fun and ra.nit == rb.nit and ra.nfev == rb.nfev
        assert ra.task == rb.task and ra.n_calls == rb.n_calls and ra.best_loss == rb.best_loss


def test_chunk_size_and_batching_invariance(dh, calib_golden):
    cal = _cal(dh, calib_golden)
    surf = cal._get_surface()
    x0s = _starts(calib_golden, 6)
    ref, _ = surf.calibrate_lbfgs(x0s, 100.0, 0.05, 128, maxiter=40, chunk=8)
    for chunk in (1, 3):
        got, _ = surf.calibrate_lbfgs(x0s, 100.0, 0.05, 128, maxiter=40, chunk=chunk)
        _same(got, ref)
    alone = [surf.calibrate_lbfgs(x0s[i:i + 1], 100.0, 0.05, 128, maxiter=40, chunk=5)[0][0]
             for i in range(len(x0s))]
    _same(alone, ref)
    tasks = {r.task for r in ref}
    assert tasks <= {4401, 4402, 5504, 8000}, tasks


def test_maxiter_stop(dh, calib_golden):
    cal = _cal(dh, calib_golden)
    surf = cal._get_surface()
    x0 = _starts(calib_golden, 2)[1:2]
    (r,), _ = surf.calibrate_lbfgs(x0, 100.0, 0.05, 128, maxiter=3)
    assert r.nit == 3 and r.task == 5504 and r.warnflag == 1


def test_device_replays_bitwise_on_cpu_build(dh, calib_golden):
    import test_lbfgs_device_algo as T
    lib = C.CDLL(os.path.join(ROOT, "tests", "native", "liblbhost.so"))
    lib.lbh_begin.argtypes = [C.c_void_p, T._D]
    lib.lbh_point.argtypes = [C.c_void_p, T._D]
    lib.lbh_set_fg.argtypes = [C.c_void_p, C.c_double, T._D]
    lib.lbh_resume.argtypes = [C.c_void_p] + [C.c_int] * 3 + [C.c_double] * 2
    lib.lbh_result.argtypes = [C.c_void_p, T._D, T._D, C.POINTER(C.c_int)]
    cal = _cal(dh, calib_golden)
    surf = cal._get_surface()
    x0s = _starts(calib_golden, 5)
    surf.ctx.set_lb_trace(100000)
    try:
        res, _ = surf.calibrate_lbfgs(x0s, 100.0, 0.05, 128, maxiter=300, maxfun=1071)
        tr = surf.ctx.read_lb_trace()
    finally:
        surf.ctx.set_lb_trace(0)
    assert len(tr) == sum(r.n_calls for r in res) // 14
    eps = np.finfo(float).eps
    for s, r in enumerate(res):
        rows = tr[tr[:, 0] == s]
        rows = rows[np.argsort(rows[:, 1])]
        assert np.array_equal(rows[:, 1], np.arange(len(rows)))
        st = C.create_string_buffer(lib.lbh_state_size())
        x0 = np.ascontiguousarray(x0s[s])
        more = lib.lbh_begin(st, x0.ctypes.data_as(T._D))
        xe = np.empty(13)
        k = 0
        while more:
            lib.lbh_point(st, xe.ctypes.data_as(T._D))
            assert np.array_equal(xe, rows[k, 3:16]), (s, k)
            g = np.ascontiguousarray(rows[k, 16:29])
            lib.lbh_set_fg(st, rows[k, 2], g.ctypes.data_as(T._D))
            more = lib.lbh_resume(st, 300, 1071, 20, (1e-9 / eps) * eps, 1e-6)
            k += 1
        assert k == len(rows) == r.nfev
        x = np.empty(13)
        fv = C.c_double()
        info = (C.c_int * 4)()
        lib.lbh_result(st, x.ctypes.data_as(T._D), C.byref(fv), info)
        assert np.array_equal(x, np.array(r.x[:])) and fv.value == r.fun
        assert list(info) == [r.nit, r.nfev, r.task, r.warnflag]


def test_invalid_prices_mark_the_loss_on_both_drivers(dh, calib_golden):
    """A start whose prices are invalid (v0 = e^40 overflows the CF: NaN prices) has loss 1e10 at
    every point (lbfgs_calibrator.py:152-158).  The device driver's loss requests store each
    tile's partial and its invalid-price count; both drivers must end the same way: ABNORMAL at x0
    with fun = 1e10 and the same request count."""
    from dhcos.calibrator import run_starts, run_starts_device
    x0 = np.array(calib_golden["calibrate_seed0_starts"][0]["x0"], dtype=float)
    x0[0] = x0[5] = 40.0
    (dev, _), = run_starts_device(_cal(dh, calib_golden), [x0], 300)
    (host, _), = run_starts(_cal(dh, calib_golden), [x0], 300)
    assert dev.fun == host.fun == 1e10
    assert (dev.nit, dev.nfev, dev.message) == (host.nit, host.nfev, host.message)
    assert np.array_equal(dev.x, host.x) and np.array_equal(dev.x, x0)


def test_nan_market_price_gives_nan_loss_on_both_drivers(dh, calib_golden):
    """A NaN (or infinite) market price makes every loss NaN in the reference (rel = NaN at that
    option).  The device driver's loss launches carry each tile's invalid-price count apart from
    its sum, so the NaN stays a NaN there too (not 1e10); the gradient is NaN, so the pgtol test
    fails as in SciPy, and the line search's trial points are NaN (their prices are invalid:
    1e10).  Both drivers end as SciPy does: ABNORMAL at x0 after 21 requests, fun = the last
    trial's loss."""
    from dhcos.calibrator import run_starts, run_starts_device
    x0 = np.array(calib_golden["calibrate_seed0_starts"][1]["x0"], dtype=float)
    for bad in (float("nan"), float("inf")):
        mkt = [dict(o) for o in calib_golden["test_market"]]
        mkt[4]["price"] = bad
        cal = dh.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
        assert np.isnan(cal.compute_loss(x0))
        (dev, _), = run_starts_device(cal, [x0], 300)
        (host, _), = run_starts(dh.DoubleHestonJumpCalibrator(100.0, 0.05, mkt), [x0], 300)
        assert np.array_equal(dev.fun, host.fun, equal_nan=True)
        assert (dev.nit, dev.nfev, dev.message) == (host.nit, host.nfev, host.message) == \
            (0, 21, "ABNORMAL: ")
        assert np.array_equal(dev.x, host.x) and np.array_equal(dev.x, x0)


def test_degenerate_markets_fall_back_to_reference_semantics(dh, calib_golden):
    """'' option type (every loss 1e10) and an empty market (NaN) have nothing to optimise; the
    device driver hands them to the host driver and returns the reference's result."""
    mkt = [dict(o) for o in calib_golden["test_market"]]
    mkt[0]["option_type"] = ""
    for market in (mkt, []):
        r = dh.DoubleHestonJumpCalibrator(100.0, 0.05, market).calibrate(
            maxiter=10, multi_start=1, driver="device")
        h = dh.DoubleHestonJumpCalibrator(100.0, 0.05, market).calibrate(maxiter=10, multi_start=1)
        assert (r.final_loss, r.success, r.message, r.iterations) == \
            (h.final_loss, h.success, h.message, h.iterations)
    assert not r.success


def _sharded_worker(rank, world, port, out_dir, market):
    import pickle
    import torch.distributed as dist
    import dhcos
    from dhcos import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        np.random.seed(0 if rank == 0 else 4321 + rank)     # x0s are drawn on rank 0
        cal = dhcos.DoubleHestonJumpCalibrator(100.0, 0.05, market)
        res = D.calibrate_sharded(cal, maxiter=300, multi_start=4, driver="device")
        with open(os.path.join(out_dir, f"rank{rank}.pkl"), "wb") as fh:
            pickle.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_device_driver_equals_single_process(dh, calib_golden, tmp_path):
    """Two ranks (gloo) sharing the GPU, each running its starts on the device driver, return
    the single-process result bit for bit (a start's trajectory does not depend on which starts
    share its launches)."""
    import pickle
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    market = calib_golden["test_market"]
    mp.spawn(_sharded_worker, args=(2, port, str(tmp_path), market), nprocs=2, join=True)
    np.random.seed(0)
    want = dh.DoubleHestonJumpCalibrator(100.0, 0.05, market).calibrate(300, 4, driver="device")
    for r in range(2):
        got = pickle.load(open(tmp_path / f"rank{r}.pkl", "rb"))
        assert got.final_loss == want.final_loss and got.iterations == want.iterations
        assert got.message == want.message and got.parameters == want.parameters
        np.testing.assert_array_equal(got.model_prices, want.model_prices)
