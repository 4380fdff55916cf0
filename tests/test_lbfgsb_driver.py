"""The single-threaded L-BFGS-B driver (dhcos.calibrator.lbfgsb_steps / run_starts) against
scipy.optimize.minimize(method='L-BFGS-B', jac=True): same setulb inputs in the same order, so
x, fun, nit, nfev, message and success must agree bit for bit -- on smooth problems, on the
Feller-style kink that ends in 'ABNORMAL' (the reference's guess-0 start), and at
the maxiter / maxfun stops.  CPU only (the objectives here are NumPy)."""
import numpy as np
import pytest
from scipy.optimize import minimize

from dhcos.calibrator import (FD_ABS_STEP, N_PARAMS, _minimize_start, fd_request_points,
                              lbfgsb_steps, run_starts)
from oracle import dh_oracle as O


def _drive(gen, fun):
    x = next(gen)
    try:
        while True:
            x = gen.send(fun(np.copy(x)))
    except StopIteration as stop:
        return stop.value


def _rosen(x):
    f = np.sum(100.0 * (x[1:] - x[:-1] ** 2) ** 2 + (1 - x[:-1]) ** 2)
    g = np.zeros_like(x)
    g[:-1] += -400.0 * x[:-1] * (x[1:] - x[:-1] ** 2) - 2 * (1 - x[:-1])
    g[1:] += 200.0 * (x[1:] - x[:-1] ** 2)
    return f, g


def _kinked_fd(x):
    """sum x^2 + 1000 max(0, x0 x1 - 0.5) with SciPy's forward-difference gradient."""
    def f(z):
        return float(np.sum(z * z) + 1000.0 * max(0.0, z[0] * z[1] - 0.5))
    X, dx = fd_request_points(x, FD_ABS_STEP)
    fv = np.array([f(r) for r in X])
    return fv[0], (fv[1:] - fv[0]) / dx


def _same(a, b):
    assert np.array_equal(a.x, b.x), (a.x, b.x)
    assert a.fun == b.fun and a.nit == b.nit and a.nfev == b.nfev
    assert a.message == b.message and a.success == b.success


@pytest.mark.parametrize("fun,x0,maxiter,maxfun", [
    (_rosen, np.linspace(-1.2, 1.0, N_PARAMS), 300, 1071),
    (_rosen, np.full(N_PARAMS, 3.0), 5, 1071),               # maxiter stop
    (_rosen, np.full(N_PARAMS, -2.0), 300, 7),               # maxfun stop
    (_kinked_fd, np.array([0.8, 0.9] + [0.3] * (N_PARAMS - 2)), 300, 1071),
])
def test_driver_matches_scipy_minimize(fun, x0, maxiter, maxfun):
    want = minimize(fun=fun, x0=x0, method="L-BFGS-B", jac=True,
                    options={"maxiter": maxiter, "ftol": 1e-9, "gtol": 1e-6, "maxfun": maxfun})
    got = _drive(lbfgsb_steps(x0, maxiter, maxfun), fun)
    _same(got, want)


class _OracleCal:
    """A calibrator stand-in whose loss_batch is the CPU oracle (tests only)."""

    def __init__(self, market, spot, r, N):
        self.market, self.spot, self.r, self.N = market, spot, r, N
        self.n_calls, self.best_loss = 0, np.inf

    def loss_batch(self, X, track=True):
        return np.array([O.loss(x, self.market, self.spot, self.r, self.N) for x in X])

    def loss_and_grad(self, x):
        X, dx = fd_request_points(x)
        f = self.loss_batch(X)
        return f[0], (f[1:] - f[0]) / dx


def test_run_starts_lockstep_and_sequential_match_minimize(calib_golden):
    """run_starts over three starts of the reference's test market (N = 32 to keep the CPU
    oracle quick): lockstep and sequential equal per-start scipy.optimize.minimize runs."""
    mkt = calib_golden["test_market"]
    cal = _OracleCal(mkt, 100.0, 0.05, 32)                 # tests/test_suite.py:274-302 market
    x0 = np.array(calib_golden["fd_guess0"]["x0"])
    x0s = [x0, x0 + 0.05 * np.sin(np.arange(N_PARAMS)), x0 - 0.04 * np.cos(np.arange(N_PARAMS))]
    lock = run_starts(cal, x0s, 12, lockstep=True)
    seq = run_starts(cal, x0s, 12, lockstep=False)
    for s, x in enumerate(x0s):
        want = _minimize_start(cal.loss_and_grad, x, 12)
        _same(lock[s][0], want)
        _same(seq[s][0], want)


def test_warm_start_hook_replaces_start_zero_only(calib_golden):
    """calibrate(x0=...) (the FFN warm-start hook): start 0 becomes the given
    point (dict of model parameters or unconstrained vector); the random starts are unchanged."""
    from dhcos.calibrator import DoubleHestonJumpCalibrator
    cal = DoubleHestonJumpCalibrator(100.0, 0.05, calib_golden["test_market"])
    np.random.seed(3)
    plain = cal.start_points(4)
    prm = cal.transform_params(plain[1] + 0.01)
    np.random.seed(3)
    warm = cal.start_points(4, x0=prm)
    np.testing.assert_allclose(warm[0], plain[1] + 0.01, rtol=0, atol=1e-12)
    for a, b in zip(warm[1:], plain[1:]):
        assert np.array_equal(a, b)
    np.random.seed(3)
    vec = cal.start_points(4, x0=plain[2])
    assert np.array_equal(vec[0], plain[2]) and np.array_equal(vec[3], plain[3])


def test_fd_models_equals_per_point_transforms():
    """fd_models (the SciPy driver's per-request transforms, three ufunc calls over the request)
    equals x_to_model of every FD point fd_request_points_many forms, bit for bit: at ordinary
    points, where the absolute step vanishes (|x| ~ 1e9: the relative step), at +-0, and with a
    NaN component (no step vanishes there: NaN - NaN compares unequal to 0)."""
    from dhcos.calibrator import fd_models, fd_request_points_many, x_to_model
    rs = np.random.RandomState(7)
    for case in range(40):
        S = 1 + case % 3
        X0 = rs.normal(0.0, 1.5, size=(S, N_PARAMS))
        if case % 4 == 1:
            X0[rs.randint(S), rs.randint(N_PARAMS)] = rs.choice([1e9, -3e9, 7.5e8])
        if case % 4 == 2:
            X0[rs.randint(S), rs.randint(N_PARAMS)] = rs.choice([0.0, -0.0])
        if case % 4 == 3:
            X0[rs.randint(S), rs.randint(N_PARAMS)] = np.nan
        P = fd_models(X0)
        X, _ = fd_request_points_many(X0)
        want = x_to_model(X).reshape(S, N_PARAMS + 1, N_PARAMS)
        with np.errstate(invalid="ignore"):
            assert np.array_equal(P[0].view(np.int64), want[:, 0].view(np.int64)), case
            for i in range(N_PARAMS):        # point i + 1 moves component i only
                assert np.array_equal(P[1][:, i].view(np.int64),
                                      want[:, i + 1, i].view(np.int64)), (case, i)
