"""Why calibrate() is compared on robust properties, not on its trajectory (CPU, oracle only).

L-BFGS-B with SciPy's forward differences (h = 1e-8) turns ~1e-14 loss noise into ~1e-6
relative gradient noise; on the reference's test market the line searches of starts 1 and 2 are
sensitive to that.  Here the reference algorithm itself (the CPU oracle, bitwise equal to the
reference on the KATs) is rerun with its prices perturbed by 1e-15 relative: start 1's iteration
count and final loss move, start 0 (the Feller-kink start) does not.
"""
import numpy as np
from scipy.optimize import minimize

from oracle import dh_oracle as O


def _run(market, x0, eps, seed):
    mk = np.array([o["price"] for o in market])
    K = [o["strike"] for o in market]
    T = [o["maturity"] for o in market]
    rs = np.random.RandomState(seed)

    def loss(x):
        p = O.to_params(x)
        pr = O.price_many(p, 100.0, K, T, 0.05, True, 128)
        pr = pr * (1 + eps * rs.uniform(-1, 1, pr.size))
        return np.mean(((pr - mk) / mk) ** 2) + O.feller(p)

    def fg(x):
        X, dx = O.fd_points(x)
        f = np.array([loss(xx) for xx in X])
        return f[0], O.fd_grad(f, dx)

    with np.errstate(all="ignore"):
        return minimize(fg, x0, method="L-BFGS-B", jac=True,
                        options={"maxiter": 300, "ftol": 1e-9, "gtol": 1e-6, "maxfun": 1071})


def test_start1_trajectory_moves_under_1e15_noise(calib_golden):
    market = calib_golden["test_market"]
    x1 = np.array(calib_golden["calibrate_seed0_starts"][1]["x0"])
    outcomes = {(r.nit, round(float(r.fun), 10)) for r in
                (_run(market, x1, 0.0, 0), _run(market, x1, 1e-15, 1), _run(market, x1, 1e-15, 2))}
    assert len(outcomes) >= 2, outcomes


def test_start0_is_robust(calib_golden):
    market = calib_golden["test_market"]
    want = calib_golden["calibrate_seed0_starts"][0]
    for eps, seed in ((0.0, 0), (1e-14, 3)):
        r = _run(market, np.array(want["x0"]), eps, seed)
        assert r.nit == 0 and r.nfev == 21 and r.message == want["message"]
