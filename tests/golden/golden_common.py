"""Shared pieces of the fixture generators in tests/golden/ (test infrastructure only).

``reference_guess`` restates lbfgs_calibrator.py:179-234 (get_initial_guess) and :89-109
(inverse_transform_params) in plain NumPy, independently of dhcos.calibrator.
``pinned_start_points`` first checks that restatement against the reference's own draws
(tests/golden/calib.json ``guesses_seed0``: np.random.seed(0), guess types 0, 1, 2, 1 on the
reference's test market, made by importing the reference), then checks that the calibrator's
``start_points`` gives the same starts on the fixture's surface, and only then returns them -- so
a fixture's starts are the reference algorithm's, not the product's.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from oracle import dh_oracle as O  # noqa: E402

# lbfgs_calibrator.py:184-188 (and the type-1 template, :192-196), in the reference's dict order
_BASE = {"v1_0": 0.04, "kappa1": 2.5, "theta1": 0.04, "sigma1": 0.3, "rho1": -0.7,
         "v2_0": 0.04, "kappa2": 0.5, "theta2": 0.04, "sigma2": 0.2, "rho2": -0.5,
         "lambda_j": 0.15, "mu_j": -0.04, "sigma_j": 0.08}


def reference_guess(guess_type, market, spot):
    """get_initial_guess(guess_type) of lbfgs_calibrator.py:179-234 (global np.random)."""
    if guess_type == 0:
        params = dict(_BASE)
    elif guess_type == 1:
        params = {}
        for name, value in _BASE.items():                  # :198-206, dict order
            span = 0.15 if name in ("rho1", "rho2", "mu_j") else 0.20
            params[name] = value * (1 + np.random.uniform(-span, span))
        params["rho1"] = np.clip(params["rho1"], -0.95, -0.3)   # :209-210
        params["rho2"] = np.clip(params["rho2"], -0.95, -0.3)
    else:                                                  # :212-232
        atm = [o for o in market if 0.95 < o["strike"] / spot < 1.05]
        if atm:
            avg_price = np.mean([o["price"] for o in atm])
            avg_maturity = np.mean([o["maturity"] for o in atm])
            iv = (avg_price / spot) / np.sqrt(avg_maturity)
            iv = max(0.01, min(0.1, iv))
        else:
            iv = 0.04
        params = {"v1_0": iv, "kappa1": 2.0, "theta1": iv, "sigma1": 0.4, "rho1": -0.6,
                  "v2_0": iv, "kappa2": 0.7, "theta2": iv, "sigma2": 0.25, "rho2": -0.4,
                  "lambda_j": 0.12, "mu_j": -0.03, "sigma_j": 0.07}
    return O.from_params(np.array([params[n] for n in O.PARAM_NAMES]))   # :89-109


def pinned_start_points(cal, n_starts, seed=0):
    """The n_starts starts calibrate() draws under np.random.seed(seed) (guess type s % 3),
    cross-checked three ways (module docstring); leaves np.random after the draws."""
    with open(os.path.join(ROOT, "tests", "golden", "calib.json")) as fh:
        g = json.load(fh)
    np.random.seed(0)
    mine = [reference_guess(t, g["test_market"], 100.0) for t in (0, 1, 2, 1)]
    assert all(np.array_equal(a, np.array(b)) for a, b in zip(mine, g["guesses_seed0"])), \
        "restated get_initial_guess differs from the reference's draws"
    np.random.seed(seed)
    want = [reference_guess(s % 3, cal.market_options, cal.spot) for s in range(n_starts)]
    state = np.random.get_state()
    np.random.seed(seed)
    got = cal.start_points(n_starts)
    assert all(np.array_equal(a, b) for a, b in zip(got, want)), "calibrator start points differ"
    np.random.set_state(state)
    return want
