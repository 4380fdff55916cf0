"""Drop-in ``DoubleHestonJumpCalibrator`` / ``CalibrationResult`` on the gfx950 objective kernel.

Reference: src/calibration/lbfgs_calibrator.py (class at :44-336, dataclass at :21-41).

What changes relative to the reference, and what does not:
  * ``compute_loss(x)`` keeps its exact semantics (n_calls, best_loss, 1e10 on invalid prices,
    inf on zero market prices, NaN on an empty market) but prices the whole surface in one launch.
  * ``calibrate()`` still drives SciPy's L-BFGS-B with the same options.  Instead of letting SciPy
    call the objective 14 times per function+gradient request (1 base + 13 forward differences,
    scipy/optimize/_numdiff.py:498-511,592-596), it hands SciPy ``jac=True`` and evaluates the 14
    points SciPy would have evaluated in ONE launch, forming the gradient with SciPy's own
    formula ``(f_i - f_0) / ((x_i + h) - x_i)``.  ``maxfun`` is rescaled so the stop rule
    ``nfev > maxfun`` fires at the same request count.  Multi-start runs in lockstep: every live
    start's 14 points share one launch (S = 14 x starts param sets).
  * Starts are independent, so the per-start trajectory does not depend on how many starts share
    a launch; the best start is chosen with the reference's strict ``<`` in start order.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Dict, List

import numpy as np
from scipy.optimize import minimize

from . import _native
from .pricer import resolve_call

INVALID_LOSS = 1e10                 # lbfgs_calibrator.py:152-158,176-177
FD_ABS_STEP = 1e-8                  # SciPy L-BFGS-B default eps (scipy/_lbfgsb_py.py:290)
SCIPY_MAXFUN = 15000                # SciPy L-BFGS-B default maxfun
N_PARAMS = 13

PARAM_NAMES = ["v1_0", "kappa1", "theta1", "sigma1", "rho1",
               "v2_0", "kappa2", "theta2", "sigma2", "rho2",
               "lambda_j", "mu_j", "sigma_j"]
# transform kind per slot of x (lbfgs_calibrator.py:62-87): exp / tanh / identity
_EXP = np.array([0, 1, 2, 3, 5, 6, 7, 8, 10, 12])
_TANH = np.array([4, 9])
_IDENT = 11

# literature start (lbfgs_calibrator.py:184-188) and the type-2 template (:226-232)
_BASE_GUESS = {"v1_0": 0.04, "kappa1": 2.5, "theta1": 0.04, "sigma1": 0.3, "rho1": -0.7,
               "v2_0": 0.04, "kappa2": 0.5, "theta2": 0.04, "sigma2": 0.2, "rho2": -0.5,
               "lambda_j": 0.15, "mu_j": -0.04, "sigma_j": 0.08}
_PERTURB_15 = ("rho1", "rho2", "mu_j")      # +-15% for these, +-20% otherwise (:201-206)


@dataclass
class CalibrationResult:
    """Same fields, order and defaults as lbfgs_calibrator.py:21-41."""
    date: str
    spot: float
    risk_free: float
    parameters: Dict[str, float]
    market_prices: np.ndarray
    model_prices: np.ndarray
    market_options: List[Dict]
    final_loss: float
    calibration_time: float = None
    success: bool = True
    iterations: int = None
    message: str = ""


# pickles name the reference's module (lbfgs_calibrator.py), see ../lbfgs_calibrator.py
CalibrationResult.__module__ = "lbfgs_calibrator"

def x_to_model(X: np.ndarray) -> np.ndarray:
    """Unconstrained x [..., 13] -> model params [..., 13] (exp / tanh / identity)."""
    X = np.asarray(X, dtype=np.float64)
    P = np.empty_like(X)
    P[..., _EXP] = np.exp(X[..., _EXP])
    P[..., _TANH] = np.tanh(X[..., _TANH])
    P[..., _IDENT] = X[..., _IDENT]
    return P


def feller_penalty(P: np.ndarray) -> np.ndarray:
    """1000 * sum_j max(0, sigma_j^2 - 2 kappa_j theta_j) with Python ``max(0, v)`` semantics."""
    v1 = P[..., 3] ** 2 - 2 * P[..., 1] * P[..., 2]
    v2 = P[..., 8] ** 2 - 2 * P[..., 6] * P[..., 7]
    return 1000.0 * (np.where(v1 > 0, v1, 0.0) + np.where(v2 > 0, v2, 0.0))


def fd_request_points(x0, h=FD_ABS_STEP):
    """The points SciPy 1.15 evaluates for one function+gradient request with jac=None:
    x0 and x0 + h_i e_i, plus dx_i = (x0_i + h_i) - x0_i.  h_i falls back to the relative step
    sqrt(eps) * sign(x0_i) * max(1, |x0_i|) where the absolute step vanishes."""
    x0 = np.asarray(x0, dtype=np.float64).ravel()
    n = x0.size
    sign = (x0 >= 0).astype(float) * 2 - 1
    hv = np.full(n, float(h))
    hv = np.where(((x0 + hv) - x0) == 0,
                  np.sqrt(np.finfo(np.float64).eps) * sign * np.maximum(1.0, np.abs(x0)), hv)
    X = np.repeat(x0[None, :], n + 1, axis=0)
    idx = np.arange(n)
    X[idx + 1, idx] += hv
    dx = X[idx + 1, idx] - x0
    return X, dx


class DoubleHestonJumpCalibrator:
    """Calibrates the 13 Double-Heston + jump parameters to a list of market options."""

    def __init__(self, spot: float, risk_free_rate: float, market_options: List[Dict], *,
                 N: int = 128, device=None):
        self.spot = spot
        self.risk_free_rate = risk_free_rate
        self.market_options = market_options
        self.market_prices = np.array([opt["price"] for opt in market_options])
        self.param_names = list(PARAM_NAMES)
        self.n_calls = 0
        self.best_loss = np.inf
        self.N = int(N)            # the reference hard-wires pricing() default N=128 (:150)
        self.device = device
        self._surface = None
        self._surface_ok = None    # False when an option_type is '' (every loss is then 1e10)
        self.loss_evals = 0        # param sets evaluated over the object's life (all starts)

    # ---- transforms (lbfgs_calibrator.py:62-116) ---------------------------------------
    def transform_params(self, x: np.ndarray) -> Dict[str, float]:
        vals = x_to_model(np.asarray(x, dtype=np.float64)[:N_PARAMS])
        return {name: vals[i] for i, name in enumerate(PARAM_NAMES)}

    def inverse_transform_params(self, params: Dict[str, float]) -> np.ndarray:
        x = np.zeros(N_PARAMS)
        for i, name in enumerate(PARAM_NAMES):
            v = params[name]
            if i in _TANH:
                x[i] = np.arctanh(np.clip(v, -0.999, 0.999))
            elif i == _IDENT:
                x[i] = v
            else:
                x[i] = np.log(v)
        return x

    def compute_feller_penalty(self, params: Dict[str, float]) -> float:
        s1, k1, t1 = params["sigma1"], params["kappa1"], params["theta1"]
        s2, k2, t2 = params["sigma2"], params["kappa2"], params["theta2"]
        return 1000.0 * (max(0, s1 ** 2 - 2 * k1 * t1) + max(0, s2 ** 2 - 2 * k2 * t2))

    # ---- device surface -----------------------------------------------------------------
    def _get_surface(self):
        if self._surface_ok is None:
            try:
                flags = [resolve_call(o["option_type"]) for o in self.market_options]
            except Exception:          # '' / non-string option types: the reference returns 1e10
                self._surface_ok = False
                return None
            ctx = _native.default_context(self.device)
            K = [o["strike"] for o in self.market_options]
            T = [o["maturity"] for o in self.market_options]
            self._surface = _native.Surface(ctx, K, T, flags, self.market_prices)
            self._surface_ok = True
        return self._surface if self._surface_ok else None

    def _records(self, X: np.ndarray):
        P = x_to_model(X)
        rec = np.empty((P.shape[0], _native.PARAM_STRIDE))
        rec[:, :13] = P
        rec[:, 13] = self.spot
        rec[:, 14] = self.risk_free_rate
        rec[:, 15] = 0.0
        return P, rec

    def loss_batch(self, X: np.ndarray, track: bool = True) -> np.ndarray:
        """compute_loss for every row of X [S, 13] in one launch (reference semantics per row)."""
        X = np.atleast_2d(np.asarray(X, dtype=np.float64))
        S = X.shape[0]
        self.loss_evals += S
        if track:
            self.n_calls += S
        M = len(self.market_options)
        P, rec = self._records(X)
        pen = feller_penalty(P)
        if M == 0:                              # np.mean([]) -> nan
            return np.full(S, np.nan)
        surf = self._get_surface()
        if surf is None:
            return np.full(S, INVALID_LOSS)
        sse, bad, _ = surf.loss_terms(rec, self.N)
        loss = np.where(bad > 0, INVALID_LOSS, sse / M + pen)
        if track:
            valid = loss[bad == 0]
            if valid.size:
                lo = valid[np.argmin(np.where(np.isnan(valid), np.inf, valid))]
                if lo < self.best_loss:
                    self.best_loss = lo
        return loss

    def compute_loss(self, x: np.ndarray) -> float:
        """Relative MSE + Feller penalty (lbfgs_calibrator.py:118-177)."""
        return float(self.loss_batch(np.asarray(x, dtype=np.float64)[None, :N_PARAMS])[0])

    def compute_loss_and_grad(self, x: np.ndarray, eps: float = FD_ABS_STEP):
        """(f, g) exactly as SciPy's 2-point forward difference would form them, from one launch
        of the 14 points (x and x + h e_i)."""
        X, dx = fd_request_points(x, eps)
        f = self.loss_batch(X)
        return f[0], (f[1:] - f[0]) / dx

    # ---- initial guesses (lbfgs_calibrator.py:179-234) --------------------------------------
    def get_initial_guess(self, guess_type: int = 0) -> np.ndarray:
        if guess_type == 0:
            params = dict(_BASE_GUESS)
        elif guess_type == 1:
            params = {}
            for name, base in _BASE_GUESS.items():        # global RNG, dict order
                span = 0.15 if name in _PERTURB_15 else 0.20
                params[name] = base * (1 + np.random.uniform(-span, span))
            for name in ("rho1", "rho2"):
                params[name] = np.clip(params[name], -0.95, -0.3)
        else:
            atm = [o for o in self.market_options if 0.95 < o["strike"] / self.spot < 1.05]
            iv = 0.04
            if atm:
                avg_p = np.mean([o["price"] for o in atm])
                avg_t = np.mean([o["maturity"] for o in atm])
                iv = max(0.01, min(0.1, (avg_p / self.spot) / np.sqrt(avg_t)))
            params = {"v1_0": iv, "kappa1": 2.0, "theta1": iv, "sigma1": 0.4, "rho1": -0.6,
                      "v2_0": iv, "kappa2": 0.7, "theta2": iv, "sigma2": 0.25, "rho2": -0.4,
                      "lambda_j": 0.12, "mu_j": -0.03, "sigma_j": 0.07}
        return self.inverse_transform_params(params)

    # ---- calibration (lbfgs_calibrator.py:236-336) ------------------------------------------
    def _model_prices(self, params: Dict[str, float]) -> np.ndarray:
        surf = self._get_surface()
        if surf is None:
            raise IndexError("string index out of range")   # what the reference raises here
        rec = np.empty((1, _native.PARAM_STRIDE))
        rec[0, :13] = [params[n] for n in PARAM_NAMES]
        rec[0, 13:] = (self.spot, self.risk_free_rate, 0.0)
        return surf.price(rec, self.N)[0]

    def calibrate(self, maxiter: int = 300, multi_start: int = 3, *, lockstep: bool = True,
                  x0s=None) -> CalibrationResult:
        """Multi-start L-BFGS-B; returns the best start (strict ``<`` in start order)."""
        start_time = time.time()
        # draw every start's x0 in start order (the only consumer of the global RNG, :256)
        if x0s is None:
            x0s = [self.get_initial_guess(guess_type=s % 3) for s in range(multi_start)]
        outcomes = run_starts(self, x0s, maxiter, lockstep=lockstep)
        best_result, best_loss = None, np.inf
        for s, out in enumerate(outcomes):
            if out is None:                       # the start raised: except -> continue (:316)
                continue
            res, t_done = out
            if res.fun < best_loss:
                best_loss = res.fun
                params = self.transform_params(res.x)
                try:
                    model = self._model_prices(params)
                except _native.NativeError:
                    raise
                except Exception:
                    continue
                best_result = CalibrationResult(
                    date="", spot=self.spot, risk_free=self.risk_free_rate, parameters=params,
                    market_prices=self.market_prices, model_prices=model,
                    market_options=self.market_options, final_loss=res.fun,
                    calibration_time=t_done - start_time, success=res.success,
                    iterations=res.nit, message=res.message)
        if best_result is None:
            best_result = CalibrationResult(
                date="", spot=self.spot, risk_free=self.risk_free_rate,
                parameters={name: 0.0 for name in self.param_names},
                market_prices=self.market_prices, model_prices=np.zeros_like(self.market_prices),
                market_options=self.market_options, final_loss=np.inf,
                calibration_time=time.time() - start_time, success=False, iterations=0,
                message="All optimization starts failed")
        return best_result


# ----------------------------------------------------------------------------------------------
# lockstep multi-start driver
# ----------------------------------------------------------------------------------------------
class _StartState:
    """Per-start bookkeeping that mirrors the reference's per-start resets (:253-254)."""

    def __init__(self):
        self.n_calls = 0
        self.best_loss = np.inf


class _Lockstep:
    """Collects the function+gradient requests of all live starts and serves them with one
    launch.  Each start runs SciPy's minimize in its own thread; the last thread to arrive
    evaluates the whole batch.  A start's values depend only on its own x, so results equal the
    sequential run bit for bit."""

    def __init__(self, cal: DoubleHestonJumpCalibrator, n: int):
        self.cal = cal
        self.live = n
        self.pending = {}
        self.results = {}
        self.cv = threading.Condition()
        self.states = [_StartState() for _ in range(n)]
        self.launches = 0

    def _run_batch(self):
        ids = sorted(self.pending)
        pts = [fd_request_points(self.pending[i]) for i in ids]
        X = np.concatenate([p[0] for p in pts])
        try:
            f = self.cal.loss_batch(X, track=False)
            self.launches += 1
            for j, sid in enumerate(ids):
                fj = f[j * (N_PARAMS + 1):(j + 1) * (N_PARAMS + 1)]
                st = self.states[sid]
                st.n_calls += N_PARAMS + 1
                ok = fj[fj != INVALID_LOSS]
                if ok.size:
                    lo = np.min(np.where(np.isnan(ok), np.inf, ok))
                    if lo < st.best_loss:
                        st.best_loss = lo
                self.results[sid] = (fj[0], (fj[1:] - fj[0]) / pts[j][1])
        except BaseException as e:  # hand the failure to every waiting start
            for sid in ids:
                self.results[sid] = e
        self.pending.clear()
        self.cv.notify_all()

    def request(self, sid, x):
        with self.cv:
            self.pending[sid] = np.array(x, dtype=np.float64)
            if len(self.pending) >= self.live:
                self._run_batch()
            while sid not in self.results:
                self.cv.wait()
            r = self.results.pop(sid)
        if isinstance(r, BaseException):
            raise r
        return r

    def finish(self):
        with self.cv:
            self.live -= 1
            if self.pending and len(self.pending) >= self.live:
                self._run_batch()


def _minimize_start(fun, x0, maxiter):
    # jac=True: nfev counts one per request, SciPy's FD path counts 14 -> rescale maxfun so the
    # `nfev > maxfun` stop fires at the same request (scipy/_lbfgsb_py.py:466-469)
    return minimize(fun=fun, x0=x0, method="L-BFGS-B", jac=True,
                    options={"maxiter": maxiter, "ftol": 1e-9, "gtol": 1e-6,
                             "maxfun": SCIPY_MAXFUN // (N_PARAMS + 1)})


def run_starts(cal: DoubleHestonJumpCalibrator, x0s, maxiter: int, lockstep: bool = True):
    """Run one L-BFGS-B per x0; returns [(OptimizeResult, t_done) | None] in start order."""
    n = len(x0s)
    outcomes = [None] * n
    if n == 0:
        return outcomes
    if not lockstep or n == 1:
        for s, x0 in enumerate(x0s):
            cal.n_calls, cal.best_loss = 0, np.inf
            try:
                res = _minimize_start(cal.compute_loss_and_grad, x0, maxiter)
                outcomes[s] = (res, time.time())
            except _native.NativeError:
                raise
            except Exception:
                outcomes[s] = None
        return outcomes
    ls = _Lockstep(cal, n)
    errors = [None] * n

    def worker(s):
        try:
            res = _minimize_start(lambda x: ls.request(s, x), x0s[s], maxiter)
            outcomes[s] = (res, time.time())
        except BaseException as e:  # noqa: BLE001 -- reference: except -> continue
            errors[s] = e
        finally:
            ls.finish()

    threads = [threading.Thread(target=worker, args=(s,), daemon=True) for s in range(n)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in errors:
        if isinstance(e, _native.NativeError):
            raise e
    last = ls.states[-1]
    cal.n_calls, cal.best_loss = last.n_calls, last.best_loss   # state after the last start
    cal.lockstep_launches = ls.launches
    return outcomes
