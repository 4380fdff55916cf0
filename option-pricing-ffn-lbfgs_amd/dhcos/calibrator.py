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
  * SciPy's optimizer itself is driven through its reverse-communication entry point
    (``scipy.optimize._lbfgsb.setulb``) by ``lbfgsb_steps``, a line-for-line restatement of
    ``_minimize_lbfgsb``'s loop for jac=True and no bounds: one Python thread advances every
    start, so a lockstep iteration costs one launch plus the setulb calls, with no thread
    hand-offs.  Same setulb inputs in the same order, so the same trajectory as ``minimize``.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from operator import itemgetter
from dataclasses import dataclass
from typing import Dict, List

import numpy as np
from scipy.optimize import OptimizeResult, _lbfgsb, minimize
from scipy.optimize._lbfgsb_py import status_messages, task_messages
from threadpoolctl import ThreadpoolController

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
    X, dx = fd_request_points_many(np.asarray(x0, dtype=np.float64).reshape(1, -1), h)
    return X, dx[0]


_SQRT_EPS = float(np.sqrt(np.finfo(np.float64).eps))


_EXP_MASK = np.zeros(N_PARAMS, dtype=bool)
_EXP_MASK[_EXP] = True


def fd_models(X0, h=FD_ABS_STEP, out=None):
    """[2, S, 13]: the model params (x_to_model) of every x0 row and of x0 + h, h as
    fd_request_points_many forms it.  NumPy's exp / tanh as the reference's transform_params
    calls them element by element (the same SIMD loops, so the same bits), in place in one
    [2S, 13] array (out: the caller's [2, S, 13] buffer, e.g. _native.FgChannel.model_out): the
    per-iteration host cost of the SciPy driver (tests/test_gpu_parity.py holds fg() to
    fg_from_losses() bit for bit)."""
    X0 = np.asarray(X0, dtype=np.float64)
    S = X0.shape[0]
    P = np.empty((2 * S, N_PARAMS)) if out is None else out.reshape(2 * S, N_PARAMS)
    P[:S] = X0
    Xh = P[S:]
    np.add(X0, h, out=Xh)
    d = Xh - X0
    if np.count_nonzero(d) != d.size:                 # some step vanishes (d == 0); NaN counts
        vanish = d == 0                                # as nonzero, as in (Xh - X0) == 0
        sign = np.where(X0 >= 0, 1.0, -1.0)
        Xh[...] = X0 + np.where(vanish, _SQRT_EPS * sign * np.maximum(1.0, np.abs(X0)), h)
    np.exp(P, out=P, where=_EXP_MASK)                 # identity where the mask is off
    np.tanh(P[:, 4], out=P[:, 4])
    np.tanh(P[:, 9], out=P[:, 9])
    return P.reshape(2, S, N_PARAMS)


def _custom_loss(cal):
    """True when a subclass replaces compute_loss or loss_batch: its losses must then be used
    (the reference's minimize calls self.compute_loss), not the native request."""
    cls = type(cal)
    return (cls.compute_loss is not DoubleHestonJumpCalibrator.compute_loss
            or cls.loss_batch is not DoubleHestonJumpCalibrator.loss_batch)


class _StartRaised(Exception):
    """fg_from_losses' compute_loss path: start ``j`` of the group raised; ``rows`` holds the
    [j, 14] losses of the starts before it (each point evaluated once, as the reference's
    per-start minimize calls would)."""

    def __init__(self, j, rows):
        super().__init__(j)
        self.j, self.rows = j, rows


def _fg_rows(F, dx):
    """(f0, g, low) of [S, 14] losses: SciPy's forward difference and the smallest valid loss
    (NaN never wins, 1e10 is not valid)."""
    G = (F[:, 1:] - F[:, :1]) / dx
    low = np.min(np.where((F == INVALID_LOSS) | np.isnan(F), np.inf, F), axis=1)
    return F[:, 0].copy(), G, low


def fg_from_losses(cal, X0):
    """fg_batch through the calibrator's own losses (``compute_loss`` per point when a subclass
    replaces it, else ``loss_batch``): the 14 points of each request, their losses, SciPy's
    forward difference and the smallest valid loss.  With a ``compute_loss`` override the starts
    are evaluated one after another and a start that raises ends the call with ``_StartRaised``
    (the losses of the starts before it attached), so no point is ever evaluated twice."""
    S = X0.shape[0]
    X, dx = fd_request_points_many(X0)
    custom = getattr(type(cal), "compute_loss", DoubleHestonJumpCalibrator.compute_loss)
    if custom is not DoubleHestonJumpCalibrator.compute_loss and hasattr(cal, "market_options"):
        n0 = cal.n_calls
        rows = []
        try:
            for j in range(S):
                pts = X[j * (N_PARAMS + 1):(j + 1) * (N_PARAMS + 1)]
                try:
                    rows.append([cal.compute_loss(x) for x in pts])
                except _native.NativeError:
                    raise
                except Exception as exc:      # noqa: BLE001 -- the reference drops this start
                    raise _StartRaised(j, np.array(rows, dtype=np.float64).reshape(
                        len(rows), N_PARAMS + 1)) from exc
        finally:
            cal.n_calls = n0            # run_starts keeps the per-start counts
        F = np.array(rows, dtype=np.float64).reshape(S, N_PARAMS + 1)
    else:
        F = cal.loss_batch(X, track=False).reshape(S, N_PARAMS + 1)
    return _fg_rows(F, dx)


def fd_request_points_many(X0, h=FD_ABS_STEP):
    """fd_request_points for every row of X0 [S, n]: -> X [S * (n + 1), n] (per start x0 then
    x0 + h_i e_i, start-major) and dx [S, n].  Elementwise the same arithmetic."""
    X0 = np.asarray(X0, dtype=np.float64)
    S, n = X0.shape
    hv = np.full((S, n), float(h))
    vanish = ((X0 + hv) - X0) == 0
    if vanish.any():
        sign = (X0 >= 0).astype(float) * 2 - 1
        hv[vanish] = (_SQRT_EPS * sign * np.maximum(1.0, np.abs(X0)))[vanish]
    X = np.repeat(X0[:, None, :], n + 1, axis=1)
    idx = np.arange(n)
    X[:, idx + 1, idx] += hv
    dx = X[:, idx + 1, idx] - X0
    return X.reshape(S * (n + 1), n), dx


class DoubleHestonJumpCalibrator:
    """Calibrates the 13 Double-Heston + jump parameters to a list of market options."""

    def __init__(self, spot: float, risk_free_rate: float, market_options: List[Dict], *,
                 N: int = 128, device=None):
        self.spot = spot
        self.risk_free_rate = risk_free_rate
        self.market_options = market_options
        self.market_prices = np.array(list(map(itemgetter("price"), market_options)))
        self.param_names = list(PARAM_NAMES)
        self.n_calls = 0
        self.best_loss = np.inf
        self.N = int(N)            # the reference hard-wires pricing() default N=128 (:150)
        self.device = device
        self._surface = None
        self._surface_ok = None    # False when an option_type is '' (every loss is then 1e10)
        self._strikes = self._maturities = None   # _option_arrays
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
            opts = self.market_options
            try:
                # resolve_call once per distinct type string (10,000-option surfaces hold two)
                types = list(map(itemgetter("option_type"), opts))
                rule = {t: resolve_call(t) for t in set(types)}
                flags = list(map(rule.__getitem__, types))
            except Exception:          # '' / non-string option types: the reference returns 1e10
                self._surface_ok = False
                return None
            ctx = _native.default_context(self.device)
            K, T = self._option_arrays()
            self._surface = _native.Surface(ctx, K, T, flags, self.market_prices)
            self._surface_ok = True
        return self._surface if self._surface_ok else None

    def _option_arrays(self):
        """The options' strikes and maturities as NumPy arrays, built once (np.array of the
        dicts' values: float64 for numbers, another dtype when a value is not one)."""
        if self._strikes is None:
            opts = self.market_options
            self._strikes = np.array(list(map(itemgetter("strike"), opts)))
            self._maturities = np.array(list(map(itemgetter("maturity"), opts)))
        return self._strikes, self._maturities

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

    def fg_batch(self, X0: np.ndarray):
        """One SciPy function+gradient request per row of X0 [S, 13] in one launch:
        -> (f [S], g [S, 13], low [S] = smallest valid loss of each request's 14 points).
        Natively (dh_surface_fg: FD points, Feller and the gradient formed in C++ around one loss
        request; the transforms by NumPy, fd_models) unless a subclass replaces loss_batch,
        whose values are then used the same way."""
        X0 = np.atleast_2d(np.asarray(X0, dtype=np.float64))
        native = not _custom_loss(self)
        surf = self._get_surface() if native and len(self.market_options) else None
        if surf is None:
            return fg_from_losses(self, X0)
        self.loss_evals += X0.shape[0] * (N_PARAMS + 1)
        return surf.fg(X0, self.spot, self.risk_free_rate, self.N, model=fd_models(X0))

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
            iv = 0.04
            K, T = self._option_arrays()
            P = self.market_prices
            if (K.dtype.kind in "fi" and T.dtype.kind in "fi" and P.dtype.kind in "fi"
                    and isinstance(self.spot, (float, int))):
                # the reference's ATM filter and means over arrays: the same IEEE division and
                # comparisons per option, and np.mean of the same values in the same order
                m = K / self.spot
                atm = (0.95 < m) & (m < 1.05)
                if atm.any():
                    avg_p = np.mean(P[atm])
                    avg_t = np.mean(T[atm])
                    iv = max(0.01, min(0.1, (avg_p / self.spot) / np.sqrt(avg_t)))
            else:                   # values that are not plain numbers: the reference's loop
                atm = [o for o in self.market_options if 0.95 < o["strike"] / self.spot < 1.05]
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

    def start_points(self, multi_start: int, x0=None):
        """The starts calibrate() runs: get_initial_guess(s % 3) in start order (the only
        consumer of the global RNG, lbfgs_calibrator.py:256).  x0 -- the warm-start hook the
        reference's docs describe for an FFN prediction (docs/METHODOLOGY.md:112-134, no code
        there) -- replaces start 0's literature guess: a dict of the 13 model parameters, or an
        unconstrained 13-vector.  Start 0 draws no random numbers, so the other starts are
        unchanged."""
        x0s = [self.get_initial_guess(guess_type=s % 3) for s in range(multi_start)]
        if x0 is not None and multi_start > 0:
            x0s[0] = (self.inverse_transform_params(x0) if isinstance(x0, dict)
                      else np.asarray(x0, dtype=np.float64).reshape(N_PARAMS).copy())
        return x0s

    def calibrate(self, maxiter: int = 300, multi_start: int = 3, *, lockstep: bool = True,
                  x0s=None, x0=None, driver: str = "scipy") -> CalibrationResult:
        """Multi-start L-BFGS-B; returns the best start (strict ``<`` in start order).

        driver="scipy": SciPy's own setulb on the host, one launch per lockstep request (the
        reference's optimizer, bit for bit).  driver="device": the device-resident L-BFGS-B
        (dh_calibrate_lbfgs: the loss launches and the optimizer steps run back to back on the
        GPU, the host checks for finished starts every few iterations); same algorithm and
        stopping rules, with the subspace step rounded differently (csrc/dh_lbfgs.h)."""
        start_time = time.time()
        # draw every start's x0 in start order (the only consumer of the global RNG, :256)
        if x0s is None:
            x0s = self.start_points(multi_start, x0)
        if driver == "device":
            outcomes = run_starts_device(self, x0s, maxiter)
        elif driver == "scipy":
            outcomes = run_starts(self, x0s, maxiter, lockstep=lockstep)
        else:
            raise ValueError(f"driver must be 'scipy' or 'device', not {driver!r}")
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
# L-BFGS-B through SciPy's reverse-communication interface
# ----------------------------------------------------------------------------------------------
def lbfgsb_steps(x0, maxiter, maxfun, m=10, ftol=1e-9, gtol=1e-6, maxls=20):
    """Generator restating ``scipy.optimize._lbfgsb_py._minimize_lbfgsb`` (SciPy 1.15.3, the
    ``while True`` loop around ``_lbfgsb.setulb``) for ``jac=True`` and no bounds, with the
    objective evaluated by the caller: it yields the point x at which it needs (f, g) and
    receives them through ``send``; its return value (``StopIteration.value``) is the
    OptimizeResult.  The evaluation bookkeeping is ``ScalarFunction``'s
    (scipy/optimize/_differentiable_functions.py): x0 is evaluated at construction (nfev = 1)
    and a point is re-evaluated only when it differs from the last one (``np.array_equal``)."""
    factr = ftol / np.finfo(float).eps
    pgtol = gtol
    x0 = np.asarray(x0).ravel()
    n = x0.size
    sf_x = x0.astype(np.float64)                     # ScalarFunction.__init__: f and g at x0
    sf_f, sf_g = yield sf_x
    nfev = 1
    nbd = np.zeros(n, np.int32)
    low_bnd = np.zeros(n, np.float64)
    upper_bnd = np.zeros(n, np.float64)
    x = np.array(x0, dtype=np.float64)
    f = np.array(0.0, dtype=np.int32)
    g = np.zeros((n,), dtype=np.int32)
    wa = np.zeros(2 * m * n + 5 * n + 11 * m * m + 8 * m, np.float64)
    iwa = np.zeros(3 * n, dtype=np.int32)
    task = np.zeros(2, dtype=np.int32)
    ln_task = np.zeros(2, dtype=np.int32)
    lsave = np.zeros(4, dtype=np.int32)
    isave = np.zeros(44, dtype=np.int32)
    dsave = np.zeros(29, dtype=np.float64)
    n_iterations = 0
    while True:
        g = g.astype(np.float64)
        _lbfgsb.setulb(m, x, low_bnd, upper_bnd, nbd, f, g, factr, pgtol, wa, iwa, task, lsave,
                       isave, dsave, maxls, ln_task)
        if task[0] == 3:
            if not (x == sf_x).all():                # ScalarFunction.fun_and_grad: np.array_equal
                                                     # (same shapes, so its elementwise test)
                sf_x = x.astype(np.float64)
                sf_f, sf_g = yield sf_x
                nfev += 1
            f, g = sf_f, sf_g
        elif task[0] == 1:
            n_iterations += 1
            if n_iterations >= maxiter:
                task[0] = 5
                task[1] = 504
            elif nfev > maxfun:
                task[0] = 5
                task[1] = 502
        else:
            break
    if task[0] == 4:
        warnflag = 0
    elif nfev > maxfun or n_iterations >= maxiter:
        warnflag = 1
    else:
        warnflag = 2
    msg = status_messages[task[0]] + ": " + task_messages[task[1]]
    return OptimizeResult(fun=f, jac=g, nfev=nfev, njev=nfev, nit=n_iterations,
                          status=warnflag, message=msg, x=x, success=(warnflag == 0))


_BLAS = None


def _single_threaded_blas():
    """Context that pins the BLAS pools (SciPy's OpenBLAS, which setulb calls on 13-vectors and
    10x10 blocks) to one thread.  With the default pool (OMP_NUM_THREADS threads) every setulb call
    pays thread wake-ups worth several times its arithmetic.  Problem sizes are far below
    OpenBLAS's split thresholds, so the results are the same bits (tests/test_lbfgsb_driver.py)."""
    global _BLAS
    if _BLAS is None:
        _BLAS = ThreadpoolController()
    return _BLAS.limit(limits=1, user_api="blas")


# jac=True: nfev counts one per request, SciPy's FD path counts 14 -> rescale maxfun so the
# `nfev > maxfun` stop fires at the same request (scipy/_lbfgsb_py.py:466-469)
_MAXFUN = SCIPY_MAXFUN // (N_PARAMS + 1)


def _minimize_start(fun, x0, maxiter):
    """``minimize(method='L-BFGS-B', jac=True)`` with the reference's options (kept as the
    independent cross-check of ``lbfgsb_steps`` in the tests)."""
    return minimize(fun=fun, x0=x0, method="L-BFGS-B", jac=True,
                    options={"maxiter": maxiter, "ftol": 1e-9, "gtol": 1e-6,
                             "maxfun": _MAXFUN})


class _StartState:
    """Per-start bookkeeping that mirrors the reference's per-start resets (:253-254)."""

    def __init__(self):
        self.n_calls = 0
        self.best_loss = np.inf


def _native_surface(cal, group_starts):
    """The surface whose request slots (dh_surface_fg_begin / _end through _native.FgChannel) a
    loop may drive directly for groups of up to group_starts starts, or None: subclassed losses
    and fg_batch overrides (their values must be used), markets without a surface, and groups too
    large for one asynchronous request take the generic _fg path."""
    if group_starts * (N_PARAMS + 1) > _native_async_max_sets():
        return None
    cls = type(cal)
    if (not isinstance(cal, DoubleHestonJumpCalibrator)
            or cls.fg_batch is not DoubleHestonJumpCalibrator.fg_batch
            or _custom_loss(cal) or not len(cal.market_options)):
        return None
    return cal._get_surface()


def _pipeline_surface(cal, n_starts, force=None):
    """The surface the pipelined loop may use, or None: one start, no native channel for half
    the starts (_native_surface; more groups hold fewer), or force False ($DHCOS_SCIPY_PIPELINE = 0 when force is
    None) keep the lockstep loop.  Round 4 measured the pipeline ahead on every bench surface once
    both loops drive prepared slots (C1 calibrate(300, 3) 5.0 vs 5.6 ms, C2 6.0 vs 6.8 ms)."""
    if force is None:
        force = {"0": False, "1": True}.get(os.environ.get("DHCOS_SCIPY_PIPELINE", ""))
    if force is False or n_starts < 2:
        return None
    return _native_surface(cal, -(-n_starts // 2))


def _pipeline_groups(surf, n_starts):
    """How many groups (request slots, each on its own stream: _slot_ctx) the pipelined loop
    splits the starts into: one per start, up to _native.FG_SLOTS.  A one-start request's 14
    records then travel in its launch's kernel arguments (libdhcos KargParams) instead of mapped
    host memory.  Measured with the native loop (round 5, calibrate(300, 3), medians of 7, one
    box): C2 4.73 ms with three groups against 4.79 ms with two, C3 8.42 / 8.76 ms; before the
    records moved to the arguments two groups were faster on C2 and C3 (4.64 / 4.75 ms,
    8.68 / 8.91 ms) and three on C1 (3.98 / 4.20 ms).  $DHCOS_SCIPY_GROUPS overrides."""
    env = os.environ.get("DHCOS_SCIPY_GROUPS", "")
    G = int(env) if env else _native.FG_SLOTS
    return max(1, min(G, n_starts, _native.FG_SLOTS))


def _slot_ctx(surf, k):
    """Request slot k's context: the surface's own for slot 0; for the others, by default, a
    context of their own on the same device (Context.slot_context: its own stream and scratch, so
    two groups' requests may run on the GPU at once); $DHCOS_SCIPY_STREAMS=0 keeps every slot on
    the surface's context (one stream)."""
    if os.environ.get("DHCOS_SCIPY_STREAMS", "") == "0":
        return surf.ctx
    return surf.ctx.slot_context(k)


def _native_async_max_sets():
    return 1024                        # dh_surface_fg_begin: 14 S <= 1024 (include/dhcos.h)


def run_starts(cal: DoubleHestonJumpCalibrator, x0s, maxiter: int, lockstep: bool = True,
               pipeline=None):
    """Run one L-BFGS-B per x0; returns [(OptimizeResult, t_done) | None] in start order.

    lockstep: every live start's function+gradient request shares one launch (S = 14 x live
    starts); otherwise the starts run one after the other.  pipeline (with lockstep, >= 2
    starts; None: by the market's size, _pipeline_surface): the starts form two groups whose
    requests alternate on the device, so one group's setulb steps run on the host while the
    other's request runs (_advance_pipelined).  A start's
    values depend only on its own x (the kernels are batch-composition invariant), so all three
    give the same results."""
    n = len(x0s)
    outcomes = [None] * n
    if n == 0:
        return outcomes
    gens = [lbfgsb_steps(x0, maxiter, _MAXFUN) for x0 in x0s]
    states = [_StartState() for _ in range(n)]
    order = [list(range(n))] if lockstep else [[s] for s in range(n)]
    surf = _pipeline_surface(cal, n, pipeline) if (lockstep and pipeline is not False) else None
    with _single_threaded_blas():
        # cal.request_trace (a list; tests): every request's (start, x, f, g) in the order the
        # starts consumed them -- recorded by the Python loops, which the native loop equals bit
        # for bit (tests/test_gpu_parity.py::test_native_loop_equals_python_loop).  The native
        # loop is loaded only where a native surface will use it.
        traced = getattr(cal, "request_trace", None) is not None
        if surf is not None:
            loop = None if traced else _scipy_loop()
            G = _pipeline_groups(surf, n)
            groups = [list(range(k, n, G)) for k in range(G)]
            cal.pipeline_groups = groups
            if loop is not None:
                _run_native(loop, cal, surf, x0s, groups, maxiter, states, outcomes)
            else:
                _advance_pipelined(cal, surf, gens, states, outcomes, groups)
        else:
            nsurf = None if traced else _native_surface(cal, max(len(g) for g in order))
            loop = _scipy_loop() if nsurf is not None else None
            if loop is not None:
                launches = 0
                for group in order:
                    # one native run per group over the group's own starts (ids remapped), so
                    # the sequential starts cost O(n) setup, not O(n^2)
                    sub = [None] * len(group)
                    _run_native(loop, cal, nsurf, [x0s[s] for s in group],
                                [list(range(len(group)))], maxiter, [states[s] for s in group],
                                sub)
                    for j, s in enumerate(group):
                        outcomes[s] = sub[j]
                    launches += cal.lockstep_launches
                cal.lockstep_launches = launches
            else:
                _advance(cal, gens, states, order, outcomes)
    cal.start_stats = [(st.n_calls, st.best_loss) for st in states]
    last = states[-1]
    cal.n_calls, cal.best_loss = last.n_calls, last.best_loss   # state after the last start
    return outcomes


def _fg(cal, X0):
    return cal.fg_batch(X0) if hasattr(cal, "fg_batch") else fg_from_losses(cal, X0)


def _fg_per_start(cal, ids, X0, gens, pending, exc=None):
    """A group request that raised (a subclass's loss): the reference runs each start in its own
    try/except (lbfgs_calibrator.py:258-317), so only a start whose own request raises is dropped.
    With ``exc`` a _StartRaised (per-point compute_loss), the starts before the raising one keep
    the losses already computed, the raising start is dropped and the evaluation goes on after it
    -- every point evaluated exactly once.  Otherwise (a loss_batch override, which evaluates the
    group at once) the group's starts are re-evaluated one at a time (a start's values do not
    depend on the batch) and the raising ones dropped.  -> the survivors' (ids, f0, G, lows)."""
    keep, rows = [], []

    def one_by_one(js):
        for j in js:
            try:
                rows.append(_fg(cal, X0[j:j + 1]))
                keep.append(ids[j])
            except _native.NativeError:
                raise
            except Exception:          # noqa: BLE001 -- reference: except -> continue
                gens[ids[j]].close()
                del pending[ids[j]]

    if not isinstance(exc, _StartRaised):
        one_by_one(range(len(ids)))
    off = 0
    while isinstance(exc, _StartRaised):
        j = off + exc.j
        if exc.j:
            _, dx = fd_request_points_many(X0[off:j])
            rows.append(_fg_rows(exc.rows, dx))
            keep.extend(ids[off:j])
        gens[ids[j]].close()
        del pending[ids[j]]
        off, exc = j + 1, None
        if off < len(ids):
            try:
                rows.append(_fg(cal, X0[off:]))
                keep.extend(ids[off:])
            except _native.NativeError:
                raise
            except _StartRaised as nxt:
                exc = nxt
            except Exception:          # noqa: BLE001 -- not the per-point path: one by one
                one_by_one(range(off, len(ids)))
    if not keep:
        return keep, None, None, None
    return (keep, np.concatenate([r[0] for r in rows]), np.concatenate([r[1] for r in rows]),
            np.concatenate([r[2] for r in rows]))


def _advance(cal, gens, states, order, outcomes):
    """run_starts' loop: one launch per lockstep request, setulb steps per start.  On a native
    market the requests go through one prepared request slot (_native.FgChannel on slot 0:
    zero-copy points in, a spin-wait on the request's event, no per-call argument marshalling),
    else through cal.fg_batch; both give the same values (fg_batch is dh_surface_fg)."""
    launches = 0
    surf = _native_surface(cal, max(len(g) for g in order)) if order else None
    chan = None if surf is None else _native.FgChannel(surf, 0, max(len(g) for g in order),
                                                       cal.spot, cal.risk_free_rate, cal.N)
    busy = False

    def fg(X0):
        nonlocal busy
        if chan is None:
            return _fg(cal, X0)
        fd_models(X0, out=chan.model_out(X0.shape[0]))
        cal.loss_evals += X0.shape[0] * (N_PARAMS + 1)
        chan.begin(X0)
        busy = True
        out = chan.end()
        busy = False
        return out

    try:
        for group in order:
            pending = {}
            for sid in group:
                pending[sid] = next(gens[sid])
            while pending:
                ids = sorted(pending)
                X0 = np.array([pending[sid] for sid in ids])   # = np.stack, ~3 us sooner
                try:
                    f0, G, lows = fg(X0)
                except _native.NativeError:
                    raise
                except Exception as exc:   # some start's loss raised: drop that start only
                    ids, f0, G, lows = _fg_per_start(cal, ids, X0, gens, pending, exc)
                    if not ids:
                        continue
                launches += 1
                _consume(states, gens, pending, outcomes, ids, f0, G, lows,
                         getattr(cal, "request_trace", None))
    finally:
        if busy:                       # unwinding with the slot's request in flight
            try:
                surf.ctx.fg_cancel(0)
            except Exception:          # noqa: BLE001 -- unwinding: the first error wins
                pass
    cal.lockstep_launches = launches


def _consume(states, gens, pending, outcomes, ids, f0, G, lows, trace=None):
    """A request's results to its starts' generators (the bookkeeping of _advance); trace (a
    list) gets each start's (start, x, f, g)."""
    for j, sid in enumerate(ids):
        if trace is not None:
            trace.append((sid, np.array(pending[sid], dtype=np.float64), float(f0[j]),
                          np.array(G[j], dtype=np.float64)))
        st = states[sid]
        st.n_calls += N_PARAMS + 1
        if lows[j] < st.best_loss:
            st.best_loss = lows[j]
        try:
            pending[sid] = gens[sid].send((f0[j], G[j]))
        except StopIteration as stop:
            outcomes[sid] = (stop.value, time.time())
            del pending[sid]
        except Exception:      # noqa: BLE001 -- reference: except -> continue
            del pending[sid]


def _advance_pipelined(cal, surf, gens, states, outcomes, groups):
    """run_starts' pipelined loop: group k (_pipeline_groups) on request slot k
    (dh_surface_fg_begin / _end).  Group k's results are consumed, its next request enqueued
    behind the other groups', then the next group's results are awaited: the host's setulb steps
    of one group overlap the device's requests of the others.  The per-start values and
    bookkeeping are _advance's."""
    n = len(gens)
    n_groups = len(groups)
    pending = {sid: next(gens[sid]) for sid in range(n)}
    inflight = [None] * n_groups
    busy = [False] * n_groups          # slot k holds a request of this loop (fg_begin .. fg_end)
    launches = 0
    # the two slots with their arguments prepared once (_native.FgChannel: the per-request host
    # path is a row copy in, one foreign call each way, three small copies out)
    chans = [_native.FgChannel(surf, k, max(1, len(groups[k])), cal.spot, cal.risk_free_rate,
                               cal.N, ctx=_slot_ctx(surf, k)) for k in range(n_groups)]

    def submit(k):
        ids = [sid for sid in groups[k] if sid in pending]
        inflight[k] = None
        if not ids:
            return
        X0 = chans[k].x_rows(len(ids))                 # the rows straight into the slot
        for j, sid in enumerate(ids):
            X0[j] = pending[sid]
        try:
            fd_models(X0, out=chans[k].model_out(len(ids)))
        except Exception:          # reference: except -> continue, for the raising start only
            keep = []
            for j, sid in enumerate(ids):
                try:
                    fd_models(X0[j:j + 1])
                    keep.append(j)
                except Exception:  # noqa: BLE001
                    gens[sid].close()
                    del pending[sid]
            if not keep:
                return
            ids, X0 = [ids[j] for j in keep], X0[keep]
            fd_models(X0, out=chans[k].model_out(len(ids)))
        cal.loss_evals += X0.shape[0] * (N_PARAMS + 1)
        chans[k].begin(X0)
        inflight[k] = ids
        busy[k] = True

    # the slots belong to the surface's context (the per-thread default context): whatever ends
    # this loop -- an error, a KeyboardInterrupt -- must leave no request in flight in them
    try:
        for k in range(n_groups):
            submit(k)
        while any(f is not None for f in inflight):
            for k in range(n_groups):
                ids = inflight[k]
                if ids is None:
                    continue
                inflight[k] = None
                f0, G, lows = chans[k].end()
                busy[k] = False
                launches += 1
                _consume(states, gens, pending, outcomes, ids, f0, G, lows,
                         getattr(cal, "request_trace", None))
                submit(k)
    finally:
        for k in range(n_groups):
            if busy[k]:
                try:
                    chans[k].ctx.fg_cancel(k)
                except Exception:      # noqa: BLE001 -- unwinding: the first error wins
                    pass
    cal.lockstep_launches = launches


_LOOP = None


def _scipy_loop():
    """The native request loop (dhcos._scipy_loop, csrc/dh_scipy_loop.cpp), or None where the
    Python loop runs: $DHCOS_NATIVE_LOOP = 0, or NumPy's error state set to raise / call on a
    floating-point error (fd_models may then raise for one start, which the Python loop drops
    alone).  The module is part of the build (make -C option-pricing-ffn-lbfgs_amd/csrc): a
    missing one is an error, not a silent fallback."""
    global _LOOP
    if os.environ.get("DHCOS_NATIVE_LOOP", "") == "0":
        return None
    if any(v in ("raise", "call") for v in np.geterr().values()):
        return None
    if _LOOP is None:
        try:
            from . import _scipy_loop as mod
        except ImportError as exc:
            raise _native.NativeError(
                "dhcos/_scipy_loop is not built; run `make -C option-pricing-ffn-lbfgs_amd/csrc` "
                "(or set DHCOS_NATIVE_LOOP=0 for the Python loop)") from exc
        _LOOP = mod
    return _LOOP


_LBFGSB_M = 10


def _lbfgsb_arrays(x0):
    """One start's setulb arrays as lbfgsb_steps allocates them (x = x0, no bounds), plus the
    float64 g the loop hands to setulb."""
    n, m = N_PARAMS, _LBFGSB_M
    return (np.array(np.asarray(x0).ravel(), dtype=np.float64), np.zeros(n, np.float64),
            np.zeros(n, np.float64), np.zeros(n, np.int32),
            np.zeros(2 * m * n + 5 * n + 11 * m * m + 8 * m, np.float64),
            np.zeros(3 * n, dtype=np.int32), np.zeros(2, dtype=np.int32),
            np.zeros(4, dtype=np.int32), np.zeros(44, dtype=np.int32), np.zeros(29, np.float64),
            np.zeros(2, dtype=np.int32), np.zeros(n, np.float64))


def _loop_consts(maxiter):
    return (_LBFGSB_M, 1e-9 / np.finfo(float).eps, 1e-6, 20, int(maxiter), _MAXFUN,
            FD_ABS_STEP, _SQRT_EPS)


def _loop_results(rows, arrs, maxiter, states, outcomes, ids):
    """The native loop's per-start rows -> _StartState counters and lbfgsb_steps' OptimizeResult
    (the same fields and message) for the starts in ids that finished."""
    for s in ids:
        state, f, g, nfev, nit, t_done, n_calls, best = rows[s]
        states[s].n_calls, states[s].best_loss = n_calls, best
        if state != 0:
            continue                                   # dropped: setulb raised (except -> continue)
        task = arrs[s][6]
        if task[0] == 4:
            warnflag = 0
        elif nfev > _MAXFUN or nit >= maxiter:
            warnflag = 1
        else:
            warnflag = 2
        msg = status_messages[task[0]] + ": " + task_messages[task[1]]
        res = OptimizeResult(fun=np.float64(f), jac=np.array(g), nfev=nfev, njev=nfev, nit=nit,
                             status=warnflag, message=msg, x=arrs[s][0], success=(warnflag == 0))
        outcomes[s] = (res, t_done)


def _run_native(loop, cal, surf, x0s, groups, maxiter, states, outcomes):
    """run_starts' request loop in native code (csrc/dh_scipy_loop.cpp): _advance_pipelined with
    several groups (each slot on its own context, _slot_ctx), _advance's lockstep loop with one;
    the same setulb calls, fd_models bits and per-start bookkeeping (tests/test_scipy_loop.py;
    tests/test_gpu_parity.py holds the two loops' calibrations equal bit for bit).  The contexts'
    request slots are held for the call."""
    arrs = [_lbfgsb_arrays(x0) for x0 in x0s]
    chans = [_native.FgChannel(surf, k, max(1, len(g)), cal.spot, cal.risk_free_rate, cal.N,
                               ctx=_slot_ctx(surf, k) if len(groups) > 1 else surf.ctx)
             for k, g in enumerate(groups)]
    dev = chans[0].loop_device()
    dev = dev[:3] + (tuple(ch.ctx.handle.value for ch in chans),) + dev[4:]
    with contextlib.ExitStack() as stack:
        for c in {id(ch.ctx): ch.ctx for ch in chans}.values():
            stack.enter_context(c._lock)
        rc, launches, evals, rows = loop.run(dev, [list(g) for g in groups],
                                             [ch.loop_slot() for ch in chans], arrs,
                                             _lbfgsb.setulb, np.exp, np.tanh,
                                             _loop_consts(maxiter))
    cal.loss_evals += evals
    cal.lockstep_launches = launches
    _native._check(rc)
    _loop_results(rows, arrs, maxiter, states, outcomes, [s for g in groups for s in g])


def run_starts_device(cal: DoubleHestonJumpCalibrator, x0s, maxiter: int):
    """run_starts on the device-resident L-BFGS-B (dh_calibrate_lbfgs): every start's requests
    and optimizer steps run on the GPU; returns [(OptimizeResult, t_done)] in start order.
    Markets whose loss is constant (an option type of '' -> 1e10, no options -> NaN) have
    nothing to optimise on the device and take the host driver, which reproduces the
    reference's result for them."""
    n = len(x0s)
    if n == 0:
        return []
    surf = cal._get_surface()
    if surf is None or len(cal.market_options) == 0:
        return run_starts(cal, x0s, maxiter)
    t0 = time.time()
    res, launches = surf.calibrate_lbfgs(np.stack([np.asarray(x, dtype=np.float64)[:N_PARAMS]
                                                   for x in x0s]),
                                         cal.spot, cal.risk_free_rate, cal.N, maxiter=maxiter,
                                         maxfun=_MAXFUN)
    outcomes = []
    for r in res:
        msg = status_messages[r.task // 1000] + ": " + task_messages[r.task % 1000]
        opt = OptimizeResult(fun=float(r.fun), jac=None, nfev=r.nfev, njev=r.nfev, nit=r.nit,
                             status=r.warnflag, message=msg, x=np.array(r.x[:]),
                             success=(r.warnflag == 0))
        outcomes.append((opt, t0 + r.t_done))
    cal.start_stats = [(r.n_calls, r.best_loss) for r in res]
    cal.n_calls, cal.best_loss = res[-1].n_calls, res[-1].best_loss   # state after the last start
    cal.loss_evals += sum(r.n_calls for r in res)
    cal.lockstep_launches = launches
    return outcomes
