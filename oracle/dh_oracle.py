"""CPU oracle for the Double-Heston + Merton-jump COS pricer and the calibration objective.

TEST INFRASTRUCTURE ONLY.  This module is a plain NumPy restatement of the reference algorithm
(zenthepen/Option-Pricing-FFN-LBFGS).  It is imported by tests/, by __graft_entry__.smoke()
(as the checker) and by bench.py's ``cpu_baseline`` leg (as the timed CPU stand-in for the
reference).  The product path (option-pricing-ffn-lbfgs_amd/dhcos) never imports it and has no
CPU fallback.

Pinning: every function here is checked against golden vectors produced by running the reference
itself in the build container (tests/golden/make_golden.py -> tests/golden/*.json|npz), see
tests/test_oracle_golden.py.

Two pricers are provided:
  * ``price_scalar``  -- follows the reference's per-option structure: one complex CF evaluation per
    COS term, then a per-term chi/psi loop (double_heston.py:160-192).  This is the CPU baseline.
  * ``price_vec``     -- the same arithmetic vectorised over the COS terms (fast checker).

Parameter vector order (13): v01 kappa1 theta1 sigma1 rho1 v02 kappa2 theta2 sigma2 rho2
lambda_j mu_j sigma_j  (double_heston.py:26-27, lbfgs_calibrator.py:53-57).
"""
from __future__ import annotations

import math

import numpy as np

PARAM_NAMES = ("v1_0", "kappa1", "theta1", "sigma1", "rho1", "v2_0", "kappa2", "theta2",
               "sigma2", "rho2", "lambda_j", "mu_j", "sigma_j")
INVALID_LOSS = 1e10          # lbfgs_calibrator.py:152-158,176-177
FD_STEP = 1e-8               # scipy/_lbfgsb_py.py:290 eps default (absolute step)


# ----------------------------------------------------------------------------------------------
# characteristic function  (double_heston.py:48-97)
# ----------------------------------------------------------------------------------------------
def _heston_factor(u, tau, kappa, theta, sigma, rho):
    """One variance factor: returns (B_j, A_j) in the 'little Heston trap' form.

    beta = kappa - i rho sigma u                     (double_heston.py:64,67,70)
    d    = sqrt(beta^2 + sigma^2 u (u + i))          (:64-65)
    g    = (beta - d) / (beta + d)                   (:67-68)
    B    = (beta - d)/sigma^2 * (1 - e)/(1 - g e),  e = exp(-d tau)   (:70-71)
    A    = kappa theta / sigma^2 * ((beta - d) tau - 2 log((1 - g e)/(1 - g)))  (:85-87)
    """
    beta = kappa - rho * sigma * 1j * u
    d = np.sqrt(beta ** 2 + sigma ** 2 * u * (u + 1j))
    bm = beta - d
    g = bm / (beta + d)
    e = np.exp(-d * tau)
    B = (bm / sigma ** 2) * ((1 - e) / (1 - g * e))
    A = (kappa * theta / sigma ** 2) * (bm * tau - 2 * np.log((1 - g * e) / (1 - g)))
    return B, A


def _heston_factor_stable(u, tau, kappa, theta, sigma, rho):
    """_heston_factor's (B_j, A_j) without its cancellation at small sigma -- NOT the reference's
    operation order: a probe of how far the reference's own arithmetic is from the exact value
    (tests/test_gpu_shadow.py).  beta - d = -sigma^2 u (u + i) / (beta + d), B = -u (u + i)(1 - e)
    / D, log((1 - g e)/(1 - g)) = log(1 + w), w = (beta - d)(1 - e) / (2 d), D = (beta + d) -
    (beta - d) e: the same quantities, no division of an O(sigma^2) difference by sigma^2."""
    beta = kappa - rho * sigma * 1j * u
    uu = u * (u + 1j)
    d = np.sqrt(beta ** 2 + sigma ** 2 * uu)
    bp = beta + d
    c = uu / bp                                   # -(beta - d) / sigma^2
    bm = -c * sigma ** 2
    e = np.exp(-d * tau)
    D = bp - bm * e
    B = -uu * (1 - e) / D
    w = bm * (1 - e) / (2 * d)
    logq = 0.5 * np.log1p(2 * w.real + (w.real ** 2 + w.imag ** 2)) + \
        1j * np.arctan2(w.imag, 1 + w.real)
    A = kappa * theta * (-c * tau - 2 * logq / sigma ** 2)
    return B, A


def cf(u, tau, prm, r, q=0.0, stable=False):
    """phi(u) = exp(A + B1 v01 + B2 v02) * phi_jump(u)   (double_heston.py:82-96).

    ``u`` may be a scalar or an ndarray; the drift term carries the jump compensator
    lambda (exp(mu + sigma_j^2/2) - 1) and no log(S0) term.  stable: the factors in the
    cancellation-free form (_heston_factor_stable; a probe, not the reference's arithmetic).
    """
    v01, k1, t1, s1, r1, v02, k2, t2, s2, r2, lam, muj, sj = prm
    hf = _heston_factor_stable if stable else _heston_factor
    B1, A1 = hf(u, tau, k1, t1, s1, r1)
    B2, A2 = hf(u, tau, k2, t2, s2, r2)
    comp = np.exp(muj + 0.5 * sj ** 2) - 1
    A = (r - q - lam * comp) * 1j * u * tau
    A = A + A1
    A = A + A2
    jump = np.exp(lam * tau * (np.exp(1j * u * muj - 0.5 * sj ** 2 * u ** 2) - 1))
    return np.exp(A + B1 * v01 + B2 * v02) * jump


# ----------------------------------------------------------------------------------------------
# truncation range (double_heston.py:100-139)
# ----------------------------------------------------------------------------------------------
def _factor_cumulants(T, r, v0, kap, vbar, eta, rho):
    """Per-factor c1, c2.  Q1: each factor adds r*T to c1 (double_heston.py:107, used twice)."""
    ekt = np.exp(-kap * T)
    c1 = r * T + (1 - ekt) * (vbar - v0) / (2 * kap) - vbar * T / 2
    c2 = 1 / (8 * np.power(kap, 3)) * (
        eta * T * kap * ekt * (v0 - vbar) * (8 * kap * rho - 4 * eta)
        + kap * rho * eta * (1 - ekt) * (16 * vbar - 8 * v0)
        + 2 * vbar * kap * T * (-4 * kap * rho * eta + np.power(eta, 2) + 4 * np.power(kap, 2))
        + np.power(eta, 2) * ((vbar - 2 * v0) * np.exp(-2 * kap * T) + vbar * (6 * ekt - 7) + 2 * v0)
        + 8 * np.power(kap, 2) * (v0 - vbar) * (1 - ekt))
    return c1, c2


def trunc_range(prm, S0, K, T, r, L=10.0):
    """[a, b] = c1 -/+ L sqrt|c2|, then widened to contain log(K/S0) -/+ 0.1 (Q2, :131-137)."""
    v01, k1, t1, s1, r1, v02, k2, t2, s2, r2, lam, muj, sj = prm
    c1a, c2a = _factor_cumulants(T, r, v01, k1, t1, s1, r1)
    c1b, c2b = _factor_cumulants(T, r, v02, k2, t2, s2, r2)
    c1 = c1a + c1b + lam * T * muj
    c2 = c2a + c2b + lam * T * (sj ** 2 + muj ** 2)
    half = L * np.sqrt(np.abs(c2))
    a, b = c1 - half, c1 + half
    x = np.log(K / S0)
    return min(a, x - 0.1), max(b, x + 0.1)


# ----------------------------------------------------------------------------------------------
# cosine payoff coefficients (double_heston.py:141-158)
# ----------------------------------------------------------------------------------------------
def chi(k, c, d, a, b):
    """Cosine coefficient of e^y on [c, d]; k == 0 -> e^d - e^c."""
    if k == 0:
        return np.exp(d) - np.exp(c)
    w = k * np.pi / (b - a)
    ed, ec = np.exp(d), np.exp(c)
    s = np.cos(w * (d - a)) * ed - np.cos(w * (c - a)) * ec
    s = s + w * np.sin(w * (d - a)) * ed
    s = s - w * np.sin(w * (c - a)) * ec
    return (1.0 / (1 + w ** 2)) * s


def psi(k, c, d, a, b):
    """Cosine coefficient of 1 on [c, d]; k == 0 -> d - c."""
    if k == 0:
        return d - c
    w = k * np.pi / (b - a)
    return (1.0 / w) * (np.sin(w * (d - a)) - np.sin(w * (c - a)))


def is_call_type(option_type: str) -> bool:
    """Q3: first character upper-cased == 'C' is a call, anything else a put; '' raises."""
    return option_type.upper()[0] == "C"


# ----------------------------------------------------------------------------------------------
# COS price
# ----------------------------------------------------------------------------------------------
def price_scalar(prm, S0, K, T, r, is_call, N=128, q=0.0):
    """Per-option scalar-structured COS price (mirrors double_heston.py:160-192 step by step)."""
    xK = np.log(K / S0)
    a, b = trunc_range(prm, S0, K, T, r)
    ks = np.arange(N)
    us = ks * np.pi / (b - a)
    phis = np.array([cf(u, T, prm, r, q) for u in us])
    V = np.zeros(N)
    scale = 2.0 / (b - a)
    for k in range(N):
        if is_call:
            V[k] = scale * (S0 * chi(k, xK, b, a, b) - K * psi(k, xK, b, a, b))
        else:
            V[k] = scale * (K * psi(k, a, xK, a, b) - S0 * chi(k, a, xK, a, b))
    terms = np.real(phis * np.exp(-1j * us * a)) * V
    terms[0] *= 0.5
    return np.exp(-r * T) * np.sum(terms)


def price_vec(prm, S0, K, T, r, is_call, N=128, q=0.0):
    """Same arithmetic as price_scalar, vectorised over the N COS terms."""
    xK = np.log(K / S0)
    a, b = trunc_range(prm, S0, K, T, r)
    k = np.arange(N, dtype=np.float64)
    u = k * np.pi / (b - a)
    phi = cf(u, T, prm, r, q)
    c, d = (xK, b) if is_call else (a, xK)
    ed, ec = np.exp(d), np.exp(c)
    with np.errstate(divide="ignore", invalid="ignore"):
        cd, cc = np.cos(u * (d - a)), np.cos(u * (c - a))
        sd, sc = np.sin(u * (d - a)), np.sin(u * (c - a))
        ch = (1.0 / (1 + u ** 2)) * (cd * ed - cc * ec + u * sd * ed - u * sc * ec)
        ps = (1.0 / u) * (sd - sc)
    ch[0] = ed - ec
    ps[0] = d - c
    if is_call:
        V = (2.0 / (b - a)) * (S0 * ch - K * ps)
    else:
        V = (2.0 / (b - a)) * (K * ps - S0 * ch)
    terms = np.real(phi * np.exp(-1j * u * a)) * V
    terms[0] *= 0.5
    return np.exp(-r * T) * np.sum(terms)


def price_surface(prm, S0, K, T, r, is_call, N=128, q=0.0):
    """price_vec for every option of a surface under one parameter set, as [M, N] arrays (the
    fixture generators' fast checker for 1,024-option calibrations): per option the same
    expressions as price_vec, broadcast over the options (tests/test_oracle_golden.py holds it
    to price_vec at 1e-13)."""
    K = np.asarray(K, dtype=np.float64).reshape(-1)
    T = np.asarray(T, dtype=np.float64).reshape(-1)
    call = np.broadcast_to(np.asarray(is_call, dtype=bool), K.shape)
    xK = np.log(K / S0)
    v01, k1, t1, s1, r1, v02, k2, t2, s2, r2, lam, muj, sj = prm
    c1a, c2a = _factor_cumulants(T, r, v01, k1, t1, s1, r1)       # trunc_range, per option
    c1b, c2b = _factor_cumulants(T, r, v02, k2, t2, s2, r2)
    c1 = c1a + c1b + lam * T * muj
    c2 = c2a + c2b + lam * T * (sj ** 2 + muj ** 2)
    half = 10.0 * np.sqrt(np.abs(c2))
    a = np.minimum(c1 - half, xK - 0.1)
    b = np.maximum(c1 + half, xK + 0.1)
    k = np.arange(N, dtype=np.float64)[None, :]
    u = k * np.pi / (b - a)[:, None]
    phi = cf(u, T[:, None], prm, r, q)
    c = np.where(call, xK, a)[:, None]
    d = np.where(call, b, xK)[:, None]
    A = a[:, None]
    ed, ec = np.exp(d), np.exp(c)
    with np.errstate(divide="ignore", invalid="ignore"):
        cd, cc = np.cos(u * (d - A)), np.cos(u * (c - A))
        sd, sc = np.sin(u * (d - A)), np.sin(u * (c - A))
        ch = (1.0 / (1 + u ** 2)) * (cd * ed - cc * ec + u * sd * ed - u * sc * ec)
        ps = (1.0 / u) * (sd - sc)
    ch[:, 0] = (ed - ec)[:, 0]
    ps[:, 0] = (d - c)[:, 0]
    scale = (2.0 / (b - a))[:, None]
    Kc = K[:, None]
    V = np.where(call[:, None], scale * (S0 * ch - Kc * ps), scale * (Kc * ps - S0 * ch))
    terms = np.real(phi * np.exp(-1j * u * A)) * V
    terms[:, 0] *= 0.5
    return np.exp(-r * T) * np.sum(terms, axis=1)


def price_surface_grouped(prm, S0, K, T, r, is_call, N=128, q=0.0, stable=False):
    """price_surface with the characteristic function evaluated once per distinct (T, a, b) --
    the reference evaluates it per option (double_heston.py:168), on the same u_k = k pi / (b - a)
    and tau = T for every option of such a group, so the values are the same; everything per
    option (the range, chi / psi, V, the sum) is price_surface's expressions.  The trajectory-
    shadowing tests' checker at 10,000 options x N = 512 (tests/test_gpu_shadow.py;
    tests/test_oracle_golden.py holds it to price_surface).  stable: the CF in the
    cancellation-free form (cf(stable=True)), the exact-value probe of the shadowing tests."""
    K = np.asarray(K, dtype=np.float64).reshape(-1)
    T = np.asarray(T, dtype=np.float64).reshape(-1)
    call = np.broadcast_to(np.asarray(is_call, dtype=bool), K.shape)
    xK = np.log(K / S0)
    v01, k1, t1, s1, r1, v02, k2, t2, s2, r2, lam, muj, sj = prm
    c1a, c2a = _factor_cumulants(T, r, v01, k1, t1, s1, r1)       # trunc_range, per option
    c1b, c2b = _factor_cumulants(T, r, v02, k2, t2, s2, r2)
    c1 = c1a + c1b + lam * T * muj
    c2 = c2a + c2b + lam * T * (sj ** 2 + muj ** 2)
    half = 10.0 * np.sqrt(np.abs(c2))
    a = np.minimum(c1 - half, xK - 0.1)
    b = np.maximum(c1 + half, xK + 0.1)
    k = np.arange(N, dtype=np.float64)[None, :]
    key = np.stack([T, a, b], axis=1)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    ug = k * np.pi / (uniq[:, 2] - uniq[:, 1])[:, None]
    phi_g = cf(ug, uniq[:, 0][:, None], prm, r, q, stable=stable)
    A_g = uniq[:, 1][:, None]
    rot_g = phi_g * np.exp(-1j * ug * A_g)                        # phi(u_k) e^{-i u_k a} per group
    u = ug[inv]
    c = np.where(call, xK, a)[:, None]
    d = np.where(call, b, xK)[:, None]
    A = a[:, None]
    ed, ec = np.exp(d), np.exp(c)
    with np.errstate(divide="ignore", invalid="ignore"):
        cd, cc = np.cos(u * (d - A)), np.cos(u * (c - A))
        sd, sc = np.sin(u * (d - A)), np.sin(u * (c - A))
        ch = (1.0 / (1 + u ** 2)) * (cd * ed - cc * ec + u * sd * ed - u * sc * ec)
        ps = (1.0 / u) * (sd - sc)
    ch[:, 0] = (ed - ec)[:, 0]
    ps[:, 0] = (d - c)[:, 0]
    scale = (2.0 / (b - a))[:, None]
    Kc = K[:, None]
    V = np.where(call[:, None], scale * (S0 * ch - Kc * ps), scale * (Kc * ps - S0 * ch))
    terms = np.real(rot_g[inv]) * V
    terms[:, 0] *= 0.5
    return np.exp(-r * T) * np.sum(terms, axis=1)


def loss_surface(x, K, T, is_call, mkt, spot, r, N=128):
    """compute_loss (lbfgs_calibrator.py:118-177) on a surface through price_surface_grouped:
    (loss, prices); 1e10 on any NaN / inf / <= 0 price (Q5)."""
    p = to_params(x)
    with np.errstate(all="ignore"):
        model = price_surface_grouped(p, spot, K, T, r, is_call, N)
        if not np.all(np.isfinite(model)) or np.any(model <= 0):
            return INVALID_LOSS, model
        rel = (model - mkt) / mkt
        return np.mean(rel ** 2) + feller(p), model


def price_many(params, S0, K, T, r, is_call, N=128, q=0.0, scalar=False):
    """Loop helper: arrays broadcast over options; returns an ndarray of prices."""
    params = np.atleast_2d(np.asarray(params, dtype=np.float64))
    n = max(len(params), np.size(K))
    bc = lambda v: np.broadcast_to(np.asarray(v, dtype=np.float64), (n,))  # noqa: E731
    S0, K, T, r, q = bc(S0), bc(K), bc(T), bc(r), bc(q)
    ic = np.broadcast_to(np.asarray(is_call, dtype=bool), (n,))
    Ns = np.broadcast_to(np.asarray(N, dtype=np.int64), (n,))
    P = np.broadcast_to(params, (n, 13)) if len(params) == 1 else params
    fn = price_scalar if scalar else price_vec
    with np.errstate(all="ignore"):
        return np.array([fn(P[i], S0[i], K[i], T[i], r[i], bool(ic[i]), int(Ns[i]), q[i])
                         for i in range(n)], dtype=np.float64)


# ----------------------------------------------------------------------------------------------
# calibration objective (lbfgs_calibrator.py:62-177) and SciPy's forward-difference batch
# ----------------------------------------------------------------------------------------------
_EXP_IDX = (0, 1, 2, 3, 5, 6, 7, 8, 10, 12)
_TANH_IDX = (4, 9)


def to_params(x):
    """x (unconstrained) -> 13 model params: exp / tanh / identity (lbfgs_calibrator.py:62-87)."""
    x = np.asarray(x, dtype=np.float64)
    p = np.empty(13)
    for i in _EXP_IDX:
        p[i] = np.exp(x[i])
    for i in _TANH_IDX:
        p[i] = np.tanh(x[i])
    p[11] = x[11]
    return p


def from_params(p):
    """Inverse transform with rho clipped to +-0.999 (lbfgs_calibrator.py:89-109)."""
    x = np.empty(13)
    for i in _EXP_IDX:
        x[i] = np.log(p[i])
    for i in _TANH_IDX:
        x[i] = np.arctanh(np.clip(p[i], -0.999, 0.999))
    x[11] = p[11]
    return x


def feller(p):
    """1000 * (max(0, s1^2 - 2 k1 t1) + max(0, s2^2 - 2 k2 t2))  (lbfgs_calibrator.py:111-116)."""
    return 1000.0 * (max(0, p[3] ** 2 - 2 * p[1] * p[2]) + max(0, p[8] ** 2 - 2 * p[6] * p[7]))


def loss(x, market, spot, r, N=128, scalar=False):
    """compute_loss semantics: 1e10 on any NaN/inf/<=0 price or bad option_type (Q5)."""
    p = to_params(x)
    mkt = np.array([o["price"] for o in market], dtype=np.float64)
    model = []
    with np.errstate(all="ignore"):
        for o in market:
            try:
                call = is_call_type(o["option_type"])
            except Exception:
                return INVALID_LOSS
            fn = price_scalar if scalar else price_vec
            v = fn(p, spot, o["strike"], o["maturity"], r, call, N)
            if np.isnan(v) or np.isinf(v) or v <= 0:
                return INVALID_LOSS
            model.append(v)
        rel = (np.array(model) - mkt) / mkt
        return np.mean(rel ** 2) + feller(p)


def fd_points(x0, h=FD_STEP):
    """The 14 points SciPy 1.15.3 evaluates per function+gradient request for jac=None:
    x0, then x0 + h e_i with dx_i = (x0_i + h) - x0_i recomputed (scipy/_numdiff.py:498-511,
    592-596); zero dx falls back to the relative step sqrt(eps)*sign*max(1,|x|)."""
    x0 = np.asarray(x0, dtype=np.float64)
    sign = (x0 >= 0).astype(float) * 2 - 1
    hv = np.full(x0.shape, h)
    dx = (x0 + hv) - x0
    hv = np.where(dx == 0, np.sqrt(np.finfo(float).eps) * sign * np.maximum(1.0, np.abs(x0)), hv)
    X = np.repeat(x0[None, :], x0.size + 1, axis=0)
    dxs = np.empty(x0.size)
    for i in range(x0.size):
        X[1 + i, i] += hv[i]
        dxs[i] = X[1 + i, i] - x0[i]
    return X, dxs


def fd_grad(fvals, dxs):
    f0 = fvals[0]
    return np.array([(fvals[1 + i] - f0) / dxs[i] for i in range(len(dxs))])


if __name__ == "__main__":  # tiny self-check against the survey KAT (double_heston.py demo)
    prm = [0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3, 0.5, -0.05, 0.10]
    print(price_scalar(prm, 100.0, 100.0, 1.0, 0.05, True), price_vec(prm, 100.0, 100.0, 1.0, 0.05, True),
          math.nan)
