"""The CF cut's bound (csrc/dh_kernels.hip cir_log_laplace / cf_cut_passes), restated in NumPy
and checked against the oracle's characteristic function (oracle/dh_oracle.py, the reference's
double_heston.py:48-97 restated): |phi(u)| <= M(u) = prod_i E[exp(-u^2 (1 - rho_i^2) I_i / 2)]
(the CIR Laplace transform of each factor's integrated variance), M decreasing in u.  So a
table's entries past the first passing candidate are below the tail cut's delta, and the
kernels may skip evaluating them.  CPU only."""
import mpmath as mp
import numpy as np
import pytest

from oracle import dh_oracle as O

LO = np.array([0.025, 1.5, 0.025, 0.2, -0.85, 0.02, 0.3, 0.025, 0.1, -0.7, 0.05, -0.08, 0.03])
HI = np.array([0.08, 4.5, 0.065, 0.5, -0.4, 0.07, 1.2, 0.07, 0.35, -0.2, 0.25, -0.01, 0.12])


def cir_log_laplace(s, tau, v0, kap, th, sig):
    g = np.sqrt(kap * kap + 2.0 * sig * sig * s)
    e = np.exp(-(g * tau))
    den = (g + kap) * (1.0 - e) + 2.0 * g * e
    B = 2.0 * s * (1.0 - e) / den
    A = (2.0 * kap * th / (sig * sig)) * (np.log(2.0 * g) + 0.5 * (kap - g) * tau - np.log(den))
    return A - B * v0


def log_bound(prm, u, tau):
    v01, k1, t1, s1, r1, v02, k2, t2, s2, r2 = prm[:10]
    return (cir_log_laplace(0.5 * u * u * (1 - r1 * r1), tau, v01, k1, t1, s1) +
            cir_log_laplace(0.5 * u * u * (1 - r2 * r2), tau, v02, k2, t2, s2))


@pytest.mark.parametrize("seed", range(6))
def test_cf_modulus_below_laplace_bound(seed):
    rs = np.random.RandomState(seed)
    # the generator's ranges, and wider: small sigma, rho near -1/+1, long and short maturities
    lo, hi = LO.copy(), HI.copy()
    if seed >= 3:
        lo[[3, 8]], hi[[3, 8]] = 0.05, 1.5
        lo[[4, 9]], hi[[4, 9]] = -0.99, 0.99
    for _ in range(20):
        prm = lo + (hi - lo) * rs.rand(13)
        tau = rs.choice([0.02, 0.1, 0.5, 1.0, 2.0, 5.0])
        u = np.concatenate([np.linspace(1e-3, 5, 50), np.geomspace(5, 2000, 200)])
        with np.errstate(all="ignore"):
            lphi = np.log(np.abs(O.cf(u, tau, prm, 0.03)))
        lm = log_bound(prm, u, tau)
        ok = np.isfinite(lphi) & (lphi > -700.0)     # not subnormal: the oracle's modulus there
                                                     # carries the subnormal's few bits only
        assert np.all(lphi[ok] <= lm[ok] + 1e-9 * np.maximum(1.0, np.abs(lm[ok]))), (prm, tau)
        assert np.all(np.diff(lm) <= 1e-12 * np.maximum(1.0, np.abs(lm[1:])))   # decreasing


def test_fp32_bound_within_margin():
    """The kernels test the bound in fp32 (cir_log_laplace_f32, the kernel's form) against
    log(delta / 2) - 0.01: the fp32 log-bound must stay within that margin of the fp64 one where
    the test is decided (log-bound > -1e3), on the generator's ranges."""
    rs = np.random.RandomState(9)
    worst = 0.0
    for _ in range(100):
        prm = LO + (HI - LO) * rs.rand(13)
        tau = rs.choice([0.02, 0.1, 0.5, 1.0, 2.0, 5.0])
        u = np.geomspace(1.0, 3000.0, 60)
        l64 = log_bound(prm, u, tau) + np.log(2 * 100.0 / (4.0 * (1 + u * u)))
        v01, k1, t1, s1, r1, v02, k2, t2, s2, r2 = prm[:10]
        f = np.float32
        l32 = np.array([
            cir_log_laplace_f32(f(0.5) * f(uu) * f(uu) * (f(1) - f(r1) * f(r1)), tau, v01, k1, t1,
                                s1) +
            cir_log_laplace_f32(f(0.5) * f(uu) * f(uu) * (f(1) - f(r2) * f(r2)), tau, v02, k2, t2,
                                s2) +
            float(np.log(f(2 * 100.0) / (f(4.0) * (f(1) + f(uu) ** 2)))) for uu in u])
        sel = l64 > -1e3
        worst = max(worst, float(np.max(np.abs(l32[sel] - l64[sel]))))
    print("max |fp32 - fp64| log-bound", worst)
    assert worst < 1e-3


def cir_log_laplace_f32(s, tau, v0, kap, th, sig):
    """csrc/dh_kernels.hip cir_log_laplace (the cancellation-free form) in fp32, operation for
    operation (NumPy's correctly rounded exp / log stand in for the native-rate v_exp / v_log)."""
    f = np.float32
    s, tau, v0, kap, th, sig = (f(v) for v in (s, tau, v0, kap, th, sig))
    with np.errstate(all="ignore"):
        s2 = sig * sig
        g = np.sqrt(kap * kap + f(2) * s2 * s)
        gk = g + kap
        x = g * tau
        if x < 1:
            p = f(1 / 39916800)
            for c in (1 / 3628800, 1 / 362880, 1 / 40320, 1 / 5040, 1 / 720, 1 / 120, 1 / 24,
                      1 / 6, 0.5):
                p = p * -x + f(c)
            h = p * (x * x)
            om = x - h
            e = f(1) - om
        else:
            e = np.exp(-x)
            om = f(1) - e
            h = x - om
        y = (s2 * s * om) / (gk * g)
        if y < 0.125:
            q = f(1 / 9)
            for c in (1 / 8, 1 / 7, 1 / 6, 1 / 5, 0.25, 1 / 3, 0.5):
                q = q * y + f(c)
            rm1 = q * y
        else:
            rm1 = (-np.log(f(1) - y) - y) / y
        D = (h - om * rm1) / g
        A = -((f(2) * kap * th * s) / gk) * D
        B = (f(2) * s * om) / (gk * om + f(2) * g * e)
        return float(A - B * v0)


def cir_log_laplace_mp(s, tau, v0, kap, th, sig):
    """The textbook form at 60 digits: the exact value the fp32 forms are held to."""
    with mp.workdps(60):
        s, tau, v0, kap, th, sig = (mp.mpf(float(v)) for v in (s, tau, v0, kap, th, sig))
        g = mp.sqrt(kap * kap + 2 * sig * sig * s)
        e = mp.exp(-g * tau)
        den = (g + kap) * (1 - e) + 2 * g * e
        A = (2 * kap * th / (sig * sig)) * (mp.log(2 * g) + (kap - g) * tau / 2 - mp.log(den))
        return float(A - 2 * s * (1 - e) / den * v0)


def test_fp32_bound_small_vol_of_vol():
    """at small vol-of-vol the textbook A = (2 kappa theta / sigma^2)[...] scales the
    fp32 rounding of a difference of O(1) logs by 2 kappa theta / sigma^2 (off by ~3 in the log at
    sigma = 1e-4), so a candidate could pass early and the CF cut drop terms that matter.  The
    kernel's cancellation-free form stays within 1e-4 relative of the exact log-bound for sigma
    down to 1e-6 (kappa theta / sigma^2 up to ~1e11), kappa from 1e-4, maturities 0.01..5 and v0
    of 0 -- far inside the 0.01 log-margin of the test."""
    rs = np.random.RandomState(11)
    worst, n = 0.0, 0
    for _ in range(1500):
        sig = 10 ** rs.uniform(-6, np.log10(0.05)) if rs.rand() < 0.7 else 10 ** rs.uniform(-1.3, 0.3)
        kap, th = 10 ** rs.uniform(-4, 1), 10 ** rs.uniform(-3, -0.5)
        v0 = 0.0 if rs.rand() < 0.3 else 10 ** rs.uniform(-3, -0.5)
        tau, u, rho = 10 ** rs.uniform(-2, 0.7), 10 ** rs.uniform(0, 4), rs.uniform(-0.99, 0.99)
        s = 0.5 * u * u * (1 - rho * rho)
        exact = cir_log_laplace_mp(s, tau, v0, kap, th, sig)
        if exact < -1e3:                 # far past any threshold: not where the test decides
            continue
        got = cir_log_laplace_f32(s, tau, v0, kap, th, sig)
        worst = max(worst, abs(got - exact) / max(1.0, abs(exact)))
        n += 1
    print(f"max rel |fp32 - exact| log-bound over {n} points: {worst:.2e}")
    assert n > 500 and worst < 1e-4
