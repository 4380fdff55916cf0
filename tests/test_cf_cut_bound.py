"""The CF cut's bound (csrc/dh_kernels.hip cir_log_laplace / cf_cut_passes), restated in NumPy
and checked against the oracle's characteristic function (oracle/dh_oracle.py, the reference's
double_heston.py:48-97 restated): |phi(u)| <= M(u) = prod_i E[exp(-u^2 (1 - rho_i^2) I_i / 2)]
(the CIR Laplace transform of each factor's integrated variance), M decreasing in u.  So a
table's entries past the first passing candidate are below the tail cut's delta, and the
kernels may skip evaluating them.  CPU only."""
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
    """The kernels test the bound in fp32 against log(delta / 2) - 0.01: the fp32 log-bound must
    stay within that margin of the fp64 one where the test is decided (log-bound > -1e3)."""
    rs = np.random.RandomState(9)
    worst = 0.0
    for _ in range(200):
        prm = LO + (HI - LO) * rs.rand(13)
        tau = rs.choice([0.02, 0.1, 0.5, 1.0, 2.0, 5.0])
        u = np.geomspace(1.0, 3000.0, 400)
        l64 = log_bound(prm, u, tau) + np.log(2 * 100.0 / (4.0 * (1 + u * u)))
        with np.errstate(all="ignore"):
            l32 = (log_bound(prm.astype(np.float32), u.astype(np.float32), np.float32(tau)) +
                   np.log(np.float32(2 * 100.0) / (np.float32(4.0) * (1 + u.astype(np.float32) ** 2))))
        sel = l64 > -1e3
        worst = max(worst, float(np.max(np.abs(l32[sel].astype(np.float64) - l64[sel]))))
    print("max |fp32 - fp64| log-bound", worst)
    assert worst < 1e-3
