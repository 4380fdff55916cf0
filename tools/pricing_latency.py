"""Latency of the reference's single-option API, DoubleHeston(...).pricing(N=128), through the
host C-ABI (dh_price_pairs): median per call over repeated calls on one context."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402

from dhcos import DoubleHeston  # noqa: E402


def main():
    dh = DoubleHeston(S0=100.0, K=100.0, T=1.0, r=0.05, v01=0.04, kappa1=2.0, theta1=0.04,
                      sigma1=0.3, rho1=-0.5, v02=0.04, kappa2=1.5, theta2=0.04, sigma2=0.2,
                      rho2=-0.3, lambda_j=0.5, mu_j=-0.05, sigma_j=0.1, option_type="call")
    for _ in range(20):
        dh.pricing()
    ts = []
    for _ in range(500):
        t0 = time.perf_counter()
        p = dh.pricing()
        ts.append(time.perf_counter() - t0)
    print(f"pricing(): median {np.median(ts) * 1e6:.1f} us, p10 {np.percentile(ts, 10) * 1e6:.1f} us "
          f"(price {p:.15f})")
    for n in (15, 1024):
        rs = np.random.RandomState(0)
        K = 100 * rs.uniform(0.8, 1.2, n)
        T = rs.uniform(0.1, 2.0, n)
        prm = np.tile([0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3, 0.5, -0.05, 0.1], (n, 1))
        DoubleHeston.price_batch(prm, 100.0, K, T, 0.05, "C")
        ts = []
        for _ in range(100):
            t0 = time.perf_counter()
            DoubleHeston.price_batch(prm, 100.0, K, T, 0.05, "C")
            ts.append(time.perf_counter() - t0)
        print(f"price_batch({n} pairs): median {np.median(ts) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
