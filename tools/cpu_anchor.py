#!/usr/bin/env python3
"""Anchor the CPU baseline to the reference: time the reference's own DoubleHeston.pricing(N)
(/root/reference/src/models/double_heston.py:160-192, imported read-only) and the oracle's
scalar restatement (oracle.dh_oracle.price_scalar, what bench.py's cpu_baseline times on the GPU
box) side by side on the same options, one process, in this container; write
profiles/cpu_anchor.json with the per-option times, their ratio and the CPU model.

The reference never travels to the GPU box: bench.py only reads the committed JSON (the ratio
and this container's CPU model) to state how its port-based baseline relates to the reference.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_anchor.py [--budget SECONDS_PER_LEG]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("DHCOS_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(REF, "src/models"))

from double_heston import DoubleHeston  # noqa: E402  (reference, read-only)
from oracle import dh_oracle as O       # noqa: E402

PNAMES = ["v01", "kappa1", "theta1", "sigma1", "rho1", "v02", "kappa2", "theta2",
          "sigma2", "rho2", "lambda_j", "mu_j", "sigma_j"]
GEN_LO = np.array([0.025, 1.5, 0.025, 0.2, -0.85, 0.02, 0.3, 0.025, 0.1, -0.7, 0.05, -0.08, 0.03])
GEN_HI = np.array([0.08, 4.5, 0.065, 0.5, -0.4, 0.07, 1.2, 0.07, 0.35, -0.2, 0.25, -0.01, 0.12])


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def options(n, seed=11):
    """The bench's C3 ranges: K/S in [0.8, 1.2], T in [0.1, 2], puts below the spot."""
    rs = np.random.RandomState(seed)
    prm = GEN_LO + (GEN_HI - GEN_LO) * rs.rand(13)
    K = 100.0 * rs.uniform(0.8, 1.2, n)
    T = rs.uniform(0.1, 2.0, n)
    return prm, K, T, K >= 100.0


def time_leg(fn, n_opts, budget):
    done, t0 = 0, time.perf_counter()
    while done < n_opts and (time.perf_counter() - t0 < budget or done < 8):
        fn(done)
        done += 1
    return done, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=8.0, help="seconds per (leg, N)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_anchor.json"))
    args = ap.parse_args()
    prm, K, T, call = options(4000)
    rows = []
    for N in (128, 256, 512):
        def ref(i):
            dh = DoubleHeston(S0=100.0, K=K[i], T=T[i], r=0.03,
                              option_type="C" if call[i] else "P", **dict(zip(PNAMES, prm)))
            return dh.pricing(N=N)

        def port(i):
            return O.price_scalar(prm, 100.0, K[i], T[i], 0.03, bool(call[i]), N)

        with np.errstate(all="ignore"):
            n_ref, t_ref = time_leg(ref, K.size, args.budget)
            n_port, t_port = time_leg(port, K.size, args.budget)
            m = min(n_ref, n_port, 64)
            diff = max(abs(ref(i) - port(i)) / abs(ref(i)) for i in range(m))
        rows.append({"N": N, "reference_ms_per_option": t_ref / n_ref * 1e3,
                     "port_ms_per_option": t_port / n_port * 1e3,
                     "reference_over_port_time": (t_ref / n_ref) / (t_port / n_port),
                     "options_timed": [n_ref, n_port], "max_rel_diff_first_64": diff})
        print(json.dumps(rows[-1]), flush=True)
    out = {"cpu_model": cpu_model(), "cores_used": 1, "python": platform.python_version(),
           "numpy": np.__version__,
           "what": "reference DoubleHeston.pricing(N) (double_heston.py:160-192) vs "
                   "oracle.dh_oracle.price_scalar, one process each, the same options "
                   "(K/S in [0.8, 1.2], T in [0.1, 2], puts below the spot, r = 0.03)",
           "rows": rows}
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
