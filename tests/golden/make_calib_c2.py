#!/usr/bin/env python3
"""Generate the C2-surface calibration fixtures: the reference algorithm's single-start
calibration on bench.py's 1,024-option C2 surface (32 K/S x 32 T) at N = 256.

  --start 0 (default) -> tests/golden/calib_c2_single_start.json: calibrate(300, 1) as configs[1]
      of BASELINE.json states it, from the literature guess (start 0, which draws no random
      numbers).  That start sits on the Feller kink: every member ends ABNORMAL at nit 0 after 21
      requests (round 4).
  --start 1 -> tests/golden/calib_c2_start1.json: calibrate(300, 1, x0=...) from start 1 of
      calibrate(300, 3) under np.random.seed(0) (guess type 1, a draw of the global RNG): a start
      that iterates (VERDICT r4 "missing" 3).

Test infrastructure.  The market is built as bench.py make_surface(32, 32, N=256) builds it, but
priced by the oracle (oracle/dh_oracle.py, the reference's pricer restated; its vectorised form,
within ~1e-13 of the reference): model prices at a seed-1 draw of the generator's ranges, times
(1 + N(0, 0.02)) with seed 2, calls, S0 = 100, r = 0.03.  The start comes from
golden_common.pinned_start_points (a restatement of lbfgs_calibrator.py:179-234 checked against
the reference's own draws in tests/golden/calib.json, and against the calibrator).  The losses are
the oracle's at N = 256 (oracle.price_surface: price_vec's bits over the whole market), driven by
scipy.optimize.minimize exactly as lbfgs_calibrator.py:259-269 calls it (the 2-point forward
difference SciPy forms, h = 1e-8).  Member 0 is noise-free; members 1.. multiply every price by
(1 + eps U(-1, 1)), eps = the GPU's measured relative price difference from the reference's
pricer on this surface (tests/golden/gpu_price_noise.json, measure_price_noise.py), so the ensemble
spans the outcomes that depend on last bits.

Usage:  python tests/golden/make_calib_c2.py [--start 1] [--members 8] [--procs 8]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from golden_common import ROOT, O, pinned_start_points  # noqa: E402
from make_calib_noise import (GEN_HI, GEN_LO, HISTORY, N_MAX, measured_eps,  # noqa: E402
                              member_eps, run_start)

N = 256


def surface_c2():
    S0, r = 100.0, 0.03
    kk, tt = np.meshgrid(np.linspace(0.8, 1.2, 32) * S0, np.linspace(0.1, 2.0, 32))
    K, T = kk.ravel(), tt.ravel()
    true = GEN_LO + (GEN_HI - GEN_LO) * np.random.RandomState(1).rand(13)
    model = O.price_many(true, S0, K, T, r, True, N)
    mkt = model * (1 + np.random.RandomState(2).normal(0, 0.02, K.size))
    return [{"strike": float(k), "maturity": float(t), "price": float(p), "option_type": "call"}
            for k, t, p in zip(K, T, mkt)], S0, r


def _member(args):
    market, x0, m, S0, r, eps = args
    e = member_eps("c2", m, N_MAX["c2"]) if eps is None else (0.0 if m == 0 else eps)
    return dict(run_start(market, np.array(x0), e, 7000 + m, S0=S0, r=r, N=N, surface=True),
                eps=e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=0, choices=[0, 1])
    ap.add_argument("--members", type=int, default=24)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--eps", type=float, default=None,
                    help="member noise scale (default: the measured C2 max, gpu_price_noise.json)")
    a = ap.parse_args()
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd"))
    from dhcos.calibrator import DoubleHestonJumpCalibrator   # start_points: NumPy only
    market, S0, r = surface_c2()
    x0 = pinned_start_points(DoubleHestonJumpCalibrator(S0, r, market, N=N), 3)[a.start].tolist()
    eps, eps_src = (a.eps, "--eps") if a.eps is not None else measured_eps("c2")
    eps_r, src_r = measured_eps("c2", "rms")
    with mp.get_context("fork").Pool(a.procs) as pool:
        members = pool.map(_member, [(market, x0, m, S0, r, a.eps) for m in range(a.members)])
    for m, mb in enumerate(members):
        print(m, mb, flush=True)
    funs = [mb["fun"] for mb in members]
    name = "calib_c2_single_start.json" if a.start == 0 else "calib_c2_start1.json"
    out = {"what": f"calibrate(300, 1) of the reference algorithm (oracle losses at N = 256, "
                   f"SciPy L-BFGS-B) on bench.py's C2 surface priced by the oracle, from start "
                   f"{a.start} of calibrate(300, 3) under np.random.seed(0); member 0 noise-free, "
                   f"members 1.. prices x (1 + eps U(-1, 1)), eps = {eps:.3e} ({eps_src}) for "
                   f"members 1 .. {N_MAX['c2'] - 1}"
                   + ("" if a.eps is not None else f", {eps_r:.3e} ({src_r}) after"),
           "history": HISTORY, "N": N, "market": market, "S0": S0, "r": r, "x0": x0,
           "start": a.start, "eps": eps, "eps_rms": eps_r,
           "members": members, "fun_min": min(funs), "fun_max": max(funs),
           "nit_min": min(mb["nit"] for mb in members),
           "nit_max": max(mb["nit"] for mb in members)}
    with open(os.path.join(HERE, name), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
