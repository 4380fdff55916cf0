#!/usr/bin/env python3
"""Measure the GPU's relative price differences from the reference's pricer on the surfaces the
calibration noise ensembles are built on (VERDICT r4 "weak" 1 / "next" 4): the scale at which
make_calib_noise.py / make_calib_c2.py perturb their members' prices.

Test infrastructure, run ON THE GPU BOX:  python tests/golden/measure_price_noise.py
-> gpurun_out/gpu_price_noise.json (committed as tests/golden/gpu_price_noise.json).

For each surface -- the reference's test market (tests/test_suite.py:274-302, N = 128), the 5 x 5
synthetic surface (N = 128) and bench.py's 1,024-option C2 surface (N = 256), all with the
fixtures' own markets -- and for each of its fixture's starts x0 and 8 points around each
(x0 + N(0, 0.05) in the unconstrained coordinates, seed 5: where an optimizer's trial points go),
the GPU prices (the fast path a calibration runs, Surface.price) against
oracle.dh_oracle.price_scalar (the reference's per-option structure, bitwise its prices on the
KATs): max and RMS of |p_gpu - p_ref| / |p_ref| per point, and over the surface.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
from oracle import dh_oracle as O  # noqa: E402


def surfaces():
    with open(os.path.join(HERE, "calib.json")) as fh:
        g = json.load(fh)
    yield "test_market", g["test_market"], 100.0, 0.05, 128, \
        [s["x0"] for s in g["calibrate_seed0_starts"]]
    with open(os.path.join(HERE, "calib_noise_5x5.json")) as fh:
        g = json.load(fh)
    yield "5x5", g["market"], g["S0"], g["r"], 128, g["x0s"]
    with open(os.path.join(HERE, "calib_c2_single_start.json")) as fh:
        g = json.load(fh)
    yield "c2", g["market"], g["S0"], g["r"], g["N"], [g["x0"]]


def main():
    import torch  # noqa: F401  (one HIP runtime with the library)
    from dhcos import _native
    from dhcos.calibrator import x_to_model
    ctx = _native.default_context()
    out = {}
    rs = np.random.RandomState(5)
    for name, market, S0, r, N, x0s in surfaces():
        K = np.array([o["strike"] for o in market], dtype=np.float64)
        T = np.array([o["maturity"] for o in market], dtype=np.float64)
        call = np.array([O.is_call_type(o["option_type"]) for o in market])
        surf = _native.Surface(ctx, K, T, call)
        X = []
        for x0 in x0s:
            X.append(np.array(x0))
            X.extend(np.array(x0) + rs.normal(0, 0.05, 13) for _ in range(8))
        X = np.array(X)
        rec = np.zeros((len(X), 16))
        rec[:, :13], rec[:, 13], rec[:, 14] = x_to_model(X), S0, r
        gpu = surf.price(rec, N)
        rows = []
        for i, x in enumerate(X):
            p = O.to_params(x)
            with np.errstate(all="ignore"):
                ref = np.array([O.price_scalar(p, S0, k, t, r, c, N)
                                for k, t, c in zip(K, T, call)])
            ok = np.isfinite(ref) & (ref > 0)
            d = np.abs(gpu[i][ok] - ref[ok]) / np.abs(ref[ok])
            rows.append({"max": float(d.max()), "rms": float(np.sqrt(np.mean(d ** 2))),
                         "valid": int(ok.sum())})
            print(name, i, rows[-1], flush=True)
        out[name] = {"N": N, "options": len(market), "points": len(X),
                     "max_rel": max(r_["max"] for r_ in rows),
                     "rms_rel": float(np.sqrt(np.mean([r_["rms"] ** 2 for r_ in rows]))),
                     "per_point": rows}
        surf.close()
    out["what"] = ("GPU fast-path prices (Surface.price) vs oracle price_scalar (the reference's "
                   "per-option pricer) at each fixture start and 8 points around it: relative "
                   "differences")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "gpu_price_noise.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in out.items():
        if isinstance(v, dict):
            print(k, "max", v["max_rel"], "rms", v["rms_rel"])


if __name__ == "__main__":
    main()
