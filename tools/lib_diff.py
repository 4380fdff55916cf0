"""Word-for-word comparison of two builds of libdhcos on the same inputs (GPU).

Usage:  python tools/lib_diff.py <libA.so> <libB.so>
Each library runs in its own subprocess (the ctypes binding loads one library per process) on a
fixed set of workloads -- C1/C2/C3-shaped surfaces (price and loss mode, split and fused paths),
a generator-shaped small-tile batch, paired pricing and the building-block entry points -- and
the outputs are compared bitwise.  Prints the max relative difference per workload and exits
non-zero if any differs (a kernel change meant to preserve results must show "identical"; one
that changes rounding shows the size of the change relative to each row's price scale).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(out_path):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
    from dhcos import _native
    ctx = _native.default_context()
    rs = np.random.RandomState(7)
    lo = np.array([0.025, 1.5, 0.025, 0.2, -0.85, 0.02, 0.3, 0.025, 0.1, -0.7, 0.05, -0.08, 0.03])
    hi = np.array([0.08, 4.5, 0.065, 0.5, -0.4, 0.07, 1.2, 0.07, 0.35, -0.2, 0.25, -0.01, 0.12])
    res = {}
    for name, P, nK, nT, N in [("c1", 14, 5, 3, 128), ("c2", 14, 32, 32, 256),
                               ("c3", 42, 100, 100, 512), ("n2048", 3, 64, 2, 2048)]:
        rec = np.zeros((P, 16))
        rec[:, :13] = lo + (hi - lo) * rs.rand(P, 13)
        rec[:, 13], rec[:, 14] = 100.0, 0.03
        kk, tt = np.meshgrid(np.linspace(0.8, 1.2, nK) * 100, np.linspace(0.1, 2.0, nT))
        K, T = kk.ravel(), tt.ravel()
        K[:2] = [4.0, 900.0]
        call = (np.arange(K.size) % 3) != 0
        mkt = 1.0 + rs.rand(K.size)
        surf = _native.Surface(ctx, K, T, call, mkt)
        for path in (1, 2):
            ctx.set_path(path)
            res[f"{name}_price_p{path}"] = surf.price(rec, N)
            sse, bad, pr = surf.loss_terms(rec, N, want_prices=True)
            res[f"{name}_sse_p{path}"], res[f"{name}_bad_p{path}"] = sse, bad
        ctx.set_path(0)
    # generator-shaped batch (small-tile kernel) and paired pricing
    P = 70000
    rec = np.zeros((P, 16))
    rec[:, :13] = lo + (hi - lo) * rs.rand(P, 13)
    rec[:, 13], rec[:, 14] = 100.0 * np.exp(rs.normal(0, 0.05, P)), 0.03
    Krel = np.tile(np.linspace(80.0, 120.0, 8), 4)
    T = np.repeat([0.25, 0.5, 1.0, 2.0], 8)
    g = _native.Surface(ctx, Krel, T, np.ones(32, np.int8), strike_mode=_native.STRIKE_PCT_SPOT)
    res["gen"] = g.price(rec, 128)
    res["pairs"] = ctx.price_pairs(rec[:500], 100 * rs.uniform(0.7, 1.3, 500), rs.uniform(0.05, 3, 500),
                                   rs.rand(500) < 0.5, 128)
    u = np.linspace(0.0, 60.0, 301)
    res["cf"] = ctx.cf(rec[0], u, 0.7)
    a, b = ctx.trunc_range(rec[:50], 100 * rs.uniform(0.5, 2, 50), rs.uniform(0.05, 3, 50))
    res["trunc"] = np.concatenate([a, b])
    np.savez(out_path, **{k: np.asarray(v) for k, v in res.items()})


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--run":
        run_one(sys.argv[2])
        return
    libs = sys.argv[1:3]
    outs = []
    with tempfile.TemporaryDirectory() as td:
        for i, lib in enumerate(libs):
            path = os.path.join(td, f"o{i}.npz")
            env = dict(os.environ, DHCOS_LIB=os.path.abspath(lib))
            subprocess.run([sys.executable, __file__, "--run", path], env=env, check=True)
            outs.append(dict(np.load(path)))
    bad = 0
    for k in outs[0]:
        a, b = outs[0][k], outs[1][k]
        same = np.array_equal(a.view(np.uint8), b.view(np.uint8)) if a.dtype == b.dtype else False
        with np.errstate(all="ignore"):
            # error relative to the row's price scale (deep-OTM prices of ~1e-20 carry no digits)
            a2, b2 = np.atleast_2d(a.astype(float)), np.atleast_2d(b.astype(float))
            scale = np.maximum(np.max(np.abs(a2), axis=-1, keepdims=True), 1e-300)
            rel = float(np.nanmax(np.abs(a2 - b2) / scale)) if not same else 0.0
        print(f"{k:18s} {'identical' if same else f'DIFFERS max |diff|/row scale {rel:.3e}'}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
