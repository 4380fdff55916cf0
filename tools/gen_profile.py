#!/usr/bin/env python3
"""End-to-end profile of generate_synthetic_calibrations(n, as_arrays=True) by stage, on the GPU
box (where the 1M-sample run spends its time): the native legacy-NumPy draw,
the GPU pricing through the host API (params up, prices down), and the host assembly (noise,
losses, dates, columnar arrays); medians of --reps runs after one warm-up.

usage: python tools/gen_profile.py [--n 1000000] [--reps 5] [--out profiles/r03_generator_e2e.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime with libdhcos)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd"))
from dhcos import generator as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out")
    a = ap.parse_args()
    stages = {"draw": [], "price": [], "assemble": [], "total": []}
    for rep in range(a.reps + 1):
        np.random.seed(0)
        t0 = time.perf_counter()
        p, s, nz = G.draw_paths(a.n)
        t1 = time.perf_counter()
        model = G.price_grid(p, s)
        t2 = time.perf_counter()
        res = G.assemble(p, s, nz, model, None, as_arrays=True, verbose=False)
        t3 = time.perf_counter()
        del res, p, s, nz, model
        if rep:                                   # rep 0 is the warm-up
            for k, v in zip(stages, (t1 - t0, t2 - t1, t3 - t2, t3 - t0)):
                stages[k].append(v)
    # the API call itself: the draw on a worker thread, each pricing chunk as soon as it is drawn
    pipe = []
    for rep in range(a.reps + 1):
        np.random.seed(0)
        t0 = time.perf_counter()
        res = G.generate_synthetic_calibrations(a.n, None, as_arrays=True, verbose=False)
        t1 = time.perf_counter()      # before the result is freed (releasing ~0.5 GB of pages)
        del res
        if rep:
            pipe.append(t1 - t0)
    out = {k: float(np.median(v)) for k, v in stages.items()}
    out["generate_synthetic_calibrations"] = float(np.median(pipe))
    out.update(samples=a.n, options_per_sample=15, reps=a.reps, cpu=platform.processor() or None,
               call="draw_paths + price_grid (host API, N=128) + assemble(as_arrays=True), one "
                    "after the other; generate_synthetic_calibrations(n, as_arrays=True): the "
                    "API, draw and pricing overlapped")
    try:
        with open("/proc/cpuinfo") as fh:
            out["cpu"] = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
