"""Timeline of one generate_synthetic_calibrations(1_000_000, as_arrays=True) call (after warm-up):
when each pricing chunk waited for the draw, ran its host-API call, and when the assembly and the
final columnar step ran.  Wrappers add ~1 us per call."""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd"))
from dhcos import _native, generator as G  # noqa: E402

EV = []
T0 = [0.0]


def mark(name, t0, t1):
    EV.append((name, (t0 - T0[0]) * 1e3, (t1 - T0[0]) * 1e3))


def wrap(owner, name):
    fn = getattr(owner, name)

    def timed(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            mark(name, t0, time.perf_counter())
    setattr(owner, name, timed)


for name in ("price_cols",):
    wrap(_native.Surface, name)
wrap(_native.GenDraw, "ready")
wrap(_native.GenDraw, "finish")
wrap(_native, "gen_assemble")
wrap(G, "assemble")
wrap(G, "trading_dates_array")
wrap(_native.pinned, "__enter__")
wrap(_native.pinned, "__exit__")
for rep in range(4):
    EV.clear()
    np.random.seed(0)
    T0[0] = time.perf_counter()
    res = G.generate_synthetic_calibrations(1_000_000, None, as_arrays=True, verbose=False)
    tot = (time.perf_counter() - T0[0]) * 1e3
    del res
    print(f"rep {rep}: total {tot:.1f} ms")
for name, a, b in sorted(EV, key=lambda e: e[1]):
    print(f"  {name:22s} {a:7.2f} -> {b:7.2f} ms ({b - a:6.2f})")
