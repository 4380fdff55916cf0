"""generate_synthetic_calibrations(1_000_000, as_arrays=True) under np.random.seed(0): the device
draw (default) and the host draw, a few calls each (the first of each warms the caches), with the
device path's own stage times (seconds from the call's start)."""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime with libdhcos)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd"))
from dhcos import generator as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for draw in ("device", "host", "device"):
    ts = []
    for _ in range(reps):
        np.random.seed(0)
        t0 = time.perf_counter()
        out = G.generate_synthetic_calibrations(n, None, as_arrays=True, verbose=False, draw=draw)
        ts.append(time.perf_counter() - t0)
        del out
        if draw == "device":
            st = G.last_device_stats
            print(f"  device stages: twister {st['twister_s'] * 1e3:.1f} walk {st['walk_s'] * 1e3:.1f} "
                  f"first chunk {st['first_chunk_s'] * 1e3:.1f} native total {st['total_s'] * 1e3:.1f} ms"
                  f"  rerun {st['ar1_segments_rerun']}", flush=True)
    print(f"{draw}: " + " ".join(f"{t * 1e3:.1f}" for t in ts) + f" ms (median {np.median(ts) * 1e3:.1f})",
          flush=True)
