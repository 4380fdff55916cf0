"""Probe: calibrate(300, 3) with the SciPy driver on a bench surface, and the native loop's
host-time split (setulb / fd_models / begin / end / whole loop) per calibration."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from dhcos import _scipy_loop  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c1"]
opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])


N_RUNS = int(sys.argv[3]) if len(sys.argv) > 3 else 7


def runs(drv, n=N_RUNS):
    t = []
    for _ in range(n):
        cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
        np.random.seed(0)
        t0 = time.perf_counter()
        cal.calibrate(300, 3, driver=drv)
        t.append(time.perf_counter() - t0)
    return np.array(t) * 1e3, cal


for rnd in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    _scipy_loop.stats()
    t, cal = runs("scipy")
    st = np.array(_scipy_loop.stats()) / N_RUNS / 1e3
    L = cal.lockstep_launches
    print(f"round {rnd} scipy: median {np.median(t):.2f} ms, {L} launches; per calibration (us) "
          f"setulb {st[0]:.0f} models {st[1]:.0f} begin {st[2]:.0f} end {st[3]:.0f} loop {st[4]:.0f}; "
          f"per launch begin {st[2] / L:.2f} end {st[3] / L:.2f} setulb {st[0] / L:.2f} "
          f"models {st[1] / L:.2f}", flush=True)
    t, _ = runs("device")
    print(f"round {rnd} device: median {np.median(t):.2f} ms", flush=True)
