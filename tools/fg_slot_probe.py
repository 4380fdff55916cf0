"""Host view of one SciPy-driver request on the C1 surface (S = 2 starts): FgChannel.begin and end
back to back, fd_models, and the same loss request issued through the device-pointer call on the
context's stream and waited for (the request's round trip: launch, kernel, completion), against
the launch call alone.  (Surface.loss_dev(stream=0) means the context's stream; wait on that
stream, not on torch's null stream.)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dhcos import _native  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator, fd_models  # noqa: E402

cfg = bench.CONFIGS["c1"]
opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
surf = cal._get_surface()
ctx = surf.ctx
X0 = np.array(cal.start_points(2))
ch = _native.FgChannel(surf, 0, 2, S0, r, cfg["N"])


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


t_b, t_e = [], []
for _ in range(2000):
    t0 = time.perf_counter()
    ch.begin(X0)
    t1 = time.perf_counter()
    ch.end()
    t_b.append(t1 - t0)
    t_e.append(time.perf_counter() - t1)
print(f"FgChannel begin median {np.median(t_b) * 1e6:.2f} us, end (incl. the wait) median "
      f"{np.median(t_e) * 1e6:.2f} us")
print(f"fd_models: {per_call(lambda: fd_models(X0, out=ch.model_out(2))):.2f} us")
d = torch.from_numpy(bench.step_params(cal, 1, 2, seed=1)[0]).cuda()
sse = torch.empty(28, dtype=torch.float64, device="cuda")
bad = torch.empty(28, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()


def launch():
    surf.loss_dev(d.data_ptr(), 28, sse.data_ptr(), bad.data_ptr(), N=cfg["N"])


def round_trip():
    launch()
    ctx.synchronize()


print(f"loss request round trip (launch + kernel + wait) on the context's stream: "
      f"{per_call(round_trip, 1000):.2f} us")
print(f"launch call alone (requests queued back to back): {per_call(launch, 500):.2f} us")
ctx.synchronize()
