"""A/B timing of the COS kernel modes on one surface (HIP events on one stream, interleaved).

Usage: python tools/kernel_ab.py [--config c2] [--reps 50]
Prints median kernel ms for: loss mode (one fused launch), price mode (prices to HBM, no loss
reduction) and, for reference, exact (validation) mode.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import bench  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--modes", default="loss,price,exact")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    S = 14 * cfg["starts"]
    host = bench.step_params(cal, 4, cfg["starts"], seed=0)
    d_par = torch.from_numpy(host).to(dev)
    sse = torch.empty(S, dtype=torch.float64, device=dev)
    bad = torch.empty(S, dtype=torch.int32, device=dev)
    out = torch.empty((S, surf.M), dtype=torch.float64, device=dev)
    N = cfg["N"]
    modes = {
        "loss": lambda i: surf.loss_dev(d_par[i].data_ptr(), S, sse.data_ptr(), bad.data_ptr(),
                                        N=N, stream=sp),
        "price": lambda i: surf.price_dev(d_par[i].data_ptr(), S, out.data_ptr(), N=N, stream=sp),
    }
    want = args.modes.split(",")
    modes = {k: v for k, v in modes.items() if k in want}
    times = {k: [] for k in modes}
    for rep in range(args.reps):
        for name, fn in modes.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn(rep % 4)
            e1.record(stream)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1))
    for k, v in times.items():
        print(f"{args.config} {k:6s} median {np.median(v) * 1e3:8.2f} us  min {np.min(v) * 1e3:8.2f} us")
    torch.cuda.synchronize()
    if "exact" not in want:
        return
    cal._get_surface().ctx.set_exact(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    modes["loss"](0)
    torch.cuda.synchronize()
    e0.record(stream)
    modes["loss"](0)
    e1.record(stream)
    torch.cuda.synchronize()
    print(f"{args.config} exact  {e0.elapsed_time(e1) * 1e3:8.2f} us")
    surf.ctx.set_exact(False)


if __name__ == "__main__":
    main()
