"""Request time of C3's fused loss launch against the number of param sets (tables = sets x 100
maturity groups), to see the grid's round quantization: 1,024 resident blocks, so 40.96 sets
fill four rounds exactly.  Median of HIP-event timings over back-to-back launches.

Usage: python tools/c3_sets_sweep.py [--sets 28,36,40,41,42,44] [--reps 30]
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--sets", default="28,32,36,38,40,41,42,44,48")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--inner", type=int, default=20)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    sets = [int(s) for s in args.sets.split(",")]
    rows = np.concatenate([bench.step_params(cal, 4, cfg["starts"], seed=s)[0]
                           for s in range(1 + max(sets) // (14 * cfg["starts"]))])
    d_par = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    sse = torch.empty(max(sets), dtype=torch.float64, device=dev)
    bad = torch.empty(max(sets), dtype=torch.int32, device=dev)
    N = cfg["N"]
    res = {s: [] for s in sets}
    for s in sets:                                  # warm every grid size once
        surf.loss_dev(d_par.data_ptr(), s, sse.data_ptr(), bad.data_ptr(), N=N, stream=sp)
    torch.cuda.synchronize()
    for _ in range(args.reps):
        for s in sets:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.inner):
                surf.loss_dev(d_par.data_ptr(), s, sse.data_ptr(), bad.data_ptr(), N=N, stream=sp)
            e1.record(stream)
            torch.cuda.synchronize()
            res[s].append(e0.elapsed_time(e1) / args.inner)
    for s in sets:
        us = np.median(res[s]) * 1e3
        print(f"{args.config} sets {s:3d} tables {s * cfg['nT']:5d}"
              f"  {us:7.2f} us/request  {us / s:6.3f} us/set")


if __name__ == "__main__":
    main()
