"""Phase breakdown of the device L-BFGS-B step kernel (lb_step_kernel) from s_memtime stamps in
the request trace (diagnostic build: make -C option-pricing-ffn-lbfgs_amd/csrc stamps).

Usage: python tools/lbstep_stamps.py [--config c2] [--starts 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DHCOS_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(
    ROOT, "option-pricing-ffn-lbfgs_amd", "dhcos", "libdhcos_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--starts", type=int, default=3)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    np.random.seed(0)
    x0s = np.stack([cal.get_initial_guess(s % 3) for s in range(args.starts)])
    surf.calibrate_lbfgs(x0s, S0, r, cfg["N"])                 # warm-up
    surf.ctx.set_lb_trace(1 << 16)
    res, launches = surf.calibrate_lbfgs(x0s, S0, r, cfg["N"])
    tr = surf.ctx.read_lb_trace()
    surf.ctx.set_lb_trace(0)
    keep = tr[:, 32] > 0
    sub = tr[keep][:, [32, 31, 38, 39, 33]]       # start, sidx, loads issued, loads landed, t_load
    st = tr[keep][:, 32:38]
    print(f"{args.config} {args.starts} starts: {len(st)} consumed requests, {launches} iterations")
    names = ["load state", "consume request", "state machine", "emit request", "store state"]
    for i, nm in enumerate(names):
        c = st[:, i + 1] - st[:, i]
        print(f"  {nm:16s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}  "
              f"max {c.max():8.0f} cycles")
    if (sub[:, 1:4] > 0).all():
        for i, nm in enumerate(["  kernargs/sidx", "  issue loads", "  loads landed", "  tile sums"]):
            c = sub[:, i + 1] - sub[:, i]
            print(f"  {nm:16s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}")
    life = st[:, 5] - st[:, 0]
    print(f"  lifetime median {np.median(life):8.0f}  max {life.max():8.0f}")


if __name__ == "__main__":
    main()
