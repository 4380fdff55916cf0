"""Phase breakdown of the COS kernel from in-kernel s_memtime stamps (diagnostic build).

Usage:  make -C option-pricing-ffn-lbfgs_amd/csrc stamps
        python tools/stamps.py [--config c2] [--mode loss|price]
Stamps per block: [0] realtime start, [1] start, [2] setup done (params, truncation range),
[3] table built (phase 1), [4] options done (phase 2, before clamp rebuilds), [5] clamp rebuilds
done, [6] loss hand-off done, [7] realtime end.  Shares are read, not absolute lengths (the
stamps themselves serialise the block).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DHCOS_LIB"] = os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd", "dhcos",
                                       "libdhcos_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--mode", default="loss")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    S = 14 * cfg["starts"]
    host = bench.step_params(cal, 2, cfg["starts"], seed=0)
    for _ in range(3):   # warm-up
        surf.loss_terms(host[0], cfg["N"])
    surf.ctx.debug_stamps(True)
    if args.mode == "loss":
        surf.loss_terms(host[1], cfg["N"])
    else:
        surf.price(host[1], cfg["N"])
    st = surf.ctx.read_stamps().astype(np.int64)
    surf.ctx.debug_stamps(False)
    st = st[st[:, 1] > 0]
    t0 = st[:, 1].min()
    span = st[:, 6].max() - t0
    rt = (st[:, 7].max() - st[:, 0].min()) / 100e6          # s_memrealtime is 100 MHz
    clk = span / rt / 1e9 if rt > 0 else float("nan")
    print(f"{args.config} {args.mode}: blocks {len(st)}  span {span} cycles  ~{rt * 1e6:.1f} us"
          f"  clock ~{clk:.2f} GHz")
    names = ["start skew", "setup", "phase1 table", "phase2 options", "phase2b clamp", "loss"]
    cols = [st[:, 1] - t0, st[:, 2] - st[:, 1], st[:, 3] - st[:, 2], st[:, 4] - st[:, 3],
            st[:, 5] - st[:, 4], st[:, 6] - st[:, 5]]
    for nm, c in zip(names, cols):
        print(f"  {nm:15s} median {np.median(c):9.0f}  p90 {np.percentile(c, 90):9.0f}  "
              f"max {c.max():9.0f} cycles")
    life = st[:, 6] - st[:, 1]
    print(f"  block lifetime  median {np.median(life):9.0f}  max {life.max():9.0f}")
    end = st[:, 6] - t0
    print(f"  block end       median {np.median(end):9.0f}  p90 {np.percentile(end, 90):9.0f}")


if __name__ == "__main__":
    main()
