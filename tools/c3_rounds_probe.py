"""How the C3 request's time grows with its table count (the block-round tail): the C3 surface
(100 maturity groups, N = 512) under 14 x S param sets for S = 1 .. 8 starts, i.e. 1,400 ..
11,200 fused blocks over 1,024 resident slots; median isolated-request time (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402

cfg = bench.CONFIGS["c3"]
opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
surf = cal._get_surface()
st = torch.cuda.Stream()
for S in range(1, 9):
    host = bench.step_params(cal, 24, S, seed=7)
    d = torch.from_numpy(host).cuda()
    sse = torch.empty((24, 14 * S), dtype=torch.float64, device="cuda")
    bad = torch.empty((24, 14 * S), dtype=torch.int32, device="cuda")

    def run(j):
        surf.loss_dev(d[j].data_ptr(), 14 * S, sse[j].data_ptr(), bad[j].data_ptr(), N=cfg["N"],
                      stream=st.cuda_stream)
    for j in range(4):
        run(j)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        ms = bench.event_ms(lambda j: run(4 + j), st, 20)
    tables = 14 * S * 100
    print(f"starts {S}: {tables:6d} tables ({tables / 1024:5.2f} rounds of 1,024): {ms * 1e3:7.2f} us, "
          f"{ms * 1e3 / (tables / 1024):6.2f} us per round", flush=True)
