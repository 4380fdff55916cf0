"""Request time against the number of param sets (blocks) on one surface: separates a block's
latency (few blocks per CU) from the CU's issue throughput (many blocks per CU).  Run on the GPU
box: python tools/occupancy_probe.py [c3|c2] -> one JSON line per S."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = bench.CONFIGS[cfgname]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = bench.DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    groups = len({o["maturity"] for o in opts})
    host = bench.step_params(cal, 8, 3, seed=100)          # [8, 42, 16]
    for S in [1, 2, 3, 5, 7, 10, 14, 21, 28, 35, 42]:
        rows = np.concatenate([host[i] for i in range(8)])[: S * 8].reshape(8, S, 16)
        d_p = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
        d_sse = torch.empty((8, S), dtype=torch.float64, device=dev)
        d_bad = torch.empty((8, S), dtype=torch.int32, device=dev)

        def run(j):
            surf.loss_dev(d_p[j % 8].data_ptr(), S, d_sse[j % 8].data_ptr(),
                          d_bad[j % 8].data_ptr(), N=cfg["N"], stream=stream.cuda_stream)
        for j in range(20):
            run(j)
        torch.cuda.synchronize()
        iso = bench.event_ms(run, stream, 40)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for j in range(100):
            run(j)
        e1.record(stream)
        torch.cuda.synchronize()
        b2b = e0.elapsed_time(e1) / 100
        print(json.dumps({"config": cfgname, "S": S, "blocks": S * groups,
                          "isolated_us": round(iso * 1e3, 2), "back_to_back_us": round(b2b * 1e3, 2),
                          "us_per_block_slot": round(b2b * 1e3 / max(1.0, S * groups / 1024), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
