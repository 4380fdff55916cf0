"""Debug: device-driver requests of the C2 iterating start where GPU prices differ from the oracle."""
import json, os, sys
import numpy as np
import torch  # noqa
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import dhcos
from dhcos import _native
from dhcos.calibrator import x_to_model
from oracle import dh_oracle as O
g = json.load(open(os.path.join(ROOT, "tests/golden/calib_c2_start1.json")))
mk, S0, r, N = g["market"], g["S0"], g["r"], g["N"]
x0 = np.array(g["x0"])
cal = dhcos.DoubleHestonJumpCalibrator(S0, r, mk, N=N)
surf = cal._get_surface()
surf.ctx.set_lb_trace(100000)
res = cal.calibrate(maxiter=300, x0s=[x0], driver="device")
tr = surf.ctx.read_lb_trace()
surf.ctx.set_lb_trace(0)
tr = tr[np.argsort(tr[:, 1])]
K = np.array([o["strike"] for o in mk]); T = np.array([o["maturity"] for o in mk])
call = np.array([o["option_type"].upper()[0] == "C" for o in mk]); m = np.array([o["price"] for o in mk])
for k in (120, 121, 122, 123):
    x = tr[k, 3:16]
    prm = x_to_model(x[None])[0]
    rec = np.zeros((1, 16)); rec[0, :13], rec[0, 13], rec[0, 14] = prm, S0, r
    pg = surf.price(rec, N)[0]
    po = O.price_surface_grouped(prm, S0, K, T, r, call, N)
    rel = np.abs(pg - po) / np.abs(po)
    j = int(np.argmax(rel))
    print(k, "f", tr[k, 2], "max rel", rel.max(), "at", j, "K", K[j], "T", T[j], pg[j], po[j],
          "n>1e-8", int(np.sum(rel > 1e-8)))
    print("   params", prm.tolist())
    ctx = surf.ctx
    ctx.set_exact(True)
    pe = surf.price(rec, N)[0]
    ctx.set_exact(False)
    ctx.set_tail_cut(False)
    pn = surf.price(rec, N)[0]
    ctx.set_tail_cut(True)
    print("   exact-mode at j", pe[j], "tail-cut off", pn[j], "scalar oracle",
          O.price_scalar(prm, S0, K[j], T[j], r, bool(call[j]), N))
