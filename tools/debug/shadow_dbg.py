"""Debug: device-driver requests of the C2 iterating start whose f differs from the host path."""
import json, os, sys
import numpy as np
import torch  # noqa
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import dhcos
from dhcos.calibrator import x_to_model, feller_penalty
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
print("device", res.iterations, res.message, res.final_loss, "requests", len(tr))
X = tr[:, 3:16]
f_host, g_host, _ = cal.fg_batch(X)
K = np.array([o["strike"] for o in mk]); T = np.array([o["maturity"] for o in mk])
call = np.array([o["option_type"].upper()[0] == "C" for o in mk]); m = np.array([o["price"] for o in mk])
bad = np.flatnonzero(np.abs(tr[:, 2] - f_host) > 1e-9 * np.abs(f_host))
print("mismatching requests (device f vs host-path f):", bad[:20], len(bad))
for k in bad[:4]:
    x = X[k]
    fo, p = O.loss_surface(x, K, T, call, m, S0, r, N)
    prm = x_to_model(x[None])[0]
    print(k, "f_dev", tr[k, 2], "f_host", f_host[k], "f_oracle", fo, "feller", feller_penalty(prm[None]))
    print("   x", x.tolist())
    print("   params", prm.tolist())
    print("   g_dev", tr[k, 16:29].tolist())
    print("   g_host", g_host[k].tolist())
