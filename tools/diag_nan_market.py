"""Diagnostic: device L-BFGS-B request trace on a NaN-market calibration, replayed through the
CPU build of the same state machine (tests/native/liblbhost.so); prints where they part."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: F401,E402
import dhcos  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests", "golden", "calib.json")))
x0 = np.array(g["calibrate_seed0_starts"][1]["x0"], dtype=float)
mkt = [dict(o) for o in g["test_market"]]
mkt[4]["price"] = float("nan")
cal = dhcos.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
surf = cal._get_surface()
surf.ctx.set_lb_trace(1000)
res, _ = surf.calibrate_lbfgs(x0[None], 100.0, 0.05, 128, maxiter=300, maxfun=1071)
tr = surf.ctx.read_lb_trace()
surf.ctx.set_lb_trace(0)
r = res[0]
print("device:", r.nit, r.nfev, r.task, r.fun)
tr = tr[np.argsort(tr[:, 1])]
for row in tr:
    print("req", int(row[1]), "f", row[2], "x0..2", row[3:6], "g0..2", row[16:19])
lib = C.CDLL(os.path.join(ROOT, "tests", "native", "liblbhost.so"))
D = C.POINTER(C.c_double)
lib.lbh_begin.argtypes = [C.c_void_p, D]
lib.lbh_point.argtypes = [C.c_void_p, D]
lib.lbh_set_fg.argtypes = [C.c_void_p, C.c_double, D]
lib.lbh_resume.argtypes = [C.c_void_p] + [C.c_int] * 3 + [C.c_double] * 2
st = C.create_string_buffer(lib.lbh_state_size())
more = lib.lbh_begin(st, np.ascontiguousarray(x0).ctypes.data_as(D))
xe = np.empty(13)
k = 0
eps = np.finfo(float).eps
while more and k < len(tr):
    lib.lbh_point(st, xe.ctypes.data_as(D))
    same = np.array_equal(xe, tr[k, 3:16], equal_nan=True)
    print("cpu req", k, "x0..2", xe[:3], "same point" if same else "DIFFERENT")
    gg = np.ascontiguousarray(tr[k, 16:29])
    lib.lbh_set_fg(st, tr[k, 2], gg.ctypes.data_as(D))
    more = lib.lbh_resume(st, 300, 1071, 20, (1e-9 / eps) * eps, 1e-6)
    k += 1
print("cpu more", more, "after", k)
