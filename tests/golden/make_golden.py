#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ by running the REFERENCE implementation.

This script is the only place in the repository that touches /root/reference, and it only
runs in the build container (the reference never travels to the GPU box).  It imports the
reference's three modules read-only (PYTHONDONTWRITEBYTECODE=1 keeps the tree pristine),
evaluates them on seeded inputs and writes plain data files:

  kat.json            known-answer prices / CF / chi-psi values / truncation ranges
  pricing_grid.npz    ~1.6k random (param set, option, N) -> price, a, b
  calib.json          calibrator transforms, losses, one FD batch, minimize() and
                      calibrate() outcomes on the reference's own test market
  generator.json      generate_synthetic_calibrations() under np.random.seed(0)
  cf_complex.json     characteristic_function at complex phi (scalars and one array)

Reference call sites exercised (file:line in /root/reference):
  src/models/double_heston.py:48-97   characteristic_function
  src/models/double_heston.py:100-139 truncationRange
  src/models/double_heston.py:141-158 chi_k / psi_k
  src/models/double_heston.py:160-192 pricing
  src/calibration/lbfgs_calibrator.py:62-336 transforms, loss, initial guesses, calibrate
  src/data/synthetic_generator.py:25-234 generate_synthetic_calibrations
  tests/test_suite.py:196-321 pricing sanity params and the calibration test market

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--skip-calibrate]
                                                                       [--only-cf-complex]
"""
import json
import os
import sys
import time

import numpy as np

REF = os.environ.get("DHCOS_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
for sub in ("src/models", "src/calibration", "src/data"):
    sys.path.insert(0, os.path.join(REF, sub))

from double_heston import DoubleHeston  # noqa: E402  (reference)
import lbfgs_calibrator as ref_cal      # noqa: E402  (reference)
from scipy.optimize import minimize     # noqa: E402

PNAMES = ["v01", "kappa1", "theta1", "sigma1", "rho1", "v02", "kappa2", "theta2",
          "sigma2", "rho2", "lambda_j", "mu_j", "sigma_j"]
# synthetic_generator.py:75-89 ranges, in the reference's dict order
GEN_RANGES = [(0.025, 0.080), (1.5, 4.5), (0.025, 0.065), (0.20, 0.50), (-0.85, -0.40),
              (0.020, 0.070), (0.30, 1.20), (0.025, 0.070), (0.10, 0.35), (-0.70, -0.20),
              (0.05, 0.25), (-0.08, -0.01), (0.03, 0.12)]

DEMO = [0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3]  # double_heston.py:208-218


def f(x):
    return float(x)


def make(S0, K, T, r, p, typ, q=0.0):
    kw = dict(zip(PNAMES, p))
    return DoubleHeston(S0=S0, K=K, T=T, r=r, option_type=typ, q=q, **kw)


def kat():
    out = {"prices": [], "cf": [], "chipsi": [], "trunc": []}

    def add(S0, K, T, r, p, typ, N, q=0.0, tag=""):
        dh = make(S0, K, T, r, p, typ, q)
        try:
            price = f(dh.pricing(N=N))
        except Exception as e:  # record the exception class (Q3: '' -> IndexError)
            price = type(e).__name__
        a, b = dh.truncationRange()
        out["prices"].append(dict(tag=tag, S0=S0, K=K, T=T, r=r, q=q, params=list(p),
                                  option_type=typ, N=N, price=price, a=f(a), b=f(b)))

    jumps = DEMO + [0.5, -0.05, 0.10]
    nojump = DEMO + [0.0, 0.0, 0.0]
    testp = DEMO + [0.1, 0.0, 0.1]  # tests/test_suite.py:197-201
    for typ in ("C", "P"):
        add(100.0, 100.0, 1.0, 0.05, jumps, typ, 128, tag="demo_jumps")
        add(100.0, 100.0, 1.0, 0.05, nojump, typ, 128, tag="demo_nojump")
    add(100.0, 100.0, 1.0, 0.05, testp, "call", 128, tag="test_3_1_atm")
    for K in (90, 95, 100, 105, 110):
        add(100.0, float(K), 1.0, 0.05, testp, "call", 128, tag="test_3_2_strike")
    for T in (0.25, 0.5, 1.0):
        add(100.0, 100.0, T, 0.05, testp, "call", 128, tag="test_3_3_maturity")
    for (S, K, T) in ((100, 100, 0.25), (100, 100, 2.0), (100, 80, 1.0), (100, 120, 1.0)):
        add(float(S), float(K), T, 0.05, testp, "call", 128, tag="test_3_4_finite")
    add(100.0, 100.0, 1.0, 0.05, testp, "put", 128, tag="put_atm")
    # option_type normalisation quirk (Q3): first letter upper()=='C' -> call, else put
    for typ in ("c", "Call", "CALL", "p", "Put", "x", "straddle"):
        add(100.0, 95.0, 0.5, 0.05, testp, typ, 128, tag="type_" + typ)
    add(100.0, 95.0, 0.5, 0.05, testp, "", 128, tag="type_empty")
    # clamp-active truncation ranges (Q2) and deep OTM/ITM
    for K in (5.0, 50.0, 200.0, 5000.0):
        for typ in ("C", "P"):
            add(100.0, K, 0.05, 0.05, jumps, typ, 128, tag="clamp")
    # N variants incl. tiny and non-power-of-two
    for N in (1, 2, 7, 64, 100, 256, 512, 1000, 2048):
        add(100.0, 100.0, 1.0, 0.05, jumps, "C", N, tag="N_variant")
        add(100.0, 110.0, 0.5, 0.05, jumps, "P", N, tag="N_variant")
    # dividend yield only enters the CF drift (Q4)
    add(100.0, 100.0, 1.0, 0.05, jumps, "C", 128, q=0.02, tag="dividend")
    add(100.0, 100.0, 1.0, 0.05, jumps, "P", 128, q=0.02, tag="dividend")
    add(100.0, 100.0, 1.0, 0.0, jumps, "C", 128, tag="zero_rate")

    dh = make(100.0, 100.0, 1.0, 0.05, jumps, "C")
    for u in (0.0, 1e-6, 0.5, 1.0, 3.7, 10.0, 42.0, 100.0, 250.0):
        for tau in (0.1, 1.0, 2.0):
            c = complex(dh.characteristic_function(u, tau))
            out["cf"].append(dict(params=jumps, r=0.05, q=0.0, u=u, tau=tau, re=c.real, im=c.imag))
    for k in (0, 1, 2, 5, 17, 127, 511):
        for (c, d, a, b) in ((0.0, 3.0, -2.9, 3.0), (-0.1, 2.5, -3.1, 2.5),
                             (-2.0, 0.05, -2.0, 2.2)):
            out["chipsi"].append(dict(k=k, c=c, d=d, a=a, b=b,
                                      chi=f(dh.chi_k(k, c, d, a, b)),
                                      psi=f(dh.psi_k(k, c, d, a, b))))
    for T in (0.05, 0.25, 1.0, 3.0):
        for K in (50.0, 100.0, 150.0):
            d2 = make(100.0, K, T, 0.03, jumps, "C")
            a, b = d2.truncationRange()
            a5, b5 = d2.truncationRange(L=5)
            out["trunc"].append(dict(params=jumps, S0=100.0, K=K, T=T, r=0.03,
                                     a=f(a), b=f(b), a_L5=f(a5), b_L5=f(b5)))
    return out


def cf_complex():
    """characteristic_function at complex phi (double_heston.py:48-97 documents phi : complex):
    the damped-integrand shifts u - i alpha used by Fourier pricers, upper-half-plane points, and
    complex values with a zero imaginary part, as np.complex128 scalars and as one array."""
    jumps = DEMO + [0.5, -0.05, 0.10]
    other = [0.06, 3.1, 0.05, 0.45, -0.8, 0.03, 0.6, 0.06, 0.3, -0.25, 0.2, -0.06, 0.09]
    rows = []
    for p, r, q in ((jumps, 0.05, 0.0), (other, 0.03, 0.01)):
        dh = make(100.0, 100.0, 1.0, r, p, "C", q)
        for u in (0.0, 0.3, 1.0, 4.5, 20.0, 75.0):
            for im in (-1.5, -1.0, -0.5, 0.0, 0.25, 1.0):
                for tau in (0.1, 1.0, 2.5):
                    c = complex(dh.characteristic_function(np.complex128(complex(u, im)), tau))
                    rows.append(dict(params=p, r=r, q=q, re_phi=u, im_phi=im, tau=tau,
                                     re=c.real, im=c.imag))
    dh = make(100.0, 100.0, 1.0, 0.05, jumps, "C")
    z = np.array([0.5 - 1.0j, 2.0 + 0.5j, 10.0 - 0.25j, 0.0 + 0.0j])
    c = dh.characteristic_function(z, 0.7)
    return {"points": rows,
            "array": dict(params=jumps, r=0.05, q=0.0, tau=0.7, re_phi=list(map(f, z.real)),
                          im_phi=list(map(f, z.imag)), re=list(map(f, c.real)),
                          im=list(map(f, c.imag)))}


def grid(n=1600, seed=1234):
    rs = np.random.RandomState(seed)
    Ns = np.array([64, 128, 128, 128, 256, 512])
    rows = []
    for i in range(n):
        p = [rs.uniform(lo, hi) for (lo, hi) in GEN_RANGES]
        if i % 10 == 9:  # wider stress: vol-of-vol, correlations, jumps, Feller violations
            p[3] = rs.uniform(0.5, 1.2); p[8] = rs.uniform(0.3, 0.9)
            p[4] = rs.uniform(-0.99, 0.5); p[9] = rs.uniform(-0.99, 0.5)
            p[10] = rs.uniform(0.0, 2.0); p[11] = rs.uniform(-0.3, 0.2)
        S0 = float(rs.uniform(50, 150))
        K = float(S0 * rs.uniform(0.8, 1.2))
        T = float(rs.uniform(0.1, 2.0))
        r = float(rs.choice([0.0, 0.03, 0.05]))
        q = float(rs.choice([0.0, 0.0, 0.0, 0.015]))
        is_call = int(rs.rand() < 0.5)
        N = int(Ns[rs.randint(len(Ns))])
        dh = make(S0, K, T, r, p, "C" if is_call else "P", q)
        a, b = dh.truncationRange()
        rows.append(p + [S0, K, T, r, q, is_call, N, f(dh.pricing(N=N)), f(a), f(b)])
    A = np.array(rows, dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "pricing_grid.npz"),
                        params=A[:, :13], S0=A[:, 13], K=A[:, 14], T=A[:, 15], r=A[:, 16],
                        q=A[:, 17], is_call=A[:, 18].astype(np.int8),
                        N=A[:, 19].astype(np.int32), price=A[:, 20], a=A[:, 21], b=A[:, 22])


def test_market(r=0.05):
    """tests/test_suite.py:274-302: 15 clean calls at the 'true' params."""
    true = DEMO + [0.1, 0.0, 0.1]
    mkt = []
    for T in (0.25, 0.5, 1.0):
        for K in (90, 95, 100, 105, 110):
            price = f(make(100.0, K, T, r, true, "call").pricing(N=128))
            mkt.append({"strike": K, "maturity": T, "price": price, "option_type": "call"})
    return mkt


def fd_batch(cal, x0, h=1e-8):
    """Mirror of SciPy 1.15.3 2-point abs-step FD (scipy/optimize/_numdiff.py:498-511,592-596)."""
    f0 = cal.compute_loss(x0.copy())
    fs, g = [f(f0)], []
    for i in range(x0.size):
        x1 = x0.copy()
        x1[i] += h
        dx = x1[i] - x0[i]
        fi = cal.compute_loss(x1)
        fs.append(f(fi))
        g.append(f((fi - f0) / dx))
    return fs, g


def calib(skip_calibrate=False):
    out = {}
    mkt = test_market()
    out["test_market"] = mkt
    cal = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
    np.random.seed(0)
    guesses = [cal.get_initial_guess(t) for t in (0, 1, 2, 1)]
    out["guesses_seed0"] = [list(map(f, g)) for g in guesses]
    out["transform"] = [{k: f(v) for k, v in cal.transform_params(g).items()} for g in guesses]
    out["feller"] = [f(cal.compute_feller_penalty(cal.transform_params(g))) for g in guesses]
    out["loss_at_guesses"] = [f(cal.compute_loss(g)) for g in guesses]
    rs = np.random.RandomState(7)
    xs = [guesses[0] + rs.normal(0, 0.3, 13) for _ in range(6)]
    out["loss_random_x"] = [dict(x=list(map(f, x)), loss=f(cal.compute_loss(x))) for x in xs]
    fs, g = fd_batch(cal, guesses[0])
    out["fd_guess0"] = dict(x0=list(map(f, guesses[0])), f=fs, g=g)
    fs, g = fd_batch(cal, guesses[2])
    out["fd_guess2"] = dict(x0=list(map(f, guesses[2])), f=fs, g=g)
    cal.n_calls = 0
    f_inval = cal.compute_loss(np.array([5.0] * 13))  # absurd params -> invalid prices
    out["loss_absurd"] = dict(x=[5.0] * 13, loss=f(f_inval), n_calls=cal.n_calls)
    # edge markets (Q6): a zero market price -> inf ; empty market -> nan ; '' type -> 1e10
    m0 = [dict(o) for o in mkt[:3]]
    m0[1]["price"] = 0.0
    c0 = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, m0)
    me = [dict(o) for o in mkt[:3]]
    me[2]["option_type"] = ""
    ce = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, me)
    cempty = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, [])
    out["edge"] = dict(zero_price=f(c0.compute_loss(guesses[0])),
                       empty_type=f(ce.compute_loss(guesses[0])),
                       empty_market=f(cempty.compute_loss(guesses[0])))
    # test 4.1 (tests/test_suite.py:305-314): plain minimize, default gtol
    cal = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
    t = time.time()
    res = minimize(fun=cal.compute_loss, x0=cal.get_initial_guess(), method="L-BFGS-B",
                   options={"maxiter": 200, "ftol": 1e-9})
    out["test_4_1"] = dict(fun=f(res.fun), nit=int(res.nit), nfev=int(res.nfev),
                           message=str(res.message), success=bool(res.success),
                           x=list(map(f, res.x)), seconds=time.time() - t,
                           n_calls=cal.n_calls, best_loss=f(cal.best_loss))
    if skip_calibrate:
        return out
    # calibrate(300, 3) under seed 0, plus each start replayed individually
    np.random.seed(0)
    cal = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
    t = time.time()
    r = cal.calibrate(maxiter=300, multi_start=3)
    out["calibrate_seed0"] = dict(final_loss=f(r.final_loss), iterations=int(r.iterations),
                                  message=str(r.message), success=bool(r.success),
                                  parameters={k: f(v) for k, v in r.parameters.items()},
                                  model_prices=list(map(f, r.model_prices)),
                                  seconds=time.time() - t)
    np.random.seed(0)
    cal = ref_cal.DoubleHestonJumpCalibrator(100.0, 0.05, mkt)
    starts = []
    for s in range(3):
        cal.n_calls = 0
        cal.best_loss = np.inf
        x0 = cal.get_initial_guess(guess_type=s % 3)
        res = minimize(fun=cal.compute_loss, x0=x0, method="L-BFGS-B",
                       options={"maxiter": 300, "ftol": 1e-9, "gtol": 1e-6, "disp": False})
        starts.append(dict(x0=list(map(f, x0)), fun=f(res.fun), nit=int(res.nit),
                           nfev=int(res.nfev), message=str(res.message),
                           success=bool(res.success), x=list(map(f, res.x)),
                           n_calls=cal.n_calls, best_loss=f(cal.best_loss)))
    out["calibrate_seed0_starts"] = starts
    return out


def generator():
    import synthetic_generator as ref_gen  # noqa: E402  (reference)
    import contextlib
    import io
    np.random.seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        res = ref_gen.generate_synthetic_calibrations(n_samples=6, save_path="/tmp/_golden_gen.pkl")
    os.remove("/tmp/_golden_gen.pkl")
    return [dict(date=r.date, spot=f(r.spot), risk_free=f(r.risk_free),
                 parameters={k: f(v) for k, v in r.parameters.items()},
                 market_prices=list(map(f, r.market_prices)),
                 model_prices=list(map(f, r.model_prices)),
                 strikes=[f(o["strike"]) for o in r.market_options],
                 maturities=[f(o["maturity"]) for o in r.market_options],
                 final_loss=f(r.final_loss), message=r.message) for r in res]


def main():
    skip = "--skip-calibrate" in sys.argv
    t0 = time.time()
    with open(os.path.join(OUT, "cf_complex.json"), "w") as fh:
        json.dump(cf_complex(), fh, indent=1)
    if "--only-cf-complex" in sys.argv:           # round 3: the complex-phi fixture alone
        return
    with open(os.path.join(OUT, "kat.json"), "w") as fh:
        json.dump(kat(), fh, indent=1)
    print("kat done", time.time() - t0, flush=True)
    grid()
    print("grid done", time.time() - t0, flush=True)
    with open(os.path.join(OUT, "generator.json"), "w") as fh:
        json.dump(generator(), fh, indent=1)
    print("generator done", time.time() - t0, flush=True)
    with open(os.path.join(OUT, "calib.json"), "w") as fh:
        json.dump(calib(skip), fh, indent=1)
    print("calib done", time.time() - t0, flush=True)


if __name__ == "__main__":
    main()
