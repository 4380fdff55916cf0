"""calibrate()'s per-start exception semantics (lbfgs_calibrator.py:258-317: each start's minimize
runs in its own try/except, so a start whose loss raises is dropped and the others go on) under
lockstep batching, and a subclass's compute_loss being the loss that is optimised (the reference's
minimize calls self.compute_loss).  CPU only: the losses are the oracle's (test infrastructure)."""
import numpy as np
import pytest

from dhcos.calibrator import DoubleHestonJumpCalibrator, run_starts
from oracle import dh_oracle as O

N_CPU = 32           # COS terms: keeps the scalar oracle quick


class OracleLossCal(DoubleHestonJumpCalibrator):
    """compute_loss = the oracle's restatement of lbfgs_calibrator.py:118-177."""

    def compute_loss(self, x):
        self.n_calls += 1
        return O.loss(np.asarray(x), self.market_options, self.spot, self.risk_free_rate, self.N)

    def _model_prices(self, params):                 # the best start's re-pricing, on the CPU
        prm = np.array([params[n] for n in self.param_names])
        return np.array([O.price_scalar(prm, self.spot, o["strike"], o["maturity"],
                                        self.risk_free_rate, O.is_call_type(o["option_type"]),
                                        self.N) for o in self.market_options])


class RaisingCal(OracleLossCal):
    """Raises for every point of the start whose mu_j (x[11], identity transform) is near the
    type-2 guess's -0.03 (start 2); the other starts never come near it in two iterations."""

    def compute_loss(self, x):
        if x[11] > -0.0315:
            raise ValueError("injected failure")
        return super().compute_loss(x)


def _same(a, b):
    assert np.array_equal(a.x, b.x) and a.fun == b.fun and a.nit == b.nit
    assert a.message == b.message


def test_lockstep_drops_only_the_raising_start(calib_golden):
    mkt = calib_golden["test_market"]
    np.random.seed(0)
    x0s = OracleLossCal(100.0, 0.05, mkt, N=N_CPU).start_points(3)
    assert x0s[2][11] == pytest.approx(-0.03) and x0s[0][11] < -0.0315 and x0s[1][11] < -0.0315
    got = run_starts(RaisingCal(100.0, 0.05, mkt, N=N_CPU), x0s, 2, lockstep=True)
    want = run_starts(OracleLossCal(100.0, 0.05, mkt, N=N_CPU), x0s[:2], 2, lockstep=True)
    assert got[2] is None                       # the raising start is dropped (except: continue)
    for s in (0, 1):                            # the others run exactly as without it
        _same(got[s][0], want[s][0])


def test_calibrate_result_skips_the_raising_start(calib_golden):
    mkt = calib_golden["test_market"]
    np.random.seed(0)
    cal = RaisingCal(100.0, 0.05, mkt, N=N_CPU)
    x0s = cal.start_points(3)
    res = cal.calibrate(maxiter=2, x0s=x0s)
    ref = OracleLossCal(100.0, 0.05, mkt, N=N_CPU)
    outs = run_starts(ref, x0s[:2], 2)
    best = min((o[0] for o in outs), key=lambda r: r.fun)
    assert res.final_loss == best.fun and res.iterations == best.nit


def test_subclass_compute_loss_is_what_calibrate_optimises(calib_golden):
    """The losses SciPy sees are the subclass's compute_loss values: f at x0 equals it."""
    mkt = calib_golden["test_market"]
    cal = OracleLossCal(100.0, 0.05, mkt, N=N_CPU)
    x0 = cal.get_initial_guess(0)
    f, g, low = cal.fg_batch(x0[None, :])
    assert f[0] == cal.compute_loss(x0)
    assert np.all(np.isfinite(g))


class CountingRaisingCal(RaisingCal):
    """RaisingCal that records every point its compute_loss evaluates (raising ones too)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.seen = []

    def compute_loss(self, x):
        self.seen.append(np.array(x, copy=True))
        return super().compute_loss(x)


class CountingCal(OracleLossCal):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.seen = []

    def compute_loss(self, x):
        self.seen.append(np.array(x, copy=True))
        return super().compute_loss(x)


def test_raising_start_costs_no_duplicate_evaluations(calib_golden):
    """A start raising in the middle of a lockstep group: the starts before it keep the losses
    already computed and the group goes on after it, so every point is evaluated exactly once --
    the reference's per-start minimize calls (a re-evaluation had counted the earlier
    starts' points twice in the subclass's side effects).  The raising start's points up to the
    raise are evaluated once too, as the reference's would be."""
    mkt = calib_golden["test_market"]
    np.random.seed(0)
    x0s = OracleLossCal(100.0, 0.05, mkt, N=N_CPU).start_points(3)
    x0s = [x0s[0], x0s[2], x0s[1]]                  # the raising start (mu_j = -0.03) in the middle
    cal = CountingRaisingCal(100.0, 0.05, mkt, N=N_CPU)
    got = run_starts(cal, x0s, 2, lockstep=True)
    ref = CountingCal(100.0, 0.05, mkt, N=N_CPU)
    want = run_starts(ref, [x0s[0], x0s[2]], 2, lockstep=True)
    assert got[1] is None
    _same(got[0][0], want[0][0])
    _same(got[2][0], want[1][0])
    ok = [x for x in cal.seen if x[11] <= -0.0315]
    bad = [x for x in cal.seen if x[11] > -0.0315]
    assert len(ok) == len(ref.seen)                 # no point of a surviving start twice
    assert len(bad) == 1                            # the raising start: its first point only


def _guess2_loop(cal):
    """get_initial_guess(2)'s implied volatility as lbfgs_calibrator.py:211-222 forms it: the ATM
    filter and the two means over lists of the option dicts' values."""
    atm = [o for o in cal.market_options if 0.95 < o["strike"] / cal.spot < 1.05]
    iv = 0.04
    if atm:
        avg_p = np.mean([o["price"] for o in atm])
        avg_t = np.mean([o["maturity"] for o in atm])
        iv = max(0.01, min(0.1, (avg_p / cal.spot) / np.sqrt(avg_t)))
    return iv


@pytest.mark.parametrize("case", ["floats", "int_strikes", "no_atm", "edges", "mixed_prices"])
def test_atm_guess_over_arrays_equals_the_loop(case):
    """The type-2 guess filters and averages over cached arrays: the same iv bits as the
    reference's loop over the dicts, on float and int strikes, no ATM option, strikes on the
    filter's edges (0.95 S and 1.05 S are out) and int/float prices."""
    rs = np.random.RandomState({"floats": 1, "int_strikes": 2, "no_atm": 3, "edges": 4,
                                "mixed_prices": 5}[case])
    S = 100.0
    n = 500
    K = rs.uniform(70, 130, n)
    if case == "int_strikes":
        K = [int(k) for k in K]
    elif case == "no_atm":
        K = np.concatenate([rs.uniform(60, 94, n // 2), rs.uniform(106, 140, n - n // 2)])
    elif case == "edges":
        K = np.concatenate([[95.0, 105.0, 95.0000000001, 104.9999999999], K[4:]])
    T = rs.uniform(0.05, 2.0, n)
    P = rs.uniform(0.5, 30.0, n)
    prices = [int(p) if (case == "mixed_prices" and i % 3 == 0) else float(p)
              for i, p in enumerate(P)]
    opts = [{"strike": k if isinstance(k, int) else float(k), "maturity": float(t), "price": p,
             "option_type": "call"} for k, t, p in zip(K, T, prices)]
    cal = DoubleHestonJumpCalibrator(S, 0.03, opts)
    iv = _guess2_loop(cal)
    x = cal.get_initial_guess(2)
    assert x[0] == np.log(iv) and x[2] == np.log(iv)          # v1_0, theta1: log of iv
    if case == "no_atm":
        assert iv == 0.04
