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
