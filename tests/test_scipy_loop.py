"""The SciPy driver's native request loop (dhcos._scipy_loop, csrc/dh_scipy_loop.cpp) against the
Python loop it replaces (dhcos.calibrator.lbfgsb_steps + fd_models + _consume), on the CPU: the
device is replaced by Python callables that price a synthetic objective from the slot's model
buffer, and check on every request that the loop's model params are fd_models' bits.

Every per-start outcome -- x, fun, jac, nit, nfev, message, n_calls, best loss -- must be the
same bits, and the launch count the pipelined loop's (the GPU counterpart:
tests/test_gpu_parity.py::test_native_loop_equals_python_loop)."""
import numpy as np
import pytest

from dhcos import calibrator as CM

N = 13
INVALID = 1e10
TARGET = np.array([0.04, 2.0, 0.04, 0.3, -0.6, 0.05, 0.8, 0.05, 0.2, -0.4, 0.1, -0.05, 0.08])
SCALE = np.array([0.01, 1.0, 0.01, 0.1, 0.2, 0.01, 0.3, 0.01, 0.05, 0.2, 0.05, 0.02, 0.02])


def _losses(P, invalid_above=None):
    """A synthetic loss of model params [k, 13]: weighted squares plus a ripple; 1e10 (the
    reference's invalid-price loss) where P[:, 1] exceeds invalid_above.  invalid_above = "kink":
    weighted absolute values plus a smooth part instead (a kink at TARGET, where the line search
    fails; the gradient differs from point to point, so a restored one is told apart)."""
    z = (P - TARGET) / SCALE
    if isinstance(invalid_above, str):
        return np.sum(np.abs(z), axis=1) + 1e-3 * np.sum(z * z + z, axis=1)
    f = np.sum(z * z, axis=1) * 1e-3 + 1e-4 * np.sin(3.0 * P[:, 0] / SCALE[0])
    if invalid_above is not None:
        f = np.where(P[:, 1] > invalid_above, INVALID, f)
    return f


def _fg(X0, model, invalid_above=None):
    """(f [S], g [S, 13], low [S]) as dh_surface_fg_end forms them from the 14 points' losses."""
    S = X0.shape[0]
    _, dx = CM.fd_request_points_many(X0)
    f, g, low = np.empty(S), np.empty((S, N)), np.empty(S)
    for j in range(S):
        pts = np.repeat(model[0, j][None], N + 1, axis=0)
        for i in range(N):
            pts[i + 1, i] = model[1, j, i]
        fl = _losses(pts, invalid_above)
        f[j] = fl[0]
        g[j] = (fl[1:] - fl[0]) / dx[j]
        ok = np.isfinite(fl) & (fl != INVALID)
        low[j] = fl[ok].min() if ok.any() else np.inf
    return f, g, low


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def _native(x0s, groups, maxiter, invalid_above=None, setulb=None):
    loop = CM._scipy_loop()
    assert loop is not None, "dhcos._scipy_loop is built with the library (csrc/Makefile)"
    arrs = [CM._lbfgsb_arrays(x0) for x0 in x0s]
    slots = []
    for g in groups:
        sm = max(1, len(g))
        slots.append((np.empty((sm, N)), np.empty(2 * sm * N), np.empty(sm), np.empty((sm, N)),
                      np.empty(sm), [None] + [np.empty(2 * S * 10) for S in range(1, sm + 1)],
                      [None] + [np.empty(2 * S * 2) for S in range(1, sm + 1)]))
    seen = []

    def begin(k, S):
        x, m, f, g, low = slots[k][:5]
        X0 = x[:S].copy()
        want = CM.fd_models(X0)
        got = m[:2 * S * N].reshape(2, S, N)
        assert np.array_equal(_bits(got), _bits(want)), "native fd_models differs from NumPy's"
        f[:S], g[:S], low[:S] = _fg(X0, got, invalid_above)
        seen.append((k, S))

    rc, launches, evals, rows = loop.run((begin, lambda k, S: None), [list(g) for g in groups],
                                         slots, arrs, setulb or CM._lbfgsb.setulb, np.exp,
                                         np.tanh, CM._loop_consts(maxiter))
    assert rc == 0 and launches == len(seen)
    assert evals == 14 * sum(S for _, S in seen)
    states = [CM._StartState() for _ in x0s]
    outcomes = [None] * len(x0s)
    CM._loop_results(rows, arrs, maxiter, states, outcomes, [s for g in groups for s in g])
    return outcomes, states, launches


def _python(x0, maxiter, invalid_above=None):
    """One start through lbfgsb_steps with the same requests -> (result, n_calls, best, requests)."""
    gen = CM.lbfgsb_steps(x0, maxiter, CM._MAXFUN)
    x = next(gen)
    n_calls, best, req = 0, np.inf, 0
    while True:
        X0 = np.array([x])
        f, g, low = _fg(X0, CM.fd_models(X0), invalid_above)
        req += 1
        n_calls += 14
        if low[0] < best:
            best = low[0]
        try:
            x = gen.send((f[0], g[0]))
        except StopIteration as stop:
            return stop.value, n_calls, best, req


def _starts(n, seed):
    rs = np.random.RandomState(seed)
    base = CM.DoubleHestonJumpCalibrator.inverse_transform_params(
        None, dict(zip(CM.PARAM_NAMES, TARGET)))
    return [base + rs.normal(0, 0.4, N) for _ in range(n)]


def _same(res, want):
    assert np.array_equal(_bits(res.x), _bits(want.x))
    assert _bits(np.array([res.fun]))[0] == _bits(np.array([want.fun]))[0]
    assert np.array_equal(_bits(res.jac), _bits(want.jac))
    assert (res.nit, res.nfev, res.njev, res.status, res.success, res.message) == \
        (want.nit, want.nfev, want.njev, want.status, want.success, want.message)


@pytest.mark.parametrize("n,maxiter,G", [(3, 300, 2), (3, 300, 3), (3, 300, 1), (1, 300, 1),
                                         (4, 5, 2), (5, 300, 2), (6, 300, 4)])
def test_native_loop_equals_python_loop(n, maxiter, G):
    """G groups of starts on G request slots (run_starts' pipelined loop; G = 1: lockstep)."""
    x0s = _starts(n, 7 + n)
    groups = [list(range(k, n, G)) for k in range(G)]
    outcomes, states, launches = _native(x0s, groups, maxiter)
    reqs = []
    for s, x0 in enumerate(x0s):
        want, n_calls, best, req = _python(x0, maxiter)
        res, t_done = outcomes[s]
        _same(res, want)
        assert (states[s].n_calls, states[s].best_loss) == (n_calls, best)
        assert t_done > 0
        reqs.append(req)
    # one request per live start group per round: a group runs as long as its longest start
    assert launches == sum(max(reqs[s] for s in g) for g in groups if g)


def test_native_loop_invalid_losses_and_sequential_groups():
    """Points whose loss is the invalid 1e10 (excluded from the best loss), and the
    one-start-at-a-time order (lockstep=False: one single-start group per call)."""
    x0s = _starts(3, 21)
    for s, x0 in enumerate(x0s):
        outcomes, states, launches = _native([x0], [[0]], 300, invalid_above=2.5)
        want, n_calls, best, req = _python(x0, 300, invalid_above=2.5)
        _same(outcomes[0][0], want)
        assert (states[0].n_calls, states[0].best_loss, launches) == (n_calls, best, req)


def test_native_loop_line_search_failure():
    """A start on a kink: the line search fails (ABNORMAL), setulb restores the previous iterate's
    x and gradient in its arrays, and the result carries them as lbfgsb_steps' does."""
    x0 = CM.DoubleHestonJumpCalibrator.inverse_transform_params(None, dict(zip(CM.PARAM_NAMES,
                                                                               TARGET)))
    outcomes, states, launches = _native([x0, x0 + 0.01], [[0], [1]], 300, invalid_above="kink")
    for s, x in enumerate([x0, x0 + 0.01]):
        want, n_calls, best, req = _python(x, 300, invalid_above="kink")
        _same(outcomes[s][0], want)
        assert (states[s].n_calls, states[s].best_loss) == (n_calls, best)
    assert outcomes[0][0].message.startswith("ABNORMAL")


def test_native_loop_keeps_what_setulb_writes_into_g(monkeypatch):
    """setulb may write the g it receives (on a failed line search it restores the previous
    iterate's gradient there), and lbfgsb_steps keeps that array as its g.  A setulb that scales g
    after every NEW_X step makes any difference in that bookkeeping change the trajectory."""
    real = CM._lbfgsb.setulb

    def setulb(*a):
        real(*a)
        if a[11][0] == 1:                        # task NEW_X
            np.multiply(a[6], 1.0 + 2.0 ** -20, out=a[6])

    x0s = _starts(2, 13)
    outcomes, states, launches = _native(x0s, [[0], [1]], 300, setulb=setulb)
    monkeypatch.setattr(CM._lbfgsb, "setulb", setulb)
    for s, x0 in enumerate(x0s):
        want, n_calls, best, req = _python(x0, 300)
        _same(outcomes[s][0], want)


def test_native_loop_vanishing_step():
    """A coordinate where x + 1e-8 == x takes SciPy's relative step (fd_models' fallback)."""
    x0s = _starts(2, 5)
    x0s[1][11] = 3e8
    outcomes, states, launches = _native(x0s, [[0], [1]], 8)
    for s, x0 in enumerate(x0s):
        want, n_calls, best, req = _python(x0, 8)
        _same(outcomes[s][0], want)


def test_native_loop_propagates_device_errors():
    """An exception raised by the device call ends the loop and propagates."""
    loop = CM._scipy_loop()
    arrs = [CM._lbfgsb_arrays(x0) for x0 in _starts(2, 3)]
    slot = (np.empty((2, N)), np.empty(2 * 2 * N), np.empty(2), np.empty((2, N)), np.empty(2),
            [None, np.empty(20), np.empty(40)], [None, np.empty(4), np.empty(8)])

    def begin(k, S):
        raise RuntimeError("device gone")

    with pytest.raises(RuntimeError, match="device gone"):
        loop.run((begin, lambda k, S: None), [[0, 1]], [slot], arrs, CM._lbfgsb.setulb, np.exp,
                 np.tanh, CM._loop_consts(300))
    with pytest.raises(ValueError):
        loop.run((begin, lambda k, S: None), [[0, 5]], [slot], arrs, CM._lbfgsb.setulb, np.exp,
                 np.tanh, CM._loop_consts(300))


def test_native_loop_off_under_numpy_raise_mode(monkeypatch):
    """NumPy's raise / call error modes and DHCOS_NATIVE_LOOP=0 keep the Python loop (which drops
    a start whose transforms raise, alone)."""
    assert CM._scipy_loop() is not None
    with np.errstate(over="raise"):
        assert CM._scipy_loop() is None
    monkeypatch.setenv("DHCOS_NATIVE_LOOP", "0")
    assert CM._scipy_loop() is None
