"""The generator's native host draw (dh_gen_draw: NumPy's legacy MT19937 / uniform / polar gauss
restated in C++) against NumPy itself and against the reference's own output.  CPU only: the
function is host code in libdhcos.so and needs no device.

Bar: bit-identical draws and an identical continuation of the global np.random stream."""
import numpy as np
import pytest

from dhcos import generator as G


# n >= 4096 takes the three-pass draw (dh_gen_rng.cpp), n > 65536 crosses one of its chunks
@pytest.mark.parametrize("seed,n,pre", [(0, 3000, 0), (7, 1, 1), (123, 257, 3), (99, 0, 1),
                                        (5, 4096, 0), (11, 66000, 1), (13, 5000, 2)])
def test_native_draw_equals_numpy_loop(seed, n, pre):
    """pre = scalar normals drawn first, so the stream starts with / without a cached gauss."""
    np.random.seed(seed)
    for _ in range(pre):
        np.random.normal()
    want = G.draw_paths_numpy(n)
    after_want = np.random.random(7)
    np.random.seed(seed)
    for _ in range(pre):
        np.random.normal()
    got = G.draw_paths(n)
    after_got = np.random.random(7)
    for a, b in zip(got, want):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert np.array_equal(after_got, after_want)


def test_native_draw_reproduces_reference_samples(gen_golden):
    """np.random.seed(0); generate_synthetic_calibrations(6) in the reference: its parameters and
    spots, and its market prices formed from its own model prices and our noise draws."""
    np.random.seed(0)
    params, spots, noise = G.draw_paths(len(gen_golden))
    for i, w in enumerate(gen_golden):
        assert list(params[i]) == list(w["parameters"].values())
        assert spots[i] == w["spot"]
        model = np.array(w["model_prices"])
        assert np.array_equal(model + noise[i] * model, np.array(w["market_prices"]))


def test_native_draw_rejects_bad_arguments():
    import ctypes as C
    from dhcos import _native
    lib = _native.load()
    key = np.zeros(624, dtype=np.uint32)
    pos, hg, cg = C.c_int32(625), C.c_int32(0), C.c_double(0.0)
    lo, hi = np.zeros(13), np.ones(13)
    out = [np.empty((2, 13)), np.empty(2), np.empty((2, 15))]
    args = [key.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(pos), C.byref(hg), C.byref(cg), 2,
            _native._ptr(lo), _native._ptr(hi), 15, 0.9, 100.0, 0.0, 0.01, 0.02] + \
        [_native._ptr(a) for a in out]
    assert lib.dh_gen_draw(*args) == -1          # mt_pos outside [0, 624]
    pos.value = 624
    args[4] = -1
    assert lib.dh_gen_draw(*args) == -1          # negative sample count


@pytest.mark.parametrize("seed,n,pre", [(0, 0, 0), (7, 1, 1), (5, 4096, 0), (11, 140000, 1)])
def test_progress_draw_equals_draw(seed, n, pre):
    """dh_gen_draw_progress on its worker thread (_native.GenDraw, what
    generate_synthetic_calibrations overlaps with the GPU pricing): the same rows, the same
    continuation of np.random, and rows published only once complete (read at each ready())."""
    np.random.seed(seed)
    for _ in range(pre):
        np.random.normal()
    want = G.draw_paths(n)
    after_want = np.random.random(7)
    np.random.seed(seed)
    for _ in range(pre):
        np.random.normal()
    d = G.draw_paths_async(n)
    for e in range(0, n + 1, 65536):
        d.ready(e)                                   # rows < e final from here on
        assert np.array_equal(d.params[:e], want[0][:e]) and np.array_equal(d.spots[:e], want[1][:e])
        assert np.array_equal(d.noise[:e], want[2][:e])
    got = d.finish()
    after_got = np.random.random(7)
    for a, b in zip(got, want):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert np.array_equal(after_got, after_want)


def test_progress_draw_requires_counter():
    import ctypes as C
    from dhcos import _native
    lib = _native.load()
    np.random.seed(0)
    key = np.ascontiguousarray(np.random.get_state()[1], dtype=np.uint32)
    pos, hg, cg = C.c_int32(624), C.c_int32(0), C.c_double(0.0)
    lo, hi = np.zeros(13), np.ones(13)
    out = [np.empty((2, 13)), np.empty(2), np.empty((2, 15))]
    args = [key.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(pos), C.byref(hg), C.byref(cg), 2,
            _native._ptr(lo), _native._ptr(hi), 15, 0.9, 100.0, 0.0, 0.01, 0.02] + \
        [_native._ptr(a) for a in out]
    assert lib.dh_gen_draw_progress(*args, None) == -1        # no progress counter
    done = C.c_int64(0)
    assert lib.dh_gen_draw_progress(*args, C.byref(done)) == 0 and done.value == 2


def test_gen_assemble_into_row_slices():
    """gen_assemble(out=...) on row chunks (generate_synthetic_calibrations assembles each
    priced chunk while the next is drawn and priced) == one call on all rows, bit for bit."""
    from dhcos import _native
    rs = np.random.RandomState(4)
    n, m = 1000, 15
    model = rs.rand(n, m) + 0.5
    noise = rs.normal(0, 0.02, (n, m))
    spots = 100 + rs.rand(n)
    k = np.tile(np.array([90.0, 95, 100, 105, 110]), 3)
    want = _native.gen_assemble(model, noise, spots, k)
    got = (np.empty((n, m)), np.empty(n), np.empty((n, m)))
    for s in range(0, n, 300):
        e = min(n, s + 300)
        _native.gen_assemble(model[s:e], noise[s:e], spots[s:e], k, tuple(a[s:e] for a in got))
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    with pytest.raises(_native.NativeError):
        _native.gen_assemble(model, noise, spots, k, (got[0][:, :3], got[1], got[2]))


def test_trading_dates_match_reference_loop():
    """synthetic_generator.py:59-67's weekend-skipping loop, restated here as the check."""
    from datetime import datetime, timedelta

    def loop(n):
        out, cur = [], datetime(2022, 1, 3)
        for _ in range(n):
            while cur.weekday() >= 5:
                cur += timedelta(days=1)
            out.append(cur.strftime("%Y-%m-%d"))
            cur += timedelta(days=1)
        return out

    for n in (0, 1, 5, 6, 7, 11, 2500):
        got = G.trading_dates(n)
        assert got == loop(n) and all(type(d) is str for d in got)


def test_trading_dates_array_equals_numpy_formatting():
    """The columnar path's dates (integer-formatted U10 code points) equal np.datetime_as_string
    of the same business days, to 10^6 samples (year 5855) and past year 9999 (NumPy's own
    formatting takes over)."""
    for n in (0, 1, 4, 5, 6, 1000, 1_000_000, 2_700_000):
        days = np.busday_offset("2022-01-03", np.arange(n), roll="forward")
        got = G.trading_dates_array(n)
        assert np.array_equal(got, np.datetime_as_string(days, unit="D")), n
        assert got.size == n


@pytest.mark.parametrize("pos", [1, 311, 623, 624])
def test_native_draw_any_stream_position(pos):
    """The three-pass draw reads the MT19937 words a generation at a time and pairs them into
    doubles; an odd entry position makes a double straddle a twist.  Same bits, same end state."""
    np.random.seed(3)
    st = list(np.random.get_state())
    st[2] = pos
    np.random.set_state(tuple(st))
    want = G.draw_paths_numpy(4500)
    after_want = np.random.get_state()
    np.random.set_state(tuple(st))
    got = G.draw_paths(4500)
    after_got = np.random.get_state()
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert np.array_equal(after_got[1], after_want[1]) and after_got[2:] == after_want[2:]


@pytest.mark.parametrize("n,m", [(5, 15), (5000, 15), (300, 1), (300, 7), (300, 8), (300, 9),
                                 (200, 32), (100, 129), (50, 300)])
def test_native_assemble_equals_numpy(n, m):
    """dh_gen_assemble (market = model + noise model, loss = np.mean of rel^2, absolute strikes)
    against the NumPy expressions of the reference (synthetic_generator.py:141-157), bit for bit,
    below and above the worker-team threshold and across np.mean's pairwise-sum block sizes."""
    from dhcos import _native
    rs = np.random.RandomState(n + m)
    model = np.abs(rs.standard_normal((n, m))) * 10 + 1e-3
    noise = rs.normal(0, 0.02, (n, m))
    spots = 100 * np.exp(rs.normal(0, 0.1, n))
    k_rel = rs.uniform(80, 120, m)
    market, loss, strikes = _native.gen_assemble(model, noise, spots, k_rel)
    want_mkt = model + noise * model
    assert np.array_equal(market, want_mkt)
    assert np.array_equal(loss, np.array([np.mean(((model[i] - want_mkt[i]) / want_mkt[i]) ** 2)
                                          for i in range(n)]))
    assert np.array_equal(strikes, (k_rel[None, :] * spots[:, None]) / 100.0)


@pytest.mark.parametrize("n_opt,threads,pre", [(15, 3, 0), (15, 7, 1), (0, 4, 1), (1, 5, 0),
                                               (2, 16, 1), (15, 16, 2)])
def test_parallel_draw_equals_numpy_loop(monkeypatch, n_opt, threads, pre):
    """The parallel draw (twister, acceptance bits, walk, chunk workers, sweep; dh_gen_rng.cpp)
    for every team size and grid width, with and without a gauss cached at entry: the same draws
    and the same continuation of np.random as NumPy's own per-sample loop.  n spans several of the
    draw's 16k-sample chunks, and n_opt = 0 / 1 exercise a cached value served past a chunk's
    first sample."""
    monkeypatch.setenv("DHCOS_GEN_THREADS", str(threads))
    n = 40000
    strikes = np.arange(max(n_opt, 1))[:n_opt] + 90.0
    mats = np.array([1.0])
    np.random.seed(31 + n_opt)
    for _ in range(pre):
        np.random.normal()
    want = G.draw_paths_numpy(n, strikes, mats)
    after_want = np.random.random(5)
    np.random.seed(31 + n_opt)
    for _ in range(pre):
        np.random.normal()
    got = G.draw_paths(n, strikes, mats)
    after_got = np.random.random(5)
    for a, b in zip(got, want):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert np.array_equal(after_got, after_want)


def test_parallel_draw_small_runs_repeated(monkeypatch):
    """Draws just above the parallel threshold, repeated: the stream bound's last block lies past
    the bound (no candidate pairs) and the bit workers may reach it before the walk ends; it must
    be skipped, not sized negative (a race that aborted the process)."""
    monkeypatch.setenv("DHCOS_GEN_THREADS", "16")
    np.random.seed(5)
    want = G.draw_paths_numpy(4096)
    for _ in range(60):
        np.random.seed(5)
        got = G.draw_paths(4096)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)


def _state_vec():
    name, key, pos, hg, c = np.random.get_state()
    return np.concatenate([np.asarray(key, dtype=np.float64), [pos, hg, c]])


# (n, ranks, chunk, pre): empty and one-sample draws, blocks of one chunk, chunks of 7 samples
# (cached gauss values carried across many chunk starts), ranks with empty blocks, a draw
# straddling many generations, and the 16k-sample chunks generate_sharded uses
@pytest.mark.parametrize("n,world,chunk,pre", [(0, 2, 7, 0), (1, 3, 7, 1), (2, 4, 1, 2),
                                                (15, 2, 7, 1), (40, 4, 3, 3), (5000, 3, 7, 0),
                                                (70001, 2, 1 << 14, 1), (70001, 5, 1000, 2)])
def test_locate_draw_located_sweep_equal_the_draw(n, world, chunk, pre):
    """The sharded draw's three pieces -- dh_gen_locate (one rank: twister, acceptance bitmaps,
    walk; no sample drawn), dh_gen_draw_located (each rank its own chunks) and dh_gen_sweep (the
    AR(1) blend and spot walk carried rank to rank) -- give dh_gen_draw's samples bit for bit,
    and locate leaves np.random's state exactly where the draw leaves it."""
    from dhcos import _native
    from dhcos import distributed as D
    np.random.seed(1000 + n)
    np.random.random(pre)
    for _ in range(pre % 2):
        np.random.normal()
    st = np.random.get_state()
    want = G.draw_paths(n)
    want_state = _state_vec()
    np.random.set_state(st)
    starts = D.chunk_starts(n, world, chunk)
    drawn0 = _native.gen_drawn_samples()
    loc, end = G.locate_samples(_state_vec(), n, starts)
    assert _native.gen_drawn_samples() == drawn0          # locating draws nothing
    assert np.array_equal(end, want_state)
    carry, parts = np.zeros(14), []
    for r in range(world):
        lo, hi = D.sample_block(n, r, world)
        m = (starts >= lo) & (starts < hi)
        blk = G.draw_block(loc[m], starts[m], hi) if hi > lo else (
            np.empty((0, 13)), np.empty(0), np.empty((0, 15)))
        carry = G.sweep_block(blk[0], blk[1], lo, carry)
        parts.append(blk)
    assert _native.gen_drawn_samples() - drawn0 == n
    for k in range(3):
        assert np.array_equal(np.concatenate([p[k] for p in parts]), want[k]), k


def test_located_states_are_numpy_states():
    """A located state is np.random's own state at that sample: set into NumPy, its next draws
    are the sample's uniforms and gauss values."""
    np.random.seed(3)
    np.random.normal()
    st = np.random.get_state()
    n, at = 200, np.array([0, 57, 199])
    loc, _ = G.locate_samples(_state_vec(), n, at)
    np.random.set_state(st)
    lo, hi = G._ranges()
    ref = G.draw_paths_numpy(n)
    for j, i in enumerate(at):
        np.random.set_state(("MT19937", loc[j, :624].astype(np.uint32), int(loc[j, 624]),
                             int(loc[j, 625]), float(loc[j, 626])))
        raw = np.random.uniform(lo, hi)
        if i == 0:
            assert np.array_equal(raw, ref[0][0])
        else:                 # the blend: alpha prev + (1 - alpha) raw
            assert np.array_equal(G.ALPHA * ref[0][i - 1] + (1 - G.ALPHA) * raw, ref[0][i])
            np.random.normal(0.0003, 0.01)
        assert np.array_equal(np.random.normal(0, 0.02, 15), ref[2][i])


def test_sharded_draw_rejects_bad_arguments():
    from dhcos import _native
    st = np.zeros(627)
    st[624] = 625                                         # pos outside [0, 624]
    with pytest.raises(_native.NativeError):
        _native.gen_locate(st, 10, 15, [0])
    st[624] = 624
    with pytest.raises(_native.NativeError):
        _native.gen_locate(st, 10, 15, [5, 2])            # starts must not decrease
    with pytest.raises(_native.NativeError):
        _native.gen_locate(st, 10, 15, [11])              # past the draw
    np.random.seed(0)
    loc, _ = _native.gen_locate(_state_vec(), 10, 15, [0])
    bad = loc.copy()
    bad[0, 3] = 0.5                                       # a key word that is no uint32
    lo, hi = G._ranges()
    with pytest.raises(_native.NativeError):
        _native.gen_draw_located(bad, [0], 10, lo, hi, 15, 0.0003, 0.01, 0.02)
    with pytest.raises(_native.NativeError):
        _native.gen_draw_located(loc, [0], -1, lo, hi, 15, 0.0003, 0.01, 0.02)
