"""Batch path of the synthetic calibration-data generator on the gfx950 pricer.

Reference: src/data/synthetic_generator.py:25-234.  Per sample the reference draws 13 uniforms,
blends them AR(1) (alpha = 0.9) into the previous sample, random-walks the spot, prices a 5 x 3
call grid one option at a time and adds 2% Gaussian noise to each price.  Pricing consumes no
randomness, and the samples' positions in the stream depend on the data only through the polar
method's acceptances, so this implementation

  1. the host runs only the serial part of the legacy ``np.random`` stream: NumPy's MT19937
     recurrence and the walk over the polar acceptances, which gives each sample its first
     double (state taken from and handed back to ``np.random``);
  2. the device re-creates the stream's words, draws every sample's uniforms and normals in the
     reference's order (13 uniforms, one spot normal for i > 0, 15 noise normals; glibc's log
     restated so the gauss values are NumPy's bits), runs the AR(1) blend and the spot walk,
  3. prices all samples x options (strikes K_relative * spot / 100.0, exactly the reference's
     expression, :125) and applies the noise and the per-sample loss with the reference's NumPy
     expressions, chunk by chunk behind the host walk, into page-locked output arrays
     (``_native.gen_device``).

``draw="host"`` keeps the round-4 pipeline (``dh_gen_draw``: the same draws on the host's
threads, priced chunk by chunk); ``draw_paths_numpy`` is the per-sample NumPy loop of the tests.

Output: ``list[CalibrationResult]`` pickled to ``save_path`` (as the reference), or, with
``as_arrays=True``, a dict of columnar arrays (no per-sample Python objects, for 10^6 samples).
"""
from __future__ import annotations

import pickle
from datetime import datetime, timedelta

import threading

import numpy as np

from . import _native
from .calibrator import CalibrationResult

# synthetic_generator.py:75-89, in the reference's dict order
PARAM_RANGES = {
    "v1_0": (0.025, 0.080), "kappa1": (1.5, 4.5), "theta1": (0.025, 0.065),
    "sigma1": (0.20, 0.50), "rho1": (-0.85, -0.40), "v2_0": (0.020, 0.070),
    "kappa2": (0.30, 1.20), "theta2": (0.025, 0.070), "sigma2": (0.10, 0.35),
    "rho2": (-0.70, -0.20), "lambda_j": (0.05, 0.25), "mu_j": (-0.08, -0.01),
    "sigma_j": (0.03, 0.12),
}
STRIKES_PCT = np.array([90, 95, 100, 105, 110])   # :91
MATURITIES = np.array([0.25, 0.5, 1.0])           # :92
SPOT_BASE = 100.0                                  # :93
RISK_FREE = 0.03                                   # :94
ALPHA = 0.9                                        # :108


def _civil(z):
    """Proleptic Gregorian (year, month, day) of day numbers z since 1970-01-01 (H. Hinnant's
    days-to-civil algorithm, vectorised in int64)."""
    z = z + 719468
    era = np.floor_divide(z, 146097)
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = np.where(mp < 10, mp + 3, mp - 9)
    return yoe + era * 400 + (m <= 2), m, d


def trading_dates_array(n):
    """Weekdays from 2022-01-03 as a '<U10' array of 'YYYY-MM-DD' (synthetic_generator.py:59-67):
    the reference's weekend-skipping loop as integer day arithmetic, formatted natively into the
    code points of a U10 array (dh_gen_dates; np.datetime_as_string's per-element formatting,
    then NumPy's integer passes, were most of a 1M-sample run's host time); past year 9999 NumPy's
    formatting.  The strings are the reference's."""
    if int(n) == 0:
        return np.array([], dtype="U10")
    out = _native.gen_dates(18995, n)          # 18995 = days(1970-01-01, 2022-01-03), a Monday
    if out is not None:
        return out
    i = np.arange(int(n), dtype=np.int64)
    # 2022-01-03 is a Monday: sample i falls on Monday + 7 (i // 5) + i % 5 (the reference's
    # weekday loop, no holidays; np.busday_offset gives the same days, ~10x slower)
    days = np.int64(18995) + 7 * (i // 5) + i % 5          # 18995 = days(1970-01-01, 2022-01-03)
    y, m, d = _civil(days)
    if y[-1] > 9999:                               # 5-digit years: NumPy's own formatting
        return np.datetime_as_string(days.astype("datetime64[D]"), unit="D")
    c = np.empty((days.size, 10), np.uint32)
    c[:, 0], c[:, 1], c[:, 2], c[:, 3] = y // 1000, y // 100 % 10, y // 10 % 10, y % 10
    c[:, 5], c[:, 6], c[:, 8], c[:, 9] = m // 10, m % 10, d // 10, d % 10
    c += ord("0")
    c[:, 4] = c[:, 7] = ord("-")
    return c.view("U10").ravel()


def trading_dates(n):
    """trading_dates_array as a list of Python strings (the reference's per-record dates)."""
    return trading_dates_array(n).tolist()


def draw_paths(n_samples, strikes=STRIKES_PCT, maturities=MATURITIES):
    """Host part: RNG in reference order + AR(1) params + spot walk, natively (dh_gen_draw).
    Returns (params [n,13], spots [n], noise [n, n_opts]) and leaves np.random's state where the
    reference's loop leaves it."""
    lo = np.array([v[0] for v in PARAM_RANGES.values()])
    hi = np.array([v[1] for v in PARAM_RANGES.values()])
    n_opt = len(strikes) * len(maturities)
    return _native.gen_draw(n_samples, lo, hi, n_opt, ALPHA, SPOT_BASE, 0.0003, 0.01, 0.02)


def draw_paths_async(n_samples, strikes=STRIKES_PCT, maturities=MATURITIES):
    """draw_paths on a worker thread (_native.GenDraw): its rows can be consumed as they are
    finished (``ready(e)``); ``finish()`` returns what draw_paths returns."""
    lo = np.array([v[0] for v in PARAM_RANGES.values()])
    hi = np.array([v[1] for v in PARAM_RANGES.values()])
    n_opt = len(strikes) * len(maturities)
    return _native.GenDraw(n_samples, lo, hi, n_opt, ALPHA, SPOT_BASE, 0.0003, 0.01, 0.02)


# samples per located chunk of the sharded draw (a rank's chunks are drawn in parallel)
LOCATE_CHUNK = 1 << 14


def _ranges():
    lo = np.array([v[0] for v in PARAM_RANGES.values()])
    hi = np.array([v[1] for v in PARAM_RANGES.values()])
    return lo, hi


def locate_samples(state, n_samples, starts, n_opt=len(STRIKES_PCT) * len(MATURITIES)):
    """The serial part of an n_samples draw from the np.random state ``state`` ([627]): the
    generator's state at each sample index of ``starts`` (dh_gen_locate) -> (loc [n, 627], the
    state the whole draw leaves [627]).  No sample is drawn."""
    return _native.gen_locate(state, n_samples, n_opt, starts)


def draw_block(loc, starts, i_end, n_opt=len(STRIKES_PCT) * len(MATURITIES)):
    """Samples [starts[0], i_end) from their located chunk states (dh_gen_draw_located): (raw
    params, spot returns, noise); sweep_block then applies the AR(1) blend and the spot walk."""
    lo, hi = _ranges()
    return _native.gen_draw_located(loc, starts, i_end, lo, hi, n_opt, 0.0003, 0.01, 0.02)


def sweep_block(params, rets, i0, carry):
    """AR(1) blend (:105-109) and spot walk (:112-116) of a drawn block of samples [i0, ...), in
    place (rets become spots), from the previous sample's row ``carry`` [14] -> this block's last
    row (dh_gen_sweep)."""
    return _native.gen_sweep(params, rets, i0, ALPHA, SPOT_BASE, carry)


def draw_paths_numpy(n_samples, strikes=STRIKES_PCT, maturities=MATURITIES):
    """draw_paths as a per-sample NumPy loop (the reference's calls, vectorised per sample);
    kept as the tests' cross-check of the native draw."""
    lo = np.array([v[0] for v in PARAM_RANGES.values()])
    hi = np.array([v[1] for v in PARAM_RANGES.values()])
    n_opt = len(strikes) * len(maturities)
    params = np.empty((n_samples, 13))
    spots = np.empty(n_samples)
    noise = np.empty((n_samples, n_opt))
    prev, spot = None, SPOT_BASE
    for i in range(n_samples):
        draw = np.random.uniform(lo, hi)                       # 13 draws, dict order (:101-102)
        if prev is not None:
            cur = ALPHA * prev + (1 - ALPHA) * draw            # (:105-109)
        else:
            cur = draw
        if i > 0:
            spot = spot * (1 + np.random.normal(0.0003, 0.01))  # (:112-116)
        noise[i] = np.random.normal(0, 0.02, n_opt)           # one per option, grid order (:141)
        params[i], spots[i], prev = cur, spot, cur
    return params, spots, noise


def grid_surface(ctx, strikes=STRIKES_PCT, maturities=MATURITIES):
    """The call grid (T outer, K inner -- the reference's loop order) as a surface of strikes in
    percent of each sample's spot, cached on the context (one per grid: creating and destroying
    it per call cost a device allocation and a synchronising free per call).
    -> (surface, K_rel [m], T [m])."""
    Krel = np.tile(np.asarray(strikes, dtype=np.float64), len(maturities))
    T = np.repeat(np.asarray(maturities, dtype=np.float64), len(strikes))
    grids = ctx.__dict__.setdefault("_grid_surfaces", {})
    key = (Krel.tobytes(), T.tobytes())
    surf = grids.get(key)
    if surf is None:
        surf = grids[key] = _native.Surface(ctx, Krel, T, np.ones(T.size, dtype=np.int8),
                                            strike_mode=_native.STRIKE_PCT_SPOT)
    return surf, Krel, T


# the last device draw's timings (seconds from the call's start; dh_gen_device's stats): when the
# twister and the walk (the host's serial part) ended, when the first chunk went to the device,
# when the call returned
last_device_stats = {}


def generate_device(n_samples, N=128, device=None, strikes=STRIKES_PCT, maturities=MATURITIES,
                    r=RISK_FREE):
    """The whole batch path on the device (dh_gen_device) from np.random's state, which it
    advances as the reference's loop does.  -> dict(params, spots, market, model, loss, strikes,
    dates ('<U10'), maturities)."""
    ctx = _native.default_context(device)
    surf, Krel, T = grid_surface(ctx, strikes, maturities)
    lo, hi = _ranges()
    n = int(n_samples)
    # the device forms the dates while years have four digits (n <= ~2M samples from 2022)
    dates_dev = n <= 2_000_000
    st = np.zeros(8)
    out = _native.gen_device(surf, n, lo, hi, ALPHA, SPOT_BASE, 0.0003, 0.01, 0.02, r, Krel, N=N,
                             first_day=18995 if dates_dev else None, stats=st)
    if not dates_dev:
        out["dates"] = trading_dates_array(n)
    last_device_stats.clear()
    last_device_stats.update(twister_s=st[0], walk_s=st[1], first_chunk_s=st[2], total_s=st[3],
                             ar1_segments_rerun=int(st[4]), chunks=int(st[7]))
    out["maturities"] = T
    return out


def price_grid(params, spots, N=128, strikes=STRIKES_PCT, maturities=MATURITIES, r=RISK_FREE,
               chunk=1 << 18, device=None, ready=None, on_chunk=None):
    """GPU: price every sample's call grid (T outer, K inner -- the reference's loop order).
    ``ready(e)``, if given, is called before rows [s, e) are read (a draw still in progress,
    _native.GenDraw); the chunks, and so the launches and the bits, are the same either way.
    ``on_chunk(s, e, out)``, if given, is called after rows [s, e) of ``out`` are priced."""
    ctx = _native.default_context(device)
    surf, Krel, T = grid_surface(ctx, strikes, maturities)
    n = params.shape[0]
    out = np.empty((n, T.size))
    if ready is not None:
        # rows are still being written (a draw in progress): a converting copy would snapshot
        # rows the draw has not finished, so the arrays must be the draw's own
        for a in (params, spots):
            if a.dtype != np.float64 or not a.flags.c_contiguous:
                raise ValueError("price_grid(ready=...): params / spots must be the draw's "
                                 "C-contiguous float64 arrays")
    else:
        params = np.ascontiguousarray(params, dtype=np.float64)
        spots = np.ascontiguousarray(spots, dtype=np.float64)
    # the rows move by DMA from / into the page-locked arrays; the device forms the records
    with _native.pinned(params, spots, out):
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            if ready is not None:
                ready(e)
            surf.price_cols(params[s:e], spots[s:e], r, N, out=out[s:e])
            if on_chunk is not None:
                on_chunk(s, e, out)
    return out


def generate_synthetic_calibrations(n_samples: int = 500,
                                    save_path: str = "lbfgs_calibrations_synthetic.pkl", *,
                                    N: int = 128, device=None, as_arrays: bool = False,
                                    verbose: bool = True, draw: str = "device"):
    """Generate ``n_samples`` synthetic calibrations (synthetic_generator.py:25-234).  By default
    the draws, recursions, pricing and assembly run on the device behind the host's serial walk of
    the RNG stream (generate_device); ``draw="host"``: the native host draw on a worker thread,
    each chunk priced on the GPU as soon as the draw has finished it."""
    if draw not in ("device", "host"):
        raise ValueError("draw must be 'device' or 'host'")
    if draw == "device" and int(n_samples) > 0:
        o = generate_device(n_samples, N=N, device=device)
        return assemble(o["params"], o["spots"], None, o["model"], save_path, as_arrays=as_arrays,
                        verbose=verbose, N=N, assembled=(o["market"], o["loss"], o["strikes"]),
                        dates=o["dates"])
    d = draw_paths_async(n_samples)
    dates = []                         # the columnar dates depend on n only: formed meanwhile
    t_dates = threading.Thread(target=lambda: dates.append(trading_dates_array(n_samples)))
    if as_arrays:
        t_dates.start()
    n_opt = d.noise.shape[1]
    Krel = np.tile(STRIKES_PCT, len(MATURITIES))
    asm = (np.empty((n_samples, n_opt)), np.empty(n_samples), np.empty((n_samples, n_opt)))
    workers, errors = [], []

    def assemble_rows(s, e, model):
        # dh_gen_assemble of the priced rows on a worker thread (the ctypes call releases the
        # GIL) while the next chunk is drawn and priced; row-wise, so the same bits
        def work():
            try:
                _native.gen_assemble(model[s:e], d.noise[s:e], d.spots[s:e], Krel,
                                     tuple(a[s:e] for a in asm))
            except BaseException as exc:          # re-raised by the caller after the join
                errors.append(exc)
        t = threading.Thread(target=work)
        t.start()
        workers.append(t)

    try:
        # chunks of 65,536 rows (the draw's own): the first is priced as soon as the draw
        # publishes it, and the last leaves the least pricing after the draw ends
        model = price_grid(d.params, d.spots, N=N, device=device, ready=d.ready,
                           on_chunk=assemble_rows, chunk=1 << 16)
    finally:
        params, spots, noise = d.finish()
        for t in workers:
            t.join()
        if as_arrays:
            t_dates.join()
    if errors:
        raise errors[0]
    return assemble(params, spots, noise, model, save_path, as_arrays=as_arrays,
                    verbose=verbose, N=N, assembled=asm, dates=dates[0] if dates else None)


def assemble(params, spots, noise, model, save_path, *, as_arrays=False, verbose=True, N=128,
             assembled=None, dates=None):
    """Host part after pricing: noise, per-sample loss, output records (:141-183)."""
    say = print if verbose else (lambda *a, **k: None)
    n_samples = params.shape[0]
    say("=" * 70)
    say("GENERATING SYNTHETIC HISTORICAL CALIBRATIONS (MI355X batch path)")
    say("=" * 70)
    say(f"  samples: {n_samples}   save path: {save_path}   COS terms: {N}")
    # the columnar output keeps the dates as one '<U10' array: 10^6 Python strings were most of
    # the host time of a 1M-sample run (profiles/r03_generator_e2e.json)
    if dates is None:
        dates = trading_dates_array(n_samples) if as_arrays else trading_dates(n_samples)
    names = list(PARAM_RANGES.keys())
    Krel = np.tile(STRIKES_PCT, len(MATURITIES))
    Tg = np.repeat(MATURITIES, len(STRIKES_PCT))
    # market = model + noise * model (:141-142), loss = mean(((model - market)/market)^2)
    # (:154-157) and the absolute strikes in one native pass, NumPy's bits
    # (_native.gen_assemble: dh_gen_assemble)
    if assembled is None:
        market, losses, strikes = _native.gen_assemble(model, noise, spots, Krel)
    else:                                # formed chunk by chunk during the pricing
        market, losses, strikes = assembled
    if as_arrays:
        result = dict(dates=dates, spot=spots, risk_free=RISK_FREE, params=params,
                      param_names=names, market_prices=market, model_prices=model,
                      strikes=strikes, maturities=Tg, final_loss=losses)
        if save_path:
            np.savez(save_path if save_path.endswith(".npz") else save_path + ".npz",
                     **{k: v for k, v in result.items() if k != "param_names"},
                     param_names=np.array(names))
        return result
    calibrations = []
    for i in range(n_samples):
        opts = [{"strike": Krel[j] * spots[i] / 100.0, "maturity": Tg[j],
                 "price": market[i, j], "option_type": "call"} for j in range(Tg.size)]
        calibrations.append(CalibrationResult(
            date=dates[i], spot=spots[i], risk_free=RISK_FREE,
            parameters={nm: params[i, k] for k, nm in enumerate(names)},
            market_prices=market[i], model_prices=model[i], market_options=opts,
            final_loss=losses[i], calibration_time=None, success=True, iterations=None,
            message="Synthetic data (not from real calibration)"))
        if verbose and (i + 1) % 50 == 0 and n_samples <= 10000:
            say(f"  Progress: {i + 1}/{n_samples} ({(i + 1) / n_samples * 100:.1f}%)")
    if save_path:
        with open(save_path, "wb") as fh:
            pickle.dump(calibrations, fh)
    if verbose and n_samples:
        errs = np.abs((model - market) / market) * 100
        say(f"  mean loss {np.mean(losses):.6f}  median {np.median(losses):.6f}  "
            f"spot {spots[0]:.2f} -> {spots[-1]:.2f}  mean |err| {np.mean(errs):.2f}%")
    return calibrations
