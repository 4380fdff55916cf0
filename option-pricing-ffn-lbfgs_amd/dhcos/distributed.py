"""Multi-GPU sharding of the hot path: one process per GPU, ``torch.distributed``
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).  Nothing on the data path
is exchanged: the shards are independent and each rank drives its own GPU.

  * ``calibrate_sharded``: the starts of ``calibrate(maxiter, multi_start)`` are dealt
    round-robin over the ranks (start s on rank s % world); each rank runs its starts in lockstep
    on its own GPU, then ONE all-gather of a fixed-size record per start (status, fun, success,
    nit, nfev, time, x[13], message bytes) gives every rank the whole table, and the best start is
    chosen exactly as the reference does -- strict ``<`` over starts in start order
    (lbfgs_calibrator.py:271-299).  Start x0s are drawn on rank 0 in start order from the global
    ``np.random`` stream (the reference's only RNG consumer, :256) and broadcast with rank 0's
    RNG state after the draws, so the result, ``n_calls`` / ``best_loss`` (those of the last
    start) and every rank's ``np.random`` stream afterwards equal the single-process
    ``calibrate`` with the same RNG state.
  * ``generate_sharded``: rank r owns a contiguous block of samples and draws only those.  Rank 0
    runs the serial part of the draw alone -- the MT19937 twister, the polar acceptance bitmaps
    and the walk (dh_gen_locate), no sample drawn -- and broadcasts the generator's state at the
    start of every rank's chunks (627 words each).  Each rank draws its own chunks
    (dh_gen_draw_located), the AR(1) blend and spot walk pass rank to rank (the previous block's
    last row, 14 doubles, one broadcast per rank: dh_gen_sweep), each rank prices its block, and
    one gather brings the blocks (params, spots, noise, prices) to rank 0, which builds and saves
    the reference output.  Bit for bit the single-process draw (synthetic_generator.py:98-141);
    every rank's ``np.random`` ends where rank 0's draw leaves it.

Only collectives on small host-side records and (generator) the price block are used; the COS
kernels never wait on another rank.  The collectives run over ``torch.distributed`` (a process
group) or, for callers without torch, over the library's own RCCL communicator
(``comm=_native.Comm``: dh_comm_broadcast / dh_allgather_best).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from . import _native
from .calibrator import (CalibrationResult, DoubleHestonJumpCalibrator, N_PARAMS, run_starts,
                         run_starts_device)

_MSG_BYTES = 64                        # SciPy messages are <= 52 characters
# status, start, fun, success, nit, nfev, t_rel, n_calls, best_loss, x[13]
_REC = 9 + N_PARAMS
_REC_I64 = _REC + _MSG_BYTES // 8


def _comm_device(group=None, device=None):
    """Device on which collectives of this group take tensors (RCCL: the rank's GPU, the one its
    kernels run on: _native.resolve_device)."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", _native.resolve_device(device))
    return torch.device("cpu")


def _world(group=None, comm=None):
    if comm is not None:
        return comm.rank, comm.world
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _broadcast_f64(arr, shape, group=None, device=None, comm=None, root=0):
    """Broadcast a float64 array from rank ``root`` (bit-exact)."""
    if comm is not None:
        buf = (np.array(arr, dtype=np.float64).reshape(shape) if comm.rank == root
               else np.zeros(shape))
        return comm.broadcast(buf, root)
    dev = _comm_device(group, device)
    t = torch.empty(shape, dtype=torch.float64, device=dev)
    if dist.get_rank(group) == root:
        t.copy_(torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64).reshape(shape)))
    src = dist.get_global_rank(group, root) if group is not None else root
    dist.broadcast(t, src=src, group=group)
    return t.cpu().numpy()


def _gather_rows(block, group=None, device=None, comm=None):
    """Rank 0 gets every rank's float64 block (same shape on every rank) as [world, *shape] in
    rank order; other ranks get None (the native communicator all-gathers)."""
    rank, world = _world(group, comm)
    blk = np.ascontiguousarray(block, dtype=np.float64)
    if comm is not None:
        out = comm.allgather(blk)
        return out if rank == 0 else None
    dev = _comm_device(group, device)
    mine = torch.from_numpy(blk).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)] if rank == 0 else None
    dst = dist.get_global_rank(group, 0) if group is not None else 0
    dist.gather(mine, parts, dst=dst, group=group)
    return np.stack([p.cpu().numpy() for p in parts]) if rank == 0 else None


def start_shard(n_starts: int, rank: int, world: int):
    """Start indices owned by ``rank`` (round-robin keeps the guess types mixed per rank)."""
    return list(range(rank, n_starts, world))


def _encode(s, out, t0, stats=(0, np.inf)):
    """Fixed-size int64 record of one start's outcome (doubles bit-cast, message as bytes).
    stats: the start's (n_calls, best_loss), kept whether or not the start finished."""
    rec = np.zeros(_REC_I64, dtype=np.int64)
    d = np.zeros(_REC, dtype=np.float64)
    d[1] = s
    d[2] = np.nan                      # no outcome: never the best (dh_allgather_best's rule)
    d[7], d[8] = stats
    if out is not None:
        res, t_done = out
        d[0] = 1.0
        d[2] = res.fun
        d[3] = 1.0 if res.success else 0.0
        d[4] = res.nit
        d[5] = res.nfev
        d[6] = t_done - t0
        d[9:] = res.x
        msg = str(res.message).encode("utf-8")[:_MSG_BYTES]
        rec[_REC:] = np.frombuffer(msg.ljust(_MSG_BYTES, b"\0"), dtype=np.int64)
    rec[:_REC] = d.view(np.int64)
    return rec


def _decode(rec):
    d = rec[:_REC].view(np.float64)
    stats = (int(d[7]), float(d[8]))
    if d[0] != 1.0:
        return int(d[1]), None, stats
    msg = rec[_REC:].tobytes().rstrip(b"\0").decode("utf-8", "replace")
    return int(d[1]), dict(fun=float(d[2]), success=bool(d[3]), nit=int(d[4]), nfev=int(d[5]),
                           t_rel=float(d[6]), x=d[9:].copy(), message=msg), stats


def gather_start_records(local, n_starts, group=None, device=None, comm=None):
    """All-gather the per-start records of every rank -> ([n_starts] decoded outcomes,
    [n_starts] (n_calls, best_loss))."""
    rank, world = _world(group, comm)
    n_max = (n_starts + world - 1) // world
    buf = np.zeros((n_max, _REC_I64), dtype=np.int64)
    buf[:, :_REC] = np.full(_REC, -1.0).view(np.int64)      # padding rows: start index -1
    for i, rec in enumerate(local):
        buf[i] = rec
    if comm is not None:              # RCCL moves the records' bytes unchanged (a copy)
        allr, _ = comm.allgather_best(buf.view(np.float64), col_start=1, col_fun=2)
        parts = list(allr.view(np.int64).reshape(world, n_max, _REC_I64))
    else:
        dev = _comm_device(group, device)
        mine = torch.from_numpy(buf).to(dev)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        parts = [p.cpu().numpy() for p in parts]
    table, stats = [None] * n_starts, [(0, np.inf)] * n_starts
    for p in parts:
        for row in p:
            s, out, st = _decode(row)
            if 0 <= s < n_starts:
                table[s], stats[s] = out, st
    return table, stats


def _rng_state_vec():
    """np.random's legacy MT19937 state as float64 (uint32 key words are exact in a double)."""
    name, key, pos, has_gauss, cached = np.random.get_state()
    if name != "MT19937":
        raise ValueError(f"unsupported bit generator {name}")
    return np.concatenate([np.asarray(key, dtype=np.float64), [pos, has_gauss, cached]])


def _set_rng_state_vec(v):
    key = v[:624].astype(np.uint32)
    np.random.set_state(("MT19937", key, int(v[624]), int(v[625]), float(v[626])))


def calibrate_sharded(cal: DoubleHestonJumpCalibrator, maxiter: int = 300, multi_start: int = 3,
                      *, group=None, x0s=None, x0=None,
                      driver: str = "scipy", comm=None) -> CalibrationResult:
    """``cal.calibrate(maxiter, multi_start, x0s=x0s, x0=x0, driver=driver)`` with the starts
    sharded over the process group (or the ranks of ``comm``, a ``_native.Comm``).  Every rank
    returns the same ``CalibrationResult`` and ends with the same ``cal.n_calls`` /
    ``cal.best_loss`` and ``np.random`` state."""
    rank, world = _world(group, comm)
    if world == 1 and comm is None:
        return cal.calibrate(maxiter=maxiter, multi_start=multi_start, x0s=x0s, x0=x0,
                             driver=driver)
    if driver not in ("scipy", "device"):
        raise ValueError(f"driver must be 'scipy' or 'device', not {driver!r}")
    t0 = time.time()
    dev = cal.device
    block = None
    if rank == 0:           # draws in start order (:256), then the state the draws left behind
        if x0s is None:
            x0s = cal.start_points(multi_start, x0)
        block = np.concatenate([np.asarray(x0s, dtype=np.float64).reshape(-1),
                                _rng_state_vec()])
    block = _broadcast_f64(block, (multi_start * N_PARAMS + 627,), group, dev, comm)
    x0s = block[:multi_start * N_PARAMS].reshape(multi_start, N_PARAMS)
    _set_rng_state_vec(block[multi_start * N_PARAMS:])
    mine = start_shard(multi_start, rank, world)
    run = run_starts_device if driver == "device" else run_starts
    outcomes = run(cal, [x0s[s] for s in mine], maxiter) if mine else []
    stats_local = getattr(cal, "start_stats", None) if mine else []
    local = [_encode(s, o, t0, stats_local[i] if stats_local else (0, np.inf))
             for i, (s, o) in enumerate(zip(mine, outcomes))]
    table, stats = gather_start_records(local, multi_start, group, dev, comm)
    if multi_start > 0:     # the per-start resets (:253-254): the state after the last start
        cal.n_calls, cal.best_loss = stats[multi_start - 1]

    best, best_loss = None, np.inf
    for s, out in enumerate(table):          # strict < in start order (:271)
        if out is None:
            continue
        if out["fun"] < best_loss:
            best_loss = out["fun"]
            params = cal.transform_params(out["x"])
            try:
                model = cal._model_prices(params)
            except _native.NativeError:
                raise
            except Exception:
                continue
            best = CalibrationResult(
                date="", spot=cal.spot, risk_free=cal.risk_free_rate, parameters=params,
                market_prices=cal.market_prices, model_prices=model,
                market_options=cal.market_options, final_loss=out["fun"],
                calibration_time=out["t_rel"], success=out["success"], iterations=out["nit"],
                message=out["message"])
    if best is None:
        best = CalibrationResult(
            date="", spot=cal.spot, risk_free=cal.risk_free_rate,
            parameters={name: 0.0 for name in cal.param_names},
            market_prices=cal.market_prices, model_prices=np.zeros_like(cal.market_prices),
            market_options=cal.market_options, final_loss=np.inf,
            calibration_time=time.time() - t0, success=False, iterations=0,
            message="All optimization starts failed")
    return best


def sample_block(n: int, rank: int, world: int):
    """Contiguous [lo, hi) block of samples owned by ``rank``."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def chunk_starts(n: int, world: int, chunk: int):
    """The located chunk starts of every rank's block, in sample order: each block cut into
    ``chunk``-sample chunks (the same list on every rank)."""
    out = []
    for r in range(world):
        lo, hi = sample_block(n, r, world)
        out.extend(range(lo, hi, chunk))
    return np.array(out, dtype=np.int64)


# what the last generate_sharded call did on this rank (instrumentation: samples this process
# drew natively, its block, and the stages' seconds)
last_generate_stats: dict = {}


def generate_sharded(n_samples: int = 500,
                     save_path: str = "lbfgs_calibrations_synthetic.pkl", *, N: int = 128,
                     as_arrays: bool = False, verbose: bool = True, group=None, price_fn=None,
                     device=None, comm=None):
    """``generate_synthetic_calibrations`` with the draw and the pricing sharded over the process
    group (module docstring).  Rank 0 returns (and saves) the reference output; other ranks return
    None."""
    from . import generator as G

    rank, world = _world(group, comm)
    if world == 1 and comm is None and price_fn is None:
        # one rank: the single-process API itself (draw, pricing and assembly overlapped)
        return G.generate_synthetic_calibrations(n_samples, save_path, N=N, device=device,
                                                 as_arrays=as_arrays, verbose=verbose)
    price_fn = price_fn or (lambda p, s: G.price_grid(p, s, N=N, device=device))
    n_opt = len(G.STRIKES_PCT) * len(G.MATURITIES)
    n = int(n_samples)
    t0 = time.perf_counter()
    drawn0 = _native.gen_drawn_samples()
    lo, hi = sample_block(n, rank, world)
    starts = chunk_starts(n, world, G.LOCATE_CHUNK)
    # rank 0: the serial part of the draw (twister, acceptance bitmaps, walk), no sample drawn;
    # every rank gets the states at all chunk starts and the state the whole draw leaves
    shape = (starts.size + 1, _native.GEN_LOC_WORDS)
    block = None
    if rank == 0:
        loc, end = G.locate_samples(_rng_state_vec(), n, starts, n_opt)
        block = np.concatenate([loc, end[None, :]])
    block = _broadcast_f64(block, shape, group, device, comm)
    _set_rng_state_vec(block[-1])
    t_loc = time.perf_counter()
    mine = (starts >= lo) & (starts < hi)
    if hi > lo:
        params, spots, noise = G.draw_block(block[:-1][mine], starts[mine], hi, n_opt)
    else:
        params, spots, noise = np.empty((0, 13)), np.empty(0), np.empty((0, n_opt))
    t_draw = time.perf_counter()
    # the AR(1) blend and the spot walk carry across blocks: rank r sweeps its block from rank
    # r - 1's last row and hands its own last row on (a block that is empty passes it through)
    carry = np.zeros(14)
    for r in range(world):
        if rank == r:
            carry = G.sweep_block(params, spots, lo, carry)
        if r < world - 1:
            carry = _broadcast_f64(carry, (14,), group, device, comm, root=r)
    t_sweep = time.perf_counter()
    model = price_fn(params, spots) if hi > lo else np.empty((0, n_opt))
    t_price = time.perf_counter()
    # one gather: every block's params, spots, noise and prices to rank 0
    per = (n + world - 1) // world
    width = 13 + 1 + 2 * n_opt
    buf = np.zeros((per, width))
    buf[:hi - lo, :13], buf[:hi - lo, 13] = params, spots
    buf[:hi - lo, 14:14 + n_opt], buf[:hi - lo, 14 + n_opt:] = noise, model
    allb = _gather_rows(buf, group, device, comm)
    t_gather = time.perf_counter()
    last_generate_stats.clear()
    last_generate_stats.update(
        rank=rank, world=world, block=(lo, hi), samples=n,
        samples_drawn=_native.gen_drawn_samples() - drawn0,
        seconds={"locate_broadcast": t_loc - t0, "draw": t_draw - t_loc,
                 "sweep_chain": t_sweep - t_draw, "price": t_price - t_sweep,
                 "gather": t_gather - t_price})
    if rank != 0:
        return None
    rows = allb.reshape(world * per, width)[:n]
    params = np.ascontiguousarray(rows[:, :13])
    spots = np.ascontiguousarray(rows[:, 13])
    noise = np.ascontiguousarray(rows[:, 14:14 + n_opt])
    model = np.ascontiguousarray(rows[:, 14 + n_opt:])
    return G.assemble(params, spots, noise, model, save_path, as_arrays=as_arrays,
                      verbose=verbose, N=N)
