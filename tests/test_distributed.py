"""Multi-process (gloo, world_size 2, CPU) tests of dhcos.distributed: the sharded multi-start and
the sharded generator must return exactly what the single-process path returns.

No GPU here, so the per-rank objective / pricer is the CPU oracle (test infrastructure, used as a
stand-in for the device surface): what is under test is the sharding, the record exchange and the
reference's best-start rule, not the kernels (those are covered by test_gpu_parity.py)."""
import os
import pickle
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from dhcos import distributed as D
from dhcos import generator as G
from dhcos.calibrator import DoubleHestonJumpCalibrator
from oracle import dh_oracle as O

SPOT, R = 100.0, 0.05


def _market():
    prm = np.array([0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3, 0.1, 0.0, 0.1])
    out = []
    for T in (0.25, 0.5, 1.0):
        for K in (90.0, 95.0, 100.0, 105.0, 110.0):
            out.append({"strike": K, "maturity": T, "option_type": "call",
                        "price": float(O.price_vec(prm, SPOT, K, T, R, True, 64)) * 1.01})
    return out


class OracleCalibrator(DoubleHestonJumpCalibrator):
    """The calibrator with its device surface replaced by the CPU oracle (N = 64)."""

    def loss_batch(self, X, track=True):
        X = np.atleast_2d(np.asarray(X, dtype=np.float64))
        if track:
            self.n_calls += X.shape[0]
        return np.array([O.loss(x, self.market_options, self.spot, self.risk_free_rate, self.N)
                         for x in X])

    def _model_prices(self, params):
        p = np.array([params[n] for n in self.param_names])
        return np.array([O.price_vec(p, self.spot, o["strike"], o["maturity"],
                                     self.risk_free_rate, True, self.N)
                         for o in self.market_options])


def oracle_price_fn(params, spots, N=64):
    Krel = np.tile(G.STRIKES_PCT.astype(float), len(G.MATURITIES))
    T = np.repeat(G.MATURITIES, len(G.STRIKES_PCT))
    out = np.empty((params.shape[0], T.size))
    for i in range(params.shape[0]):
        K = Krel * spots[i] / 100.0
        out[i] = [O.price_vec(params[i], spots[i], K[j], T[j], G.RISK_FREE, True, N)
                  for j in range(T.size)]
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


WARM = {"v1_0": 0.05, "kappa1": 1.8, "theta1": 0.045, "sigma1": 0.28, "rho1": -0.55,
        "v2_0": 0.035, "kappa2": 1.2, "theta2": 0.04, "sigma2": 0.22, "rho2": -0.35,
        "lambda_j": 0.12, "mu_j": -0.02, "sigma_j": 0.09}


def _worker(rank, world, port, out_dir, n_starts, n_samples):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    os.environ.pop("DHCOS_DEVICE", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dhcos import _native
        dev = _native.resolve_device()          # the rank's own GPU under torch.distributed
        # only rank 0's RNG state matters: x0s and generator draws are broadcast from it
        np.random.seed(0 if rank == 0 else 1234 + rank)
        cal = OracleCalibrator(SPOT, R, _market(), N=64)
        res = D.calibrate_sharded(cal, maxiter=2, multi_start=n_starts)
        stats = (cal.n_calls, cal.best_loss)
        rng_after_cal = np.random.random(4)
        cal_w = OracleCalibrator(SPOT, R, _market(), N=64)
        res_w = D.calibrate_sharded(cal_w, maxiter=2, multi_start=n_starts, x0=WARM)
        np.random.seed(7 if rank == 0 else 99)
        gen = D.generate_sharded(n_samples, os.path.join(out_dir, f"gen{rank}.pkl"), N=64,
                                 verbose=False, price_fn=oracle_price_fn)
        rng_after_gen = np.random.random(4)
        with open(os.path.join(out_dir, f"rank{rank}.pkl"), "wb") as fh:
            pickle.dump({"res": res, "gen": gen, "stats": stats, "rng_cal": rng_after_cal,
                         "res_w": res_w, "rng_gen": rng_after_gen, "dev": dev}, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n_starts", [(2, 4), (3, 2)])
def test_sharded_equals_single_process(tmp_path, world, n_starts):
    n_samples = 5
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_starts, n_samples),
             nprocs=world, join=True)
    got = [pickle.load(open(tmp_path / f"rank{r}.pkl", "rb")) for r in range(world)]

    np.random.seed(0)
    cal = OracleCalibrator(SPOT, R, _market(), N=64)
    want = cal.calibrate(maxiter=2, multi_start=n_starts)
    want_stats = (cal.n_calls, cal.best_loss)
    want_rng = np.random.random(4)
    want_w = OracleCalibrator(SPOT, R, _market(), N=64).calibrate(maxiter=2,
                                                                   multi_start=n_starts, x0=WARM)
    for rank, g in enumerate(got):      # every rank holds the same, reference-identical result
        assert g["dev"] == rank         # LOCAL_RANK (no device here: modulo nothing)
        for r, w in ((g["res"], want), (g["res_w"], want_w)):
            assert r.final_loss == w.final_loss
            assert r.iterations == w.iterations
            assert r.message == w.message
            assert r.success == w.success
            assert r.parameters == w.parameters
            np.testing.assert_array_equal(r.model_prices, w.model_prices)
        assert g["stats"] == want_stats                     # n_calls / best_loss of the last start
        np.testing.assert_array_equal(g["rng_cal"], want_rng)   # every rank's RNG continues alike

    np.random.seed(7)
    p, s, nz = G.draw_paths(n_samples)
    want_rng_gen = np.random.random(4)
    for g in got:
        np.testing.assert_array_equal(g["rng_gen"], want_rng_gen)
    ref = G.assemble(p, s, nz, oracle_price_fn(p, s), None, verbose=False)
    gen = got[0]["gen"]
    assert len(gen) == n_samples
    for a, b in zip(gen, ref):
        np.testing.assert_array_equal(a.market_prices, b.market_prices)
        np.testing.assert_array_equal(a.model_prices, b.model_prices)
        assert a.parameters == b.parameters and a.spot == b.spot and a.date == b.date
        assert a.final_loss == b.final_loss
    assert all(g["gen"] is None for g in got[1:])
    # rank 0 saved the reference-format pickle; it names lbfgs_calibrator.CalibrationResult
    raw = open(tmp_path / "gen0.pkl", "rb").read()
    assert b"lbfgs_calibrator" in raw and b"CalibrationResult" in raw


def fake_price_fn(params, spots):
    """A cheap deterministic stand-in for the pricer (what is under test is the partitioned draw,
    the carry chain and the gather, not the prices): positive, row-dependent."""
    return np.outer(spots, np.arange(1.0, 16.0)) * params[:, :1] + params[:, 1:2]


def _gen_worker(rank, world, port, out_dir, n_samples):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    os.environ["DHCOS_GEN_THREADS"] = "4"          # two ranks share the container's 8 CPUs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        np.random.seed(11 if rank == 0 else 500 + rank)   # only rank 0's state matters
        np.random.random(3)
        np.random.normal()                                # a cached gauss at entry
        out = D.generate_sharded(n_samples, None, as_arrays=True, verbose=False,
                                 price_fn=fake_price_fn)
        stats = dict(D.last_generate_stats)
        rng_after = np.random.random(4)
        if rank == 0:
            np.savez(os.path.join(out_dir, "gen.npz"),
                     **{k: v for k, v in out.items() if k not in ("param_names", "risk_free")})
        with open(os.path.join(out_dir, f"gstats{rank}.pkl"), "wb") as fh:
            pickle.dump({"stats": stats, "rng": rng_after}, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_generate_sharded_partitions_the_draw(tmp_path):
    """a gloo world-2 generate_sharded(1_000_000) equals the single process
    bit for bit (every output array and the RNG continuation), and each rank draws at most 55%
    of the samples (the library's own count of the samples this process drew): rank 0 only
    locates the chunk starts of rank 1's block (twister, acceptance bitmaps, walk), it does not
    draw them."""
    n, world = 1_000_000, 2
    mp.spawn(_gen_worker, args=(world, _free_port(), str(tmp_path), n), nprocs=world, join=True)
    np.random.seed(11)
    np.random.random(3)
    np.random.normal()
    p, s, nz = G.draw_paths(n)
    want_rng = np.random.random(4)
    want = G.assemble(p, s, nz, fake_price_fn(p, s), None, as_arrays=True, verbose=False)
    got = np.load(tmp_path / "gen.npz")
    for k in ("dates", "spot", "params", "market_prices", "model_prices", "strikes",
              "maturities", "final_loss"):
        assert np.array_equal(got[k], want[k]), k
    for r in range(world):
        g = pickle.load(open(tmp_path / f"gstats{r}.pkl", "rb"))
        np.testing.assert_array_equal(g["rng"], want_rng)
        lo, hi = g["stats"]["block"]
        assert g["stats"]["samples_drawn"] == hi - lo <= 0.55 * n, g["stats"]


def test_shard_helpers():
    assert D.start_shard(8, 1, 3) == [1, 4, 7]
    assert sorted(sum((D.start_shard(64, r, 8) for r in range(8)), [])) == list(range(64))
    blocks = [D.sample_block(10, r, 4) for r in range(4)]
    assert blocks == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert D.sample_block(2, 3, 4) == (2, 2)
    s, out, st = D._decode(D._encode(5, None, 0.0, (28, 0.5)))
    assert s == 5 and out is None and st == (28, 0.5)


def test_resolve_device(monkeypatch):
    from dhcos import _native
    monkeypatch.delenv("DHCOS_DEVICE", raising=False)
    assert _native.resolve_device(3) == 3
    assert _native.resolve_device() == 0            # no process group: device 0
    monkeypatch.setenv("DHCOS_DEVICE", "2")
    assert _native.resolve_device() == 2


def _reference_best(rows):
    """lbfgs_calibrator.py:271-275: starts in order, best_loss = inf, strict <."""
    best, best_loss = -1, np.inf
    for s, fun in sorted(((r[1], r[2]) for r in rows if r[1] >= 0), key=lambda t: t[0]):
        if fun < best_loss:
            best, best_loss = int(s), fun
    return best


def test_best_start_matches_reference_rule():
    """dh_best_start (host only, the selection dh_allgather_best applies after its RCCL gather):
    start order, strict <, NaN and inf never win, padding rows (start < 0) ignored, ties go to the
    earlier start -- on records gathered in rank order, not start order."""
    from dhcos import _native
    rs = np.random.RandomState(7)
    for trial in range(200):
        n = rs.randint(0, 20)
        rows = np.zeros((n + 3, 5))
        rows[:, 1] = -1.0                                   # padding
        starts = rs.permutation(n)
        for i, s in enumerate(starts):
            rows[i, 1] = s
            rows[i, 2] = rs.choice([np.nan, np.inf, 1e10, 0.5, 0.25, rs.rand()])
        rs.shuffle(rows)
        assert _native.best_start(rows, 1, 2) == _reference_best(rows), (trial, rows)
    assert _native.best_start(np.zeros((0, 5)), 1, 2) == -1
    with pytest.raises(_native.NativeError):
        _native.best_start(np.zeros((2, 3)), 1, 5)


def test_missing_outcome_record_never_wins():
    """A start without an outcome travels with fun = NaN, so the native selection skips it."""
    rec = D._encode(3, None, 0.0)
    d = rec[:D._REC].view(np.float64)
    assert d[1] == 3 and np.isnan(d[2])
    s, out, stats = D._decode(rec)
    assert s == 3 and out is None and stats == (0, np.inf)


def test_resolve_device_under_process_group(monkeypatch):
    """Under torch.distributed on a multi-GPU node the device is resolved once per process group
    (ADVICE r5): a gloo job that never touched CUDA puts rank LOCAL_RANK on its own GPU (not every
    rank on torch's default GPU 0), and the library's own CUDA tensors that follow (the first
    collective's tensors on that GPU initialise CUDA without a set_device, leaving torch's current
    device at 0) do not move later calls to GPU 0; a rank that set its device before its first
    call (set_device(5), or an explicit set_device(0) under LOCAL_RANK = 3) keeps that device.
    (GPUs simulated: 8 visible.)"""
    import torch
    from dhcos import _native
    monkeypatch.delenv("DHCOS_DEVICE", raising=False)
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setattr(_native, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    cur = {"dev": 0, "init": False}
    monkeypatch.setattr(torch.cuda, "current_device", lambda: cur["dev"])
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: cur["init"])

    def group(then):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
        try:
            then()
        finally:
            dist.destroy_process_group()

    def no_cuda_state_first():
        assert _native.resolve_device() == 3          # no CUDA state: LOCAL_RANK
        cur.update(dev=0, init=True)                  # the first collective's tensors init CUDA
        assert _native.resolve_device() == 3          # ... and do not move the rank to GPU 0
        cur.update(dev=5, init=True)
        assert _native.resolve_device() == 3          # fixed for the group's lifetime

    def set_device_first(dev):
        def run():
            cur.update(dev=dev, init=True)            # the rank's own set_device before any call
            assert _native.resolve_device() == dev
            cur.update(dev=7)
            assert _native.resolve_device() == dev
        return run

    cur.update(dev=0, init=False)
    group(no_cuda_state_first)
    group(set_device_first(5))
    group(set_device_first(0))                        # set_device(0) under LOCAL_RANK = 3
    monkeypatch.setenv("LOCAL_RANK", "11")
    cur.update(dev=0, init=False)
    group(lambda: _native.resolve_device() == 3 or pytest.fail("modulo the visible GPUs"))
