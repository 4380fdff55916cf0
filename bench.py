#!/usr/bin/env python3
"""Benchmark: option-prices/sec (+ calibrations/sec) of the COS calibration objective on MI355X.

Default workload "c3" (BASELINE.json configs[2]): the metric is quoted at COS N = 128, which no
single-GPU config runs, so the line is the largest single-GPU configuration -- the north star's
10k-option calibration: a 10,000-option synthetic surface (100 K/S in linspace(0.8, 1.2) x 100 T
in linspace(0.1, 2.0), puts below the spot and calls at or above it, S0 = 100, r = 0.03, market =
model at a seed-1 parameter draw x (1 + N(0, 0.02)), seed 2), COS N = 512, 3 lockstep L-BFGS-B
starts.  One step = one lockstep function+gradient request = 3 starts x the 14 SciPy forward-
difference points (13 parameters + base) priced over all 10,000 options and reduced to 42 losses:
420,000 option prices per step.  Each step uses a different x (different param sets), all inputs
resident in HBM before the timed region; the steps are issued back to back on one stream.
Also: --config c2 (configs[1]: 1,024 options, N = 256, one start), c1, c4 (64 starts), c5 (the
generator batch, 1M x 32 options).

Multi-GPU (torchrun, one process per GPU): weak scaling -- every rank runs its own independent
requests (multi-start sharding has no data-path collective); timing is the max over ranks;
value = all ranks' prices / that time.

Also reported: the roofline of the request kernel (HIP events on its stream; frac = the fp64
flops the hardware executed per request, from the committed rocprofv3 counter pass, over this
run's request time), full calibrations of the same surface (calibrations/sec, both optimizer
drivers) and a CPU baseline (the scalar-structured NumPy port in oracle/, timed on a bounded
sample on rank 0, anchored to the reference by profiles/cpu_anchor.json).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch                      # imported first: torch and libdhcos share one HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from dhcos import _native                                      # noqa: E402
from dhcos.distributed import calibrate_sharded                # noqa: E402
from dhcos.calibrator import (DoubleHestonJumpCalibrator,      # noqa: E402
                              fd_request_points, x_to_model)

# Algorithmic work = fp64 flops of the implemented algorithm (FMA = 2, add/mul = 1, each
# elementary function at the flops its gfx950 implementation executes), frozen here
# (DESIGN.md section 4):
#   FLOP_TAB  per COS-table entry (p, T, k): fast-form CF, phase, T2/T4 k-sums -- the table
#             kernel's executed fp64 flops per entry on C3 (rocprofv3 PMC, profiles/r01_c3_pmc.csv:
#             1.807 GFLOP / 2,150,400 entries; 852 on C5)
#   FLOP_TERM per (param set, option, k >= 1): 3 fma + one complex rotation (2 mul + 2 fma)
#   FLOP_OPT  per (param set, option): log-strike, e^{i G th} sincos, final sum, loss term
# The SURVEY 8(d) convention (716 per CF, 120 per option-term) is reported beside it; it charges
# per-term trig the kernels replace by a rotation recurrence, so it exceeds the peak.
FLOP_TAB = 840
FLOP_TERM = 12
FLOP_OPT = 110
PEAK_FP64_TFLOPS = 78.6   # MI355X fp64 vector peak (spec)
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)
SIMDS = 1024              # 256 CUs x 4 SIMDs
NS_FP64_WAVE_INST = 2.05  # fully fed v_fma_f64 issue per SIMD, ns per wave-instruction (ubench)
# SURVEY 8(d) algorithmic bytes: per option K, T, market price 8 B each + type 1 B, read once per
# launch; per param set 13 x 8 B in; out 8 B per price (pricing / generator) or per set (loss)
BYTES_8D_OPTION = 25
BYTES_8D_SET = 104
BYTES_8D_OUT = 8

GEN_LO = np.array([0.025, 1.5, 0.025, 0.2, -0.85, 0.02, 0.3, 0.025, 0.1, -0.7, 0.05, -0.08, 0.03])
GEN_HI = np.array([0.08, 4.5, 0.065, 0.5, -0.4, 0.07, 1.2, 0.07, 0.35, -0.2, 0.25, -0.01, 0.12])


def make_surface(nK, nT, seed_params=1, seed_noise=2, S0=100.0, r=0.03, N=256, put_itm=False):
    """Synthetic market of SURVEY 8(d): model prices at a seed-1 draw, 2% noise (seed 2)."""
    kk, tt = np.meshgrid(np.linspace(0.8, 1.2, nK) * S0, np.linspace(0.1, 2.0, nT))
    K, T = kk.ravel(), tt.ravel()
    call = np.ones(K.size, dtype=bool) if not put_itm else (K >= S0)
    true = GEN_LO + (GEN_HI - GEN_LO) * np.random.RandomState(seed_params).rand(13)
    rec = np.zeros((1, 16))
    rec[0, :13], rec[0, 13], rec[0, 14] = true, S0, r
    ctx = _native.default_context()
    model = _native.Surface(ctx, K, T, call).price(rec, N)[0]
    mkt = model * (1 + np.random.RandomState(seed_noise).normal(0, 0.02, K.size))
    opts = [{"strike": float(k), "maturity": float(t), "price": float(p),
             "option_type": "call" if c else "put"} for k, t, p, c in zip(K, T, mkt, call)]
    return opts, S0, r


def step_params(cal, n_steps, starts, seed):
    """[n_steps, 14*starts, 16] param records: FD points around distinct x per step."""
    rs = np.random.RandomState(seed)
    x0 = cal.get_initial_guess(0)
    out = np.empty((n_steps, 14 * starts, 16))
    for i in range(n_steps):
        X = np.concatenate([fd_request_points(x0 + rs.normal(0, 0.05, 13))[0] for _ in range(starts)])
        out[i, :, :13] = x_to_model(X)
        out[i, :, 13], out[i, :, 14], out[i, :, 15] = cal.spot, cal.risk_free_rate, 0.0
    return out


def _cpu_worker(args):
    """One CPU process of the baseline: price options of the workload one by one with the
    scalar-structured NumPy port for budget_s seconds (strided start so workers differ)."""
    opts, prm, S0, r, N, budget_s, start = args
    from oracle import dh_oracle as O
    n, t0 = 0, time.perf_counter()
    with np.errstate(all="ignore"):
        while True:
            o = opts[(start + n * 37) % len(opts)]
            O.price_scalar(prm, S0, o["strike"], o["maturity"], r, o["option_type"] == "call", N)
            n += 1
            if time.perf_counter() - t0 > budget_s and n >= 16:
                break
    return n, time.perf_counter() - t0


def cpu_model():
    """This host's CPU model (the cpu_baseline's cores)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def reference_anchor(N):
    """The reference's pricing(N) time over the port's, measured side by side in the build
    container (tools/cpu_anchor.py -> profiles/cpu_anchor.json; the reference never travels to the
    GPU box), at the nearest N measured."""
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_anchor.json")) as fh:
            a = json.load(fh)
    except (OSError, ValueError):
        return None
    row = min(a["rows"], key=lambda r: abs(r["N"] - N))
    return {"reference_over_port_time": row["reference_over_port_time"], "at_N": row["N"],
            "reference_ms_per_option": row["reference_ms_per_option"],
            "port_ms_per_option": row["port_ms_per_option"],
            "measured_on": a["cpu_model"], "source": "profiles/cpu_anchor.json"}


def cpu_baseline(cal_opts, S0, r, N, budget_s=12.0, cores=None):
    """Scalar-structured NumPy port (oracle/) of the reference pricer on `cores` host processes
    (default: 16, the GPU box's CPU share), each on a bounded sample of the
    workload's options.  Must run before this process touches the GPU: the pool forks."""
    import multiprocessing as mp
    from oracle import dh_oracle as O
    cores = int(cores or min(16, os.cpu_count() or 1))
    x = DoubleHestonJumpCalibrator(S0, r, cal_opts).get_initial_guess(0)
    prm = O.to_params(x)
    jobs = [(cal_opts, prm, S0, r, N, budget_s, 101 * i) for i in range(cores)]
    if cores == 1:
        res = [_cpu_worker(jobs[0])]
    else:
        # close + join (not the context manager's terminate()): the workers exit on their own,
        # so a profiled bench run carries no SIGTERM abort traces of them
        pool = mp.get_context("fork").Pool(cores)
        try:
            res = pool.map(_cpu_worker, jobs)
        finally:
            pool.close()
            pool.join()
    n = sum(c for c, _ in res)
    rate = sum(c / t for c, t in res)
    wall = max(t for _, t in res)
    out = {"value": rate, "unit": "option-prices/s", "cores": cores, "kind": "port",
           "cpu_model": cpu_model(), "per_core": rate / cores,
           "sample": f"{n} options of the workload priced one by one at N={N} by "
                     f"oracle.dh_oracle.price_scalar (reference algorithm restated) in "
                     f"{cores} processes x {wall:.1f} s"}
    anchor = reference_anchor(N)
    if anchor:
        out["reference_anchor"] = anchor
        out["reference_equivalent_value"] = rate / anchor["reference_over_port_time"]
    return out


def cpu_options(cfg):
    """The workload's option list, built without the GPU (for the CPU baseline)."""
    if cfg.get("gen"):
        Krel = np.tile(np.linspace(80.0, 120.0, 8), 4)
        T = np.repeat([0.25, 0.5, 1.0, 2.0], 8)
        return [{"strike": float(k), "maturity": float(t), "option_type": "call", "price": 1.0}
                for k, t in zip(Krel, T)], 100.0, 0.03
    S0, r = 100.0, 0.03
    kk, tt = np.meshgrid(np.linspace(0.8, 1.2, cfg["nK"]) * S0, np.linspace(0.1, 2.0, cfg["nT"]))
    K, T = kk.ravel(), tt.ravel()
    call = np.ones(K.size, dtype=bool) if not cfg["put_itm"] else (K >= S0)
    return [{"strike": float(k), "maturity": float(t), "price": 1.0,
             "option_type": "call" if c else "put"} for k, t, c in zip(K, T, call)], S0, r


def kernel_label(ctx):
    """Kernels of the last request on ctx (after the bench's own launches)."""
    if ctx.last_path == _native.PATH_FUSED:
        return "cos_fused_kernel (after table_prologue_kernel on grids of >= 8,192 tables)"
    if ctx.last_path == _native.PATH_GEN:
        return "cos_gen_kernel (fused small-tile generator kernel, one launch per batch)"
    return "cos_table_kernel + cos_option[_small]_kernel"


def _pmc(config):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh).get(config, {})
    except (OSError, ValueError):
        return {}


def pmc_traffic(config):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc summary."""
    return _pmc(config).get("hbm_bytes_per_launch")


def pmc_executed(config, ker_ms, launches=1):
    """Executed fp64 flops of one request (rocprofv3 SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 x 64
    lanes of its kernels, FMA = 2, committed under profiles/) over this run's request time: the
    rate the hardware sustained, independent of any counting convention."""
    ks = _pmc(config).get("kernels", {})
    fl = [k.get("exec_fp64_flop") for k in ks.values()]
    if not fl or any(f is None for f in fl):
        return None
    tf = sum(fl) * launches / (ker_ms * 1e-3) / 1e12
    out = {"exec_fp64_flop_per_request": sum(fl) * launches, "TFLOPs": round(tf, 3),
           "frac": round(tf / PEAK_FP64_TFLOPS, 4), "source": f"profiles/pmc_traffic.json [{config}]"}
    vi = [k.get("valu_insts") for k in ks.values()]
    if vi and all(v is not None for v in vi):
        # VALU issue: the request's wave-instructions at the fully fed fp64 rate per SIMD
        # (tools/ubench/valu_rates.hip) over the SIMDs x request time -- how close the kernels
        # run to the issue bound that limits them
        n = sum(vi) * launches
        out["valu_issue"] = {"valu_wave_insts": n, "ns_per_fp64_wave_inst": NS_FP64_WAVE_INST,
                             "simds": SIMDS,
                             "frac": round(n * NS_FP64_WAVE_INST * 1e-9 / (SIMDS * ker_ms * 1e-3), 4)}
    return out


def make_roofline(flop_conv, survey_flop, t_ms, executed, traffic, alg_bytes, label,
                  **extra):
    """The roofline object over t_ms, one request's time (the smaller of the isolated HIP-event
    time and the back-to-back step time): `frac` is the counter-executed fp64 fraction of the
    request (the only hardware-anchored figure: the frozen convention charges the round-1
    kernels' flops, and SURVEY 8(d)'s per-term trig is replaced here by table + recurrence, so it
    exceeds 1 on C3); both conventions are reported beside it.  Without a committed counter pass
    for the config the frozen convention stands in (flop_basis says which).  `hbm` holds SURVEY
    8(d)'s algorithmic bytes and the counter bytes (`traffic`), each over t_ms."""
    ker_ms = t_ms
    conv_tf = flop_conv / (ker_ms * 1e-3) / 1e12
    if executed:
        ach, basis = executed["TFLOPs"], ("executed fp64 flops per request (rocprofv3 "
                                          "SQ_INSTS_VALU_*_F64 x 64 lanes, FMA = 2, "
                                          + executed["source"] + ") / request time")
        flop = executed["exec_fp64_flop_per_request"]
    else:
        ach, basis, flop = conv_tf, "frozen convention (no counter pass committed)", flop_conv
    r = {"bound": "valu_fp64", "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS,
         "unit": "TFLOP/s", "frac": round(ach / PEAK_FP64_TFLOPS, 4), "traffic": traffic,
         "flop_basis": basis, "flop_per_launch": flop, "kernel": label,
         "kernel_ms": round(ker_ms, 5),
         "valu_issue": (executed or {}).get("valu_issue"),
         "convention": {"flop_per_launch": flop_conv, "achieved_TFLOPs": round(conv_tf, 3),
                        "frac": round(conv_tf / PEAK_FP64_TFLOPS, 4),
                        "counts": f"FLOP_TAB {FLOP_TAB} / FLOP_TERM {FLOP_TERM} / FLOP_OPT "
                                  f"{FLOP_OPT} (bench.py, frozen in round 1)"},
         "survey_8d": {"flop_eq_per_launch": survey_flop,
                       "achieved_TFLOPs": round(survey_flop / (ker_ms * 1e-3) / 1e12, 3),
                       "frac": round(survey_flop / (ker_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 4),
                       "note": "716 flop-eq per CF + 120 per (set, option, k): charges per-term "
                               "trig the kernels replace by table + recurrence (DESIGN.md 4)"},
         "alg_bytes_per_launch": alg_bytes,
         "hbm": hbm_block(alg_bytes, traffic, ker_ms)}
    r.update(extra)
    return r


def hbm_block(alg_bytes, traffic, t_ms):
    """HBM side of the roofline: SURVEY 8(d)'s algorithmic bytes per launch and the rocprofv3
    counter bytes (FETCH_SIZE + WRITE_SIZE of the launch, profiles/pmc_traffic.json), each as
    GB/s over the request time, and their ratio (above 1: bytes the algorithm does not need --
    the loss hand-off's padded lines, spills, re-reads)."""
    t = t_ms * 1e-3
    out = {"alg_bytes_8d": alg_bytes, "alg_GBs": round(alg_bytes / t / 1e9, 3),
           "counter_bytes": traffic, "peak_GBs": PEAK_HBM_GBS,
           "counter_GBs": None if traffic is None else round(traffic / t / 1e9, 3),
           "counter_over_alg": None if traffic is None else round(traffic / alg_bytes, 3),
           "bytes_basis": "8(d): 25 B per option (K, T, market, type) once per launch + 104 B "
                          "per param set in + 8 B per output (price, or loss per set)"}
    out["frac"] = round((traffic if traffic is not None else alg_bytes) / t / 1e9 / PEAK_HBM_GBS,
                        6)
    return out


CONFIGS = {
    "c2": dict(nK=32, nT=32, N=256, starts=1, put_itm=False,
               workload="1,024-option synthetic surface (32 K/S x 32 T), N=256, one L-BFGS-B "
                        "function+gradient request (14 param sets) per step"),
    "c3": dict(nK=100, nT=100, N=512, starts=3, put_itm=True,
               workload="10,000-option surface (100 K/S x 100 T, puts K<S), N=512, 3 lockstep "
                        "starts x 14 param sets per step"),
    "c4": dict(nK=32, nT=32, N=256, starts=64, put_itm=False, strong=True,
               workload="64 multi-start calibrations of the 1,024-option surface (32 K/S x 32 T), "
                        "N=256: one lockstep function+gradient request of every start's 14 param "
                        "sets per step, the 64 starts sharded over the GPUs"),
    "c1": dict(nK=5, nT=3, N=128, starts=1, put_itm=False,
               workload="15-option grid (5 K x 3 T), N=128, one function+gradient request"),
    "c5": dict(gen=True, P=1_000_000, N=128,
               workload="generator batch: 1M param sets (synthetic_generator.py ranges) x 32 "
                        "calls (8 K/S in linspace(0.8, 1.2) of each sample's spot x T in "
                        "{0.25, 0.5, 1, 2}), N=128, priced in one pass per step"),
}


def calib_leg(S0, r, opts, N, n_starts, world, coll, driver, reps=3):
    """Time calibrate(maxiter=300, multi_start=n_starts) under np.random.seed(0) (starts
    sharded over the ranks at N > 1) with the given optimizer driver; max over ranks."""
    # untimed warm-up of the same driver with as many starts (first-call costs: BLAS pool,
    # surface upload paths, device buffers grown to the run's size)
    DoubleHestonJumpCalibrator(S0, r, opts, N=N).calibrate(maxiter=2, multi_start=n_starts,
                                                           driver=driver)
    # median of `reps` identical runs (each from np.random.seed(0), so the same trajectory): the
    # SciPy driver is host-bound and a single run carries the host's scheduling noise
    times = []
    for _ in range(reps):
        cal = DoubleHestonJumpCalibrator(S0, r, opts, N=N)
        if world > 1:
            dist.barrier()
        np.random.seed(0)
        t0 = time.perf_counter()
        if world > 1:
            res = calibrate_sharded(cal, maxiter=300, multi_start=n_starts, driver=driver)
        else:
            res = cal.calibrate(maxiter=300, multi_start=n_starts, driver=driver)
        times.append(time.perf_counter() - t0)
    tc = float(np.median(times))
    if world > 1:
        tt = torch.tensor([tc], dtype=torch.float64, device=coll)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tc = float(tt.item())
    return {"driver": driver, "calibrations_per_sec": 1.0 / tc, "starts_per_sec": n_starts / tc,
            "seconds": tc, "runs": reps, "iterations": int(res.iterations), "starts": n_starts,
            "final_loss": float(res.final_loss), "message": res.message,
            "lockstep_launches_rank0": int(getattr(cal, "lockstep_launches", 0)),
            "loss_evals_rank0": int(cal.loss_evals),
            "calibrate": f"calibrate(maxiter=300, multi_start={n_starts}, driver='{driver}'), "
                         "np.random.seed(0)" + (", starts sharded over ranks" if world > 1 else "")}


def _max_over_ranks(dt, world, coll):
    """Barrier, then the max of dt over the ranks (the contract's whole-job time)."""
    if world > 1:
        dist.barrier()
        tt = torch.tensor([dt], dtype=torch.float64, device=coll)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return dt


PREWARM_S = 0.25          # untimed back-to-back requests before the warm-up steps (request_bench)


def event_ms(run, stream, reps):
    """Median HIP-event time (ms) of run(j) on `stream`, one isolated call per event pair."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for j, (e0, e1) in enumerate(evs):
        e0.record(stream)
        run(j)
        e1.record(stream)
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))


def gen_batch(P, N, steps, warmup, dev, stream, rank, world=1, coll=None):
    """C5 timing: one step = price every (param set, option) of a P-sample generator batch
    (dh_surface_price_dev, strikes K_relative * spot / 100 formed on the device), after a
    host/device spot check.  -> dict(value, ms_per_step, ker_ms, P, M, N, n_chunks, surf)."""
    sptr = stream.cuda_stream
    Krel = np.tile(np.linspace(80.0, 120.0, 8), 4)
    T = np.repeat([0.25, 0.5, 1.0, 2.0], 8)
    M = T.size
    ctx = _native.default_context()
    surf = _native.Surface(ctx, Krel, T, np.ones(M, dtype=np.int8),
                           strike_mode=_native.STRIKE_PCT_SPOT)
    rs = np.random.RandomState(5 + rank)
    host = np.empty((P, 16))
    host[:, :13] = GEN_LO + (GEN_HI - GEN_LO) * rs.rand(P, 13)
    host[:, 13] = 100.0 * np.exp(np.cumsum(rs.normal(0.0003, 0.01, P)) * 0.01)  # spot walk
    host[:, 14], host[:, 15] = 0.03, 0.0
    d_params = torch.from_numpy(host).to(dev)
    d_out = torch.empty((P, M), dtype=torch.float64, device=dev)

    def run(_j=0):
        surf.price_dev(d_params.data_ptr(), P, d_out.data_ptr(), N=N, stream=sptr)

    # correctness spot check first, so that the warm-up passes run right ahead of the timed ones
    run()
    torch.cuda.synchronize()
    chk = np.arange(0, P, max(1, P // 64))
    got = d_out[torch.from_numpy(chk).to(dev)].cpu().numpy()
    ref = surf.price(host[chk], N)          # a 64-set call: the large-tile kernel (last bits differ)
    assert np.all(np.abs(got - ref) <= 1e-12 * np.abs(ref) + 1e-12), "device/host path mismatch"
    for _ in range(warmup):
        run()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    dt = _max_over_ranks(time.perf_counter() - t0, world, coll)
    ker_ms = event_ms(run, stream, max(3, min(steps, 10)))
    # launches per batch: the split path (--path split) chunks param sets so one chunk's tables
    # stay within 256 MiB (dh_kernels.hip launch_price: per set = groups x (N + 8 consts + clamp
    # words + largest group) doubles), the committed PMC bytes being per launch pair; the
    # default generator kernel (cos_gen_kernel) is one launch
    per_p = 4 * (N + 8 + 1 + 8) * 8
    n_chunks = -(-P // max(1, (256 << 20) // per_p))
    if surf.ctx.last_path == _native.PATH_GEN:      # one fused launch for the whole batch
        n_chunks = 1
    return {"value": P * M * steps * world / dt, "ms_per_step": dt / steps * 1e3,
            "ker_ms": ker_ms, "P": P, "M": M, "N": N, "n_chunks": n_chunks, "surf": surf,
            "steps": steps, "warmup": warmup}


def gen_roofline(g, config):
    """The generator batch's roofline object (over its per-batch time)."""
    P, M, N, n_chunks = g["P"], g["M"], g["N"], g["n_chunks"]
    t_ms = min(g["ker_ms"], g["ms_per_step"])
    G = 4
    flop = P * G * N * FLOP_TAB + P * M * (N - 1) * FLOP_TERM + P * M * FLOP_OPT
    survey_flop = P * G * N * 716 + P * M * N * 120
    alg_bytes = P * BYTES_8D_SET + M * BYTES_8D_OPTION + P * M * BYTES_8D_OUT
    tr = pmc_traffic(config)
    return make_roofline(flop, survey_flop, t_ms, pmc_executed(config, t_ms, n_chunks),
                         tr * n_chunks if tr else None, alg_bytes,
                         kernel_label(g["surf"].ctx) + " (all chunks of one batch, HIP events)",
                         launch_pairs=n_chunks, kernel_ms=round(g["ker_ms"], 5))


def bench_generator(args, cfg, world, rank, dev, coll, stream, cpu=None):
    """--config c5: the generator batch as the headline line."""
    g = gen_batch(cfg["P"], cfg["N"], args.steps, args.warmup, dev, stream, rank, world, coll)
    line = None
    if rank == 0:
        line = {"metric": "option-prices/sec (COS, generator batch)", "value": g["value"],
                "unit": "option-prices/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": g["ms_per_step"],
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic",
                "config": {"workload": cfg["workload"], "param_sets": g["P"], "options": g["M"],
                           "cos_terms": g["N"], "prices_per_step": g["P"] * g["M"],
                           "tail_cut": args.tail_cut, "world_size_seen": world,
                           "parallelism": f"independent batches per rank x{world}"},
                "roofline": gen_roofline(g, args.config)}
        if cpu:
            line["cpu_baseline"] = cpu
            line["speedup_vs_cpu"] = g["value"] / cpu["value"]
    e2e = None if args.no_calib else generator_end_to_end(world, rank, coll)
    if rank == 0:
        if e2e:
            line["generator_end_to_end"] = e2e
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def generator_end_to_end(world, rank, coll, n_samples=1_000_000, host_path=False):
    """generate_synthetic_calibrations(n_samples, as_arrays=True) end to end under
    np.random.seed(0): the reference's RNG draws (legacy-NumPy stream: its serial part -- the
    MT19937 twister and the walk over the polar acceptances -- on the host, everything else on the
    device at N = 1), its 5 x 3 call grid priced on the GPUs (sharded at N > 1), noise and
    per-sample losses.  host_draw_seconds = when the host's serial part ended within the call;
    host_path: also one call of the round-4 host-draw pipeline, for comparison."""
    from dhcos import generator as G
    from dhcos.distributed import generate_sharded, last_generate_stats
    if world > 1:
        dist.barrier()
    np.random.seed(0)
    t0 = time.perf_counter()
    out = generate_sharded(n_samples, None, as_arrays=True, verbose=False)
    dt = time.perf_counter() - t0
    stages = None
    if world == 1:
        st = dict(G.last_device_stats)
        stages = {k: st[k] for k in ("twister_s", "walk_s", "first_chunk_s", "total_s")}
        stages["ar1_segments_rerun"] = st["ar1_segments_rerun"]
        host_s = st["walk_s"]
    else:
        # per-stage seconds of every rank (generate_sharded's instrumentation): the max over ranks
        sec = last_generate_stats.get("seconds", {})
        keys = sorted(sec)
        v = torch.tensor([sec[k] for k in keys], dtype=torch.float64, device=coll)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        stages = {k: float(x) for k, x in zip(keys, v.tolist())}
        host_s = stages.get("locate_broadcast")
    dt = _max_over_ranks(dt, world, coll)
    del out
    t_host = None
    if host_path and world == 1:
        np.random.seed(0)
        t1 = time.perf_counter()
        G.generate_synthetic_calibrations(n_samples, None, as_arrays=True, verbose=False,
                                          draw="host")
        t_host = time.perf_counter() - t1
    if rank != 0:
        return None
    r = {"samples": n_samples, "options_per_sample": len(G.STRIKES_PCT) * len(G.MATURITIES),
         "seconds": dt, "samples_per_sec": n_samples / dt, "host_draw_seconds": host_s,
         "stages_s": stages,
         "call": "generate_synthetic_calibrations(1_000_000, as_arrays=True), np.random.seed(0)"
                 + (", sharded over ranks (generate_sharded)" if world > 1 else
                    ", device draw (dh_gen_device)")}
    if t_host is not None:
        r["host_draw_pipeline_seconds"] = t_host
    return r


def request_bench(cfg, steps, warmup, world, rank, dev, coll, stream, starts_rank=None):
    """Function+gradient requests on cfg's surface: `steps` timed back to back after `warmup`,
    each at different param sets (inputs resident in HBM), plus the median isolated request
    (HIP events) and the PCIe-inclusive host-API rate.  -> dict."""
    sptr = stream.cuda_stream
    opts, S0, r = make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    M = len(opts)
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    if starts_rank is None:
        starts_rank = cfg["starts"]
    S = 14 * starts_rank
    n_rows = steps + max(warmup, 1)
    host = step_params(cal, n_rows, starts_rank, seed=100 + rank)
    d_params = torch.from_numpy(host).to(dev)
    d_sse = torch.empty((n_rows, S), dtype=torch.float64, device=dev)
    d_bad = torch.empty((n_rows, S), dtype=torch.int32, device=dev)
    N = cfg["N"]
    ptrs = [(d_params[i].data_ptr(), d_sse[i].data_ptr(), d_bad[i].data_ptr())
            for i in range(n_rows)]
    loss_dev = surf.loss_dev

    def run(i):
        pp, ps, pb = ptrs[i % n_rows]
        loss_dev(pp, S, ps, pb, N=N, stream=sptr)

    # correctness spot check of one step against the host API (same kernel, host copies), before
    # the warm-up so that the warm-up steps run right ahead of the timed ones; the context's
    # scratch is shared, so the bench stream is drained around it
    run(steps)
    torch.cuda.synchronize()
    sse_h, bad_h, _ = surf.loss_terms(host[steps], N)
    assert np.array_equal(sse_h, d_sse[steps].cpu().numpy()), "device/host path mismatch"
    # host-API rate (PCIe-inclusive: params H2D, losses D2H, synchronous) -- reported, not
    # `value`.  Measured ahead of the warm-up: a few ms of requests that also bring the GPU from
    # the idle of the CPU-baseline leg to its sustained clock before the W warm-up steps
    prices_per_step = S * M
    n_host = max(5, min(steps, 50))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n_host):
        surf.loss_terms(host[i % n_rows], N)
    host_rate = prices_per_step * n_host / (time.perf_counter() - t0)
    # then device requests back to back for PREWARM_S of wall time (untimed, before the W warm-up
    # steps): an idle MI355X takes tens of ms to reach its sustained clock, and a 20-step timed
    # region (~1.2 ms on C3) right after a few ms of work measured 63.8 us per step against
    # 59.0 us sustained (round 5)
    n_pre = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < PREWARM_S:
        for _ in range(16):
            run(steps + n_pre % max(warmup, 1))
            n_pre += 1
        torch.cuda.synchronize()

    def timed(k):
        for i in range(warmup):
            run(steps + i)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            run(i)
        torch.cuda.synchronize()
        return _max_over_ranks(time.perf_counter() - t0, world, coll)

    dt = timed(steps)
    ker_ms = event_ms(run, stream, max(20, min(steps, 200)))
    return {"value": prices_per_step * steps * world / dt, "dt": dt,
            "ms_per_step": dt / steps * 1e3, "ker_ms": ker_ms, "S": S, "M": M, "N": N,
            "prices_per_step": prices_per_step, "opts": opts, "S0": S0, "r": r, "surf": surf,
            "host_rate": host_rate, "timed": timed, "run": run, "steps": steps,
            "prewarm_requests": n_pre,
            "groups": len({o["maturity"] for o in opts}), "n_tiles": surf.n_tiles}


def request_roofline(q, config):
    """The request's roofline object (over the smaller of its isolated and back-to-back time)."""
    S, M, N, groups, n_tiles = q["S"], q["M"], q["N"], q["groups"], q["n_tiles"]
    t_ms = min(q["ker_ms"], q["ms_per_step"])
    flop = S * groups * N * FLOP_TAB + S * M * (N - 1) * FLOP_TERM + S * M * FLOP_OPT
    alg_bytes = M * BYTES_8D_OPTION + S * BYTES_8D_SET + S * BYTES_8D_OUT
    survey_flop = S * groups * N * 716 + S * M * N * 120        # SURVEY 8(d) convention
    return make_roofline(flop, survey_flop, t_ms, pmc_executed(config, t_ms),
                         pmc_traffic(config), alg_bytes,
                         kernel_label(q["surf"].ctx) + " (one request, HIP events)",
                         kernel_ms=round(q["ker_ms"], 5),
                         time_basis="min(kernel_ms, ms_per_step): "
                                    + ("ms_per_step" if q["ms_per_step"] < q["ker_ms"]
                                       else "kernel_ms"))


def tail_cut_off_leg(q, steps=50):
    """The same requests with the adaptive tail / certified CF cut off (dh_ctx_set_tail_cut(0):
    every COS term k < N summed), to show what the cut buys."""
    ctx = q["surf"].ctx
    ctx.set_tail_cut(False)
    try:
        steps = min(steps, q["steps"])
        dt = q["timed"](steps)
        ker = event_ms(q["run"], torch.cuda.current_stream(), 20)
    finally:
        ctx.set_tail_cut(True)
    ms = dt / steps * 1e3
    return {"ms_per_step": ms, "kernel_ms": ker, "prices_per_sec": q["prices_per_step"] / (ms * 1e-3),
            "steps": steps, "cut_on_ms_per_step": q["ms_per_step"],
            "speedup_from_cut": ms / q["ms_per_step"],
            "note": "same requests, dh_ctx_set_tail_cut(0): every term k < N summed; prices "
                    "agree with the cut ones to <= 1e-13 K (tests/test_gpu_parity.py)"}


def c2_single_start_leg(world, rank, dev, coll, stream, no_calib=False):
    """configs[1] as stated: the 1,024-option N = 256 surface, its single-start request
    (14 param sets) and calibrate(300, 1) on both drivers."""
    cfg = CONFIGS["c2"]
    q = request_bench(cfg, 100, 20, world, rank, dev, coll, stream, starts_rank=1)
    out = {"workload": cfg["workload"], "ms_per_request": q["ms_per_step"],
           "kernel_ms": q["ker_ms"], "prices_per_sec": q["value"],
           "prices_per_request": q["prices_per_step"], "steps": q["steps"],
           "roofline_frac": request_roofline(q, "c2")["frac"]}
    if not no_calib:
        for drv in ("scipy", "device"):
            out[f"calibrate_1_start_{drv}"] = calib_leg(q["S0"], q["r"], q["opts"], cfg["N"], 1,
                                                        world, coll, drv)
    return out


def c1_calibration_leg(world, coll):
    """configs[0], the reference's own CPU-runnable case: calibrate(300, 3) of the 15-option
    grid on both optimizer drivers, and the SciPy driver's time over the device driver's (the
    host-bound driver's gap on the smallest surface, where the per-request round trip is all
    there is)."""
    cfg = CONFIGS["c1"]
    opts, S0, r = make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    out = {"workload": "configs[0]: " + cfg["workload"]}
    for drv in ("scipy", "device"):
        out[drv] = calib_leg(S0, r, opts, cfg["N"], 3, world, coll, drv, reps=7)
    out["scipy_over_device"] = out["scipy"]["seconds"] / out["device"]["seconds"]
    return out


REFERENCE_C1 = {"final_loss": 1.0196869185631994e-07, "iterations": 33,
                "message": "CONVERGENCE: RELATIVE REDUCTION OF F <= FACTR*EPSMCH",
                "seconds_measured_here": [132.1, 139.5], "readme_seconds": 117.8,
                "source": "SURVEY.md 3.2 / 6 (the reference run in the build container), README.md:16"}
REFERENCE_C1_START0 = {"final_loss": 9.761042426892e-05, "iterations": 0, "message": "ABNORMAL: ",
                       "seconds_measured_here": 27.7, "source": "SURVEY.md 3.2 (start 0)"}


def reference_market():
    """The reference's own calibration market (tests/test_suite.py:274-302): 15 clean calls, K in
    {90 .. 110}, T in {0.25, 0.5, 1}, priced by the reference at its true parameters, S0 = 100,
    r = 0.05 (tests/golden/calib.json, written by make_golden.py from the reference)."""
    with open(os.path.join(ROOT, "tests", "golden", "calib.json")) as fh:
        return json.load(fh)["test_market"], 100.0, 0.05


def c1_reference_market_leg(world, coll):
    """configs[0] on the reference's own market: calibrate(300, 1) and calibrate(300, 3) under
    np.random.seed(0), N = 128, both drivers, beside the reference's outcome and time."""
    opts, S0, r = reference_market()
    out = {"workload": "configs[0] on the reference's market (tests/test_suite.py:274-302): 15 "
                       "clean calls, N=128, np.random.seed(0)",
           "reference_3_starts": REFERENCE_C1, "reference_start_0": REFERENCE_C1_START0}
    for ns in (1, 3):
        for drv in ("scipy", "device"):
            c = calib_leg(S0, r, opts, 128, ns, world, coll, drv, reps=5)
            ref = REFERENCE_C1 if ns == 3 else REFERENCE_C1_START0
            rs = ref["seconds_measured_here"]
            c["speedup_vs_reference_measured"] = (np.mean(rs) if isinstance(rs, list) else rs) / \
                c["seconds"]
            out[f"calibrate_{ns}_start{'s' if ns > 1 else ''}_{drv}"] = c
    return out


def c4_sharded_leg(world, coll, reps=3):
    """configs[3]: 64 independent multi-start L-BFGS-B starts on the 1,024-option N = 256
    surface, calibrate_sharded: the starts dealt over the ranks, one all-gather (RCCL under
    nccl) of every start's record and the strict-< best start, inside the timed region; strong
    scaling (64 starts in all at any world size)."""
    cfg = CONFIGS["c4"]
    opts, S0, r = make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    out = {"workload": cfg["workload"], "scaling": "strong", "starts": cfg["starts"],
           "world_size_seen": world}
    for drv in ("scipy", "device"):
        out[drv] = calib_leg(S0, r, opts, cfg["N"], cfg["starts"], world, coll, drv, reps=reps)
    return out


def c5_leg(dev, stream, rank):
    """The metric's own N = 128: the generator batch (1M param sets x 32 options)."""
    cfg = CONFIGS["c5"]
    g = gen_batch(cfg["P"], cfg["N"], 5, 2, dev, stream, rank)
    rf = gen_roofline(g, "c5")
    generator_end_to_end(1, rank, None)          # first call: the output cache's allocations
    e2e = [generator_end_to_end(1, rank, None, host_path=(i == 1)) for i in range(3)]
    host = [r.get("host_draw_pipeline_seconds") for r in e2e if "host_draw_pipeline_seconds" in r]
    e2e = sorted(e2e, key=lambda r: r["seconds"])[1]            # the median of 3 API calls
    e2e.pop("host_draw_pipeline_seconds", None)
    if host:
        e2e["host_draw_pipeline_seconds"] = host[0]
    return {"workload": cfg["workload"], "prices_per_sec": g["value"],
            "ms_per_batch": g["ms_per_step"], "kernel_ms": g["ker_ms"], "steps": 5,
            "roofline_frac": rf["frac"], "hbm": rf["hbm"], "generator_end_to_end": e2e}


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: run N ranks under torch.distributed.run as child
    processes (never exec: nothing here has touched the GPU, and the parent only waits); rank
    0's JSON line reaches this process's stdout.  -> the launcher's exit status."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-calib", action="store_true", help="skip the full-calibration leg")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the N = 1 side legs of the c3 line (tail cut off, C2 single "
                         "start, C5 generator batch)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--path", default="auto", choices=["auto", "split", "fused"],
                    help="request kernels (libdhcos dh_ctx_set_path): auto, table+option "
                         "launches, or one fused launch")
    ap.add_argument("--tail-cut", default="on", choices=["on", "off"],
                    help="adaptive tail of the angle sums (dh_ctx_set_tail_cut; off: every COS "
                         "term summed, for A/B)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N > 1 "
                         "with several ranks on one GPU)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU-baseline processes (default min(16, os.cpu_count()))")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")

    # --gpus N launches its own N ranks when no launcher did (first, before anything touches
    # the GPU); under a launcher the world must be the one asked for
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    # CPU baseline first, on rank 0 at N = 1 only, before anything initialises the GPU (its
    # process pool forks)
    cpu = None
    if not args.no_cpu and rank == 0 and world == 1:
        c_opts, c_S0, c_r = cpu_options(cfg)
        cpu = cpu_baseline(c_opts, c_S0, c_r, cfg["N"], args.cpu_budget, args.cpu_cores)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if args.backend == "nccl":
        # one rank per GPU: RCCL refuses two ranks on one device, and a rank must never fall
        # back to a shared one silently
        if n_dev < world or local >= n_dev:
            sys.exit(f"bench.py: --gpus {world} needs {world} visible GPUs (rank {rank}, "
                     f"LOCAL_RANK {local}, {n_dev} visible); --backend gloo rehearses several "
                     "ranks on one GPU")
    else:
        if n_dev < 1:
            sys.exit("bench.py: no GPU visible")
        local = local % n_dev                # gloo rehearsal: ranks may share a GPU
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll = dev if args.backend == "nccl" else torch.device("cpu")   # collective tensors
    world_seen = dist.get_world_size() if world > 1 else 1
    if world_seen != world:
        sys.exit(f"bench.py: process group has {world_seen} ranks, expected {world}")
    if world > 1:                        # every rank on its own device under RCCL
        t = torch.tensor([local], dtype=torch.int64, device=coll)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        devs = [int(p.item()) for p in parts]
        if args.backend == "nccl" and len(set(devs)) != world:
            sys.exit(f"bench.py: ranks share GPUs under RCCL: {devs}")
    os.environ["DHCOS_DEVICE"] = str(local)
    _native.default_context().set_path({"auto": _native.PATH_AUTO, "split": _native.PATH_SPLIT,
                                        "fused": _native.PATH_FUSED}[args.path])
    _native.default_context().set_tail_cut(args.tail_cut == "on")
    # a dedicated (non-null) stream: libdhcos launches on it and the HIP events time it.  By
    # default the context's own stream (wrapped, not created: a torch.cuda.Stream() builds
    # torch's whole stream pool, dozens of HIP streams over the process's 4 hardware queues, and
    # the calibration legs measured 4-8% slower next to it; DHCOS_BENCH_STREAM=torch: that)
    if os.environ.get("DHCOS_BENCH_STREAM", "ctx") == "torch":
        stream = torch.cuda.Stream(device=dev)
    else:
        stream = torch.cuda.ExternalStream(_native.default_context().stream, device=dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream, "expected a non-default HIP stream"
    if cfg.get("gen"):
        return bench_generator(args, cfg, world, rank, dev, coll, stream, cpu)

    # c4 deals its 64 starts over the ranks (strong scaling); the others run a fixed request per
    # rank (weak scaling)
    starts_rank = -(-cfg["starts"] // world) if cfg.get("strong") else cfg["starts"]
    q = request_bench(cfg, args.steps, args.warmup, world, rank, dev, coll, stream, starts_rank)
    roofline = request_roofline(q, args.config)
    opts, S0, r, N, M = q["opts"], q["S0"], q["r"], q["N"], q["M"]

    # side legs (N = 1, the default c3 line): what the cuts buy, configs[1] as stated (single
    # start), and the metric's own N = 128 (the generator batch)
    side = {}
    if world == 1 and args.config == "c3" and not args.no_side:
        if args.tail_cut == "on":
            side["tail_cut_off"] = tail_cut_off_leg(q)
        side["c2_single_start"] = c2_single_start_leg(world, rank, dev, coll, stream,
                                                      args.no_calib)
        side["c5_generator_n128"] = c5_leg(dev, stream, rank)
        if not args.no_calib:
            side["c1_reference_market"] = c1_reference_market_leg(world, coll)
            side["c1_calibration"] = c1_calibration_leg(world, coll)
    # the north star's two 8-GPU configurations, at every world size (N = 1 is their baseline):
    # C4's 64 starts sharded with the RCCL gather, C5's generator sharded end to end
    if args.config == "c3" and not args.no_side and not args.no_calib:
        side["c4_sharded_64_starts"] = c4_sharded_leg(world, coll)
        if world > 1:
            side["c5_generator_sharded"] = generator_end_to_end(world, rank, coll)

    # ---- calibrations/sec: one full calibration of the same surface; at N > 1 its starts are
    # sharded over the ranks (dhcos.distributed; the config's starts per GPU, weak scaling; c4:
    # 64 starts in all, strong scaling).  Two optimizer drivers: SciPy's setulb on the host (the
    # reference's optimizer bit for bit, one launch + one host round trip per lockstep request)
    # and the device-resident L-BFGS-B (dh_calibrate_lbfgs) ----
    calib = calib_dev = None
    if not args.no_calib:
        n_starts = cfg["starts"] if cfg.get("strong") else cfg["starts"] * world
        calib = calib_leg(S0, r, opts, N, n_starts, world, coll, "scipy")
        calib_dev = calib_leg(S0, r, opts, N, n_starts, world, coll, "device")

    if rank == 0:
        line = {
            "metric": "option-prices/sec (COS, calibration objective) + calibrations/sec",
            "value": q["value"], "unit": "option-prices/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": q["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if cfg.get("strong") else "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": cfg["workload"], "options": M, "cos_terms": N,
                       "tail_cut": args.tail_cut, "param_sets_per_step": q["S"],
                       "prices_per_step": q["prices_per_step"], "world_size_seen": world_seen,
                       "backend": args.backend if world > 1 else None,
                       "parallelism": f"independent requests per rank x{world}"},
            "roofline": roofline,
            "host_api_prices_per_sec": q["host_rate"],
            "prewarm": {"seconds": PREWARM_S, "requests": q["prewarm_requests"],
                        "note": "untimed device requests before the warm-up steps, to the "
                                "sustained clock"},
        }
        line.update(side)
        if calib:
            line["calibration"] = calib
            line["calibration_device"] = calib_dev
        if cpu:
            line["cpu_baseline"] = cpu
            line["speedup_vs_cpu"] = q["value"] / cpu["value"]
            if calib and world == 1:
                # the same calibration on the CPU port: every loss evaluation prices M options
                for c in (calib, calib_dev):
                    cpu_s = c["loss_evals_rank0"] * M / line["cpu_baseline"]["value"]
                    c["cpu_port_seconds_extrapolated"] = cpu_s
                    c["speedup_vs_cpu"] = cpu_s / c["seconds"]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
