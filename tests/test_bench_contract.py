"""bench.py's output contract (the driver parses its last line): one JSON object with the metric
and unit of BASELINE.json, the whole-job value, the timing fields, config.workload, the roofline
object and -- on rank 0 at N = 1 -- the CPU baseline object.  Runs a short C1 bench on the GPU
(a child process, as the driver runs it); the CPU baseline leg gets a 1 s budget."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.gpu
def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--steps", "5",
           "--warmup", "2", "--no-calib", "--cpu-budget", "1", "--cpu-cores", "2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["metric"].startswith("option-prices/sec") and base["metric"].startswith(
        "option-prices/sec")
    assert line["unit"] == "option-prices/s" and line["value"] > 0
    assert (line["n_gpus"], line["steps"], line["warmup"]) == (1, 5, 2)
    assert line["higher_is_better"] is True and line["scaling"] in ("weak", "strong")
    assert line["vs_baseline"] is None and line["dtype"] == "f64"
    assert "workload" in line["config"]
    # value = prices of one step / step time (ms_per_step in milliseconds)
    per_step = line["config"]["prices_per_step"]
    assert abs(line["value"] * line["ms_per_step"] * 1e-3 - per_step) <= 1e-6 * per_step
    r = line["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = line["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["value"] > 0 and c["cores"] == 2
    assert c["sample"]


@pytest.mark.gpu
def test_bench_line_contract_two_ranks():
    """The driver's N > 1 launch shape (torch.distributed.run, one JSON line from rank 0), rehearsed
    with two gloo ranks sharing the box's one GPU: n_gpus = 2, weak scaling, value = both ranks'
    prices per step / the max-over-ranks step time, no CPU-baseline leg at N > 1."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--config", "c1", "--steps", "5", "--warmup", "2", "--no-calib",
           "--backend", "gloo"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and "cpu_baseline" not in line
    per_step = line["config"]["prices_per_step"]
    got = line["value"] * line["ms_per_step"] * 1e-3
    assert abs(got - 2 * per_step) <= 1e-6 * per_step     # prices_per_step is per rank


@pytest.mark.gpu
def test_bench_self_launches_ranks():
    """`bench.py --gpus 2` without an external launcher starts its two ranks itself (child
    processes under torch.distributed.run) and reports the world the process group saw; gloo
    lets both ranks share the box's one GPU."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c1",
           "--steps", "5", "--warmup", "2", "--no-calib", "--backend", "gloo"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["world_size_seen"] == 2


def _bench_rc(args, env_extra=None, timeout=120):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    if not env_extra or "WORLD_SIZE" not in env_extra:
        env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_bench_world_mismatch_fails():
    """A launcher's world that differs from --gpus is an error, not a silent one-rank run."""
    out = _bench_rc(["--gpus", "1", "--config", "c1", "--no-cpu"],
                    {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in out.stderr


def test_bench_rccl_ranks_need_their_gpus():
    """--gpus 2 under RCCL (the default backend) on a host with fewer than two GPUs fails loudly
    in every rank instead of running on a shared device (here: no GPU at all)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("host has two GPUs")
    out = _bench_rc(["--gpus", "2", "--config", "c1", "--no-cpu", "--no-calib"])
    assert out.returncode != 0
    assert "needs 2 visible GPUs" in out.stderr


@pytest.mark.gpu
def test_bench_side_legs_two_ranks():
    """The north star's 8-GPU configurations in the N > 1 line, rehearsed with
    two gloo ranks on the box's one GPU: C4 (64 starts sharded with the gather of their records,
    both drivers, strong scaling) and C5 (generate_sharded end to end, with the ranks' stage
    times), each reporting the world it saw."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29541",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c3", "--steps", "3",
           "--warmup", "1", "--no-cpu", "--backend", "gloo"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["world_size_seen"] == 2
    c4 = line["c4_sharded_64_starts"]
    assert c4["world_size_seen"] == 2 and c4["starts"] == 64 and c4["scaling"] == "strong"
    for drv in ("scipy", "device"):
        assert c4[drv]["starts"] == 64 and c4[drv]["calibrations_per_sec"] > 0
        assert c4[drv]["final_loss"] < 1e9
    c5 = line["c5_generator_sharded"]
    assert c5["samples"] == 1_000_000 and c5["seconds"] > 0 and "sharded" in c5["call"]
    assert set(c5["stages_s"]) >= {"locate_broadcast", "draw", "price", "gather"}
