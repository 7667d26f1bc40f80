"""bench.py's driver contract, end to end on one MI355X: one JSON line from rank 0 with the
BASELINE.json metric, whole-job value = particles x steps / max-rank time, for N=1 and for N=2
-- launched by torch.distributed.run, and by bench.py itself when no launcher is around
(2 ranks sharing cuda:0 over gloo: RCCL refuses two ranks on one device, so this rehearses the
multi-rank control flow, not xGMI)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(cmd, timeout=100):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _check(d, n, steps, warmup, total, scaling="strong"):
    assert KEYS <= set(d)
    assert d["metric"] == "self-application steps/sec (whole node) for 100k-particle soup"
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == scaling and d["dtype"] == "fp32"
    assert d["config"]["global_batch"] == total and d["config"]["particles_per_gpu"] == total / n
    assert d["value"] == pytest.approx(total * steps / (d["ms_per_step"] * steps * 1e-3), rel=1e-6)
    assert sum(d["config"]["final_census"].values()) == total


@pytest.mark.gpu
def test_bench_single_gpu_line():
    d = _run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--particles", "20000"])
    _check(d, 1, 4, 1, 20000)
    w = _run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--scaling", "weak",
              "--particles-per-gpu", "20000"])
    _check(w, 1, 4, 1, 20000, "weak")


@pytest.mark.gpu
def test_bench_two_ranks_torchrun_gloo_shared_device():
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", "29633", "bench.py", "--gpus", "2", "--steps", "3",
              "--warmup", "1", "--scaling", "weak", "--particles-per-gpu", "20000", "--share-device",
              "--backend", "gloo"])
    _check(d, 2, 3, 1, 40000, "weak")


@pytest.mark.gpu
def test_bench_launches_its_own_ranks():
    """--gpus 2 without torchrun's env: bench.py starts the ranks itself (child process)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--particles", "20000", "--share-device", "--backend", "gloo"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    _check(json.loads(lines[0]), 2, 3, 1, 20000)  # strong: one 20k soup over two ranks
