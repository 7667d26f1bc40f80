"""bench.py's launcher contract on the CPU (host rehearsal of the same engine over gloo):
``--gpus N`` without torchrun's environment starts N ranks itself and reports n_gpus = N;
a launcher whose WORLD_SIZE disagrees with ``--gpus`` makes it exit non-zero instead of
reporting a number for another GPU count."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", **kw)
    return env


def test_bench_self_launch_cpu_two_ranks():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1",
                        "--particles-per-gpu", "1500", "--train", "2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 3000 and d["config"]["device"] == "cpu"
    assert d["config"]["parallelism"] == "population-dp2"
    assert "train=2" in d["config"]["model"]  # the config string follows the actual parameters
    assert sum(d["config"]["final_census"].values()) == 3000


def test_bench_world_size_mismatch_exits_nonzero():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--device", "cpu", "--steps", "1"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
