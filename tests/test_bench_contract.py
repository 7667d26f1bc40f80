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


def _bench(*args, timeout=300):
    p = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--steps", "2", "--warmup", "1", "--train", "2",
                        *args], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_self_launch_cpu_two_ranks_weak():
    d = _bench("--gpus", "2", "--scaling", "weak", "--particles-per-gpu", "1500")
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 3000 and d["config"]["device"] == "cpu"
    assert d["scaling"] == "weak" and d["config"]["particles_per_gpu"] == 1500
    assert d["config"]["parallelism"] == "population-dp2" and d["config"]["world_size"] == 2
    assert "train=2" in d["config"]["model"]  # the config string follows the actual parameters
    assert sum(d["config"]["final_census"].values()) == 3000


def test_bench_strong_scaling_default_one_and_two_ranks():
    """strong scaling (the default) keeps ONE soup of --particles at any rank count; the
    execution knobs in force are part of the line"""
    one = _bench("--particles", "2000")
    two = _bench("--gpus", "2", "--particles", "2000")
    for d, n in ((one, 1), (two, 2)):
        assert d["scaling"] == "strong" and d["n_gpus"] == n
        assert d["config"]["global_batch"] == 2000 and d["config"]["particles_per_gpu"] == 2000 / n
        assert sum(d["config"]["final_census"].values()) == 2000
        ex = d["config"]["execution"]
        assert ex["x2_schedule"] == "serial" and ex["finish_mode"] == "batch" and ex["graph_chunks"][0] == 20
        assert set(ex["library"]) >= {"ww_wave", "rnn_wave", "soup_lanes"}
    # the same soup, bitwise: rank count does not change the census
    assert one["config"]["final_census"] == two["config"]["final_census"]


def test_bench_weak_scaling_one_rank():
    d = _bench("--scaling", "weak", "--particles-per-gpu", "1200")
    assert d["scaling"] == "weak" and d["config"]["global_batch"] == 1200


def test_bench_world_size_mismatch_exits_nonzero():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--device", "cpu", "--steps", "1"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr


def test_bench_headline_is_the_reference_order():
    """the headline `value` is the reference's own soup semantics (in place, index order); a 1-rank
    run (the driver's BENCH form) carries the Jacobi variant of the same soup beside it
    (config.jacobi), and --order synchronous swaps the two"""
    d = _bench("--particles", "1500")
    assert d["semantics"] == "reference-order" and d["config"]["order"] == "sequential"
    assert "reference (sequential) order" in d["config"]["model"]
    lv = d["config"]["ordered_levels"]
    assert lv["error"] == 0 and sum(lv["levels"]) + lv["tail"] == 1500
    assert d["config"]["ord_pipeline"] == "stream" and d["config"]["reference_order"] is None
    j = d["config"]["jacobi"]
    assert j is not None and j["semantics"] == "jacobi" and j["steps"] == d["steps"]
    assert j["ms_per_step"] > 0 and j["value"] > 0 and sum(j["final_census"].values()) == 1500
    off = _bench("--particles", "1500", "--side-steps", "0")
    assert off["config"]["jacobi"] is None and off["config"]["reference_order"] is None
    # the same reference-order soup whatever else runs in the process
    assert off["config"]["final_census"] == d["config"]["final_census"]
    sync = _bench("--particles", "1500", "--order", "synchronous")
    assert sync["semantics"] == "jacobi" and sync["config"]["jacobi"] is None
    ro = sync["config"]["reference_order"]
    assert ro["semantics"] == "reference-order" and ro["final_census"] == d["config"]["final_census"]
    assert ro["levels"]["error"] == 0
    # the old spelling of the side-measurement flag still works
    assert _bench("--particles", "1500", "--reference-order-steps", "0")["config"]["jacobi"] is None


def test_bench_reference_order_on_two_ranks():
    """the reference order shards: --gpus 2 is the sharded reference order by default, with the
    census of the 1-rank run (bitwise the same soup on any rank count); the Jacobi side number on
    several ranks is on request only"""
    two = _bench("--gpus", "2", "--particles", "1200")
    assert two["n_gpus"] == 2 and two["semantics"] == "reference-order"
    assert two["config"]["jacobi"] is None  # on request only
    one = _bench("--particles", "1200", "--side-steps", "0")
    assert two["config"]["final_census"] == one["config"]["final_census"]
    side = _bench("--gpus", "2", "--particles", "1200", "--order", "synchronous", "--side-steps", "-1")
    assert side["semantics"] == "jacobi"
    assert side["config"]["reference_order"]["final_census"] == one["config"]["final_census"]
