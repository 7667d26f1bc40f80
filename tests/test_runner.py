"""Config system, production runner (checkpoint / exact resume), metrics stream, sampled
trajectory recorder, fault injection, profiling helpers on CPU."""
import json
import os

import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.config import ExperimentConfig, RecorderConfig, RunConfig, SoupConfig
from self_replicating_neural_networks_amd.recorder import TrajectoryRecorder, load_trajectory
from self_replicating_neural_networks_amd.run import latest_checkpoint, main as run_main, run
from self_replicating_neural_networks_amd.soup_engine import SoupEngine
from self_replicating_neural_networks_amd.utils import profiling
from self_replicating_neural_networks_amd.utils.metrics import MetricsWriter, read_metrics

SOUP = SoupConfig(attacking_rate=0.2, learn_from_rate=0.2, train=2, remove_divergent=True, remove_zero=True)


def _cfg(tmp_path, **run_kw):
    kw = dict(n_total=150, generations=6, seed=4, device="cpu", graph=False)
    kw.update(run_kw)
    return ExperimentConfig(arch=ArchSpec.weightwise(2, 2), soup=SOUP, run=RunConfig(**kw)).validate()


def test_config_json_round_trip():
    cfg = ExperimentConfig(arch=ArchSpec.aggregating(4, 2, 2, shuffler="random"), soup=SOUP,
                           run=RunConfig(n_total=10, recorder=RecorderConfig(policy="subset", subset=3)))
    back = ExperimentConfig.from_json(cfg.to_json())
    assert back == cfg
    assert cfg.replace(run=dict(n_total=99)).run.n_total == 99
    with pytest.raises(ValueError):
        cfg.replace(run=dict(dtype="int8"))
    with pytest.raises(ValueError):
        RecorderConfig(policy="sometimes").validate()
    # reference Soup.params names and defaults (code/soup.py:17-18)
    d = SoupConfig().params()
    assert d["attacking_rate"] == 0.1 and d["learn_from_rate"] == 0.1 and d["train"] == 0
    assert d["learn_from_severity"] == 1


def test_runner_checkpoint_resume_is_exact(tmp_path):
    straight, _ = run(_cfg(tmp_path, generations=6), log=lambda s: None)
    ck = str(tmp_path / "ck")
    eng1, _ = run(_cfg(tmp_path, generations=4, checkpoint_dir=ck, checkpoint_every=2), log=lambda s: None)
    assert latest_checkpoint(ck).endswith("gen-000000004")
    assert not any(p.endswith(".tmp") for p in os.listdir(ck))
    eng2, out = run(_cfg(tmp_path, generations=6, checkpoint_dir=ck, checkpoint_every=2), resume=True,
                    log=lambda s: None)
    assert eng2.time == 6
    assert torch.equal(eng2.local_rows(), straight.local_rows())
    assert torch.equal(eng2.uid, straight.uid)
    assert int(eng2.next_uid) == int(straight.next_uid)
    assert out["census"] == straight.count()


def test_runner_cli_metrics_and_trajectory(tmp_path, capsys):
    ck, mp = str(tmp_path / "ck"), str(tmp_path / "m.jsonl")
    cfg = _cfg(tmp_path, metrics_path=mp, checkpoint_dir=ck, checkpoint_every=3,
               recorder=RecorderConfig(policy="subset", subset=7, every=2))
    p = tmp_path / "cfg.json"
    p.write_text(cfg.to_json())
    assert run_main(["--config", str(p), "--set", "run.generations=6"]) == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    assert lines[0]["event"] == "start" and lines[-1]["event"] == "done"
    recs = read_metrics(mp)
    assert [r["generation"] for r in recs] == [1, 2, 3, 4, 5, 6]
    for r in recs:
        assert sum(r["census"].values()) == 150
        assert abs(sum(r["fractions"].values()) - 1) < 1e-9
    assert all(r["respawns"] >= 0 for r in recs[1:])
    z = load_trajectory(os.path.join(ck, "trajectories", "trajectory-r0000.npz"))
    assert list(z["generation"]) == [2, 4, 6]
    assert z["weights"].shape == (3, 7, 14)
    assert len(set(z["slots"].tolist())) == 7


def test_trajectory_recorder_matches_engine_rows():
    eng = SoupEngine(ArchSpec.weightwise(2, 2), 64, SOUP.params(), seed=1)
    rec = TrajectoryRecorder(eng, RecorderConfig(policy="full", every=1, capacity=2))
    snaps = []
    for _ in range(3):
        eng.evolve(1)
        rec.maybe_record(eng, eng.time)
        snaps.append(eng.local_rows()[:, :14].clone())
    gen, uid, W = rec.arrays()
    assert list(gen) == [2, 3]  # ring of 2
    assert np.array_equal(W[-1], snaps[-1].numpy())
    assert np.array_equal(uid[-1], eng.uid.numpy())
    st = rec.states()
    assert all(s["class"] == "WeightwiseNeuralNetwork" for v in st.values() for s in v)


def test_inject_nan_is_detected_and_respawned():
    eng = SoupEngine(ArchSpec.weightwise(2, 2), 100, dict(SOUP.params(), attacking_rate=0.0, learn_from_rate=0.0,
                                                          train=0), seed=2)
    eng.inject_nan([3, 50])
    assert eng.count()["divergent"] >= 2
    nu = int(eng.next_uid)
    eng.evolve(1)
    assert int(eng.next_uid) >= nu + 2           # both poisoned rows were reborn with new uids
    assert torch.isfinite(eng.local_rows()[[3, 50]]).all()
    with pytest.raises(IndexError):
        eng.inject_nan([100])


def test_metrics_writer_throughput(tmp_path):
    w = MetricsWriter(str(tmp_path / "x.jsonl"), every=2)
    assert w.due(2) and not w.due(3)
    w.log(2, {"divergent": 1, "other": 3}, 4)
    r = w.log(4, {"other": 4}, 4)
    assert r["ms_per_generation"] > 0 and r["fixpoint_fraction"] == 0.0
    w.close()
    assert len(read_metrics(str(tmp_path / "x.jsonl"))) == 2


def test_profiling_helpers():
    with profiling.roctx_range("test-range"):  # no-op or real range, never raises
        pass
    t = profiling.PhaseTimer("cpu")
    with t.phase("a"):
        sum(range(1000))
    s = t.summary()
    assert s["a"]["calls"] == 1 and s["a"]["ms"] >= 0
    profiling.check_pmc_pass(profiling.PMC_SETS["valu_mfma"])
    with pytest.raises(ValueError):
        profiling.check_pmc_pass(["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                                  "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VMEM"])
    with pytest.raises(ValueError):
        profiling.check_pmc_pass(["FETCH_SIZE", "WRITE_SIZE"])  # 5 TCC slots > 4
    cmds = profiling.rocprof_commands(["python3", "bench.py"], sets=["valu_mfma", "hbm"])
    assert cmds[0][:5] == ["timeout", "-k", "10", "120", "rocprofv3"]
    assert all(c[c.index("--") + 1] == "python3" for c in cmds)  # program right after --
    assert not any("--sys-trace" in c for c in cmds)


def test_runner_runs_the_reference_order_by_default_and_resumes_it(tmp_path):
    """RunConfig.order defaults to the reference's sequential order; the runner's checkpoints
    record it and --resume continues it bitwise; a resume with the other order raises"""
    assert RunConfig().order == "sequential"
    straight, out = run(_cfg(tmp_path, generations=5), log=lambda s: None)
    assert straight.order == "sequential" and out["order"] == "sequential"
    ref = SoupEngine(ArchSpec.weightwise(2, 2), 150, SOUP.params(), seed=4, order="sequential").evolve(5)
    assert torch.equal(straight.local_rows(), ref.local_rows())
    ck = str(tmp_path / "ck")
    run(_cfg(tmp_path, generations=2, checkpoint_dir=ck, checkpoint_every=2), log=lambda s: None)
    eng, _ = run(_cfg(tmp_path, generations=5, checkpoint_dir=ck, checkpoint_every=3), resume=True,
                 log=lambda s: None)
    assert eng.order == "sequential" and eng.time == 5
    assert torch.equal(eng.local_rows(), straight.local_rows()) and torch.equal(eng.uid, straight.uid)
    with pytest.raises(ValueError, match="change its dynamics"):
        run(_cfg(tmp_path, generations=6, checkpoint_dir=ck, checkpoint_every=3, order="synchronous"), resume=True,
            log=lambda s: None)
    with pytest.raises(ValueError):
        _cfg(tmp_path, order="gauss-seidel")
