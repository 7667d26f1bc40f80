"""The production runner on the device: hipGraph generations + metrics + sampled
trajectories + checkpoint/resume, bitwise equal to an uninterrupted run."""
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.config import ExperimentConfig, RecorderConfig, RunConfig, SoupConfig
from self_replicating_neural_networks_amd.run import run

pytestmark = pytest.mark.gpu

SOUP = SoupConfig(attacking_rate=0.1, learn_from_rate=0.1, train=5, remove_divergent=True, remove_zero=True)


def _cfg(**kw):
    base = dict(n_total=20000, generations=8, seed=9, device="cuda", graph=True)
    base.update(kw)
    return ExperimentConfig(arch=ArchSpec.weightwise(2, 2), soup=SOUP, run=RunConfig(**base)).validate()


def test_runner_graph_resume_bitwise(cuda, tmp_path):
    straight, _ = run(_cfg(), log=lambda s: None)
    ck = str(tmp_path / "ck")
    run(_cfg(generations=4, checkpoint_dir=ck, checkpoint_every=2, metrics_path=str(tmp_path / "m.jsonl"),
             recorder=RecorderConfig(policy="subset", subset=100, every=2)), log=lambda s: None)
    eng, out = run(_cfg(checkpoint_dir=ck, checkpoint_every=2), resume=True, log=lambda s: None)
    assert eng.time == 8
    assert torch.equal(eng.local_rows(), straight.local_rows())
    assert torch.equal(eng.uid, straight.uid)
    assert out["census"] == straight.count()
