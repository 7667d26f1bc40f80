"""Execution knobs (config.ExecConfig): JSON round trip inside RunConfig, environment
variables as overrides, the library knobs in force, and the engines reading the config
instead of the environment.  Plus the planner's byte model against a constructed engine
(engine_bytes vs the tensors a SoupEngine really holds)."""
import json

import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.config import ExecConfig, ExperimentConfig, RunConfig
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.soup_engine import SoupEngine, _finish_batch, engine_bytes, plan_population


def test_exec_config_round_trip():
    ex = ExecConfig(finish_mode="serial", graph_chunks=(8, 4), x2_schedule="overlap", ww_wave=False, soup_lanes=2)
    cfg = ExperimentConfig(run=RunConfig(n_total=64, execution=ex))
    back = ExperimentConfig.from_json(cfg.to_json())
    assert back.run.execution == ex
    d = json.loads(cfg.to_json())["run"]["execution"]
    assert d["graph_chunks"] == [8, 4] and d["x2_schedule"] == "overlap" and d["soup_lanes"] == 2


def test_exec_config_validation():
    with pytest.raises(ValueError):
        ExecConfig(finish_mode="x").validate()
    with pytest.raises(ValueError):
        ExecConfig(graph_chunks=(3,)).validate()
    with pytest.raises(ValueError):
        ExecConfig(x2_schedule="fast").validate()


def test_environment_overrides_config(monkeypatch):
    monkeypatch.setenv("SRNN_X2_SCHEDULE", "overlap")
    monkeypatch.setenv("SRNN_GRAPH_CHUNKS", "6,2")
    monkeypatch.setenv("SRNN_FINISH_PAR", "0")
    r = ExecConfig(x2_schedule="serial").resolved()
    assert r.x2_schedule == "overlap" and r.graph_chunks == (6, 2) and r.finish_par is False


def test_engine_reads_config_not_environment():
    spec = ArchSpec.weightwise(2, 2)
    e = SoupEngine(spec, 256, dict(train=1), device="cpu", execution=ExecConfig(graph_chunks=(6, 2)))
    assert e._chunk_sizes() == [6, 2]
    assert e.execution.finish_mode == "batch"


def test_library_knobs_set_and_overridden(monkeypatch):
    try:
        ExecConfig(ww_wave=False, soup_lanes=2).apply_library()
        assert _lib.get_knob("ww_wave") == 0 and _lib.get_knob("soup_lanes") == 2
        monkeypatch.setenv("SRNN_WW_WAVE", "1")
        assert _lib.get_knob("ww_wave") == 1  # the environment variable wins
        assert ExecConfig().in_force()["library"]["ww_wave"] == 1
    finally:
        _lib.set_knob("ww_wave", -1)
        _lib.set_knob("soup_lanes", -1)
    monkeypatch.delenv("SRNN_WW_WAVE")
    assert _lib.get_knob("ww_wave") == -1


def _held_bytes(e: SoupEngine) -> int:
    seen, total = set(), 0
    for t in e._state():
        if t is None or t.data_ptr() in seen:
            continue
        seen.add(t.data_ptr())
        total += t.numel() * t.element_size()
    return total


@pytest.mark.parametrize("n,diag", [(1000, True), (5000, False), (64, True)])
def test_engine_bytes_matches_a_constructed_single_rank_engine(n, diag):
    spec = ArchSpec.weightwise(2, 2)
    e = SoupEngine(spec, n, dict(train=1), device="cpu", diagnostics=diag)
    est = engine_bytes(spec, n, diagnostics=diag)
    held = _held_bytes(e)
    if e._bs_ring is None:  # the batched-finish ring is a GPU-only buffer: add what a GPU engine holds
        nb = max(-(-n // 64), 1)
        held += _finish_batch(nb, e._chunk_sizes()) * (nb * 8 + 2) * 4
    # the model may round a few small control tensors up; never low by more than 1 %
    assert est >= held * 0.99 and est <= held * 1.05 + 512, (est, held)


def test_plan_returns_the_engine_arguments_it_assumed():
    p = plan_population(ArchSpec.weightwise(2, 2), torch.float16, world=8)
    assert p["engine_kwargs"]["diagnostics"] is False and p["engine_kwargs"]["dtype"] == torch.float16

