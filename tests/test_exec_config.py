"""Execution knobs (config.ExecConfig): JSON round trip inside RunConfig, environment
variables as overrides, the library knobs in force, and the engines reading the config
instead of the environment.  Plus the planner's byte model against a constructed engine
(engine_bytes vs the tensors a SoupEngine really holds)."""
import os
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


@pytest.mark.parametrize("val,want", [("-1", None), ("", "unset"), ("auto", None), ("0", False), ("1", True),
                                      ("off", False)])
def test_tri_state_knobs_parse_as_tri_state(monkeypatch, val, want):
    """SRNN_FIX_GROUP / SRNN_PERM_TABLE: -1 (or auto) is "by population size", not True"""
    monkeypatch.setenv("SRNN_FIX_GROUP", val)
    monkeypatch.setenv("SRNN_PERM_TABLE", val)
    r = ExecConfig(fix_group=True).resolved()
    if want == "unset":  # empty: the config's own value stays
        assert r.fix_group is True and r.perm_table is None
    else:
        assert r.fix_group is want and r.perm_table is want


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


@pytest.mark.parametrize("order", ["synchronous", "sequential"])
@pytest.mark.parametrize("n,diag", [(1000, True), (5000, False), (64, True)])
def test_engine_bytes_matches_a_constructed_single_rank_engine(n, diag, order):
    spec = ArchSpec.weightwise(2, 2)
    e = SoupEngine(spec, n, dict(train=1), device="cpu", diagnostics=diag, order=order)
    est = engine_bytes(spec, n, diagnostics=diag, order=order, epochs=2)
    held = _held_bytes(e)
    if e._bs_ring is None:  # the batched-finish ring is a GPU-only buffer: add what a GPU engine holds
        nb = max(-(-n // 64), 1)
        held += _finish_batch(nb, e._chunk_sizes()) * (nb * 8 + 2) * 4
    if order == "sequential":
        # the pending records' permutation tables (one per plan set: the next generation's plan is
        # built while this one runs) are GPU-only buffers too (train 1 + severity 1)
        assert getattr(e, "_ptab", None) is None and e._ord_pipe and e._osrc1 is not None
        held += 2 * (2 * _lib.ord_rec_total(n) * 2 * 8)
        assert est > engine_bytes(spec, n, diagnostics=diag) + n * spec.PP * 4  # W3 alone is a table
    # the model may round a few small control tensors up; never low by more than 1 %
    assert est >= held * 0.99 and est <= held * 1.05 + 512, (est, held)


@pytest.mark.parametrize("world,rank", [(8, 0), (8, 7), (3, 1)])
@pytest.mark.parametrize("exchange", ["alltoall", "allgather"])
def test_engine_bytes_of_a_sharded_reference_order_rank(world, rank, exchange):
    """order='sequential' over several ranks: the estimate covers what one rank of the sharded
    reference order really allocates -- the replicated plan and version tables of ALL turns on the
    all-gather layout (whatever `exchange` says), no permutation table"""
    from self_replicating_neural_networks_amd.parallel.dist import Dist
    spec = ArchSpec.weightwise(2, 2)
    n = 5003
    e = SoupEngine(spec, n, dict(train=1), device="cpu", dist=Dist(world=world, rank=rank), exchange=exchange,
                   order="sequential")
    assert not e.x2 and not e._ord_pipe and e._perm_table() is None
    est = engine_bytes(spec, n, world=world, exchange=exchange, order="sequential", epochs=2)
    held = _held_bytes(e)
    assert est >= held * 0.99 and est <= held * 1.05 + 512, (est, held)
    # the replicated O(n_total) buffers dominate: far more than n_total / world rows' worth
    assert est > engine_bytes(spec, n, world=world, exchange="allgather") + n * spec.PP * 4 * 2


def test_sharded_reference_order_plan_is_capped_by_the_whole_soup():
    """every rank plans all n_total turns (int32 version codes): the soup, not a shard, stays
    below 2^30, and the plan fits the replicated buffers"""
    spec = ArchSpec.weightwise(2, 2)
    p = plan_population(spec, torch.float16, world=8, order="sequential", epochs=21)
    assert p["n_total"] <= 2 ** 30 - 1
    assert p["bytes_per_gpu"] <= 0.9 * 288e9
    assert p["bytes_per_gpu"] == engine_bytes(spec, p["n_total"], world=8, dtype=torch.float16, order="sequential",
                                              epochs=21, diagnostics=False)


def test_plan_returns_the_engine_arguments_it_assumed():
    p = plan_population(ArchSpec.weightwise(2, 2), torch.float16, world=8)
    assert p["engine_kwargs"]["diagnostics"] is False and p["engine_kwargs"]["dtype"] == torch.float16
    q = plan_population(ArchSpec.weightwise(2, 2), torch.float16, world=1, order="sequential", epochs=21)
    s = plan_population(ArchSpec.weightwise(2, 2), torch.float16, world=1)
    assert q["engine_kwargs"]["order"] == "sequential"
    # the ordered buffers make a rank hold fewer particles; int32 version codes cap it below 2^30
    assert q["n_total"] < s["n_total"] and q["n_total"] <= 2 ** 30 - 1
    assert q["limited_by"] in ("hbm", "ordered version codes (int32)")



def test_every_library_knob_is_an_exec_config_field(monkeypatch):
    """each libsrnn knob (ops/_lib.py KNOBS) can be set from ExecConfig, ord_queue included"""
    assert set(ExecConfig.LIBRARY_KNOBS) == set(_lib.KNOBS)
    monkeypatch.setenv("SRNN_ORD_QUEUE", "0")
    assert ExecConfig().resolved().ord_queue is False
    monkeypatch.delenv("SRNN_ORD_QUEUE")
    try:
        ExecConfig(ord_queue=False).apply_library()
        assert _lib.get_knob("ord_queue") == 0
    finally:
        _lib.set_knob("ord_queue", -1)


def test_every_library_knob_starts_at_its_default():
    """a fresh library reports -1 (the built-in default) for every knob without its environment
    variable (a short initialiser once left the last knob at 0: the ready queue silently off)"""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in _lib.KNOB_ENV.values()}
    code = ("from self_replicating_neural_networks_amd.ops import _lib; "
            "print(sorted(set(_lib.get_knob(k) for k in _lib.KNOBS)))")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "[-1]"


def test_reference_order_stream_knobs_from_the_environment(monkeypatch):
    """the round-6 reference-order knobs: two counter-ordered graphs per chunk (bool), shadow lanes
    (int threshold, a library knob), the census beside the next generation (bool)"""
    monkeypatch.setenv("SRNN_ORD_GRAPH_SYNC", "0")
    monkeypatch.setenv("SRNN_ORD_SHADOW", "16")
    monkeypatch.setenv("SRNN_ORD_CENSUS_SIDE", "0")
    ex = ExecConfig().resolved()
    assert ex.ord_graph_sync is False and ex.ord_shadow == 16 and ex.ord_census_side is False
    assert _lib.get_knob("ord_shadow") == 16  # (the library reads the variable itself)
    monkeypatch.delenv("SRNN_ORD_SHADOW")
    assert ExecConfig().ord_graph_sync is True and _lib.get_knob("ord_shadow") == -1
    try:
        ExecConfig(ord_shadow=0).apply_library()
        assert _lib.get_knob("ord_shadow") == 0
    finally:
        _lib.set_knob("ord_shadow", -1)
    # host engines: no side stream, no counters, never a two-graph chunk
    eng = SoupEngine(ArchSpec.weightwise(2, 2), 64, dict(train=1), order="sequential")
    assert eng._osync is None and eng._ord_decouple is False and eng._chunks == []
