"""Reference-order soups on the level-scheduled generation (SoupEngine(order="sequential"),
OP_SOUP_ORDERED, csrc/srnn_ordered.h) against the serial loop (SequentialSoupEngine,
OP_SOUP_SEQ): the reference's in-place, index-ordered Soup.evolve (code/soup.py:51-87,
SURVEY S11) computed level by level must be BITWISE the serial loop -- rows, uids, actions,
counterparts, losses, respawns -- on the host and on the device."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.config import ExecConfig
from self_replicating_neural_networks_amd.models import network as N
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine
from self_replicating_neural_networks_amd.soup import Soup
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

SPECS = [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2)]
IDS = ["ww", "agg", "rnn"]
HOT = dict(attacking_rate=0.3, learn_from_rate=0.3, train=2, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)


def _bits(t):
    t = t.cpu().contiguous()
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int16)


def _same(ordered: SoupEngine, seq: SequentialSoupEngine, P: int):
    assert torch.equal(_bits(ordered.local_rows()[:, :P]), _bits(seq.W[:, :P]))
    assert torch.equal(ordered.uid.cpu(), seq.uid.cpu())
    assert int(ordered.next_uid[0]) == int(seq.next_uid[0])
    assert torch.equal(ordered.action.cpu(), seq.action.cpu())
    assert torch.equal(ordered.counterpart.cpu(), seq.counterpart.cpu())
    assert torch.equal(ordered.respawn.cpu(), seq.respawn.cpu())
    assert torch.equal(ordered.loss.cpu().view(torch.int32), seq.loss.cpu().view(torch.int32))


@pytest.mark.parametrize("spec", SPECS, ids=IDS)
@pytest.mark.parametrize("levels,pipe", [(4, "kernel"), (1, "kernel"), (4, "stream"), (4, "off")])
def test_host_ordered_generation_is_the_serial_loop(spec, levels, pipe):
    """host path of OP_SOUP_ORDERED == OP_SOUP_SEQ bitwise, generation by generation (levels=1
    sends every turn past level 0 through the tail; pipe: each generation's plan built one
    generation ahead into the other plan set -- by the generation call itself ("kernel") or by
    OP_ORD_PLAN ("stream") -- or inline ("off"))"""
    n, seed = 300, 5
    o = SoupEngine(spec, n, HOT, device="cpu", seed=seed, order="sequential",
                   execution=ExecConfig(order_levels=levels, ord_pipeline=pipe))
    assert o._ord_mode == pipe
    s = SequentialSoupEngine(spec, n, HOT, seed=seed)
    _same(o, s, spec.P)
    deep = 0
    for _ in range(4):
        o.evolve(1)
        s.evolve(1)
        _same(o, s, spec.P)
        deep = max(deep, o.ordered_levels()["max_level"])
    assert deep >= 2  # the test exercised real dependency chains
    assert o.ordered_levels()["error"] == 0


def test_host_ordered_sub_soups_and_multi_generation_evolve():
    spec = ArchSpec.weightwise(2, 2)
    p = dict(HOT, segment=10)
    o = SoupEngine(spec, 500, p, device="cpu", seed=9, order="sequential")
    s = SequentialSoupEngine(spec, 500, p, seed=9)
    o.evolve(5)
    s.evolve(5)
    _same(o, s, spec.P)


def test_ordered_differs_from_synchronous():
    """same decisions and keys: the in-place order is a different computation from Jacobi"""
    spec = ArchSpec.weightwise(2, 2)
    o = SoupEngine(spec, 200, HOT, device="cpu", seed=3, order="sequential").evolve(1)
    j = SoupEngine(spec, 200, HOT, device="cpu", seed=3).evolve(1)
    assert not torch.equal(o.local_rows(), j.local_rows())


def test_level_profile_of_the_bench_soup():
    """the headline soup's dependency DAG (attack 0.1, learn 0.1): most turns at level 0, a
    shallow tail (the reason a level-scheduled generation is fast)"""
    spec = ArchSpec.weightwise(2, 2)
    p = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, remove_divergent=True, remove_zero=True, epsilon=1e-4)
    o = SoupEngine(spec, 20000, p, device="cpu", seed=1, order="sequential").evolve(1)
    lv = o.ordered_levels()
    assert lv["levels"][0] > 0.8 * 20000 and lv["max_level"] <= 8 and lv["error"] == 0
    assert sum(lv["levels"]) + lv["tail"] == 20000


def test_ordered_order_validation():
    spec = ArchSpec.weightwise(2, 2)
    with pytest.raises(ValueError):
        SoupEngine(spec, 10, HOT, device="cpu", order="gauss")
    with pytest.raises(NotImplementedError, match="SequentialSoupEngine"):
        SoupEngine(ArchSpec.aggregating(4, 10, 3), 10, HOT, device="cpu", order="sequential")


def _ww_trainer():
    return N.TrainingNeuralNetworkDecorator(N.WeightwiseNeuralNetwork(2, 2)).with_params(epsilon=1e-4)


def test_soup_auto_mode_keeps_the_reference_order():
    small = Soup(50, _ww_trainer)
    big = Soup(500, _ww_trainer)
    assert small.mode == "sequential" and big.mode == "ordered"
    with pytest.raises(ValueError, match="mode='device'"):
        Soup(500, _ww_trainer, dist=object())
    big.with_params(train=1, remove_divergent=True, remove_zero=True)
    big.seed()
    big.evolve(2)
    assert isinstance(big.engine, SoupEngine) and big.engine.order == "sequential"
    assert sum(big.count().values()) == 500


def test_ordered_soup_records_reference_states():
    """recording keeps each particle's pre-respawn state and its counterparts as of its turn"""
    s = Soup(150, _ww_trainer, mode="ordered", seed=4).with_params(
        attacking_rate=0.3, learn_from_rate=0.2, train=1, remove_divergent=True, remove_zero=True)
    s.seed()
    s.evolve(3)
    n_states = sum(len(p.get_states()) for p in s.historical_particles.values())
    assert n_states >= 150 * 3
    acts = {st.get("action") for p in s.historical_particles.values() for st in p.get_states()}
    assert {"init", "train_self"} <= acts


@pytest.mark.gpu
@pytest.mark.parametrize("spec", SPECS, ids=IDS)
@pytest.mark.parametrize("pipe", ["kernel", "stream", "stream-1g", "off"])
def test_device_ordered_generation_is_the_serial_loop(spec, pipe):
    """device OP_SOUP_ORDERED (plan -> run by continuation -> close; the plan of the next
    generation built while this one runs -- by the last workgroups of the run launch ("kernel") or on a
    side stream ("stream": multi-generation graphs as two graphs on two streams ordered by device
    counters; "stream-1g": one graph, a fork / join per generation) -- or inline ("off")) == the
    serial loop on the same device (k_soup_seq, one lane) bitwise, eager and captured in hipGraphs"""
    n, seed = 3000, 7
    mode = pipe.split("-")[0]
    for graphs in (False, True):
        o = SoupEngine(spec, n, HOT, device="cuda", seed=seed, order="sequential",
                       execution=ExecConfig(ord_pipeline=mode, ord_graph_sync=pipe == "stream"))
        assert o._ord_mode == mode
        # the same starting rows (the device init contracts a*b+c, the host's does not)
        s = SequentialSoupEngine(spec, n, HOT, seed=seed, device="cuda", weights=o.local_rows()[:, :spec.P].cpu())
        if graphs:
            assert o.capture(warmup=1)
            s.evolve(1)  # capture runs one warmup generation eagerly
            # (every chunk validated bitwise against eager generations; the two-graph form kept)
            assert any(c[3] is not None for c in o._chunks) == (pipe == "stream")
        _same(o, s, spec.P)
        for k in (2, 4, 1, 2):  # chunks of 2 and 4, a single-generation graph between them
            o.evolve(k)
            s.evolve(k)
            _same(o, s, spec.P)
        assert o.ordered_levels()["error"] == 0
        if o._osync is not None and graphs and pipe == "stream":
            c = o._osync.cpu().tolist()  # runs / gates and plans / closes in step
            assert c[0] == c[1] and c[2] == c[3] and c[0] > 0
        o.release_graphs()


@pytest.mark.gpu
@pytest.mark.parametrize("spec", SPECS, ids=IDS)
@pytest.mark.parametrize("queue,shadow", [(True, 0), (False, 0), (True, 8), (True, 63), (False, 63)])
def test_device_ordered_queue_and_shadow_lanes(spec, queue, shadow):
    """the continuation schedules -- one ready queue per generation or per-wave lists, with or
    without shadow lanes (idle lanes of a small round repeating a busy lane's turn, publishing
    nothing) -- are all the serial loop bitwise, in two-graph chunks"""
    n, seed = 3000, 5
    ex = ExecConfig(ord_queue=queue, ord_shadow=shadow)
    try:
        ex.apply_library()
        o = SoupEngine(spec, n, HOT, device="cuda", seed=seed, order="sequential", execution=ex)
        s = SequentialSoupEngine(spec, n, HOT, seed=seed, device="cuda", weights=o.local_rows()[:, :spec.P].cpu())
        assert _lib.get_knob("ord_queue") == int(queue) and _lib.get_knob("ord_shadow") == shadow
        assert o.capture(warmup=1)
        s.evolve(1)
        for k in (2, 4, 1):
            o.evolve(k)
            s.evolve(k)
            _same(o, s, spec.P)
        assert o.ordered_levels()["error"] == 0
        o.release_graphs()
    finally:
        _lib.set_knob("ord_queue", -1)
        _lib.set_knob("ord_shadow", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [1, 2])
def test_device_ordered_tail_and_bf16_tables(levels):
    """the tail: its own launch (1 parallel level) or the last workgroup of the last level
    launch (2)"""
    spec = ArchSpec.weightwise(2, 2)
    o = SoupEngine(spec, 2000, HOT, device="cuda", seed=2, order="sequential", dtype=torch.bfloat16,
                   execution=ExecConfig(order_levels=levels))
    s = SequentialSoupEngine(spec, 2000, HOT, seed=2, dtype=torch.bfloat16, device="cuda",
                             weights=o.local_rows()[:, :spec.P].cpu())
    for _ in range(3):
        o.evolve(1)
        s.evolve(1)
        _same(o, s, spec.P)
    assert o.ordered_levels()["tail"] > 0


@pytest.mark.gpu
def test_device_ordered_headline_soup_matches_serial_loop():
    """the bench's parameters (train 20, attack 0.1, learn 0.1, respawn) at 20k particles: the
    level-scheduled generation == the device serial loop, and most turns run at level 0"""
    spec = ArchSpec.weightwise(2, 2)
    p = dict(attacking_rate=0.1, learn_from_rate=0.1, train=20, remove_divergent=True, remove_zero=True, epsilon=1e-4)
    o = SoupEngine(spec, 20_000, p, device="cuda", seed=0, order="sequential")
    s = SequentialSoupEngine(spec, 20_000, p, seed=0, device="cuda", weights=o.local_rows()[:, :spec.P].cpu())
    o.evolve(2)
    s.evolve(2)
    _same(o, s, spec.P)
    assert o.ordered_levels()["levels"][0] > 0.8 * 20_000


def test_ordered_records_equal_native_records():
    """the recorded trajectories (reference state schema: weights, time, action, counterpart uid as
    of the turn, fitted, loss) of a level-scheduled soup equal the serial loop's record, state for
    state -- counterparts that respawned at an earlier turn of the generation are the newborns"""
    params = dict(attacking_rate=0.3, learn_from_rate=0.3, train=1, remove_divergent=True, remove_zero=True)
    soups = []
    for mode in ("native", "ordered"):
        N.ParticleDecorator.next_uid = 0
        s = Soup(120, _ww_trainer, mode=mode, seed=8, device="cpu").with_params(**params)
        s.seed()
        s.evolve(4)
        soups.append(s)
    a, b = soups
    assert sorted(a.historical_particles) == sorted(b.historical_particles)
    n_cp = 0
    for uid in a.historical_particles:
        sa, sb = a.historical_particles[uid].get_states(), b.historical_particles[uid].get_states()
        assert len(sa) == len(sb), uid
        for x, y in zip(sa, sb):
            assert set(x) == set(y) and x["action"] == y["action"] and x.get("counterpart") == y.get("counterpart")
            assert x.get("time") == y.get("time") and np.array_equal(x["weights"].view(np.int32), y["weights"].view(np.int32))
            n_cp += x.get("counterpart") is not None
    assert n_cp > 0


def test_ordered_error_bits_are_sticky():
    """an error bit of one reference-order generation survives the later generations of the same
    evolve (the plan of the next generation clears every control word but that one), so count()
    still refuses the invalid rows"""
    o = SoupEngine(ArchSpec.weightwise(2, 2), 200, HOT, device="cpu", seed=1, order="sequential")
    o.evolve(1)
    assert o.ordered_error() == 0
    o._octl[_lib.ORD_ERRW] = 2  # as k_ord_count sets it for an unstored attack output
    o.evolve(3)
    assert o.ordered_error() == 2 and o.ordered_levels()["error"] == 2
    with pytest.raises(RuntimeError, match="error bits 2"):
        o.count()


@pytest.mark.gpu
def test_stream_probe_and_serialised_kernels_fall_back_to_one_graph():
    """the two-graph chunks need the side stream to run beside the current one: the probe says so on
    a normal process; with kernels serialised (AMD_SERIALIZE_KERNEL=3, like a counter-collecting
    profiler) it says no and the engine keeps one-graph chunks -- the soup bitwise the same"""
    import os
    import subprocess
    import sys
    side = torch.cuda.Stream(priority=-1)
    assert _lib.streams_concurrent(side, torch.cuda.current_stream(), torch.device("cuda", 0))
    code = """
import torch, json
from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.soup_engine import SoupEngine
hot = dict(attacking_rate=0.3, learn_from_rate=0.3, train=2, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)
o = SoupEngine(ArchSpec.weightwise(2, 2), 2000, hot, device="cuda", seed=3, order="sequential")
assert o.capture(warmup=1)
o.evolve(4)
print(json.dumps(dict(two=any(c[3] is not None for c in o._chunks), conc=o._conc,
                      rows=o.local_rows()[:, :14].contiguous().view(torch.int32).long().sum().item(),
                      uids=o.uid.sum().item(), err=o.ordered_levels()["error"])))
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for ser in ("0", "3"):
        env = dict(os.environ, AMD_SERIALIZE_KERNEL=ser)
        p = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True,
                           timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        out[ser] = __import__("json").loads(p.stdout.strip().splitlines()[-1])
    assert out["0"]["conc"] and out["0"]["two"]
    assert not out["3"]["conc"] and not out["3"]["two"]
    # (the rows' bit patterns summed: the same soup, NaN rows of divergent particles included)
    assert out["0"]["rows"] == out["3"]["rows"] and out["0"]["uids"] == out["3"]["uids"]
    assert out["0"]["err"] == out["3"]["err"] == 0
