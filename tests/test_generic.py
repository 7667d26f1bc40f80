"""Runtime-shape engine (csrc/srnn_generic.hip).

1. A/B against the templated kernels: for every instantiated shape the generic engine
   gives bitwise the same tables, losses, classes and soups (same per-particle arithmetic,
   same Philox streams) -- so the oracle-validated templated path pins the generic one.
2. The reference constructors take any width / depth / aggregates (code/network.py:222-230,
   :324-333, :465-474, :526-535): those shapes construct, self-attack, train, learn and
   live in soups (also sharded over gloo ranks) through the same API.
"""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd import ArchSpec, Population
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

TEMPLATED = [ArchSpec.weightwise(2, 2), ArchSpec.weightwise(1, 1), ArchSpec.weightwise(4, 3), ArchSpec.weightwise(8, 2),
             ArchSpec.aggregating(4, 2, 2), ArchSpec.aggregating(4, 2, 2, aggregator="max_ref"),
             ArchSpec.aggregating(4, 2, 2, shuffler="random"), ArchSpec.aggregating(4, 4, 2),
             ArchSpec.recurrent(2, 2), ArchSpec.recurrent(4, 2), ArchSpec.fft(4, 2, 2)]
REFERENCE_SHAPES = [ArchSpec.weightwise(3, 3), ArchSpec.weightwise(10, 3), ArchSpec.aggregating(4, 3, 2),
                    ArchSpec.aggregating(4, 10, 2), ArchSpec.recurrent(3, 2), ArchSpec.fft(3, 2, 2)]
ids = lambda s: f"{s.kind}-{s.aggregates}-{s.width}-{s.depth}-{s.aggregator}-{s.shuffler}"
SOUP = dict(attacking_rate=0.2, learn_from_rate=0.2, train=3, learn_from_severity=2, remove_divergent=True,
            remove_zero=True, epsilon=1e-4)


def _bits(t):
    return t.contiguous().view(torch.uint8) if t.is_floating_point() else t


def _ops(spec):
    n = 257
    uid = torch.arange(n, dtype=torch.int64) + 5
    W = torch.zeros(n, spec.PP)
    K.init_rows(spec, W, uid, 7)
    out = {"init": W.clone()}
    idx = torch.roll(torch.arange(n), 1).contiguous()
    O = torch.zeros_like(W)
    K.apply(spec, W, O, idx_f=idx, uid=uid, seed=7, ctr=3)
    out["apply"] = O
    T = W.clone()
    out["train_loss"] = K.train(spec, T, epochs=3, uid=uid, seed=7, ctr=11)
    out["train"] = T
    L = W.clone()
    out["learn_loss"] = K.learn_from(spec, L, W, idx_t=idx, epochs=2, uid=uid, seed=7, ctr=5)
    out["learn"] = L
    F = W.clone()
    c, st, tr = K.run_fixpoint(spec, F, 12, 1e-4, uid=uid, seed=7, record=True)
    out.update(fix=F, fix_cls=c, fix_steps=st, traj=tr)
    c, cnt = K.classify(spec, T, 1e-4, uid=uid, seed=7)
    out.update(cls=c, counts=cnt)
    P = W.clone()
    K.perturb(spec, P, 1e-3, uid=uid, seed=7, ctr=2)
    out["perturb"] = P
    V = W.clone()
    tts, taf = K.vary_run(spec, V, 10, 1e-4, uid=uid, seed=7)
    out.update(vary=V, tts=tts, taf=taf)
    return out


def _ab(fn):
    outs = []
    for gen in (False, True):
        _lib.set_force_generic(gen)
        try:
            outs.append(fn())
        finally:
            _lib.set_force_generic(False)
    return outs


@pytest.mark.parametrize("spec", TEMPLATED, ids=ids)
def test_generic_equals_templated_ops(spec):
    a, b = _ab(lambda: _ops(spec))
    bad = [k for k in a if not torch.equal(_bits(a[k]), _bits(b[k]))]
    assert not bad, bad


@pytest.mark.parametrize("spec", [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2)],
                         ids=ids)
def test_generic_soup_equals_fused_soup(spec):
    def soup():
        e = SoupEngine(spec, 300, SOUP, seed=3)
        e.stats = True
        e.evolve(5)
        return e.local_rows().clone(), e.uid.clone(), int(e.next_uid), e.count(), e.generic

    (wa, ua, na, ca, ga), (wb, ub, nb, cb, gb) = _ab(soup)
    assert not ga and gb  # fused templated generation vs the generic decide/evolve/respawn pipeline
    assert torch.equal(_bits(wa), _bits(wb)) and torch.equal(ua, ub) and na == nb and ca == cb


@pytest.mark.parametrize("spec", REFERENCE_SHAPES, ids=ids)
def test_reference_shapes_run_everywhere(spec):
    assert _lib.has_config(spec) and _lib.is_generic(spec, _lib.OP_TRAIN)
    pop = Population(spec, 64, seed=2)
    w0 = pop.weights().clone()
    assert torch.isfinite(w0).all() and w0.abs().sum() > 0
    pop.train(2)
    pop.self_apply(1)
    pop.learn_from(pop.W.clone(), torch.roll(torch.arange(64), 5).contiguous())
    pop.attack(torch.arange(8), torch.tensor([9, 9, 10, 11, 12, 12, 12, 13]))
    c = pop.count()
    assert sum(c.values()) == 64
    e = SoupEngine(spec, 120, SOUP, seed=4)
    e.evolve(3)
    assert e.generic and sum(e.count().values()) == 120


def test_reference_facades_any_shape():
    from self_replicating_neural_networks_amd.models.network import (AggregatingNeuralNetwork, FFTNeuralNetwork,
                                                                     RecurrentNeuralNetwork,
                                                                     TrainingNeuralNetworkDecorator,
                                                                     WeightwiseNeuralNetwork)
    from self_replicating_neural_networks_amd.oracle import core as O
    nets = [WeightwiseNeuralNetwork(3, 3), WeightwiseNeuralNetwork(10, 3), AggregatingNeuralNetwork(4, 3, 2),
            AggregatingNeuralNetwork(4, 10, 2), RecurrentNeuralNetwork(3, 2), FFTNeuralNetwork(3, 2, 2)]
    for net in nets:
        before = net.get_weights_flat()
        expect = O.apply(net.spec, before[None], before[None])[0]
        net.self_attack()
        got = net.get_weights_flat()
        # the engine fuses a*b+c (host and device alike), the oracle rounds the product: a
        # 17-step linear recurrence carries that to a few 1e-6 of the row's scale
        assert np.max(np.abs(got - expect)) <= 1e-5 * max(np.max(np.abs(expect)), 1.0), net.spec
        t = TrainingNeuralNetworkDecorator(net)
        loss = t.compiled().train()
        assert np.isfinite(loss) or net.is_diverged()


def test_repeated_victims_apply_in_order():
    """Population.attack with repeated victims: k-th attack of every victim per batched
    launch; equals applying the attacks one by one (attackers' pre-call weights)."""
    spec = ArchSpec.weightwise(2, 2)
    pop = Population(spec, 40, seed=6)
    ref = pop.W.clone()
    att = torch.tensor([0, 1, 2, 3, 4, 5, 6])
    vic = torch.tensor([10, 11, 10, 12, 10, 11, 13])
    pop.attack(att, vic)
    src = ref.clone()
    cur = ref.clone()
    for a, v in zip(att.tolist(), vic.tolist()):
        out = torch.zeros(1, spec.PP)
        K.apply(spec, torch.stack([src[a], cur[v]]), out, idx_f=torch.tensor([0]), idx_t=torch.tensor([1]),
                idx_o=torch.tensor([0]), n=1)
        cur[v] = out[0]
    assert torch.equal(pop.W, cur)
