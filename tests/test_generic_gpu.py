"""Runtime-shape engine on the MI355X (csrc/srnn_generic.hip): generic vs templated kernels
on the device (bitwise: same code, same contraction), reference shapes vs the oracle, and
soups of shapes without a templated kernel -- including the north-star
Aggregating(4, 10, 3) with shuffle_random and 16-bit tables -- eager and graph-captured."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.oracle import core as O
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

pytestmark = pytest.mark.gpu

ids = lambda s: f"{s.kind}-{s.aggregates}-{s.width}-{s.depth}-{s.shuffler}"
SOUP = dict(attacking_rate=0.2, learn_from_rate=0.2, train=3, learn_from_severity=1, remove_divergent=True,
            remove_zero=True, epsilon=1e-4)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    ok = np.all(np.isfinite(a), 1) & np.all(np.isfinite(b), 1)
    if not ok.any():
        return 0.0
    a, b = a[ok], b[ok]
    return float(np.max(np.abs(a - b) / (np.max(np.abs(b), 1, keepdims=True) + 1e-6)))


def _ops(spec, dev, n=3000):
    uid = torch.arange(n, dtype=torch.int64, device=dev) + 5
    W = torch.zeros(n, spec.PP, device=dev)
    K.init_rows(spec, W, uid, 7)
    idx = torch.roll(torch.arange(n, device=dev), 1).contiguous()
    O_ = torch.zeros_like(W)
    K.apply(spec, W, O_, idx_f=idx, uid=uid, seed=7, ctr=3)
    T = W.clone()
    tl = K.train(spec, T, epochs=3, uid=uid, seed=7, ctr=11)
    L = W.clone()
    K.learn_from(spec, L, W, idx_t=idx, epochs=2, uid=uid, seed=7, ctr=5)
    c, cnt = K.classify(spec, T, 1e-4, uid=uid, seed=7)
    torch.cuda.synchronize()
    return dict(init=W, apply=O_, train=T, train_loss=tl, learn=L, cls=c, counts=cnt)


@pytest.mark.parametrize("spec", [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2)],
                         ids=ids)
def test_generic_equals_templated_on_device(cuda, spec):
    outs = []
    for gen in (False, True):
        _lib.set_force_generic(gen)
        try:
            outs.append(_ops(spec, cuda))
        finally:
            _lib.set_force_generic(False)
    a, b = outs
    bits = lambda t: t.contiguous().view(torch.uint8) if t.is_floating_point() else t
    bad = [k for k in a if not torch.equal(bits(a[k]), bits(b[k]))]
    assert not bad, bad


@pytest.mark.parametrize("spec", [ArchSpec.weightwise(3, 3), ArchSpec.weightwise(10, 3), ArchSpec.aggregating(4, 3, 2),
                                  ArchSpec.aggregating(4, 10, 3, shuffler="random"), ArchSpec.recurrent(3, 2),
                                  ArchSpec.fft(3, 2, 2)], ids=ids)
def test_reference_shapes_on_device_vs_oracle(cuda, spec):
    # big aggregating nets (P > 64) have their own row kernels for every dtype / shuffler
    assert _lib.is_generic(spec, _lib.OP_APPLY) == (not (spec.kind == "aggregating" and spec.P > 64))
    n = 1024
    out = _ops(spec, cuda, n)
    uid = np.arange(n) + 5
    w0 = out["init"][:, :spec.P].cpu().numpy()
    assert _rel(w0, O.init(spec, uid, 7)) < (2e-3 if spec.kind == "recurrent" else 1e-4)
    idx = np.roll(np.arange(n), 1)
    oo = O.apply(spec, w0[idx], w0, seed=7, uids=uid, ctr=3)
    assert _rel(out["apply"][:, :spec.P].cpu().numpy(), oo) < 1e-4
    tw = w0.copy()
    for e in range(3):
        tw, _ = O.train_epoch(spec, tw, tw, 0.01, True, 7, uid, 11 + e)
    # linear SimpleRNN stacks explode within a few BPTT steps for most draws: rows close to
    # divergence amplify the fma-contraction differences
    assert _rel(out["train"][:, :spec.P].cpu().numpy(), tw) < (5e-2 if spec.kind == "recurrent" else 1e-3)


@pytest.mark.parametrize("spec,dtype", [(ArchSpec.aggregating(4, 10, 3), torch.float32),
                                        (ArchSpec.aggregating(4, 10, 3, shuffler="random"), torch.float32),
                                        (ArchSpec.aggregating(4, 10, 3), torch.float16),
                                        (ArchSpec.recurrent(3, 2), torch.bfloat16),
                                        (ArchSpec.weightwise(3, 3), torch.float32)],
                         ids=["agg4-10-3", "agg4-10-3-shuffle", "agg4-10-3-fp16", "rnn3-2-bf16", "ww3-3"])
def test_generic_soup_device_host_and_graph(cuda, spec, dtype):
    """north-star net in a soup: device generation == host generation (classes / uids),
    and the hipGraph replay == the eager generations bitwise"""
    n = 600
    h = SoupEngine(spec, n, SOUP, seed=9, dtype=dtype)
    d = SoupEngine(spec, n, SOUP, device=cuda, seed=9, dtype=dtype)
    assert d.generic and not d.fused
    h.evolve(3)
    d.evolve(3)
    assert torch.equal(h.uid, d.uid.cpu())
    hw, dw = h.local_rows().float().numpy(), d.local_rows().float().cpu().numpy()
    assert _rel(dw[:, :spec.P], hw[:, :spec.P]) < 5e-2  # chaotic SGD: host / device contraction differ
    g = SoupEngine(spec, n, SOUP, device=cuda, seed=9, dtype=dtype)
    e = SoupEngine(spec, n, SOUP, device=cuda, seed=9, dtype=dtype)
    g.stats = e.stats = True
    assert g.capture(warmup=1)
    e.evolve(1)
    g.evolve(4)
    e.evolve(4)
    torch.cuda.synchronize()
    assert torch.equal(g.local_rows().view(torch.uint8), e.local_rows().view(torch.uint8))
    assert torch.equal(g.uid, e.uid) and g.count() == e.count()
