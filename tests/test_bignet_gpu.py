"""Big aggregating nets (P > 64, the north-star Aggregating(4, 10, 3)) on their lane-per-
particle row kernels (csrc/srnn_bignet.hip) for every storage format and shuffler: each
operator and whole soup generations bitwise against the runtime-shape engine on the same
device (csrc/srnn_generic.hip, itself checked against the numpy oracle in
tests/test_generic_gpu.py)."""
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

pytestmark = pytest.mark.gpu

SOUP = dict(attacking_rate=0.3, learn_from_rate=0.3, train=3, learn_from_severity=2, remove_divergent=True,
            remove_zero=True, epsilon=1e-4)
DTYPES = [torch.float32, torch.bfloat16, torch.float16]
dt_id = lambda d: str(d).replace("torch.", "")


def _bits(t):
    return t.contiguous().view(torch.uint8)


def _both(fn):
    outs = []
    for gen in (False, True):
        _lib.set_force_generic(gen)
        try:
            outs.append(fn())
        finally:
            _lib.set_force_generic(False)
    return outs


@pytest.mark.parametrize("shuffler", ["none", "random"])
@pytest.mark.parametrize("dtype", DTYPES, ids=dt_id)
def test_big_ops_equal_generic(cuda, dtype, shuffler):
    spec = ArchSpec.aggregating(4, 10, 3, shuffler=shuffler)
    code = K.dtype_code(dtype)
    for op in (_lib.OP_INIT, _lib.OP_APPLY, _lib.OP_CLASSIFY, _lib.OP_TRAIN, _lib.OP_LEARN, _lib.OP_SOUP_EVOLVE):
        assert not _lib.is_generic(spec, op, code), op
    n = 1500

    def ops():
        uid = torch.arange(n, dtype=torch.int64, device=cuda) + 3
        W = torch.zeros(n, spec.PP, dtype=dtype, device=cuda)
        K.init_rows(spec, W, uid, 5)
        idx = torch.roll(torch.arange(n, device=cuda), 7).contiguous()
        A = torch.zeros_like(W)
        K.apply(spec, W, A, idx_f=idx, uid=uid, seed=5, ctr=9)
        T = W.clone()
        tl = K.train(spec, T, epochs=4, uid=uid, seed=5, ctr=2)
        L = W.clone()
        K.learn_from(spec, L, W, idx_t=idx, epochs=2, uid=uid, seed=5, ctr=4)
        c1, n1 = K.classify(spec, W, 1e-4, uid=uid, seed=5)
        c2, n2 = K.classify(spec, A, 1e-2, uid=uid, seed=5)  # chunk-constant rows: fixpoint candidates
        out = dict(init=W, apply=A, train=T, loss=tl, learn=L, cls1=c1, cnt1=n1, cls2=c2, cnt2=n2)
        if dtype == torch.float32 and shuffler == "none":
            # run_fixpoint: row phase (staged loads), chunk-state steps, staged write-back
            F = W.clone()
            fc, fs, _ = K.run_fixpoint(spec, F, 6, 1e-4, early_exit=True)
            out.update(fix=F, fix_cls=fc, fix_steps=fs)
        torch.cuda.synchronize()
        return out

    a, b = _both(ops)
    bad = [k for k in a if not torch.equal(_bits(a[k]) if a[k].is_floating_point() else a[k],
                                           _bits(b[k]) if b[k].is_floating_point() else b[k])]
    assert not bad, bad


@pytest.mark.parametrize("shuffler", ["none", "random"])
@pytest.mark.parametrize("dtype", DTYPES, ids=dt_id)
def test_big_soup_equals_generic(cuda, dtype, shuffler):
    """decide -> evolve (attacks, learn_from, self-train, respawn) -> uids -> census of the
    north-star net: specialised row kernels == runtime-shape engine, bitwise, and the
    hipGraph replay == eager"""
    spec = ArchSpec.aggregating(4, 10, 3, shuffler=shuffler)

    def soup():
        e = SoupEngine(spec, 900, SOUP, device=cuda, seed=21, dtype=dtype)
        e.stats = True
        e.evolve(4)
        torch.cuda.synchronize()
        return (e.local_rows().clone(), e.uid.clone(), e.loss.clone(), e.action.clone(), e.counterpart.clone(),
                e.respawn.clone(), e.count())

    a, b = _both(soup)
    for x, y in zip(a[:-1], b[:-1]):
        assert torch.equal(_bits(x) if x.is_floating_point() else x, _bits(y) if y.is_floating_point() else y)
    assert a[-1] == b[-1]
    assert int((a[3] == 3).sum()) > 0  # self-training happened
    g = SoupEngine(spec, 900, SOUP, device=cuda, seed=21, dtype=dtype)
    g.stats = True
    assert g.capture(warmup=1)
    e = SoupEngine(spec, 900, SOUP, device=cuda, seed=21, dtype=dtype)
    e.stats = True
    e.evolve(1)
    g.evolve(3)
    e.evolve(3)
    torch.cuda.synchronize()
    assert torch.equal(_bits(g.local_rows()), _bits(e.local_rows())) and torch.equal(g.uid, e.uid)


@pytest.mark.parametrize("spec", [ArchSpec.aggregating(4, 2, 2), ArchSpec.aggregating(4, 10, 3)],
                         ids=["agg4-2-2", "agg4-10-3"])
def test_fixpoint_after_aggregation_device_vs_host(cuda, spec):
    """Population.is_fixpoint_after_aggregation on the GPU (apply kernels, batched) == the
    host engine on the same weights (reference code/network.py:419-439)."""
    from self_replicating_neural_networks_amd.population import Population
    h = Population(spec, 600, seed=3)
    h.self_apply(2)
    d = Population(spec, 600, device=cuda, weights=h.weights(), seed=3)
    fh, ah = h.is_fixpoint_after_aggregation(2, 1e-3)
    fd, ad = d.is_fixpoint_after_aggregation(2, 1e-3)
    assert 0 < int(fh.sum()) < 600 or spec.P > 64
    assert float((fh == fd.cpu()).float().mean()) > 0.99
    ok = torch.isfinite(ah).all(1) & torch.isfinite(ad.cpu()).all(1)
    assert torch.allclose(ah[ok], ad.cpu()[ok], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("shuffler", ["none", "random"])
def test_big_soup_vs_fp32_oracle(cuda, shuffler):
    """The north-star net's soup generation (k_big_soup_evolve: attacks received, learn_from,
    self-train, respawn) against the float32 numpy oracle of the synchronous generation
    (oracle/core.py soup_generation_sync, reference code/soup.py:51-87 with an
    AggregatingNeuralNetwork(4, 10, 3) generator, :132-134), one generation at a time from the
    device's own rows for 3 generations"""
    import numpy as np
    from self_replicating_neural_networks_amd.oracle import core as O

    spec = ArchSpec.aggregating(4, 10, 3, shuffler=shuffler)
    p = dict(attacking_rate=0.3, learn_from_rate=0.3, train=3, learn_from_severity=1, remove_divergent=True,
             remove_zero=True, epsilon=1e-4)
    n = 256
    e = SoupEngine(spec, n, p, device=cuda, seed=13)
    assert not _lib.is_generic(spec, _lib.OP_SOUP_EVOLVE)  # the big-net row kernels run
    attacked = 0
    for g in range(1, 4):
        W0 = e.local_rows()[:, :spec.P].cpu().numpy().copy()
        e.evolve(1)
        torch.cuda.synchronize()
        W1, act, cp, loss, rs = O.soup_generation_sync(spec, W0, np.arange(n, dtype=np.uint64), g, 13, p)
        assert np.array_equal(e.action.cpu().numpy(), act)
        assert np.array_equal(e.counterpart.cpu().numpy(), cp)
        assert np.array_equal(e.respawn.cpu().numpy(), rs)
        keep = (rs == 0) & np.all(np.isfinite(W1), 1)
        got = e.local_rows()[:, :spec.P].cpu().numpy()[keep]
        scale = np.max(np.abs(W1[keep]), 1, keepdims=True) + 1e-6
        assert np.max(np.abs(got - W1[keep]) / scale) < 1e-5
        at, te = O.soup_decisions(13, g, n, p["attacking_rate"], p["learn_from_rate"])
        attacked += int((at >= 0).sum() + (te >= 0).sum())
    assert attacked > 0  # attacks and learn_from happened
