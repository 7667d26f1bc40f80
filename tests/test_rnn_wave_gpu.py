"""Wide / long Recurrent nets wave per particle (csrc/srnn_generic.hip k_rnn_wave):
equal to the lane-per-particle path on the same device (same operation order) and close to
the host path, for self-application, run_fixpoint + census, self-training and learn_from."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.population import Population

pytestmark = pytest.mark.gpu


def _ops(spec, dev, n=300):
    pop = Population(spec, n, device=dev, seed=4)
    W0 = pop.W.clone()
    out = {}
    pop.self_apply(2)
    out["apply"] = pop.W.clone()
    pop.W.copy_(W0)
    cls, steps, _ = K.run_fixpoint(spec, pop.W, 4, 1e-4, early_exit=True)
    out["fix"], out["cls"], out["steps"] = pop.W.clone(), cls.clone(), steps.clone()
    pop.W.copy_(W0)
    out["loss"] = pop.train(3).clone()
    out["train"] = pop.W.clone()
    pop.W.copy_(W0)
    idx = torch.roll(torch.arange(n, device=dev), 3).contiguous()
    pop.learn_from(W0.clone(), idx, epochs=2)
    out["learn"] = pop.W.clone()
    torch.cuda.synchronize() if dev != "cpu" else None
    return out


@pytest.mark.parametrize("w,d", [(8, 2), (16, 2), (12, 3)])
def test_rnn_wave_equals_lane_path(cuda, w, d):
    spec = ArchSpec.recurrent(w, d)
    outs = []
    for wave in (True, False):
        _lib.set_rnn_wave(wave)
        try:
            outs.append(_ops(spec, cuda))
        finally:
            _lib.set_rnn_wave(True)
    a, b = outs
    for k in a:
        x, y = a[k], b[k]
        if x.is_floating_point():
            assert torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x, y.view(torch.int32)
                               if y.dtype == torch.float32 else y), k
        else:
            assert torch.equal(x, y), k
    h = _ops(spec, "cpu")
    ok = torch.isfinite(h["apply"]).all(1) & torch.isfinite(a["apply"].cpu()).all(1)
    assert torch.allclose(a["apply"].cpu()[ok], h["apply"][ok], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("w,d", [(8, 2), (16, 2), (32, 2), (8, 3), (16, 3)])
def test_rnn_wave_specialised_equals_runtime_shape(cuda, w, d):
    """The width / depth-specialised wave kernels (compile-time layer tables, unrolled loops)
    are bitwise the runtime-shape wave kernel."""
    spec = ArchSpec.recurrent(w, d)
    outs = []
    for on in (True, False):
        _lib.set_rnn_spec(on)
        try:
            outs.append(_ops(spec, cuda, n=200))
        finally:
            _lib.set_rnn_spec(True)
    a, b = outs
    for k in a:
        x, y = a[k], b[k]
        if x.dtype == torch.float32:
            x, y = x.view(torch.int32), y.view(torch.int32)
        assert torch.equal(x, y), k


SOUP = dict(attacking_rate=0.2, learn_from_rate=0.2, train=2, learn_from_severity=2, remove_divergent=True,
            remove_zero=True, epsilon=1e-4)


def _soup(spec, dev, dtype, graphs):
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine

    e = SoupEngine(spec, 150, SOUP, device=dev, seed=13, dtype=dtype)
    e.stats = True
    if graphs:
        assert e.capture(warmup=1)
        e.evolve(2)
    else:
        e.evolve(3)
    torch.cuda.synchronize()
    return (e.local_rows().clone(), e.uid.clone(), e.loss.clone(), e.action.clone(), e.counterpart.clone(),
            e.respawn.clone(), e.last_census(), int(e.next_uid))


@pytest.mark.parametrize("w,d", [(8, 2), (12, 3)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["f32", "f16"])
def test_rnn_wave_soup_equals_lane_path(cuda, w, d, dtype):
    """Recurrent soup generations wave per particle (k_rnn_wave_soup: attacks, learn_from,
    self-train, respawn with inline re-init) == the lane path, bitwise; graphs == eager"""
    spec = ArchSpec.recurrent(w, d)
    outs = []
    for wave in (True, False):
        _lib.set_rnn_soup(wave)
        try:
            outs.append(_soup(spec, cuda, dtype, graphs=False))
        finally:
            _lib.set_rnn_soup(True)
    a, b = outs
    bits = lambda t: t.contiguous().view(torch.uint8) if t.is_floating_point() else t
    for k, (x, y) in enumerate(zip(a[:6], b[:6])):
        assert torch.equal(bits(x), bits(y)), k
    assert a[6:] == b[6:]
    assert int((a[3] == 3).sum()) > 0  # self-training happened
    g = _soup(spec, cuda, dtype, graphs=True)
    for k, (x, y) in enumerate(zip(g[:6], a[:6])):
        assert torch.equal(bits(x), bits(y)), k
