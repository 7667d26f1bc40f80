"""Runtime-shape Weightwise SGD on lanes-per-particle waves (csrc/srnn_generic.hip k_ww_wave:
U = next power of two >= width lanes per particle, weights / samples / activations in LDS):
bitwise equal to the lane-per-particle runtime-shape path on the same device (same operation
order, same Philox shuffles), for self-training and learn_from, fp32 and 16-bit tables, and close
to the numpy oracle."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.oracle import core as O

pytestmark = pytest.mark.gpu


def _train_learn(spec, dev, dtype, n=700, shuffle=True):
    uid = torch.arange(n, dtype=torch.int64, device=dev) + 3
    W = torch.zeros(n, spec.PP, device=dev)
    K.init_rows(spec, W, uid, 9)
    W = W.to(dtype)
    T = W.clone()
    tl = K.train(spec, T, epochs=3, uid=uid, seed=9, ctr=17, shuffle=shuffle)
    L = W.clone()
    idx = torch.roll(torch.arange(n, device=dev), 5).contiguous()
    ll = K.learn_from(spec, L, W, idx_t=idx, epochs=2, uid=uid, seed=9, ctr=4, shuffle=shuffle)
    torch.cuda.synchronize()
    return dict(train=T, train_loss=tl, learn=L, learn_loss=ll), W


@pytest.mark.parametrize("w,d", [(3, 3), (10, 3), (16, 2), (5, 4), (32, 2)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_ww_wave_equals_lane_path(cuda, w, d, dtype):
    spec = ArchSpec.weightwise(w, d)
    assert _lib.is_generic(spec, _lib.OP_TRAIN, K.dtype_code(dtype))
    outs = []
    for wave in (True, False):
        _lib.set_ww_wave(wave)
        try:
            outs.append(_train_learn(spec, cuda, dtype)[0])
        finally:
            _lib.set_ww_wave(True)
    a, b = outs
    bits = lambda t: t.contiguous().view(torch.uint8)
    bad = [k for k in a if not torch.equal(bits(a[k]), bits(b[k]))]
    assert not bad, bad


def test_ww_wave_close_to_oracle(cuda):
    spec = ArchSpec.weightwise(10, 3)
    out, W0 = _train_learn(spec, cuda, torch.float32, n=64)
    uid = np.arange(64, dtype=np.int64) + 3
    ow = W0[:, :spec.P].cpu().numpy()
    ref = ow.copy()
    ctr = 17
    for _ in range(3):
        ref, _loss = O.train_epoch(spec, ref, ref.copy(), shuffle=True, seed=9, uids=uid, ctr=ctr)
        ctr += 1
    got = out["train"][:, :spec.P].cpu().numpy()
    ok = np.all(np.isfinite(got), 1) & np.all(np.isfinite(ref), 1)
    assert ok.sum() > 32
    err = np.max(np.abs(got[ok] - ref[ok]) / (np.max(np.abs(ref[ok]), 1, keepdims=True) + 1e-6))
    assert err < 1e-4


SOUP = dict(attacking_rate=0.3, learn_from_rate=0.3, train=2, learn_from_severity=1, remove_divergent=True,
            remove_zero=True, epsilon=1e-4)


def _soup(spec, dev, dtype, graphs):
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine

    e = SoupEngine(spec, 333, SOUP, device=dev, seed=13, dtype=dtype)
    e.stats = True
    if graphs:
        assert e.capture(warmup=1)
        e.evolve(3)
    else:
        e.evolve(4)
    torch.cuda.synchronize()
    return (e.local_rows().clone(), e.uid.clone(), e.loss.clone(), e.action.clone(), e.counterpart.clone(),
            e.respawn.clone(), e.last_census(), int(e.next_uid))


@pytest.mark.parametrize("w,d", [(3, 3), (10, 3), (16, 2)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["f32", "f16"])
def test_ww_wave_soup_equals_lane_path(cuda, w, d, dtype):
    """soup generations (attacks in ascending attacker order, learn_from, self-train, respawn
    with inline re-init) on lanes-per-particle waves == the lane path, bitwise; graphs == eager"""
    spec = ArchSpec.weightwise(w, d)
    outs = []
    for wave in (True, False):
        _lib.set_ww_wave(wave)
        try:
            outs.append(_soup(spec, cuda, dtype, graphs=False))
        finally:
            _lib.set_ww_wave(True)
    a, b = outs
    bits = lambda t: t.contiguous().view(torch.uint8) if t.is_floating_point() else t
    for k, (x, y) in enumerate(zip(a[:6], b[:6])):
        assert torch.equal(bits(x), bits(y)), k
    assert a[6:] == b[6:]
    assert int((a[3] == 3).sum()) > 0  # self-training happened
    g = _soup(spec, cuda, dtype, graphs=True)
    for k, (x, y) in enumerate(zip(g[:6], a[:6])):
        assert torch.equal(bits(x), bits(y)), k


@pytest.mark.parametrize("w,d", [(3, 3), (10, 3), (16, 2), (3, 4), (10, 2), (16, 3)])
def test_ww_register_form_equals_lds_form(cuda, w, d):
    """the register-resident SGD (ww_epochs_reg) == the LDS form (knob ww_wave = 2), bitwise, for
    training, learn_from and whole single-rank soup generations"""
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine
    spec = ArchSpec.weightwise(w, d)
    outs = []
    for knob in (1, 2):
        _lib.set_knob("ww_wave", knob)
        try:
            r = _train_learn(spec, cuda, torch.float32, n=300)[0]
            e = SoupEngine(spec, 640, dict(attacking_rate=0.2, learn_from_rate=0.2, train=2, learn_from_severity=1,
                                           remove_divergent=True, remove_zero=True, epsilon=1e-4),
                           device=cuda, seed=5)
            e.evolve(3)
            torch.cuda.synchronize()
            r["soup"] = e.local_rows().clone()
            r["uid"] = e.uid.clone()
            outs.append(r)
        finally:
            _lib.set_knob("ww_wave", -1)
    a, b = outs
    bits = lambda t: t.contiguous().view(torch.uint8)
    bad = [k for k in a if not torch.equal(bits(a[k]), bits(b[k]))]
    assert not bad, bad
