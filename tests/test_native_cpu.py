"""Host path of libsrnn (the same C++ per-particle code as the HIP kernels) vs the
independent float32 numpy oracle."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.oracle import core as O

SPECS = [ArchSpec.weightwise(2, 2), ArchSpec.weightwise(1, 1), ArchSpec.weightwise(4, 3), ArchSpec.weightwise(8, 2),
         ArchSpec.aggregating(4, 2, 2), ArchSpec.aggregating(4, 2, 2, aggregator="max"),
         ArchSpec.aggregating(4, 2, 2, aggregator="max_ref"), ArchSpec.aggregating(4, 2, 2, shuffler="random"),
         ArchSpec.aggregating(2, 2, 2), ArchSpec.recurrent(2, 2), ArchSpec.recurrent(1, 1), ArchSpec.recurrent(2, 3),
         ArchSpec.fft(4, 2, 2), ArchSpec.fft(2, 2, 2),
         # shapes without a templated kernel: the runtime-shape engine (csrc/srnn_generic.hip);
         # the reference constructors take any width / depth / aggregates (code/network.py:222-535)
         ArchSpec.weightwise(3, 3), ArchSpec.weightwise(10, 3), ArchSpec.aggregating(4, 3, 2),
         ArchSpec.aggregating(4, 10, 2), ArchSpec.aggregating(4, 10, 3), ArchSpec.aggregating(5, 3, 2, shuffler="random"),
         ArchSpec.recurrent(3, 2), ArchSpec.recurrent(5, 1), ArchSpec.fft(3, 2, 2)]
IDS = [f"{s.kind}-{s.aggregates}-{s.width}-{s.depth}-{s.aggregator}-{s.shuffler}" for s in SPECS]


def rowrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    ok = np.all(np.isfinite(a), 1) & np.all(np.isfinite(b), 1)
    a, b = a[ok], b[ok]
    return float(np.max(np.abs(a - b) / (np.max(np.abs(b), 1, keepdims=True) + 1e-6))) if len(a) else 0.0


@pytest.fixture(params=SPECS, ids=IDS)
def spec(request):
    return request.param


def _pop(spec, n=300, seed=17):
    uid = torch.arange(n, dtype=torch.int64) + 3
    W = torch.zeros(n, spec.PP)
    K.init_rows(spec, W, uid, seed)
    return W, uid


def test_configs_instantiated(spec):
    assert _lib.has_config(spec)


def test_init_matches_oracle(spec):
    W, uid = _pop(spec)
    ow = O.init(spec, uid.numpy(), 17)
    tol = 1e-4 if spec.kind == "recurrent" else 1e-6  # orthogonal init: libm logf/cosf ulps
    assert rowrel(W[:, :spec.P].numpy(), ow) < tol
    assert torch.all(W[:, spec.P:] == 0)


def test_init_statistics(spec):
    if spec.kind == "recurrent":
        # recurrent kernels orthogonal: R^T R = I
        W, _ = _pop(spec, 50)
        for (r, c), o in list(zip(spec.layer_shapes, spec.offsets))[1::2]:
            R = W[:, o:o + r * c].reshape(-1, r, c)
            eye = torch.eye(r).expand(R.shape[0], r, r)
            assert torch.allclose(R.transpose(1, 2) @ R, eye, atol=1e-5)
    else:
        W, _ = _pop(spec, 4000)
        (r, c), o = spec.layer_shapes[0], 0
        lim = np.sqrt(6.0 / (r + c))
        vals = W[:, o:o + r * c].numpy().ravel()
        assert vals.min() >= -lim and vals.max() <= lim
        assert abs(vals.mean()) < 0.02 * lim * 3
        assert abs(vals.var() - lim * lim / 3) < 0.05 * lim * lim / 3


def test_apply_matches_oracle(spec):
    W, uid = _pop(spec)
    out = torch.zeros_like(W)
    idx_f = torch.roll(torch.arange(W.shape[0]), 3).contiguous()
    K.apply(spec, W, out, idx_f=idx_f, uid=uid, seed=5, ctr=11)
    ow = W[:, :spec.P].numpy()
    oo = O.apply(spec, ow[idx_f.numpy()], ow, seed=5, uids=uid.numpy(), ctr=11)
    # fma chains vs numpy float32 matmuls: the rounding difference grows with width x depth
    tol = 1e-5 if spec.width * spec.depth <= 4 else 1e-4
    assert rowrel(out[:, :spec.P].numpy(), oo) < tol


def test_train_epoch_matches_oracle(spec):
    W, uid = _pop(spec)
    ow = W[:, :spec.P].numpy().copy()
    loss = K.train(spec, W, epochs=1, lr=0.01, shuffle=True, uid=uid, seed=9, ctr=4)
    tw, tl = O.train_epoch(spec, ow, ow, 0.01, True, 9, uid.numpy(), 4)
    assert rowrel(W[:, :spec.P].numpy(), tw) < 1e-4
    assert np.allclose(loss.numpy(), tl, rtol=1e-4, atol=1e-6)


def test_learn_from_matches_oracle(spec):
    W, uid = _pop(spec)
    T, _ = _pop(spec, seed=99)
    idx = torch.randint(0, T.shape[0], (W.shape[0],), generator=torch.Generator().manual_seed(0))
    ow = W[:, :spec.P].numpy().copy()
    K.learn_from(spec, W, T, idx, epochs=1, lr=0.01, uid=uid, seed=9, ctr=2)
    tw, _ = O.train_epoch(spec, ow, T[:, :spec.P].numpy()[idx.numpy()], 0.01, True, 9, uid.numpy(), 2)
    assert rowrel(W[:, :spec.P].numpy(), tw) < 1e-4


def test_classify_matches_oracle(spec):
    W, uid = _pop(spec)
    # include known classes: zero net, NaN net
    W[0] = 0
    W[1, 0] = float("nan")
    cls, counts = K.classify(spec, W, 1e-4, uid=uid, seed=1, ctr=0)
    ocls = O.classify(spec, W[:, :spec.P].numpy(), 1e-4, seed=1, uids=uid.numpy(), ctr=0)
    assert (cls.numpy() == ocls).mean() > 0.995
    assert cls[0] == O.C_FIX_ZERO and cls[1] == O.C_DIVERGENT
    assert int(counts.sum()) == W.shape[0]


def test_run_fixpoint_matches_oracle_short():
    spec = ArchSpec.weightwise(2, 2)
    W, uid = _pop(spec, 500)
    ow = W[:, :spec.P].numpy().copy()
    cls, nsteps, _ = K.run_fixpoint(spec, W, 5, 1e-4, early_exit=True)
    w5, n5, c5 = O.run_fixpoint(spec, ow, 5, 1e-4, early_exit=True)
    assert (nsteps.numpy() == n5).mean() > 0.99
    assert rowrel(W[:, :spec.P].numpy(), w5) < 1e-3


def test_perturb_matches_oracle():
    spec = ArchSpec.weightwise(2, 2)
    W, uid = _pop(spec, 100)
    ow = W[:, :spec.P].numpy().copy()
    K.perturb(spec, W, 1e-3, uid=uid, seed=4, ctr=7)
    assert np.array_equal(W[:, :spec.P].numpy(), O.perturb(ow, 1e-3, 4, uid.numpy(), 7))


def test_identity_fixpoint_classified_fix_other():
    """The known fixpoint of code/setups/known-fixpoint-variation.py:20-25: f(x) = x[0]."""
    spec = ArchSpec.weightwise(2, 2)
    W = torch.zeros(3, spec.PP)
    W[:, 0] = 1.0   # layer0 [0][0]
    W[:, 8] = 1.0   # layer1 [0][0]
    W[:, 12] = 1.0  # layer2 [0][0]
    cls, _ = K.classify(spec, W, 1e-4)
    assert cls.tolist() == [O.C_FIX_OTHER] * 3
    before = W.clone()
    K.run_fixpoint(spec, W, 10, 1e-4, early_exit=False)
    assert torch.equal(W, before)


def test_shape_checks_raise_before_launch():
    spec = ArchSpec.weightwise(2, 2)
    with pytest.raises(ValueError):
        K.train(spec, torch.zeros(4, 14))
    with pytest.raises(IndexError):
        K.apply(spec, torch.zeros(4, 16), torch.zeros(4, 16), idx_f=torch.tensor([0, 1, 2, 9]))


def test_any_shape_runs_and_bad_layouts_fail_loudly():
    """Shapes without a templated kernel run on the runtime-shape engine; a table whose
    layout does not match the architecture is still rejected before any launch."""
    spec = ArchSpec.weightwise(5, 5)
    W = torch.zeros(2, spec.PP)
    K.init_rows(spec, W, torch.arange(2), 0)
    assert torch.isfinite(W).all() and W[:, : spec.P].abs().sum() > 0
    assert _lib.is_generic(spec, _lib.OP_INIT)
    with pytest.raises(ValueError):
        K.init_rows(spec, torch.zeros(2, spec.PP + 4), torch.arange(2), 0)


def test_orthogonal_init_follows_lapack_svd_conventions():
    """Keras' Orthogonal = U of numpy.linalg.svd: 2x2 recurrent kernels are reflections
    (det -1) and equal numpy's U of the same gaussian matrix (oracle) to float32 rounding."""
    import numpy as np
    from self_replicating_neural_networks_amd.oracle import core as O
    spec = ArchSpec.recurrent(2, 2)
    uid = torch.arange(3000, dtype=torch.int64)
    W = torch.zeros(3000, spec.PP)
    K.init_rows(spec, W, uid, 13)
    w = W[:, :spec.P].numpy()
    o = O.init(spec, np.arange(3000), 13)
    assert np.max(np.abs(w - o)) < 1e-5  # float32 Box-Muller: host libm vs numpy ulps
    off = spec.offsets[1]  # first recurrent kernel (2x2)
    R = w[:, off:off + 4].reshape(-1, 2, 2).astype(np.float64)
    assert np.allclose(np.linalg.det(R), -1.0, atol=1e-5)
    assert np.allclose(R @ R.transpose(0, 2, 1), np.eye(2), atol=1e-6)
