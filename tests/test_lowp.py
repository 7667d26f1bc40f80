"""16-bit weight tables (bf16 / fp16 storage, fp32 arithmetic; SURVEY §7.7, BASELINE.json
configs #2 and #5).  The 16-bit operators must equal the fp32 operators applied to the
widened table followed by round-to-nearest-even after every application -- bitwise, since
the per-item arithmetic is the same code (csrc/srnn_kernels.h, srnn_lowp.hip)."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd import ArchSpec, Population
from self_replicating_neural_networks_amd.io import checkpoint as ckpt
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

SPECS = [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2)]
DT = [torch.bfloat16, torch.float16]
ids = lambda x: str(x).replace("torch.", "") if isinstance(x, torch.dtype) else x.kind


def _eq(a, b):
    return torch.equal(a.float().nan_to_num(7.0, 9.0, -9.0), b.float().nan_to_num(7.0, 9.0, -9.0))


@pytest.mark.parametrize("dtype", DT, ids=ids)
@pytest.mark.parametrize("spec", SPECS, ids=ids)
def test_lowp_ops_equal_rounded_fp32(spec, dtype):
    assert _lib.has_config(spec, K.dtype_code(dtype))
    n, seed = 300, 4
    uid = torch.arange(n, dtype=torch.int64)
    W32 = torch.zeros(n, spec.PP)
    K.init_rows(spec, W32, uid, seed)
    W = torch.zeros(n, spec.PP, dtype=dtype)
    K.init_rows(spec, W, uid, seed)
    assert torch.equal(W, W32.to(dtype))                      # init: rounded glorot draws
    # attack with a rolled attacker table
    idx = torch.roll(torch.arange(n), 3).contiguous()
    out = torch.zeros_like(W)
    K.apply(spec, W, out, idx_f=idx)
    out32 = torch.zeros_like(W32)
    K.apply(spec, W.float(), out32, idx_f=idx)
    assert _eq(out, out32.to(dtype))
    # K self-applications in one launch == K rounded single steps
    Wk = W.clone()
    K.run_fixpoint(spec, Wk, 5, 1e-4, early_exit=False)
    ref = W.clone()
    for _ in range(5):
        r32 = ref.float()
        K.run_fixpoint(spec, r32, 1, 1e-4, early_exit=False)
        ref = r32.to(dtype)
    assert _eq(Wk, ref)
    # training keeps fp32 in registers across the epochs of one launch, stores rounded
    Wt = W.clone()
    K.train(spec, Wt, epochs=3, uid=uid, seed=seed)
    Wt32 = W.float()
    K.train(spec, Wt32, epochs=3, uid=uid, seed=seed)
    assert _eq(Wt, Wt32.to(dtype))
    # the census covers every row
    cls, counts = K.classify(spec, W, 1e-4)
    assert int(counts.sum()) == n


@pytest.mark.parametrize("dtype", DT, ids=ids)
def test_lowp_fixpoints(dtype):
    """Identity fixpoint and zero net are exact in 16 bits."""
    spec = ArchSpec.weightwise(2, 2)
    W = torch.zeros(3, spec.PP, dtype=dtype)
    W[0, 0] = 1.0
    W[0, spec.offsets[1]] = 1.0
    W[0, spec.offsets[2]] = 1.0
    W[2] = float("nan")
    W[2, spec.P:] = 0
    cls, _ = K.classify(spec, W, 1e-4)
    assert cls.tolist() == [2, 1, 0]  # fix_other, fix_zero, divergent


def test_lowp_population_and_checkpoint(tmp_path):
    spec = ArchSpec.weightwise(2, 2)
    pop = Population(spec, 64, seed=3, dtype=torch.bfloat16)
    assert pop.W.dtype == torch.bfloat16 and pop.W.element_size() == 2
    pop.self_apply(3)
    ckpt.save_population(pop, str(tmp_path / "p"))
    back = ckpt.load_population(str(tmp_path / "p"))
    assert back.W.dtype == torch.bfloat16 and torch.equal(back.W, pop.W)


@pytest.mark.parametrize("dtype", DT, ids=ids)
def test_lowp_soup_resume_bitwise(tmp_path, dtype):
    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.2, learn_from_rate=0.2, train=2, remove_divergent=True, remove_zero=True)
    a = SoupEngine(spec, 100, params, seed=9, dtype=dtype)
    a.evolve(3)
    ckpt.save_engine(a, str(tmp_path / "c"))
    a.evolve(3)
    b = ckpt.load_engine(str(tmp_path / "c"))
    assert b.dtype == dtype
    b.evolve(3)
    assert _eq(a.local_rows(), b.local_rows()) and torch.equal(a.uid, b.uid)


def test_lowp_any_shape_via_generic_engine():
    """16-bit tables of shapes without a templated 16-bit kernel run on the runtime-shape
    engine; for an instantiated shape the generic engine equals the templated kernel
    bitwise (same per-particle arithmetic, same rounding points)."""
    spec = ArchSpec.recurrent(2, 2)
    assert _lib.has_config(spec, _lib.DTYPE_BF16)
    W = torch.zeros(4, spec.PP, dtype=torch.bfloat16)
    K.init_rows(spec, W, torch.arange(4), 0)
    assert torch.isfinite(W.float()).all()
    with pytest.raises(TypeError):
        K.init_rows(spec, torch.zeros(4, spec.PP, dtype=torch.float64), torch.arange(4), 0)
    for dtype in (torch.bfloat16, torch.float16):
        spec = ArchSpec.weightwise(2, 2)
        outs = []
        for gen in (False, True):
            _lib.set_force_generic(gen)
            try:
                pop = Population(spec, 200, seed=3, dtype=dtype)
                pop.train(3)
                pop.self_apply(4)
                outs.append((pop.W.clone(), pop.count()))
            finally:
                _lib.set_force_generic(False)
        assert torch.equal(outs[0][0].view(torch.int16), outs[1][0].view(torch.int16))
        assert outs[0][1] == outs[1][1]
