"""Device generations against the exact float32 oracle (oracle/exact.py) and against the host
path, bitwise.  The host library now contracts a*b+c where the device does (csrc/Makefile
``-Xarch_host -mfma``), so host == oracle == device: the reference-order generation on the GPU
is pinned to an fp32 oracle directly, not through device-vs-device comparisons."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.oracle import exact as X
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

pytestmark = pytest.mark.gpu

WW = ArchSpec.weightwise(2, 2)
BENCH = dict(attacking_rate=0.1, learn_from_rate=0.1, train=20, learn_from_severity=1, remove_divergent=True,
             remove_zero=True, epsilon=1e-4)
HOT = dict(attacking_rate=0.3, learn_from_rate=0.3, train=3, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)


def _bits(t):
    return t[:, :WW.P].contiguous().cpu().view(torch.int32)


def test_device_reference_order_generation_matches_the_oracle():
    """two device reference-order generations of the benchmark soup == the exact oracle,
    row by row (max error <= 1e-5 of the row scale; bitwise in practice)"""
    n, seed = 256, 4
    o = SoupEngine(WW, n, BENCH, device="cuda", seed=seed, order="sequential")
    W = o.local_rows()[:, :WW.P].cpu().numpy().copy()
    assert X.max_row_error(W, X.init(WW, np.arange(n), seed)) == 0.0
    for g in range(1, 3):
        W = X.seq_generation(WW, W, g, seed, BENCH)[0]
        o.evolve(1)
        got = o.local_rows()[:, :WW.P].cpu().numpy()
        assert X.max_row_error(got, W) <= 1e-5, g
        W = got.copy()  # next generation from the device's rows (per-generation comparison)


@pytest.mark.parametrize("params", [BENCH, HOT], ids=["bench", "hot"])
def test_device_equals_host_bitwise(params):
    """the same soups on the device and on the host, bitwise: reference order (level-scheduled),
    the serial loop, and the synchronous fused generation"""
    n, seed = 3000, 6
    for order in ("sequential", "synchronous"):
        d = SoupEngine(WW, n, params, device="cuda", seed=seed, order=order)
        h = SoupEngine(WW, n, params, device="cpu", seed=seed, order=order)
        assert torch.equal(_bits(d.local_rows()), _bits(h.local_rows()))
        d.evolve(2)
        h.evolve(2)
        assert torch.equal(_bits(d.local_rows()), _bits(h.local_rows())), order
        assert torch.equal(d.uid.cpu(), h.uid.cpu()) and torch.equal(d.action.cpu(), h.action.cpu())
        assert torch.equal(d.loss.cpu().view(torch.int32), h.loss.cpu().view(torch.int32))
    s_d = SequentialSoupEngine(WW, 500, params, seed=seed, device="cuda")
    s_h = SequentialSoupEngine(WW, 500, params, seed=seed)
    s_d.evolve(2)
    s_h.evolve(2)
    assert torch.equal(_bits(s_d.W), _bits(s_h.W))
