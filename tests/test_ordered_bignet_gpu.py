"""The north-star net in the reference's order on the device: SoupEngine(order="sequential")
of Aggregating(4, 10, 3) (P = 280; reference code/network.py:292-439 in code/soup.py:51-87's
in-place, index-ordered generation) runs the continuation-scheduled generation with the big
nets' turn (csrc/srnn_bignet.h BigOrd: streamed version reads, chunk-state recomputes of the
attack outputs).  It must equal the HOST serial loop (SequentialSoupEngine, the runtime-shape
engine's soup_seq_one) bitwise -- rows, uids, actions, counterparts, losses, respawns -- from
the same starting rows, for fp32 / bf16 tables and shuffle_not / shuffle_random."""
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import _lib
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

pytestmark = pytest.mark.gpu

HOT = dict(attacking_rate=0.3, learn_from_rate=0.3, train=2, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)


def _bits(t):
    t = t.cpu().contiguous()
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int16)


@pytest.mark.parametrize("dtype,shuffler", [(torch.float32, "none"), (torch.bfloat16, "none"),
                                            (torch.float32, "random")], ids=["fp32", "bf16", "fp32-shuffle"])
def test_device_ordered_big_net_is_the_host_serial_loop(dtype, shuffler):
    spec = ArchSpec.aggregating(4, 10, 3, shuffler=shuffler)
    assert _lib.supports(spec, _lib.OP_SOUP_ORDERED, True, _lib.DTYPE_FP32)
    n, seed = 2000, 11
    o = SoupEngine(spec, n, HOT, device="cuda", seed=seed, order="sequential", dtype=dtype)
    o.stats = True
    s = SequentialSoupEngine(spec, n, HOT, seed=seed, dtype=dtype, weights=o.local_rows()[:, :spec.P].float().cpu())
    deep = 0
    for g in range(3):
        o.evolve(1)
        s.evolve(1)
        torch.cuda.synchronize()
        assert torch.equal(_bits(o.local_rows()[:, :spec.P]), _bits(s.W[:, :spec.P])), g
        assert torch.equal(o.uid.cpu(), s.uid.cpu())
        assert torch.equal(o.action.cpu(), s.action.cpu())
        assert torch.equal(o.counterpart.cpu(), s.counterpart.cpu())
        assert torch.equal(o.respawn.cpu(), s.respawn.cpu())
        assert torch.equal(o.loss.cpu().view(torch.int32), s.loss.cpu().view(torch.int32))
        lv = o.ordered_levels()
        assert lv["error"] == 0
        deep = max(deep, lv["max_level"])
    assert deep >= 2  # real dependency chains (recomputed and stored attack outputs)
    assert int(o.next_uid[0]) == int(s.next_uid[0])
    assert sum(o.count().values()) == n


def test_device_ordered_big_net_graphs_equal_eager():
    spec = ArchSpec.aggregating(4, 10, 3)
    a = SoupEngine(spec, 1500, HOT, device="cuda", seed=3, order="sequential")
    b = SoupEngine(spec, 1500, HOT, device="cuda", seed=3, order="sequential")
    assert b.capture(warmup=1)
    a.evolve(1)
    a.evolve(3)
    b.evolve(3)
    torch.cuda.synchronize()
    assert torch.equal(_bits(a.local_rows()), _bits(b.local_rows())) and torch.equal(a.uid, b.uid)


@pytest.mark.parametrize("shape", [(4, 8, 2), (4, 16, 2)], ids=["agg-4-8-2", "agg-4-16-2"])
def test_device_ordered_other_big_shapes(shape):
    """the other instantiated big aggregating shapes (P = 128, 384) in the reference order"""
    spec = ArchSpec.aggregating(*shape)
    n, seed = 1200, 5
    o = SoupEngine(spec, n, HOT, device="cuda", seed=seed, order="sequential")
    s = SequentialSoupEngine(spec, n, HOT, seed=seed, weights=o.local_rows()[:, :spec.P].float().cpu())
    for g in range(2):
        o.evolve(1)
        s.evolve(1)
        torch.cuda.synchronize()
        assert torch.equal(_bits(o.local_rows()[:, :spec.P]), _bits(s.W[:, :spec.P])), g
        assert torch.equal(o.uid.cpu(), s.uid.cpu()) and torch.equal(o.respawn.cpu(), s.respawn.cpu())
    assert o.ordered_levels()["error"] == 0
