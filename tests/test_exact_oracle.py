"""The engine's exact arithmetic (oracle/exact.py) against the native host path.

The host library is built with the device's contraction (csrc/Makefile ``-Xarch_host
-mfma``), so the same SRNN_HD code rounds identically on both sides; the exact oracle
replays that operation sequence in numpy.  These tests pin the host path to it at ZERO
tolerance: init, one self-application, SGD epochs, and whole reference-order soup
generations (the serial loop and the level-scheduled generation).  The GPU side
(tests/test_exact_oracle_gpu.py, ``smoke()``) compares device generations against the same
oracle, so the reference order is tied to an fp32 oracle on both sides directly."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.oracle import core as C
from self_replicating_neural_networks_amd.oracle import exact as X
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.population import Population
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

WW = ArchSpec.weightwise(2, 2)
BENCH = dict(attacking_rate=0.1, learn_from_rate=0.1, train=20, learn_from_severity=1, remove_divergent=True,
             remove_zero=True, epsilon=1e-4)
HOT = dict(attacking_rate=0.3, learn_from_rate=0.3, train=3, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.int32)


@pytest.mark.parametrize("spec", [WW, ArchSpec.weightwise(3, 3), ArchSpec.weightwise(4, 3)], ids=str)
def test_init_apply_train_bitwise(spec):
    n, seed = 257, 11
    pop = Population(spec, n, seed=seed)
    w = pop.weights().numpy()
    assert np.array_equal(_bits(w), _bits(X.init(spec, np.arange(n), seed)))
    # one self-application
    ref = X.apply(spec, w, w)
    pop.self_apply(1)
    assert np.array_equal(_bits(pop.weights().numpy()), _bits(ref))
    # three self-train epochs (epoch counters continue from the population's)
    w1 = pop.weights().numpy()
    ctr = pop.ctr
    exp, loss = X.train_epochs(spec, w1, None, 3, True, lr=pop.lr, seed=seed, uids=np.arange(n, dtype=np.uint64),
                               ctr=ctr)
    got_loss = pop.train(3)
    assert np.array_equal(_bits(pop.weights().numpy()), _bits(exp))
    if got_loss is not None:
        assert np.array_equal(_bits(np.asarray(got_loss, dtype=np.float32)), _bits(loss))


@pytest.mark.parametrize("params", [BENCH, HOT], ids=["bench", "hot"])
def test_serial_loop_is_the_exact_oracle(params):
    """host OP_SOUP_SEQ (the reference's in-place, index-order loop) == exact oracle, bitwise,
    three generations (rows, actions, counterparts, losses, respawns)"""
    n, seed = 160, 3
    s = SequentialSoupEngine(WW, n, params, seed=seed)
    W = s.W[:, :WW.P].numpy().copy()
    assert np.array_equal(_bits(W), _bits(X.init(WW, np.arange(n), seed)))
    for g in range(1, 4):
        W, act, cp, loss, rs = X.seq_generation(WW, W, g, seed, params)
        s.evolve(1)
        assert np.array_equal(_bits(s.W[:, :WW.P].numpy()), _bits(W)), g
        assert np.array_equal(s.action.numpy(), act) and np.array_equal(s.counterpart.numpy(), cp)
        assert np.array_equal(s.respawn.numpy(), rs)
        assert np.array_equal(_bits(s.loss.numpy()), _bits(loss))


def test_level_scheduled_generation_is_the_exact_oracle():
    """host OP_SOUP_ORDERED (plan / levels / tail / close) == exact oracle, turn for turn: the
    recorded pre-respawn state of every turn and the final rows"""
    n, seed = 300, 8
    o = SoupEngine(WW, n, HOT, device="cpu", seed=seed, order="sequential")
    W = o.local_rows()[:, :WW.P].numpy().copy()
    for g in range(1, 3):
        W, act, cp, loss, rs, turns = X.seq_generation(WW, W, g, seed, HOT, record_turns=True)
        o.evolve(1)
        assert np.array_equal(_bits(o.local_rows()[:, :WW.P].numpy()), _bits(W)), g
        assert np.array_equal(o.action.numpy(), act) and np.array_equal(o.respawn.numpy(), rs)
        assert o.ordered_levels()["max_level"] >= 1


def test_exact_oracle_is_close_to_the_rounded_oracle():
    """the two oracles differ only by fused vs rounded products: one epoch of SGD agrees to
    ~1e-6 of the row scale (the fused order is the engine's, the rounded one numpy's)"""
    n, seed = 64, 2
    w = X.init(WW, np.arange(n), seed)
    a, _ = X.train_epochs(WW, w, None, 1, True, seed=seed, ctr=512)
    b, _ = C.train_epoch(WW, w, w, seed=seed, ctr=512)
    assert X.max_row_error(a, b) < 1e-5
    assert X.max_row_error(X.apply(WW, w, w), C.apply(WW, w, w)) < 1e-6
