"""Golden statistical tests against the reference's published outcome numbers
(code/results/**/log.txt).  Trials are population rows, so we use many
more than the reference's 50 and compare with binomial / normal confidence bounds."""
import numpy as np
import pytest

from self_replicating_neural_networks_amd.setups import experiments as E


def within(p_hat, n, p_ref, n_ref, z=4.0):
    """|p_hat - p_ref| within z standard errors of the combined binomial estimate."""
    se = np.sqrt(p_hat * (1 - p_hat) / n + p_ref * (1 - p_ref) / n_ref) + 1e-9
    return abs(p_hat - p_ref) <= z * se


@pytest.fixture(scope="module")
def applying(tmp_path_factory):
    return E.applying_fixpoints(trials=4000, device="cpu", seed=1, root=str(tmp_path_factory.mktemp("a")))


def test_applying_fixpoints_weightwise(applying):
    c = applying["counters"][0]  # published 23 divergent / 27 fix_zero of 50
    assert c["divergent"] + c["fix_zero"] == 4000
    assert within(c["divergent"] / 4000, 4000, 23 / 50, 50)


def test_applying_fixpoints_aggregating(applying):
    c = applying["counters"][1]  # published 4 / 46
    assert c["divergent"] + c["fix_zero"] == 4000
    assert within(c["divergent"] / 4000, 4000, 4 / 50, 50)


def test_applying_fixpoints_recurrent(applying):
    c = applying["counters"][2]  # published 46 / 4
    assert c["divergent"] + c["fix_zero"] == 4000
    assert within(c["divergent"] / 4000, 4000, 46 / 50, 50)


def test_training_fixpoints_ww_and_agg(tmp_path):
    r = E.training_fixpoints(trials=200, device="cpu", seed=2, root=str(tmp_path),
                             specs=(E.WW, E.AGG))
    ww, agg = r["counters"]
    assert ww["fix_other"] >= 196        # published 50/50 fix_other
    assert agg["other"] >= 196           # published 50/50 other


def test_known_fixpoint_variation_curve(tmp_path):
    r = E.known_fixpoint_variation(trials=400, device="cpu", seed=3, root=str(tmp_path))
    pub_y = [3.63, 5.02, 6.46, 8.04, 9.61, 11.23, 12.99, 14.58, 21.95, 26.45]
    pub_z = [0, 0, 0, 0, 0.04, 1.38, 3.23, 4.84, 11.91, 16.47]
    assert np.allclose(r["ys"], pub_y, atol=1.0, rtol=0.06)
    assert np.allclose(r["zs"], pub_z, atol=0.6, rtol=0.08)
    # the float32 jump between 1e-7 and 1e-8
    assert r["ys"][8] - r["ys"][7] > 5


def test_learn_from_soup_curve(tmp_path):
    r = E.learn_from_soup(trials=100, device="cpu", seed=4, root=str(tmp_path))
    zs = np.array(r["data"][0]["zs"])
    pub = np.array([0, 1.2, 5.2, 7.4, 8.1, 9.1, 9.6, 9.8, 10.0, 9.9, 9.9])
    assert zs[0] == 0 and np.all(np.array(r["data"][0]["ys"]) < 0.2)
    assert np.max(np.abs(zs - pub)) < 1.6
    assert np.all(np.diff(zs[:6]) > -0.3)  # monotone rise with severity


def test_mixed_soup_curve(tmp_path):
    r = E.mixed_soup(trials=100, device="cpu", seed=5, root=str(tmp_path))
    ww, agg = r["data"]
    pub = np.array([0, 0, 0.7, 1.9, 3.6, 4.3, 6.0, 6.1, 8.3, 7.7, 8.8])
    assert np.max(np.abs(np.array(ww["zs"]) - pub)) < 1.6
    assert np.all(np.array(agg["zs"]) == 0)  # aggregating soups never reach non-zero fixpoints
    # aggregating zero fixpoints per 10-particle soup (code/results/exp-mixed-soup-*/log.txt:6):
    # published 0.8, 0.4, 0.4, 0.3, 0.2, 0.2, 0.2, 0.2, 0.2, 0.4, 0.3 from 10 soups per point.
    # In the reference's order (the setup's default since the level-scheduled generation) the
    # rate is ~0.41 per soup at every train count (the synchronous generation gives ~0.31).  A
    # published point averages 10 soups of ~Binomial(10, 0.041) counts: standard error ~0.2, so
    # the first point (0.8) is ~2 standard errors above 0.41 -- every point, that one included,
    # is asserted within 2.5 standard errors, the level within ~1.3 standard errors of the mean.
    pub_agg = np.array([0.8, 0.4, 0.4, 0.3, 0.2, 0.2, 0.2, 0.2, 0.2, 0.4, 0.3])
    agg_y = np.array(agg["ys"])
    assert np.all(agg_y > 0)
    assert abs(agg_y.mean() - pub_agg.mean()) < 0.12
    assert np.max(np.abs(agg_y - pub_agg)) < 0.5


def test_mixed_self_fixpoints_curve(tmp_path):
    r = E.mixed_self_fixpoints(trials=200, device="cpu", seed=6, root=str(tmp_path),
                               trains=[0, 250, 500])
    ww, agg, rnn = (np.array(d["ys"]) for d in r["data"])
    assert ww[0] < 0.45 and ww[2] > 0.8      # published 0.2 -> 1.0
    assert np.all(agg > 0.75)                 # published 0.8 .. 1.0
    assert np.all(rnn < 0.25)                 # published 0 .. 0.1


def _numpy_ww_self_attacks(n, attacks=4, eps=1e-4, seed=0, trains=0, lr=0.01):
    """Independent float32 NumPy re-derivation of the Keras WeightwiseNeuralNetwork(2, 2)
    self-attack / self-train loop of mixed-self-fixpoints.py:81-86 (network.py:213-273
    apply_to_weights with normalize_id, network.py:140-157 is_fixpoint, network.py:281-289
    compute_samples + :613-618 train = one Keras epoch of shuffled batch-size-1 SGD on MSE,
    lr 0.01; glorot_uniform kernels, linear, no bias).  Shares no code with the engine."""
    rng = np.random.default_rng(seed)
    shapes = [(4, 2), (2, 2), (2, 1)]
    W = [rng.uniform(-np.sqrt(6 / sum(s)), np.sqrt(6 / sum(s)), (n,) + s).astype(np.float32)
         for s in shapes]

    def nid(v, m):
        return v / m if m > 1 else float(v)
    pts = [(L, c, k, nid(L, 2), nid(c, s[0] - 1), nid(k, s[1] - 1))
           for L, s in enumerate(shapes) for c in range(s[0]) for k in range(s[1])]

    def apply(net, src):
        out = [w.copy() for w in src]
        for L, c, k, nl, nc, nk in pts:
            h = np.stack([src[L][:, c, k]] + [np.full(n, v, np.float32) for v in (nl, nc, nk)], 1)[:, None]
            for w in net:
                h = h @ w
            out[L][:, c, k] = h[:, 0, 0]
        return out

    def epoch(W):
        X = np.stack([np.stack([W[L][:, c, k]] + [np.full(n, v, np.float32) for v in (nl, nc, nk)], 1)
                      for L, c, k, nl, nc, nk in pts], 1)               # [n, 14, 4] samples
        order = np.argsort(rng.random((n, len(pts))), 1)                 # per-net shuffle
        W = [w.copy() for w in W]
        for j in range(len(pts)):
            x = X[np.arange(n), order[:, j]][:, None]                    # [n, 1, 4]
            hs = [x]
            for w in W:
                hs.append(hs[-1] @ w)
            d = np.float32(2) * (hs[-1] - x[:, :, :1])                   # dL/dy, L = (y - t)^2
            for L in range(len(W) - 1, -1, -1):
                g = np.swapaxes(hs[L], 1, 2) @ d
                d = d @ np.swapaxes(W[L], 1, 2)
                W[L] = W[L] - np.float32(lr) * g
        return W

    active = np.ones(n, bool)
    with np.errstate(all="ignore"):
        for _ in range(attacks):
            new = apply(W, W)
            for _ in range(trains):
                new = epoch(new)
            W = [np.where(active[:, None, None], b, a) for a, b in zip(W, new)]
            nxt = apply(W, W)
            fin = np.all([np.isfinite(w.reshape(n, -1)).all(1) for w in W], 0)
            fix = np.all([(np.abs(a - b) < eps).reshape(n, -1).all(1) & np.isfinite(b.reshape(n, -1)).all(1)
                          for a, b in zip(W, nxt)], 0)
            active &= ~(fix | ~fin)
    return fix.mean()


@pytest.mark.parametrize("trains", [0, 100])
def test_mixed_self_fixpoints_ww_independent(tmp_path, trains):
    """The published Weightwise points at trains=0 and 100 are 4/20 and 3/20; the engine
    gives ~0.43 at both.  An engine-independent NumPy derivation of the same Keras loop gives
    the same (0.425 / 0.439 at 4000 nets), so the published points are low 20-trial draws,
    not a semantic gap (profiles/r3f_published_outcomes_at_scale.md)."""
    p_np = _numpy_ww_self_attacks(4000, trains=trains, seed=trains + 1)
    r = E.mixed_self_fixpoints(trials=4000, device="cpu", seed=9, root=str(tmp_path),
                               trains=[trains], specs=(E.WW,))
    p_eng = r["data"][0]["ys"][0]
    assert 0.38 < p_np < 0.49
    assert within(p_eng, 4000, p_np, 4000)


def test_network_trajectorys_records(tmp_path):
    r = E.network_trajectorys(trials=20, device="cpu", seed=7, root=str(tmp_path))
    assert sum(r["counters"].values()) == 20
    from self_replicating_neural_networks_amd.io import refpickle as R
    import os
    t = R.load(os.path.join(r["dir"], "trajectorys.dill"))
    assert len(t.historical_particles) == 20
    states = next(iter(t.historical_particles.values()))
    assert states[0]["action"] == "init" and [s["time"] for s in states] == list(range(len(states)))


def test_training_fixpoints_recurrent_divergence():
    """1000-epoch Recurrent self-training: published 38/50 divergent, 12/50 other
    (code/results/exp-training_fixpoint-*/log.txt:9-10).  Pinned by Keras' Orthogonal
    initializer being LAPACK's SVD U (a reflection for 2x2 kernels), csrc/srnn_core.h
    lapack_u2; with a Haar orthogonal init ~48 % diverge."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        r = E.training_fixpoints(trials=400, device="cpu", seed=8, root=d, specs=(E.RNN,))
    c = r["counters"][0]
    assert c["divergent"] + c["other"] + c["fix_other"] + c["fix_zero"] + c["fix_sec"] == 400
    assert within(c["divergent"] / 400, 400, 38 / 50, 50)
    assert c["divergent"] / 400 > 0.62
