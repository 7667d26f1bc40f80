"""EP sweep drivers (related/EP/src/testSomething.py, evalSomething.py, PltData.plotPoints)
on the batched ReductionLearner: per-learner stopping rules, frozen learners, plots."""
import os

import numpy as np
import torch

from self_replicating_neural_networks_amd.related import ep_drivers as D
from self_replicating_neural_networks_amd.related.ep import ReductionLearner, check_growing


def test_lm_rule_matches_reference_loop_semantics():
    # loss falls, then grows for > 500 loops, then flattens: begin / stop / LM as the loop sees them
    curve = list(np.linspace(1.0, 0.5, 100)) + list(np.linspace(0.5, 2.0, 700)) + list(np.linspace(2.0, 1.0, 50))
    rule = D._LMRule()
    r = []
    for i, v in enumerate(curve, 1):
        r.append(v)
        if rule(r, i):
            break
    assert 100 < rule.begin < 130            # first window where the last 10 sum >= the 10 before
    assert rule.stop > rule.begin + 500 and rule.lm == r[-1]
    z = D._LMRule()
    r = []
    for i in range(1, 1200):
        r.append(0.0)
        if z(r, i):
            break
    assert z.done and z.begin == 0 and i == 1001  # 1000 exact zeros: converged fixpoint


def test_frozen_learners_keep_their_state():
    L = ReductionLearner([1, 4, 1], ["sigmoid", "linear"], feature_reduction="rfft", number_loops=30, population=3,
                         seed=1)
    rules = [lambda r, i: i >= 5, lambda r, i: i >= 12, lambda r, i: False]
    out = D.run_with_rules(L, rules)
    assert out["loops"] == [5, 12, 30]
    # a learner trained alone for 5 loops ends with the same kernels as the frozen one
    L2 = ReductionLearner([1, 4, 1], ["sigmoid", "linear"], feature_reduction="rfft", number_loops=5, population=3,
                          seed=1)
    for _ in range(5):
        L2.adadelta_step()
    assert torch.allclose(L.kernels[0][0], L2.kernels[0][0]) and torch.allclose(L.kernels[1][0], L2.kernels[1][0])


def test_sweeps_run_and_plot(tmp_path):
    r = D.check_lm_statistical(number_of_experiments=3, max_number_of_neurons=2, number_loops=40, out_dir=str(tmp_path))
    assert list(r["neurons"]) == [2, 1] and r["LM"]["avg"].shape == (2,) and r["prob_converges"].shape == (2,)
    s = D.check_scale_of_function(number_of_experiments=4, hidden=3, number_loops=30, out_dir=str(tmp_path))
    assert len(s["through_null"]) + len(s["not_through_null"]) == 4 and all(v >= 0 for v in s["through_null"])
    t = D.search_for_threshold(number_of_experiments=4, hidden=3, number_loops=30, out_dir=str(tmp_path))
    assert len(t["grow"]) + len(t["not_grow"]) == 4
    v = D.plot_value_representation(number_of_experiments=2, hidden=5, number_loops=20, out_dir=str(tmp_path))
    assert len(v["values"]) == 2 and len(v["values"][0]) == 20
    L = ReductionLearner([1, 3, 1], ["sigmoid", "linear"], feature_reduction="rfft", population=2, seed=2)
    e = D.eval_something(L, -50, 50, 1, out_dir=str(tmp_path))
    assert e["y"].shape == (2, 100) and e["fixpoint"].shape == (2,)
    for f in ("threshold.png", "throughNull_notThroughNull_-1000_1000.png", "statistical_LM_3.png"):
        assert os.path.getsize(tmp_path / f) > 0


def test_plot_points(tmp_path):
    f = D.plot_points([[0.1, 0.2], [0.05]], ["grow", "notgrow"], str(tmp_path / "p.png"), xlabel="x")
    assert os.path.getsize(f) > 0 and check_growing([1, 2, 3, 4], 2)
