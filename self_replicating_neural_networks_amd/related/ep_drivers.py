"""Experiment drivers of the reference's EP study (related/EP/src/testSomething.py,
evalSomething.py, PltData.plotPoints), on the population-batched ``ReductionLearner``.

The reference runs ONE Keras network per call and repeats calls in Python loops
(``checkLMStatistical`` = 100 x ``checkLM`` = 100 x 200 sequential trainings).  Here every
repetition of a sweep point is a learner of one batched population: all experiments of a
neuron count train together, each with its own stopping rule -- a learner that met its rule
is frozen (weights and Adadelta state restored after every later step), so its loss history
is exactly the one a sequential run that stopped there would have produced.

Stopping rules (``fit`` of related/EP/src/NeuralNetwork.py:218-286), per learner, checked
after loop i (1-based) on its loss history ``r``:

* checkLM: ``sum(r[-1000:]) == 0`` after > 1000 loops -> converged, begin_growing = 0, stop;
  first i with ``growing(r, 10)`` -> begin_growing = i; later, ``not growing(r, 10,
  check_same=False)`` and i - begin_growing > 500 -> stop_growing = i, LM = r[-1], stop.
* checkScale: ``growing(r, 10)`` or ``sum(r[-1000:]) == 0`` or i > 2500 -> stop.
* searchForThreshold: ``growing(r, 100)`` -> (r[0], True); i > 1000 -> (r[0], False).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .ep import ReductionLearner, calc_scale, check_growing, plot_line


# ------------------------------------------------------------------------------ rules
class _LMRule:
    def __init__(self):
        self.begin, self.stop, self.lm, self.done = 0, 0, 0.0, False

    def __call__(self, r: List[float], i: int) -> bool:
        if len(r) > 1000 and float(np.sum(r[-1000:])) == 0.0:
            self.begin, self.done = 0, True
            return True
        if check_growing(r, 10) and self.begin == 0:
            self.begin = i
        if self.begin > 0 and not check_growing(r, 10, check_same=False) and i - self.begin > 500:
            self.stop, self.lm, self.done = i, float(r[-1]), True
            return True
        return False


class _ScaleRule:
    def __call__(self, r: List[float], i: int) -> bool:
        return check_growing(r, 10) or float(np.sum(r[-1000:])) == 0.0 or i > 2500


class _ThresholdRule:
    def __init__(self):
        self.growing: Optional[bool] = None

    def __call__(self, r: List[float], i: int) -> bool:
        if check_growing(r, 100):
            self.growing = True
            return True
        if i > 1000:
            self.growing = False
            return True
        return False


def run_with_rules(learner: ReductionLearner, rules: Sequence, max_loops: Optional[int] = None,
                   record_features: bool = False) -> Dict:
    """Train every learner until its own rule fires (or ``max_loops``): per-learner loss
    histories (ragged), the loop count of each, optionally the reduced input per loop."""
    n = learner.n
    hist: List[List[float]] = [[] for _ in range(n)]
    feats: List[List[float]] = [[] for _ in range(n)]
    done = np.zeros(n, dtype=bool)
    loops = max_loops or learner.number_loops
    for i in range(1, loops + 1):
        if done.all():
            break
        snap = [[t.clone() for t in lst] for lst in (learner.kernels, learner.biases, learner._acc_g,
                                                      learner._acc_dx)]
        if record_features:
            x = learner.features().detach().cpu().numpy()
        loss = (learner.hill_climber_step() if learner.hill else learner.adadelta_step()).cpu().numpy()
        newly = np.zeros(n, dtype=bool)
        for k in np.nonzero(~done)[0]:
            hist[k].append(float(loss[k]))
            if record_features:
                feats[k].append(x[k].tolist())
            newly[k] = bool(rules[k](hist[k], i))
        frozen = done  # learners already stopped before this step: undo the step for them
        if frozen.any():
            m = torch.as_tensor(frozen, device=learner.device)
            for lst, old in zip((learner.kernels, learner.biases, learner._acc_g, learner._acc_dx), snap):
                for j, (cur, o) in enumerate(zip(lst, old)):
                    lst[j] = torch.where(m.view((-1,) + (1,) * (cur.dim() - 1)), o, cur)
        done = done | newly
    return dict(losses=hist, loops=[len(h) for h in hist], features=feats if record_features else None)


# ------------------------------------------------------------------------------ drivers
def test_something(number_of_neurons=(1, 2, 1), activation_functions=("sigmoid", "linear"), feature_reduction="rfft",
                   number_loops=1000, experiments=1, check_lm=False, check_scale=False, search_for_threshold=False,
                   seed=0, device="cpu", **learner_kw) -> Dict:
    """One configuration (testSomething), ``experiments`` independent runs batched."""
    L = ReductionLearner(list(number_of_neurons), list(activation_functions)[:len(number_of_neurons) - 1],
                         feature_reduction=feature_reduction, number_loops=number_loops, population=experiments,
                         seed=seed, device=device, **learner_kw)
    if check_lm:
        rules = [_LMRule() for _ in range(experiments)]
    elif check_scale:
        rules = [_ScaleRule() for _ in range(experiments)]
    elif search_for_threshold:
        rules = [_ThresholdRule() for _ in range(experiments)]
    else:
        rules = [lambda r, i: False] * experiments
    out = run_with_rules(L, rules)
    out["learner"] = L
    if check_lm:
        out.update(begin_growing=np.array([r.begin for r in rules]), stop_growing=np.array([r.stop for r in rules]),
                   lm=np.array([r.lm for r in rules]))
    if search_for_threshold:
        out.update(first=np.array([h[0] for h in out["losses"]]), growing=np.array([bool(r.growing) for r in rules]))
    return out


def check_lm(max_number_of_neurons=200, feature_reduction="rfft", number_loops=100000, experiments=1, seed=0,
             device="cpu", out_dir: Optional[str] = None) -> Dict:
    """checkLM (testSomething.py:2670-2705): hidden width from ``max_number_of_neurons`` down
    to 1 of a [1, i, 1] sigmoid/linear net; per width and experiment the loop where the MSE
    starts growing, the loop where it stops (local maximum reached) and the maximum."""
    neurons, begin, stop, lm = [], [], [], []
    for i in range(max_number_of_neurons, 0, -1):
        r = test_something([1, i, 1], ["sigmoid", "linear"], feature_reduction, number_loops, experiments,
                           check_lm=True, seed=seed + i, device=device)
        neurons.append(i)
        begin.append(r["begin_growing"])
        stop.append(r["stop_growing"])
        lm.append(r["lm"])
    res = dict(neurons=np.array(neurons), beginGrowing=np.array(begin), stopGrowing=np.array(stop), LM=np.array(lm))
    if out_dir:
        for key in ("beginGrowing", "stopGrowing", "LM"):
            plot_line(res[key].mean(1), os.path.join(out_dir, f"{key}_{feature_reduction}.png"), x=res["neurons"],
                      x_label="neurons in the hidden layer", y_label=key)
    return res


def check_lm_statistical(number_of_experiments=100, max_number_of_neurons=200, feature_reduction="rfft",
                         number_loops=100000, seed=0, device="cpu", out_dir: Optional[str] = None) -> Dict:
    """checkLMStatistical (testSomething.py:2730-2780): checkLM repeated; average / max / min
    of beginGrowing, stopGrowing, LM per width, and the probability that the MSE converges
    at once (LM not > 0)."""
    r = check_lm(max_number_of_neurons, feature_reduction, number_loops, number_of_experiments, seed, device)
    out = dict(neurons=r["neurons"])
    for key in ("beginGrowing", "stopGrowing", "LM"):
        v = r[key].astype(float)
        out[key] = dict(avg=v.mean(1), max=v.max(1), min=v.min(1))
        if out_dir:
            plot_line(np.stack([out[key]["avg"], out[key]["max"], out[key]["min"]]),
                      os.path.join(out_dir, f"statistical_{key}_{number_of_experiments}.png"), x=r["neurons"],
                      legend=("AVG", "MAX", "MIN"), text=f"feature reduction: {feature_reduction}\n"
                                                         f"experiments: {number_of_experiments}")
    out["prob_converges"] = (~(r["LM"] > 0.0)).mean(1)
    if out_dir:
        plot_line(out["prob_converges"], os.path.join(out_dir, f"statistical_probability_{number_of_experiments}.png"),
                  x=r["neurons"], y_label="P(MSE converges at once)")
    return out


def check_scale_of_function(number_of_experiments=400, hidden=76, feature_reduction="rfft", number_loops=10000,
                            seed=0, device="cpu", out_dir: Optional[str] = None) -> Dict:
    """checkScaleOfFunction (testSomething.py:2783-2815): train [1, hidden, 1] nets with the
    checkScale rule, evaluate each on -1000..999 and sort them by whether the function
    crosses zero, and whether 0 maps to 0 (3 decimals); value = the function's scale."""
    r = test_something([1, hidden, 1], ["sigmoid", "linear"], feature_reduction, number_loops,
                       number_of_experiments, check_scale=True, seed=seed, device=device)
    data = np.arange(-1000, 1000, 1)
    p = r["learner"].evaluate(data)  # [experiments, 2000]
    through, not_through, null_is_null = [], [], []
    for row in p:
        sc = calc_scale(row)
        if round(float(row[1000]), 3) == 0.0:
            null_is_null.append(sc)
        (through if (row.max() > 0 and row.min() < 0) else not_through).append(sc)
    res = dict(through_null=through, not_through_null=not_through, null_is_null=null_is_null, loops=r["loops"])
    if out_dir:
        plot_points([through, not_through, null_is_null], ["through zero", "not through zero", "0 -> 0"],
                    os.path.join(out_dir, "throughNull_notThroughNull_-1000_1000.png"), xlabel="scale of the function")
    return res


def search_for_threshold(number_of_experiments=1000, hidden=98, feature_reduction="mean", number_loops=100000001,
                         seed=0, device="cpu", out_dir: Optional[str] = None) -> Dict:
    """searchForThreshold (testSomething.py:2614-2632): the initial MSE of runs whose MSE
    climbs to a local maximum (growing over 100 loops before loop 1000) vs runs where it
    does not; plotted as points (plotResultSearchForThreshold)."""
    r = test_something([1, hidden, 1], ["linear", "sigmoid", "linear"], feature_reduction, number_loops,
                       number_of_experiments, search_for_threshold=True, seed=seed, device=device)
    grow = r["first"][r["growing"]].tolist()
    not_grow = r["first"][~r["growing"]].tolist()
    if out_dir:
        plot_points([grow, not_grow], ["grow", "notgrow"], os.path.join(out_dir, "threshold.png"),
                    xlabel="initial mean squared error")
    return dict(grow=grow, not_grow=not_grow)


def plot_value_representation(number_of_experiments=1, hidden=600, feature_reduction="mean", number_loops=10000,
                              seed=0, device="cpu", out_dir: Optional[str] = None) -> Dict:
    """plotValueRepresentation (testSomething.py:2818-2845): the reduced input value (the
    net's own representation) per loop, and whether the run converged (last 1000 losses 0)."""
    L = ReductionLearner([1, hidden, 1], ["sigmoid", "linear"], feature_reduction=feature_reduction,
                         number_loops=number_loops, population=number_of_experiments, seed=seed, device=device)
    r = run_with_rules(L, [lambda h, i: False] * number_of_experiments, record_features=True)
    values = [np.asarray(f, dtype=float)[:, 0] for f in r["features"]]
    converged = [float(np.sum(h[-1000:])) == 0.0 for h in r["losses"]]
    if out_dir:
        for k, (v, c) in enumerate(zip(values, converged)):
            plot_line(v, os.path.join(out_dir, f"{L.file_name()}_run_{k + 1}.png"), x_label="loops",
                      y_label=f"value representation {feature_reduction}", text=f"converges {str(c).upper()}")
    return dict(values=values, converged=converged)


def eval_something(learner: ReductionLearner, start=-10000, stop=10000, step=1, out_dir: Optional[str] = None) -> Dict:
    """evalSomething (evalSomething.py:40-60): a trained model's function over a value range
    and its fixpoint candidate (the reduced representation of its own weights)."""
    data = np.arange(start, stop, step)
    y = learner.evaluate(data)
    fp = learner.features().detach().cpu().numpy()[:, 0]
    if out_dir:
        for k in range(y.shape[0]):
            plot_line(y[k], os.path.join(out_dir, f"{learner.file_name()}_{start}_{stop}_{step}_{k}.png"), x=data,
                      x_label="X", y_label="Y", text=f"fixpoint: {fp[k]}")
    return dict(x=data, y=y, fixpoint=fp)


# ------------------------------------------------------------------------------ PltData
def plot_points(data, labels, filename, xlabel=""):
    """PltData.plotPoints (PltData.py:83-95): each series as dots on its own row."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure(figsize=(1600 / 96, 5))
    dots = ["ro", "go", "bo", "yo"]
    for i, row in enumerate(data):
        row = list(row)
        plt.plot(row, [i] * len(row), dots[i % len(dots)], label=labels[i])
    plt.legend()
    plt.xlabel(xlabel)
    plt.grid(True)
    os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
    plt.savefig(filename, bbox_inches="tight")
    plt.close()
    return filename
