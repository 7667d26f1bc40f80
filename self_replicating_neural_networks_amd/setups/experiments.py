"""The reference's experiment drivers (code/setups/*.py and the ``__main__`` blocks of
code/network.py / code/soup.py) as population-scale functions.

Every trial of a reference experiment is an independent particle (or an independent
soup), so a whole experiment runs as a few device launches over a ``Population`` /
segmented ``SoupEngine`` instead of Python loops over Keras models.  Defaults equal the
reference's settings; ``trials`` can be raised by orders of magnitude for tight
statistics.  Each function writes the same experiment directory as the reference
(``log.txt``, ``experiment.dill`` and the script's ``all_*.dill`` / ``trajectorys.dill``
/ ``soup.dill``) and returns the data it logged.
"""
from __future__ import annotations

from statistics import mean
from typing import Dict, List, Optional

import numpy as np
import torch

from ..arch import ArchSpec
from ..experiment import Experiment, FixpointExperiment, SoupExperiment
from ..models import network as N
from ..oracle.core import CLASS_NAMES
from ..ops import _lib
from ..population import Population, counts_dict
from ..seq_soup import SequentialSoupEngine
from ..soup import Soup
from ..soup_engine import SoupEngine
from ..utils import rng as _rng

WW = ArchSpec.weightwise(2, 2)
AGG = ArchSpec.aggregating(4, 2, 2)
RNN = ArchSpec.recurrent(2, 2)
FFT = ArchSpec.fft(4, 2, 2)


def default_device():
    return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def generate_counters() -> Dict[str, int]:
    return {"divergent": 0, "fix_zero": 0, "fix_other": 0, "fix_sec": 0, "other": 0}


def ref_name(spec: ArchSpec, quote_bias: bool = False) -> str:
    """Name string of the reference setups (sic 'activiation', code/setups/*.py)."""
    if quote_bias:
        return f"{spec.class_name} activiation='linear' use_bias='False'"
    return f"{spec.class_name} activiation='linear' use_bias=False"


def _seed(seed):
    return _rng.get_seed() if seed is None else int(seed)


def _add(counters, counts):
    for k in CLASS_NAMES:
        counters[k] += int(counts.get(k, 0))
    return counters


# ------------------------------------------------------------------------------ C17
def applying_fixpoints(trials=50, run_count=100, epsilon=1e-4, device=None, seed=None, root="experiments",
                       specs=(WW, AGG, RNN)):
    """100 self-applications of fresh nets, then classify (code/setups/applying-fixpoints.py)."""
    device = device or default_device()
    with Experiment("applying_fixpoint", root=root) as exp:
        exp.trials, exp.run_count, exp.epsilon = trials, run_count, epsilon
        all_counters, all_names = [], []
        for k, spec in enumerate(specs):
            pop = Population(spec, trials, device=device, seed=_seed(seed) + k)
            pop.self_apply(run_count)
            all_counters.append(_add(generate_counters(), pop.count(epsilon)))
            all_names.append(ref_name(spec))
        exp.save(all_counters=all_counters)
        exp.save(trajectorys=exp.without_particles())
        exp.save(all_names=all_names)
        for name, c in zip(all_names, all_counters):
            exp.log(name)
            exp.log(c)
            exp.log("\n")
    return dict(names=all_names, counters=all_counters, dir=exp.dir)


# ------------------------------------------------------------------------------ C18
def training_fixpoints(trials=50, run_count=1000, epsilon=1e-4, device=None, seed=None, root="experiments",
                       specs=(WW, AGG, RNN)):
    """1000 self-train epochs of fresh nets, then classify (code/setups/training-fixpoints.py)."""
    device = device or default_device()
    with Experiment("training_fixpoint", root=root) as exp:
        exp.trials, exp.run_count, exp.epsilon = trials, run_count, epsilon
        all_counters, all_names = [], []
        for k, spec in enumerate(specs):
            pop = Population(spec, trials, device=device, seed=_seed(seed) + k)
            pop.train(run_count)
            all_counters.append(_add(generate_counters(), pop.count(epsilon)))
            all_names.append(ref_name(spec))
        exp.save(all_counters=all_counters)
        exp.save(trajectorys=exp.without_particles())
        exp.save(all_names=all_names)
        for name, c in zip(all_names, all_counters):
            exp.log(name)
            exp.log(c)
            exp.log("\n")
    return dict(names=all_names, counters=all_counters, dir=exp.dir)


# ------------------------------------------------------------------------------ C19
def fixpoint_density(trials=100000, epsilon=1e-4, device=None, seed=None, root="experiments", specs=(WW, AGG)):
    """Classify random nets at initialisation (code/setups/fixpoint-density.py)."""
    device = device or default_device()
    with Experiment("fixpoint-density", root=root) as exp:
        exp.trials, exp.epsilon = trials, epsilon
        all_counters, all_names = [], []
        for k, spec in enumerate(specs):
            pop = Population(spec, trials, device=device, seed=_seed(seed) + k)
            all_counters.append(_add(generate_counters(), pop.count(epsilon)))
            all_names.append("ParticleDecorator activiation='linear' use_bias='False'")
        exp.save(all_counters=all_counters)
        exp.save(all_notable_nets=[])
        exp.save(all_names=all_names)
        for name, c in zip(all_names, all_counters):
            exp.log(name)
            exp.log(c)
            exp.log("\n")
    return dict(names=all_names, counters=all_counters, dir=exp.dir)


# ------------------------------------------------------------------------------ C20
def identity_fixpoint_weights() -> np.ndarray:
    """code/setups/known-fixpoint-variation.py:20-25: f(x) = x[0] for WW(2, 2)."""
    w = np.zeros(14, dtype=np.float32)
    w[0] = w[8] = w[12] = 1.0
    return w


def known_fixpoint_variation(depth=10, trials=100, max_steps=100, epsilon=1e-4, device=None, seed=None,
                             root="experiments"):
    """Perturb the identity fixpoint at scales 1, 1e-1, ... and measure time to
    divergence/zero and time still a fixpoint (code/setups/known-fixpoint-variation.py)."""
    device = device or default_device()
    with Experiment("known-fixpoint-variation", root=root) as exp:
        exp.depth, exp.trials, exp.max_steps, exp.epsilon = depth, trials, max_steps, epsilon
        exp.xs, exp.ys, exp.zs, exp.notable_nets = [], [], [], []
        scale = 1.0
        for d in range(depth):
            pop = Population(WW, trials, device=device, seed=_seed(seed) + d,
                             weights=np.tile(identity_fixpoint_weights(), (trials, 1)))
            pop.perturb(scale)
            tts, taf = pop.vary_run(max_steps, epsilon)
            exp.xs += [scale] * trials
            exp.ys += tts.cpu().numpy().astype(int).tolist()
            exp.zs += taf.cpu().numpy().astype(int).tolist()
            scale /= 10.0
        for d in range(depth):
            exp.log("variation 10e-" + str(d))
            exp.log("avg time to vergence " + str(mean(exp.ys[d * trials:(d + 1) * trials])))
            exp.log("avg time as fixpoint " + str(mean(exp.zs[d * trials:(d + 1) * trials])))
    ys = [mean(exp.ys[d * trials:(d + 1) * trials]) for d in range(depth)]
    zs = [mean(exp.zs[d * trials:(d + 1) * trials]) for d in range(depth)]
    return dict(xs=[10.0 ** -d for d in range(depth)], ys=ys, zs=zs, dir=exp.dir)


# ------------------------------------------------------------------------------ soups
def _soup_census(spec, trials, soup_size, soup_life, params, device, seed, with_sec=False, order="sequential"):
    """``trials`` independent soups as sub-soups (segments) of one engine, in the reference's
    order by default (``order="sequential"``: each sub-soup evolves particle by particle, in
    place -- code/soup.py:51-87 -- on the level-scheduled device generation, or on the host
    loop for shapes without one); ``order="synchronous"`` runs the Jacobi generation."""
    params = dict(params, segment=soup_size)
    if order == "sequential":
        dev_side = torch.device(device).type != "cpu"
        if _lib.supports(spec, _lib.OP_SOUP_ORDERED, dev_side):
            eng = SoupEngine(spec, trials * soup_size, params, device=device, seed=seed, order="sequential")
        else:
            eng = SequentialSoupEngine(spec, trials * soup_size, params, seed=seed)
    else:
        eng = SoupEngine(spec, trials * soup_size, params, device=device, seed=seed)
    eng.evolve(soup_life)
    return eng.count(with_sec=with_sec)


def learn_from_soup(soup_size=10, soup_life=100, trials=10, severities=None, epsilon=1e-4, device=None, seed=None,
                    root="experiments", specs=(WW,)):
    """Soups that only learn from each other; census vs learn_from_severity
    (code/setups/learn_from_soup.py)."""
    device = device or default_device()
    severities = severities if severities is not None else [10 * i for i in range(11)]
    with SoupExperiment("learn-from-soup", root=root) as exp:
        exp.soup_size, exp.soup_life, exp.trials = soup_size, soup_life, trials
        exp.learn_from_severity_values = list(severities)
        exp.epsilon = epsilon
        all_names, all_data = [], []
        for k, spec in enumerate(specs):
            xs, ys, zs = [], [], []
            for sev in severities:
                c = _soup_census(spec, trials, soup_size, soup_life,
                                 dict(attacking_rate=-1, learn_from_rate=0.1, train=0, learn_from_severity=sev,
                                      epsilon=epsilon), device, _seed(seed) + 1000 * k + sev, with_sec=False)
                xs.append(sev)
                ys.append(float(c["fix_zero"]) / float(trials))
                zs.append(float(c["fix_other"]) / float(trials))
            all_names.append(f"{spec.class_name} activiation='linear' use_bias=False")
            all_data.append({"xs": xs, "ys": ys, "zs": zs})
        exp.save(all_names=all_names)
        exp.save(all_data=all_data)
        for name, data in zip(all_names, all_data):
            exp.log(name)
            exp.log(data)
            exp.log("\n")
    return dict(names=all_names, data=all_data, dir=exp.dir)


def mixed_soup(soup_size=10, soup_life=5, trials=10, trains=None, epsilon=1e-4, device=None, seed=None,
               root="experiments", specs=(WW, AGG)):
    """Soups with attacks + N self-trains per generation; census vs N
    (code/setups/mixed-soup.py)."""
    device = device or default_device()
    trains = trains if trains is not None else [10 * i for i in range(11)]
    with Experiment("mixed-soup", root=root) as exp:
        exp.trials, exp.soup_size, exp.soup_life = trials, soup_size, soup_life
        exp.trains_per_selfattack_values = list(trains)
        exp.epsilon = epsilon
        all_names, all_data = [], []
        for k, spec in enumerate(specs):
            xs, ys, zs = [], [], []
            for t in trains:
                c = _soup_census(spec, trials, soup_size, soup_life,
                                 dict(attacking_rate=0.1, learn_from_rate=-1, train=t, learn_from_severity=-1,
                                      epsilon=epsilon), device, _seed(seed) + 1000 * k + t, with_sec=False)
                xs.append(t)
                ys.append(float(c["fix_zero"]) / float(trials))
                zs.append(float(c["fix_other"]) / float(trials))
            all_names.append(f"{spec.class_name} activiation='linear' use_bias=False")
            all_data.append({"xs": xs, "ys": ys, "zs": zs})
        exp.save(all_names=all_names)
        exp.save(all_data=all_data)
        for name, data in zip(all_names, all_data):
            exp.log(name)
            exp.log(data)
            exp.log("\n")
    return dict(names=all_names, data=all_data, dir=exp.dir)


# ------------------------------------------------------------------------------ C22
def mixed_self_fixpoints(trials=20, selfattacks=4, trains=None, epsilon=1e-4, device=None, seed=None,
                         root="experiments", specs=(WW, AGG, RNN)):
    """Self-attack followed by N self-train epochs, up to ``selfattacks`` times, stopping a
    net once it is divergent or a fixpoint (code/setups/mixed-self-fixpoints.py)."""
    device = device or default_device()
    trains = trains if trains is not None else [50 * i for i in range(11)]
    with Experiment("mixed-self-fixpoints", root=root) as exp:
        exp.trials, exp.selfattacks = trials, selfattacks
        exp.trains_per_selfattack_values = list(trains)
        exp.epsilon = epsilon
        all_names, all_data = [], []
        for k, spec in enumerate(specs):
            xs, ys = [], []
            for t in trains:
                pop = Population(spec, trials, device=device, seed=_seed(seed) + 1000 * k + t)
                active = torch.ones(trials, dtype=torch.bool, device=pop.device)
                for _ in range(selfattacks):
                    before = pop.W.clone()
                    pop.self_apply(1)
                    if t:
                        pop.train(t)
                    pop.W.copy_(torch.where(active[:, None], pop.W, before))
                    cls, _ = pop.classify(epsilon, with_sec=False)
                    active &= ~((cls == 0) | (cls == 1) | (cls == 2))
                    if not bool(active.any()):
                        break
                c = pop.count(epsilon)
                xs.append(t)
                ys.append(float(c["fix_zero"] + c["fix_other"]) / float(trials))
            all_names.append(ref_name(spec))
            all_data.append({"xs": xs, "ys": ys})
        exp.save(all_names=all_names)
        exp.save(all_data=all_data)
        for name, data in zip(all_names, all_data):
            exp.log(name)
            exp.log(data)
            exp.log("\n")
    return dict(names=all_names, data=all_data, dir=exp.dir)


# ------------------------------------------------------------------------------ C24
def network_trajectorys(trials=20, step_limit=100, epsilon=1e-4, spec=WW, device=None, seed=None,
                        root="experiments", name="weightwise_self_application"):
    """run_net with recorded trajectories (code/setups/network_trajectorys.py)."""
    device = device or default_device()
    with FixpointExperiment(name=name, root=root) as exp:
        pop = Population(spec, trials, device=device, seed=_seed(seed))
        exp.run_population(pop, step_limit, early_exit=True, record=True, eps=epsilon)
        exp.log(exp.counters)
        exp.save(trajectorys=exp.without_particles())
    return dict(counters=dict(exp.counters), dir=exp.dir)


# ------------------------------------------------------------------------------ C25 / C16
def _ww_trainer(epsilon=1e-4):
    return N.TrainingNeuralNetworkDecorator(N.WeightwiseNeuralNetwork(2, 2)).with_keras_params(
        activation="linear").with_params(epsilon=epsilon)


def soup_trajectorys(size=20, life=100, train=30, mode="auto", device=None, root="experiments", seed=None):
    """20-particle self-training soup with respawn, trajectories recorded
    (code/setups/soup_trajectorys.py)."""
    if seed is not None:
        _rng.set_seed(seed)
    with SoupExperiment("soup", root=root) as exp:
        soup = Soup(size, _ww_trainer, mode=mode, device=device).with_params(
            remove_divergent=True, remove_zero=True, train=train, learn_from_rate=-1)
        soup.seed()
        soup.evolve(life)
        census = soup.count()
        exp.log(census)
        exp.save(soup=soup.without_particles())
    return dict(census=census, dir=exp.dir, soup=soup)


def soup_demo(size=100, life=100, train=20, mode="auto", device=None, root="experiments", seed=None):
    """The active demo of code/soup.py:127-147."""
    if seed is not None:
        _rng.set_seed(seed)
    with SoupExperiment("soup", root=root) as exp:
        soup = Soup(size, _ww_trainer, mode=mode, device=device).with_params(
            remove_divergent=True, remove_zero=True, train=train)
        soup.seed()
        soup.evolve(life)
        census = soup.count()
        exp.log(census)
        exp.save(soup=soup.without_particles())
    return dict(census=census, dir=exp.dir)


# ------------------------------------------------------------------------------ C10
def network_demo(trials=100, step_limit=100, train_runs=1000, device=None, seed=None, root="experiments"):
    """code/network.py:629-726 active blocks: 100-trial FixpointExperiments for the
    Weightwise, Aggregating and FFT nets, then a 1000-epoch self-train run checked every
    100 epochs."""
    device = device or default_device()
    out = {}
    for k, spec in enumerate((WW, AGG, FFT)):
        with FixpointExperiment(root=root) as exp:
            pop = Population(spec, trials, device=device, seed=_seed(seed) + k)
            exp.run_population(pop, step_limit, early_exit=True, record=True)
            exp.log(exp.counters)
        out[spec.kind] = dict(exp.counters)
    with FixpointExperiment(root=root) as exp:
        # reference :670-680: ONE net trains one epoch per run_id; every 100 epochs run_net
        # self-attacks that same net in place (until fixpoint / divergence, epsilon 1e-4)
        # and training then continues from the self-attacked weights
        pop = Population(WW, 1, device=device, seed=_seed(seed) + 7)
        for run_id in range(0, train_runs + 1, 100):
            pop.train(100 if run_id else 1)
            exp.run_population(pop, step_limit, early_exit=True, eps=1e-4)
        exp.log(exp.counters)
    out["self_train"] = dict(exp.counters)
    return out


REGISTRY = {
    "applying_fixpoints": applying_fixpoints,
    "training_fixpoints": training_fixpoints,
    "fixpoint_density": fixpoint_density,
    "known_fixpoint_variation": known_fixpoint_variation,
    "learn_from_soup": learn_from_soup,
    "mixed_self_fixpoints": mixed_self_fixpoints,
    "mixed_soup": mixed_soup,
    "network_trajectorys": network_trajectorys,
    "soup_trajectorys": soup_trajectorys,
    "soup_demo": soup_demo,
    "network_demo": network_demo,
}
