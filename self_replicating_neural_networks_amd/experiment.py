"""Experiment harness with the reference's directory / log / pickle contract
(reference code/experiment.py:8-120).

``with Experiment(name, ident) as exp:`` creates ``experiments/exp-{name}-{ident}_{t}-{it}``;
``exp.log`` echoes and records messages; ``exp.save(k=v)`` writes ``k.dill``; on exit
``experiment.dill`` (particles replaced by their state lists) and ``log.txt`` are written.
Pickles are written in the reference schema (classes ``experiment.Experiment`` /
``soup.Soup``, numpy arrays, plain dicts) by ``io.refpickle`` — no dill code
objects are produced, and ``from_dill`` reads reference files with a restricted
unpickler that never executes code from the file.

Population-scale extensions: ``FixpointExperiment.run_population`` runs the per-net
``run_net`` loop for a whole population on the device in one kernel.
"""
from __future__ import annotations

import copy
import os
import time
from typing import Dict

import numpy as np
import torch

from .io import refpickle
from .oracle.core import CLASS_NAMES


class Experiment:

    @staticmethod
    def from_dill(path):
        """Load a reference-schema pickle (ours or the reference's) without executing code."""
        return refpickle.load(path)

    def __init__(self, name=None, ident=None, root="experiments"):
        self.experiment_id = "{}_{}".format(ident or "", time.time())
        self.experiment_name = name or "unnamed_experiment"
        self.next_iteration = 0
        self.log_messages = []
        self.historical_particles = {}
        self._root = root

    def __enter__(self):
        self.dir = os.path.join(self._root, "exp-{name}-{id}-{it}".format(
            name=self.experiment_name, id=self.experiment_id, it=self.next_iteration))
        os.makedirs(self.dir)
        print("** created {dir} **".format(dir=self.dir))
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        self.save(experiment=self.without_particles())
        self.save_log()
        self.next_iteration += 1

    def log(self, message, **kwargs):
        self.log_messages.append(message)
        print(message, **kwargs)

    def save_log(self, log_name="log"):
        with open(os.path.join(self.dir, "{name}.txt".format(name=log_name)), "w") as f:
            for m in self.log_messages:
                print(str(m), file=f)

    def __copy__(self):
        # the reference always copies into a base Experiment (code/experiment.py:44-48)
        c = Experiment.__new__(Experiment)
        c.__dict__ = {k: v for k, v in self.__dict__.items() if k not in ("particles", "historical_particles")}
        return c

    def without_particles(self):
        c = copy.copy(self)
        c.historical_particles = {k: (v.states if hasattr(v, "states") else v)
                                  for k, v in self.historical_particles.items()}
        return c

    def save(self, **kwargs):
        for name, value in kwargs.items():
            refpickle.dump(value, os.path.join(self.dir, "{name}.dill".format(name=name)))

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if not k.startswith("_")}


class FixpointExperiment(Experiment):
    """run_net / count of the reference (code/experiment.py:62-91)."""

    def __init__(self, **kwargs):
        kwargs["name"] = self.__class__.__name__ if "name" not in kwargs else kwargs["name"]
        super().__init__(**kwargs)
        self.counters = dict(divergent=0, fix_zero=0, fix_other=0, fix_sec=0, other=0)
        self.interesting_fixpoints = []

    def run_net(self, net, step_limit=100, run_id=0):
        i = 0
        while i < step_limit and not net.is_diverged() and not net.is_fixpoint():
            net.self_attack()
            i += 1
            if run_id:
                net.save_state(time=i)
        self.count(net)

    def count(self, net):
        if net.is_diverged():
            self.counters["divergent"] += 1
        elif net.is_fixpoint():
            if net.is_zero():
                self.counters["fix_zero"] += 1
            else:
                self.counters["fix_other"] += 1
                self.interesting_fixpoints.append(net.get_weights())
        elif net.is_fixpoint(2):
            self.counters["fix_sec"] += 1
        else:
            self.counters["other"] += 1

    # ------------------------------------------------------------------ population scale
    def run_population(self, population, step_limit=100, early_exit=True, record=False, eps=None,
                       collect_fixpoints=True) -> Dict[str, int]:
        """``run_net`` for every particle of a ``Population`` in one device launch;
        counters accumulate like repeated ``run_net`` calls."""
        eps = eps or 1e-4
        cls, nsteps, traj = population.run_fixpoint(step_limit, eps, early_exit=early_exit, record=record)
        c = np.bincount(cls.cpu().numpy().astype(np.int64), minlength=5)
        for i, name in enumerate(CLASS_NAMES):
            self.counters[name] += int(c[i])
        if collect_fixpoints:
            idx = torch.nonzero(cls == 2).flatten()
            for row in population.W[idx, : population.spec.P].cpu().numpy():
                self.interesting_fixpoints.append(population.spec.unflatten(row))
        if record:
            self._record_trajectories(population, traj.cpu().numpy(), nsteps.cpu().numpy())
        return {n: int(c[i]) for i, n in enumerate(CLASS_NAMES)}

    def _record_trajectories(self, population, traj, nsteps):
        cname = population.spec.class_name
        P = population.spec.P
        for r, uid in enumerate(population.uid.cpu().tolist()):
            states = [{"class": cname, "weights": traj[0, r, :P].copy(), "time": 0, "action": "init",
                       "counterpart": None}]
            for s in range(1, int(nsteps[r]) + 1):
                w = traj[s, r, :P]
                if np.all(np.isfinite(w)):
                    states.append({"class": cname, "weights": w.copy(), "time": s})
            self.historical_particles[uid] = states


class MixedFixpointExperiment(FixpointExperiment):
    """Self-attack followed by ``trains_per_application`` self-train epochs per step
    (code/experiment.py:94-109)."""

    def run_net(self, net, trains_per_application=100, step_limit=100, run_id=0):
        i = 0
        while i < step_limit and not net.is_diverged() and not net.is_fixpoint():
            net.self_attack()
            for _ in range(trains_per_application):
                net.compiled().train()
            i += 1
            if run_id:
                net.save_state()
        self.count(net)


class SoupExperiment(Experiment):
    pass


class IdentLearningExperiment(Experiment):

    def __init__(self):
        super().__init__(name=self.__class__.__name__)
