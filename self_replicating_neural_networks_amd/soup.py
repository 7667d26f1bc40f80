"""Soup: a population of particles that attack, learn from and self-train each other
(reference code/soup.py:10-108), with two execution modes.

* ``mode="sequential"`` — the reference algorithm exactly: particles are processed in
  index order and in place within a generation, each particle a network
  facade on the host; decisions from a seeded ``random.Random`` stream (``prng``).
  Meant for the reference's small soups (10-100 particles).
* ``mode="native"`` — the sequential algorithm on a weight table in one native call per
  ``evolve`` (``seq_soup.SequentialSoupEngine``, any size; slot-keyed Philox streams instead
  of the process-wide ``prng``; trajectory states recorded like the other modes).
* ``mode="ordered"`` — the sequential algorithm on a device weight table
  (``SoupEngine(order="sequential")``): every generation's dependency DAG is scheduled by
  level, bitwise the serial loop of ``native`` (csrc/srnn_ordered.h), any size, single rank,
  the lane-template shapes.
* ``mode="device"`` — the SYNCHRONOUS (Jacobi) generation (``SoupEngine``): every read of a
  generation comes from the generation-start weights, so a particle attacked after its own
  turn is trained before the census instead of ending the generation untrained; optionally
  sharded over the ranks of a process group.  Its statistics differ measurably from the
  reference order at large sizes (tests/test_ordered_soup.py); choose it explicitly.

``mode="auto"`` keeps the reference order: ``sequential`` for ``size <= 100``, ``ordered``
above (``native`` for shapes without a device ordered generation).  A soup sharded over a
process group (``dist``) has no reference-order generation: ``auto`` refuses it, pass
``mode="device"`` to ask for the synchronous one.
"""
from __future__ import annotations

import copy
from typing import Dict, Optional

import numpy as np
import torch

from .io.refpickle import SoupRecord
from .models.network import ParticleDecorator, inner_net, net_spec
from .oracle.core import CLASS_NAMES
from .soup_engine import ACTION_NAMES, RESPAWN_NAMES, SoupEngine
from .utils import rng as _rng


def prng():
    """Reference ``soup.prng`` (code/soup.py:6-7) on the framework's seeded stream."""
    return _rng.prng()


class Soup(object):

    def __init__(self, size, generator, mode: str = "auto", device=None, seed: Optional[int] = None,
                 dist=None, record: bool = True, **kwargs):
        self.size = size
        self.generator = generator
        self.particles = []
        self.historical_particles = {}
        self.params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, learn_from_severity=1)
        self.params.update(kwargs)
        self.time = 0
        if mode == "auto":
            if dist is not None:
                raise ValueError("Soup(mode='auto') keeps the reference's sequential order, which has no sharded "
                                 "form; pass mode='device' for the synchronous (Jacobi) sharded soup")
            mode = "sequential" if size <= 100 else "ordered"
        if mode not in ("sequential", "native", "ordered", "device"):
            raise ValueError("mode must be 'sequential', 'native', 'ordered', 'device' or 'auto'")
        if mode in ("native", "ordered") and dist is not None:
            raise ValueError("sequential-order soups are single-process (their order is serial)")
        self.mode = mode
        self.device = device
        self.seed_value = seed
        self.dist = dist
        self.record = record
        self.engine: Optional[SoupEngine] = None

    # ------------------------------------------------------------------ reference API
    def __copy__(self):
        c = Soup.__new__(Soup)
        c.__dict__ = {k: v for k, v in self.__dict__.items() if k not in ("particles", "historical_particles")}
        return c

    def without_particles(self):
        c = copy.copy(self)
        c.historical_particles = {k: (v.states if hasattr(v, "states") else v)
                                  for k, v in self.historical_particles.items()}
        return c

    def __ref_record__(self):
        """Reference schema of a pickled soup."""
        spec = None
        try:
            spec = self._spec()
        except Exception:  # pragma: no cover
            pass
        gen = {"arch": spec, "params": dict(self.params)} if spec is not None else repr(self.generator)
        hp = {k: (v.states if hasattr(v, "states") else v) for k, v in self.historical_particles.items()}
        return SoupRecord(size=self.size, generator=gen, params=dict(self.params), time=self.time,
                          historical_particles=hp)

    def with_params(self, **kwargs):
        self.params.update(kwargs)
        if self.engine is not None:
            self.engine.params.update(kwargs)
        return self

    def generate_particle(self):
        p = ParticleDecorator(self.generator())
        self.historical_particles[p.get_uid()] = p
        return p

    def get_particle(self, uid, otherwise=None):
        return self.historical_particles.get(uid, otherwise)

    def seed(self):
        if self.mode == "sequential":
            self.particles = [self.generate_particle() for _ in range(self.size)]
        else:
            self._seed_device()
        return self

    def evolve(self, iterations=1):
        if self.mode == "sequential":
            for _ in range(iterations):
                self._evolve_sequential()
        else:
            if self.engine is None:
                self._seed_device()
            shared_counter = self.dist is None or self.dist.world <= 1
            if shared_counter:
                # networks / soups created since the last evolve took uids from the process-wide
                # counter (reference S13): newborns continue after them, never reuse them
                self.engine.next_uid.clamp_(min=ParticleDecorator.next_uid)
            if self.mode == "native":
                self.engine.evolve(iterations, record=self.record)
                self.time += iterations
            else:
                for _ in range(iterations):
                    self.time += 1
                    self.engine.evolve(1, record=self.record)
            if shared_counter:
                ParticleDecorator.next_uid = max(ParticleDecorator.next_uid, int(self.engine.next_uid[0]))
            self._refresh_views()
        return self

    def count(self):
        if self.mode in ("device", "native", "ordered"):
            if self.engine is None:
                self._seed_device()
            return self.engine.count()
        counters = dict(divergent=0, fix_zero=0, fix_other=0, fix_sec=0, other=0)
        for p in self.particles:
            if p.is_diverged():
                counters["divergent"] += 1
            elif p.is_fixpoint():
                if p.is_zero():
                    counters["fix_zero"] += 1
                else:
                    counters["fix_other"] += 1
            elif p.is_fixpoint(2):
                counters["fix_sec"] += 1
            else:
                counters["other"] += 1
        return counters

    def print_all(self):
        for p in self.particles:
            p.print_weights()
            print(p.is_fixpoint())

    # ------------------------------------------------------------------ sequential (exact)
    def _evolve_sequential(self):
        self.time += 1
        for pid, particle in enumerate(self.particles):
            description = {"time": self.time}
            if prng() < self.params.get("attacking_rate"):
                other = self.particles[int(prng() * len(self.particles))]
                particle.attack(other)
                description["action"] = "attacking"
                description["counterpart"] = other.get_uid()
            if prng() < self.params.get("learn_from_rate"):
                other = self.particles[int(prng() * len(self.particles))]
                for _ in range(self.params.get("learn_from_severity", 1)):
                    particle.learn_from(other)
                description["action"] = "learn_from"
                description["counterpart"] = other.get_uid()
            for _ in range(self.params.get("train", 0)):
                particle.compiled()
                loss = particle.train(store_states=False)
                description["fitted"] = self.params.get("train", 0)
                description["loss"] = loss
                description["action"] = "train_self"
                description["counterpart"] = None
            if self.params.get("remove_divergent") and particle.is_diverged():
                new = self.generate_particle()
                self.particles[pid] = new
                description["action"] = "divergent_dead"
                description["counterpart"] = new.get_uid()
            if self.params.get("remove_zero") and particle.is_zero():
                new = self.generate_particle()
                self.particles[pid] = new
                description["action"] = "zweo_dead"
                description["counterpart"] = new.get_uid()
            particle.save_state(**description)

    # ------------------------------------------------------------------ device mode
    def _spec(self):
        return net_spec(self._probe())

    def _probe(self):
        if not hasattr(self, "_probe_net") or self._probe_net is None:
            self._probe_net = self.generator()
        return self._probe_net

    def _seed_device(self):
        probe = self._probe()
        spec = net_spec(probe)
        inner = inner_net(probe)
        params = dict(self.params)
        params.setdefault("epsilon", inner.get_params().get("epsilon", 1e-14))
        lr = probe._lr() if hasattr(probe, "_lr") else 0.01
        if self.mode == "native":
            from .seq_soup import SequentialSoupEngine
            seed = self.seed_value if self.seed_value is not None else _rng.get_seed() ^ ParticleDecorator.next_uid
            self.engine = SequentialSoupEngine(spec, self.size, params, seed=seed, lr=lr)
            base = ParticleDecorator.next_uid
            self.engine.uid.add_(base)
            self.engine.next_uid.add_(base)
            ParticleDecorator.next_uid += self.size
            self._uid_offset = base
            if self.record:
                self.engine.recorder = StateRecorder(spec.class_name)
                self.engine.recorder.record_init(self.engine, time=0)
            self._refresh_views()
            return
        device = self.device
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        seed = self.seed_value if self.seed_value is not None else _rng.get_seed() ^ ParticleDecorator.next_uid
        if self.mode == "ordered":
            from .ops import _lib
            if not _lib.supports(spec, _lib.OP_SOUP_ORDERED, torch.device(device).type != "cpu"):
                # no level-scheduled generation for this shape: the same order on the host loop
                self.mode = "native"
                return self._seed_device()
            self.engine = SoupEngine(spec, self.size, params, device=device, seed=seed, lr=lr, order="sequential")
        else:
            self.engine = SoupEngine(spec, self.size, params, device=device, seed=seed, lr=lr, dist=self.dist)
        # global uids continue the process-wide particle counter (reference S13)
        base = ParticleDecorator.next_uid
        self.engine.uid.add_(base)
        self.engine.next_uid.add_(base)
        ParticleDecorator.next_uid += self.size
        self._uid_offset = base
        if self.record:
            self.engine.recorder = StateRecorder(spec.class_name)
            self.engine.recorder.record_init(self.engine, time=0)
        self._refresh_views()

    def _refresh_views(self):
        eng = self.engine
        rec = eng.recorder
        uids = eng.uid.cpu().tolist()
        self.particles = [ParticleView(self, slot, uid, rec.states_of(uid) if rec else None)
                          for slot, uid in enumerate(uids)]
        if rec is not None:
            for uid in rec.states:
                if uid not in self.historical_particles:
                    self.historical_particles[uid] = _HistoricalParticle(uid, rec.states[uid])
        for v in self.particles:
            self.historical_particles[v.get_uid()] = v


class StateRecorder:
    """Host-side trajectory recorder of a SoupEngine (reference state schema, S14)."""

    def __init__(self, class_name):
        self.class_name = class_name
        self.states: Dict[int, list] = {}
        self._snap = None

    def states_of(self, uid):
        return self.states.setdefault(uid, [])

    def record_init(self, eng, time=0):
        W = eng.local_rows()[:, : eng.spec.P].cpu().numpy()
        for uid, w in zip(eng.uid.cpu().tolist(), W):
            if np.all(np.isfinite(w)):
                self.states_of(uid).append({"class": self.class_name, "weights": w.copy(), "time": time,
                                            "action": "init", "counterpart": None})

    def on_evolved(self, eng, rows=None, old_uid=None, ordered: bool = False):
        """Snapshot of a generation's per-particle records.  ``rows``: the pre-respawn states
        (default: the engine's output table before its respawn pass); ``ordered``: a
        reference-order generation, whose counterparts are read as of each particle's turn."""
        uid_slots = (old_uid if old_uid is not None else eng.uid).clone()
        rows = eng.rows_out if rows is None else rows
        self._snap = (rows[:, : eng.spec.P].clone(), eng.action.clone(), eng.counterpart.clone(),
                      eng.loss.clone(), eng.respawn.clone(), uid_slots)
        self._ordered = ordered

    def on_sequential_generation(self, eng, time, old_uid):
        """After one generation of a ``SequentialSoupEngine`` (its counterparts are uids)."""
        self._snap = (eng.rows_out[:, : eng.spec.P], eng.action, eng.counterpart, eng.loss, eng.respawn, old_uid)
        self.on_generation_end(eng, time, None)

    def on_generation_end(self, eng, time, uid_of_slot):
        """``uid_of_slot`` maps counterpart slots to uids (None: counterparts are uids)."""
        W, act, cp, loss, resp, old_uid = (t.cpu().numpy() for t in self._snap)
        new_uid = eng.uid.cpu().numpy()
        ordered = getattr(self, "_ordered", False)
        self._ordered = False
        train = int(eng.params.get("train", 0))
        newW = eng.local_rows()[:, : eng.spec.P].cpu().numpy()
        for j in range(W.shape[0]):
            d = {"time": time}
            a = ACTION_NAMES[int(act[j])]
            if a is not None:
                d["action"] = a
                if a == "train_self":
                    d["counterpart"] = None
                elif uid_of_slot is None:
                    d["counterpart"] = int(cp[j])
                elif ordered and int(cp[j]) < j and resp[int(cp[j])]:
                    # the counterpart's turn came first and replaced it: the newborn (reference S11/S12)
                    d["counterpart"] = int(new_uid[int(cp[j])])
                else:
                    d["counterpart"] = int(uid_of_slot[int(cp[j])])
            if a == "train_self":
                d["fitted"] = train
                d["loss"] = float(loss[j])
            if resp[j]:
                d["action"] = RESPAWN_NAMES[int(resp[j])]
                d["counterpart"] = int(new_uid[j])
                # the newborn's init state (reference ParticleDecorator.__init__)
                if np.all(np.isfinite(newW[j])):
                    self.states_of(int(new_uid[j])).append({"class": self.class_name, "weights": newW[j].copy(),
                                                            "time": 0, "action": "init", "counterpart": None})
            if np.all(np.isfinite(W[j])):
                st = {"class": self.class_name, "weights": W[j].copy()}
                st.update(d)
                self.states_of(int(old_uid[j])).append(st)
        self._snap = None


class _HistoricalParticle:
    """A dead particle: uid + recorded states."""

    def __init__(self, uid, states):
        self.uid = uid
        self.states = states

    def get_uid(self):
        return self.uid

    def get_states(self):
        return self.states


class ParticleView:
    """A live particle of a device soup: row ``slot`` of the engine's table."""

    def __init__(self, soup: Soup, slot: int, uid: int, states):
        self._soup = soup
        self.slot = slot
        self.uid = uid
        self.states = states if states is not None else []

    def get_uid(self):
        return self.uid

    def get_states(self):
        return self.states

    def get_weights_flat(self):
        eng = self._soup.engine
        return eng.local_rows()[self.slot, : eng.spec.P].cpu().numpy()

    def get_weights(self):
        return self._soup.engine.spec.unflatten(self.get_weights_flat())

    def _facade(self):
        net = self._soup.generator()
        inner_net(net).set_weights(self.get_weights_flat())
        return net

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._facade(), name)
