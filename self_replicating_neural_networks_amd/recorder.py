"""Sampled trajectory recording for large soups.

The reference keeps a full Python list of state dicts per particle and appends one every
generation (``ParticleDecorator.save_state``, code/network.py:185-198) -- fine for 20
particles, impossible for 10^8.  :class:`TrajectoryRecorder` snapshots a *sampled* set of
rows every ``every`` generations:

* the rows are gathered on the device into a staging buffer (one gather kernel on the
  compute stream), then copied to a pinned host ring buffer on a side stream, so the copy
  overlaps the next generation (double-buffered staging, event-ordered);
* the ring keeps the last ``capacity`` snapshots (weights, uid, generation);
* :meth:`states` converts them to the reference's state schema (``{uid: [{'class',
  'weights', 'time'}]}``, NaN/Inf states dropped as in code/network.py:187-188) and
  :meth:`save` writes a compressed ``.npz`` per rank.

Policies: ``full`` (every local row), ``subset`` (``subset`` evenly spaced global slots;
each rank records the ones it owns), ``none``.  Works with hipGraph replays (snapshots
are taken between generations).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import RecorderConfig


class TrajectoryRecorder:
    def __init__(self, eng, cfg: RecorderConfig):
        cfg.validate()
        self.cfg = cfg
        self.P = eng.spec.P
        self.class_name = eng.spec.class_name
        dev = eng.device
        if cfg.policy == "full":
            local = torch.arange(eng.n, dtype=torch.int64)
        elif cfg.policy == "subset":
            k = min(cfg.subset, eng.n_total)
            slots = np.unique(np.linspace(0, eng.n_total - 1, k).round().astype(np.int64))
            slots = slots[(slots >= eng.lo) & (slots < eng.hi)] - eng.lo
            local = torch.from_numpy(slots)
        else:
            local = torch.zeros(0, dtype=torch.int64)
        self.rows = local.to(dev)
        self.slots = (local + eng.lo).numpy()
        S = self.rows.numel()
        self.S = S
        pin = dev.type == "cuda"
        self.host_w = torch.empty((cfg.capacity, S, self.P), dtype=torch.float32, pin_memory=pin)
        self.host_uid = torch.empty((cfg.capacity, S), dtype=torch.int64, pin_memory=pin)
        self.host_gen = np.full(cfg.capacity, -1, dtype=np.int64)
        self.count = 0
        self.cuda = dev.type == "cuda"
        if self.cuda:
            self.stream = torch.cuda.Stream(dev)
            self.stage_w = [torch.empty((S, self.P), dtype=torch.float32, device=dev) for _ in range(2)]
            self.stage_uid = [torch.empty(S, dtype=torch.int64, device=dev) for _ in range(2)]
            self.done = [None, None]

    def due(self, generation: int) -> bool:
        return self.cfg.policy != "none" and self.S > 0 and generation % self.cfg.every == 0

    def snapshot(self, eng, generation: int):
        slot = self.count % self.cfg.capacity
        if not self.cuda:
            self.host_w[slot] = eng.local_rows()[self.rows, : self.P].float()
            self.host_uid[slot] = eng.uid[self.rows]
        else:
            b = self.count % 2
            if self.done[b] is not None:
                self.done[b].synchronize()  # staging buffer b's previous copy has landed
            cur = torch.cuda.current_stream(eng.device)
            torch.index_select(eng.local_rows()[:, : self.P], 0, self.rows, out=self.stage_w[b]) \
                if eng.local_rows().dtype == torch.float32 else \
                self.stage_w[b].copy_(eng.local_rows()[self.rows, : self.P].float())
            torch.index_select(eng.uid, 0, self.rows, out=self.stage_uid[b])
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                self.host_w[slot].copy_(self.stage_w[b], non_blocking=True)
                self.host_uid[slot].copy_(self.stage_uid[b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.done[b] = ev
        self.host_gen[slot] = generation
        self.count += 1

    def maybe_record(self, eng, generation: int):
        if self.due(generation):
            self.snapshot(eng, generation)

    def _sync(self):
        if self.cuda:
            for ev in self.done:
                if ev is not None:
                    ev.synchronize()

    def arrays(self):
        """(generation [T], uid [T, S], weights [T, S, P]) in recording order (last
        ``capacity`` snapshots)."""
        self._sync()
        T = min(self.count, self.cfg.capacity)
        order = [(self.count - T + t) % self.cfg.capacity for t in range(T)]
        return (self.host_gen[order].copy(), self.host_uid[order].numpy().copy(),
                self.host_w[order].numpy().copy())

    def states(self) -> Dict[int, List[dict]]:
        """Reference trajectory schema: {uid: [{'class', 'weights', 'time'}, ...]}."""
        gen, uid, W = self.arrays()
        out: Dict[int, List[dict]] = {}
        for t in range(len(gen)):
            for s in range(self.S):
                w = W[t, s]
                if np.all(np.isfinite(w)):
                    out.setdefault(int(uid[t, s]), []).append(
                        {"class": self.class_name, "weights": w.copy(), "time": int(gen[t])})
        return out

    def save(self, path: str, rank: int = 0) -> str:
        gen, uid, W = self.arrays()
        os.makedirs(path, exist_ok=True)
        f = os.path.join(path, f"trajectory-r{rank:04d}.npz")
        np.savez_compressed(f, generation=gen, uid=uid, weights=W, slots=self.slots)
        return f


def load_trajectory(path: str) -> Dict[str, np.ndarray]:
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
