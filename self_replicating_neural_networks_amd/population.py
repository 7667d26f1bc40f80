"""Device-resident particle populations.

``Population`` is the unit of computation of the framework: a weight table
``W[N, spec.PP]`` (one particle per row, Keras flat order) plus a uid per row.  The table
is fp32 by default; ``dtype=torch.bfloat16`` / ``torch.float16`` stores every weight state
in 16 bits (half the HBM per particle, arithmetic still fp32 -- SURVEY §7.7).
Reference-style objects (``WeightwiseNeuralNetwork``, ``ParticleDecorator``, ``Soup``) are
views of rows of a population; the batched methods here replace the reference's
per-object Python loops (``code/experiment.py:70-91``, ``code/setups/*.py`` trial loops).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from .arch import ArchSpec
from .ops import kernels as K
from .oracle.core import CLASS_NAMES


def counts_dict(counts) -> Dict[str, int]:
    c = counts.tolist() if hasattr(counts, "tolist") else list(counts)
    return {name: int(c[i]) for i, name in enumerate(CLASS_NAMES)}


class Population:
    """N particles of one architecture on one device."""

    def __init__(self, spec: ArchSpec, n: int, device="cpu", seed: int = 0, uid_start: int = 0,
                 weights: Optional[torch.Tensor] = None, lr: float = 0.01, dtype: torch.dtype = torch.float32,
                 init: bool = True):
        self.spec = spec
        self.device = torch.device(device)
        self.seed = int(seed)
        self.lr = float(lr)
        self.ctr = 0  # op counter: keys the per-particle random streams of shuffles etc.
        self.uid = torch.arange(uid_start, uid_start + n, dtype=torch.int64, device=self.device)
        K.dtype_code(dtype)
        self.W = torch.zeros((n, spec.PP), dtype=dtype, device=self.device)
        if weights is not None:
            self.set_weights(weights)
        elif init:
            K.init_rows(spec, self.W, self.uid, self.seed)

    # -------------------------------------------------------------- helpers
    def __len__(self):
        return self.W.shape[0]

    @property
    def n(self):
        return self.W.shape[0]

    def _next_ctr(self, k=1):
        c = self.ctr
        self.ctr += k
        return c

    def weights(self) -> torch.Tensor:
        """[N, P] view without the row padding."""
        return self.W[:, : self.spec.P]

    def set_weights(self, w):
        w = torch.as_tensor(np.asarray(w, dtype=np.float32) if not torch.is_tensor(w) else w, dtype=torch.float32)
        if w.dim() == 1:
            w = w[None]
        if w.shape[0] != self.n or w.shape[1] not in (self.spec.P, self.spec.PP):
            raise ValueError(f"weights must be [{self.n}, {self.spec.P}], got {tuple(w.shape)}")
        self.W.zero_()
        self.W[:, : w.shape[1]] = w.to(self.device, self.W.dtype)
        if w.shape[1] == self.spec.PP:
            self.W[:, self.spec.P:] = 0

    # -------------------------------------------------------------- dynamics
    def self_apply(self, steps: int = 1) -> "Population":
        """``self_attack`` for every particle, ``steps`` times (no early exit)."""
        K.run_fixpoint(self.spec, self.W, steps, 1e-14, early_exit=False, with_sec=False, uid=self.uid,
                       seed=self.seed, ctr=self._next_ctr(steps))
        return self

    def attack(self, attackers: torch.Tensor, victims: torch.Tensor) -> "Population":
        """victims[i] <- f_{attackers[i]}(victims[i]), all attackers using pre-call weights;
        repeated victims are applied in order (sequential per victim)."""
        attackers = attackers.to(self.device, torch.int64).contiguous()
        victims = victims.to(self.device, torch.int64).contiguous()
        m = victims.numel()
        if m == 0:
            return self
        tmp = torch.cat([self.W, self.W])  # rows [0,N): attacker snapshot, [N,2N): evolving victims
        uid2 = torch.cat([self.uid, self.uid]).contiguous()
        if torch.unique(victims).numel() == m:
            K.apply(self.spec, tmp, self.W, idx_f=attackers, idx_t=(victims + self.n).contiguous(), idx_o=victims,
                    n=m, uid=uid2, seed=self.seed, ctr=self._next_ctr())
            return self
        # several attacks on one victim, applied in call order: round k applies the k-th
        # attack of every victim (distinct victims per round, one batched launch each, in
        # place on the victim half of tmp) -- rounds = the largest multiplicity, not m
        order = torch.argsort(victims, stable=True)
        vs, at = victims[order], attackers[order]
        pos = torch.arange(m, device=self.device)
        new = torch.ones(m, dtype=torch.bool, device=self.device)
        new[1:] = vs[1:] != vs[:-1]
        rank = pos - torch.cummax(torch.where(new, pos, torch.zeros_like(pos)), 0).values
        for k in range(int(rank.max()) + 1):
            sel = rank == k
            v = (vs[sel] + self.n).contiguous()
            K.apply(self.spec, tmp, tmp, idx_f=at[sel].contiguous(), idx_t=v, idx_o=v, n=v.numel(), uid=uid2,
                    seed=self.seed, ctr=self._next_ctr())
        self.W.copy_(tmp[self.n:])
        return self

    def train(self, epochs: int = 1, shuffle: bool = True) -> torch.Tensor:
        return K.train(self.spec, self.W, epochs, self.lr, shuffle, uid=self.uid, seed=self.seed,
                       ctr=self._next_ctr(epochs))

    def learn_from(self, teachers: torch.Tensor, idx_t=None, epochs: int = 1, shuffle: bool = True) -> torch.Tensor:
        return K.learn_from(self.spec, self.W, teachers, idx_t, epochs, self.lr, shuffle, uid=self.uid,
                            seed=self.seed, ctr=self._next_ctr(epochs))

    def run_fixpoint(self, steps: int = 100, eps: float = 1e-4, early_exit: bool = True, record: bool = False,
                     with_sec: bool = True):
        return K.run_fixpoint(self.spec, self.W, steps, eps, early_exit, with_sec, record, uid=self.uid,
                              seed=self.seed, ctr=self._next_ctr(steps + 2))

    def classify(self, eps: float = 1e-4, with_sec: bool = True):
        return K.classify(self.spec, self.W, eps, with_sec, uid=self.uid, seed=self.seed, ctr=self._next_ctr())

    def count(self, eps: float = 1e-4, with_sec: bool = True) -> Dict[str, int]:
        _, counts = self.classify(eps, with_sec)
        return counts_dict(counts.cpu())

    # -------------------------------------------------------------- aggregating nets
    def aggregates(self, W: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Chunk aggregates [N, A] of aggregating-net rows (reference collect_weights +
        aggregate_average / aggregate_max, code/network.py:294-306, 389-410): chunks of
        P // A weights, the last one takes the leftovers; means summed in float64."""
        spec = self.spec
        if spec.kind != "aggregating":
            raise TypeError("aggregates are defined for aggregating nets")
        W = (self.W if W is None else W)[:, : spec.P].float()
        A, cs = spec.aggregates, spec.P // spec.aggregates
        cols = []
        for k in range(A):
            b, e = k * cs, (spec.P if k == A - 1 else (k + 1) * cs)
            ch = W[:, b:e]
            if spec.aggregator == "mean":
                cols.append((ch.double().sum(1) / (e - b)).float())
            elif spec.aggregator == "max":
                cols.append(ch.max(1).values)
            else:  # reference quirk: `weight > max and weight or max` never takes a zero
                nz = torch.where(ch != 0, ch, torch.full_like(ch, float("-inf"))).max(1).values
                cols.append(torch.maximum(ch[:, 0], nz))
        return torch.stack(cols, 1)

    def is_fixpoint_after_aggregation(self, degree: int = 1, eps: float = 1e-4):
        """Batched ``is_fixpoint_after_aggregation`` (reference code/network.py:419-439): each
        particle's net is applied ``degree`` times to (its own, then the resulting) weights
        with the population's apply kernels; a particle is a fixpoint when the result is
        finite and every chunk aggregate moved by less than ``eps``.  Returns (bool[N],
        new aggregates [N, A]); diverged particles are False (the reference returns a bare
        False for them)."""
        if degree < 1:
            raise ValueError("degree must be >= 1")
        n = self.n
        old = self.aggregates()
        tmp = torch.cat([self.W, self.W])  # rows [0, n): the nets, [n, 2n): evolving targets
        uid2 = torch.cat([self.uid, self.uid]).contiguous()
        idx_f = torch.arange(n, dtype=torch.int64, device=self.device)
        idx_t = (idx_f + n).contiguous()
        for _ in range(degree):
            out = torch.zeros_like(self.W)
            K.apply(self.spec, tmp, out, idx_f=idx_f, idx_t=idx_t, n=n, uid=uid2, seed=self.seed, ctr=self._next_ctr())
            tmp[n:] = out
        new = tmp[n:]
        finite = torch.isfinite(new[:, : self.spec.P].float()).all(1)
        new_aggs = self.aggregates(new)
        fix = finite & ((new_aggs - old).abs() < eps).all(1)
        return fix, new_aggs

    def inject_nan(self, rows) -> "Population":
        """Fault injection: NaN into the first weight of ``rows``."""
        rows = torch.as_tensor(rows, dtype=torch.int64, device=self.W.device)
        self.W[rows, 0] = float("nan")
        return self

    def perturb(self, e: float) -> "Population":
        K.perturb(self.spec, self.W, e, uid=self.uid, seed=self.seed, ctr=self._next_ctr())
        return self

    def vary_run(self, steps: int, eps: float):
        return K.vary_run(self.spec, self.W, steps, eps, uid=self.uid, seed=self.seed, ctr=self._next_ctr(2 * steps))
