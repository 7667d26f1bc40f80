"""Exact sequential soups at any size on the native engine.

The reference evolves a soup particle by particle, in place and in index order
(``Soup.evolve``, reference code/soup.py:51-87): particle j sees
the attacks, learn_from and self-training of every earlier particle of the same
generation.  ``Soup(mode="sequential")`` reproduces that with one network facade per
particle (host loop, meant for the reference's 10-100 particle soups).  This engine runs
the same algorithm on a weight table in ONE native call per ``evolve`` (OP_SOUP_SEQ,
csrc/srnn_kernels.h ``soup_seq``): the update order is serial by definition, so a CPU core
is its natural home (a single GPU lane runs the same chain slower), and 1000-particle
reference soups take milliseconds per generation instead of a per-object Python loop.

Random streams are the synchronous engine's: decisions keyed by (slot, generation), SGD
shuffles by (slot, generation), newborn init by (generation, slot); newborn uids are
numbered in index order.  ``SoupEngine`` is the synchronous (Jacobi) device counterpart;
population statistics of the two agree (tests/test_seq_soup.py).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .arch import ArchSpec
from .ops import _lib
from .ops import kernels as K
from .population import counts_dict


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class SequentialSoupEngine:
    def __init__(self, spec: ArchSpec, n: int, params: Optional[dict] = None, seed: int = 0, lr: float = 0.01,
                 shuffle: bool = True, dtype: torch.dtype = torch.float32, weights: Optional[torch.Tensor] = None,
                 device="cpu"):
        """``device="cuda"`` runs the same serial loop as one GPU lane (``k_soup_seq``; measured
        slower than the host loop -- it exists for tables that live on the device)."""
        self.spec, self.n = spec, int(n)
        self.device = torch.device(device)
        self.params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, learn_from_severity=1)
        self.params.update(params or {})
        self.seed, self.lr, self.shuffle = int(seed), float(lr), bool(shuffle)
        self.dtype_code = K.dtype_code(dtype)
        if not _lib.supports(spec, _lib.OP_SOUP_SEQ, self.device.type != "cpu", self.dtype_code):
            raise NotImplementedError(
                f"no native sequential soup loop for {spec} on {self.device.type}: the device loop exists for "
                "the instantiated lane-per-particle shapes only; use device='cpu' (any shape) or the "
                "synchronous SoupEngine")
        self.W = torch.zeros((self.n, spec.PP), dtype=dtype)
        self.uid = torch.arange(self.n, dtype=torch.int64)
        if weights is not None:
            self.W[:, : spec.P] = torch.as_tensor(weights, dtype=dtype)[:, : spec.P]
        else:
            K.init_rows(spec, self.W, self.uid, self.seed)
        self.next_uid = torch.tensor([self.n], dtype=torch.int64)
        self.gen = torch.ones(1, dtype=torch.int32)
        self.time = 0
        self.action = torch.zeros(self.n, dtype=torch.int8)
        self.counterpart = torch.full((self.n,), -1, dtype=torch.int64)
        self.loss = torch.zeros(self.n, dtype=torch.float32)
        self.respawn = torch.zeros(self.n, dtype=torch.int8)
        if self.device.type != "cpu":
            for k in ("W", "uid", "next_uid", "gen", "action", "counterpart", "loss", "respawn"):
                setattr(self, k, getattr(self, k).to(self.device))
        self.recorder = None  # StateRecorder (Soup record=True): trajectory states per generation

    def local_rows(self) -> torch.Tensor:
        return self.W

    @property
    def eps(self) -> float:
        return float(self.params.get("epsilon") or 1e-14)

    def _flags(self) -> int:
        f = _lib.FLAG_SHUFFLE if self.shuffle else 0
        if self.params.get("remove_divergent"):
            f |= _lib.FLAG_REMOVE_DIVERGENT
        if self.params.get("remove_zero"):
            f |= _lib.FLAG_REMOVE_ZERO
        return f

    def evolve(self, iterations: int = 1, record: bool = False) -> "SequentialSoupEngine":
        """``iterations`` sequential generations in one native call (action / counterpart /
        loss / respawn describe the last one).  With ``record`` (and a ``recorder``) one call
        per generation that also keeps every particle's pre-respawn state (``rows_out``) and
        the counterparts' uids at the time of each action, for the reference's trajectory
        states (code/soup.py:87)."""
        if iterations <= 0:
            return self
        if record and self.recorder is not None:
            for _ in range(int(iterations)):
                old_uid = self.uid.clone()
                self._run(1, rows_out=self.rows_out)
                self.recorder.on_sequential_generation(self, self.time, old_uid)
            return self
        self._run(int(iterations))
        return self

    @property
    def rows_out(self) -> torch.Tensor:
        if getattr(self, "_rows_out", None) is None:
            self._rows_out = torch.zeros_like(self.W)
        return self._rows_out

    def _run(self, iterations: int, rows_out: Optional[torch.Tensor] = None):
        a = _lib.SrnnArgs()
        a.n, a.n_total, a.lo = self.n, self.n, 0
        a.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        a.lr, a.eps = self.lr, self.eps
        a.attacking_rate = float(self.params.get("attacking_rate", 0.1))
        a.learn_from_rate = float(self.params.get("learn_from_rate", 0.1))
        a.epochs = int(self.params.get("train", 0))
        a.severity = int(self.params.get("learn_from_severity", 1))
        a.segment = int(self.params.get("segment", 0) or 0)
        a.flags = self._flags()
        a.steps = int(iterations)
        a.W, a.W2 = _p(self.W), _p(rows_out)
        a.gen_ptr = _p(self.gen)
        a.uid_base, a.uid_out = _p(self.next_uid), _p(self.uid)
        a.action, a.counterpart, a.loss, a.respawn = _p(self.action), _p(self.counterpart), _p(self.loss), _p(self.respawn)
        if self.device.type != "cpu":
            a.dev = 1
            a.stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.run(_lib.OP_SOUP_SEQ, self.spec, a, dtype=self.dtype_code)
        self.time += int(iterations)

    def count(self, with_sec: bool = True) -> Dict[str, int]:
        """Census (reference Soup.count, code/soup.py:89-103)."""
        _, counts = K.classify(self.spec, self.W, self.eps, with_sec=with_sec, uid=self.uid, seed=self.seed)
        return counts_dict(counts)

    def weights(self) -> torch.Tensor:
        return self.W[:, : self.spec.P].float().clone()
