"""Device soup engine: one fused generation pipeline over a sharded population.

Replaces the per-particle Python loop of ``Soup.evolve`` (reference code/soup.py:51-87)
with a *synchronous* (Jacobi) generation, computed for every particle at once:

1. ``decide``  — every rank draws the decisions of every *global* slot from Philox keyed
   by (seed, slot, generation), so pairings are known everywhere without exchanging
   indices; attacks on local victims are counted.
2. ``scan`` + ``fill`` — CSR list of attackers per local victim.
3. ``evolve`` (fused kernel, lane per particle) — received attacks in ascending attacker
   slot order using generation-start attacker weights, then ``learn_from_severity``
   epochs on the teacher's generation-start samples, then ``train`` self-train epochs,
   then divergence / zero respawn flags (reference :77-86).
4. ``scan`` + ``respawn`` — new uids are globally sequential (reference S13): rank r's
   first new uid = next_uid + sum of the respawn counts of ranks < r.
5. all-gather of the new local rows into the global generation-start table of the next
   generation (RCCL over xGMI with ``nccl``; gloo on CPU).
6. optional ``classify`` + all-reduce of the 5-bin class histogram (reference
   code/soup.py:89-103).

Differences from the sequential reference (documented in docs and tested
statistically): particle k does not see the effects of particles < k within the same
generation; every read is from the generation-start table.  ``Soup(mode="sequential")``
provides the exact reference order for small populations.

The per-generation work is graph-capturable (device generation counter, no host syncs),
so ``capture()`` records one generation into a HIP graph that is replayed per evolve().
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .arch import ArchSpec
from .ops import _lib
from .ops import kernels as K
from .parallel.dist import Dist
from .population import counts_dict

ACTION_NAMES = {0: None, 1: "attacking", 2: "learn_from", 3: "train_self"}
RESPAWN_NAMES = {1: "divergent_dead", 2: "zweo_dead"}  # sic, reference code/soup.py:84


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class SoupEngine:
    """Population-sharded soup on one device per rank."""

    def __init__(self, spec: ArchSpec, n_total: int, params: Dict, device="cpu", seed: int = 0,
                 lr: float = 0.01, shuffle: bool = True, dist: Optional[Dist] = None, weights=None):
        self.spec = spec
        self.n_total = int(n_total)
        self.params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, learn_from_severity=1)
        self.params.update(params or {})
        self.device = torch.device(device)
        self.seed = int(seed)
        self.lr = float(lr)
        self.shuffle = bool(shuffle)
        self.dist = dist or Dist()
        self.lo, self.hi = self.dist.shard(self.n_total)
        self.n = self.hi - self.lo
        if self.n_total >= 2 ** 31 - 1:
            raise ValueError("soup slots are int32 on device")
        seg = int(self.params.get("segment", 0) or 0)
        if seg and self.n_total % seg:
            raise ValueError("population size must be a multiple of the sub-soup segment")
        dev, PP = self.device, spec.PP
        i32 = dict(dtype=torch.int32, device=dev)
        if self.dist.enabled:
            # generation-start table of every global row + this rank's output rows
            self.table = torch.zeros((self.n_total, PP), dtype=torch.float32, device=dev)
            self.next_rows = torch.zeros((self.n, PP), dtype=torch.float32, device=dev)
        else:
            # ping-pong pair: generation t reads buf[p], writes buf[1-p]
            self._bufs = [torch.zeros((self.n, PP), dtype=torch.float32, device=dev) for _ in range(2)]
            self._p = 0
        self.uid = torch.arange(self.lo, self.hi, dtype=torch.int64, device=dev)
        self.next_uid = torch.full((1,), self.n_total, dtype=torch.int64, device=dev)
        self.uid_base = torch.zeros(1, dtype=torch.int64, device=dev)
        self.gen_dev = torch.ones(1, dtype=torch.int32, device=dev)  # generation about to run
        self.time = 0
        self.head = torch.full((self.n,), -1, **i32)       # first attacker of each local victim
        self.next_att = torch.full((self.n_total,), -1, **i32)  # attacker -> next attacker of its victim
        self.flags32 = torch.zeros(self.n, **i32)
        self.off = torch.zeros(self.n + 1, **i32)
        self.action = torch.zeros(self.n, dtype=torch.int8, device=dev)
        self.counterpart = torch.full((self.n,), -1, dtype=torch.int64, device=dev)
        self.loss = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.respawn = torch.zeros(self.n, dtype=torch.int8, device=dev)
        self.counts = torch.zeros(5, dtype=torch.int64, device=dev)
        self.rank_totals = torch.zeros(self.dist.world, **i32)
        tb = _lib.scan_temp_bytes(self.n) if dev.type == "cuda" and self.dist.enabled else 0
        self.scan_temp = torch.empty(max(tb, 16), dtype=torch.uint8, device=dev)
        self.cfg = _lib.make_cfg(spec)
        self.recorder = None
        self.stats = False          # classify + all-reduce every generation
        self.stats_with_sec = True
        self._graphs = None
        # initial particles: uids 0..n_total-1, keyed init (identical for any rank count)
        local = self.local_rows()
        if weights is not None:
            w = torch.as_tensor(weights, dtype=torch.float32)
            local.zero_()
            local[:, : w.shape[1]] = w[self.lo:self.hi].to(dev)
        else:
            K.init_rows(spec, local, self.uid, self.seed)
        if self.dist.enabled:
            self.next_rows.copy_(local)
            self.dist.all_gather_rows(self.table, self.next_rows, self.n_total)

    # ------------------------------------------------------------------ views
    @property
    def table_in(self) -> torch.Tensor:
        """Generation-start table read by the next generation."""
        return self.table if self.dist.enabled else self._bufs[self._p]

    @property
    def rows_out(self) -> torch.Tensor:
        return self.next_rows if self.dist.enabled else self._bufs[1 - self._p]

    def local_rows(self) -> torch.Tensor:
        """Current weights of this rank's particles ([n, PP])."""
        return self.table[self.lo:self.hi] if self.dist.enabled else self._bufs[self._p]

    @property
    def eps(self) -> float:
        return float(self.params.get("epsilon", 1e-4) or 1e-14)

    def _flags(self) -> int:
        f = _lib.FLAG_SHUFFLE if self.shuffle else 0
        if self.params.get("remove_divergent"):
            f |= _lib.FLAG_REMOVE_DIVERGENT
        if self.params.get("remove_zero"):
            f |= _lib.FLAG_REMOVE_ZERO
        return f

    def _args(self) -> _lib.SrnnArgs:
        a = _lib.SrnnArgs()
        a.n, a.n_total, a.lo = self.n, self.n_total, self.lo
        a.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        a.lr, a.eps = self.lr, self.eps
        a.attacking_rate = float(self.params.get("attacking_rate", 0.1))
        a.learn_from_rate = float(self.params.get("learn_from_rate", 0.1))
        a.epochs = int(self.params.get("train", 0))
        a.severity = int(self.params.get("learn_from_severity", 1))
        a.flags = self._flags()
        a.gen_ptr = _p(self.gen_dev)
        a.segment = int(self.params.get("segment", 0) or 0)
        if self.device.type == "cuda":
            a.dev = 1
            a.stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        return a

    # ------------------------------------------------------------------ one generation
    def _generation(self, record: bool = False):
        spec, cfg = self.spec, self.cfg
        a = self._args()
        a.W2 = _p(self.table_in)
        a.W = _p(self.rows_out)
        a.uid = _p(self.uid)
        a.i32e, a.i32f = _p(self.head), _p(self.next_att)
        a.i32c, a.i32d = _p(self.flags32), _p(self.off)
        a.action, a.counterpart, a.loss, a.respawn = _p(self.action), _p(self.counterpart), _p(self.loss), _p(self.respawn)
        a.temp, a.temp_bytes = _p(self.scan_temp), self.scan_temp.numel()
        a.uid_out = _p(self.uid)
        if self.dist.enabled:
            a.flags |= 16  # per-row respawn flags for the scan (else per-block counts)
        # head[] is -1 on entry: set at construction, reset by the evolve kernel after use
        _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
        _lib.run(_lib.OP_SOUP_EVOLVE, spec, a, cfg)
        if record and self.recorder is not None:
            self.recorder.on_evolved(self)
        if self.dist.enabled:
            # globally sequential uids: rank r starts after the respawns of ranks < r
            _lib.run(_lib.OP_SCAN, spec, a, cfg)
            self.dist.all_gather_scalar(self.rank_totals, self.off[self.n:self.n + 1])
            prefix = self.rank_totals[: self.dist.rank].sum().to(torch.int64)
            self.uid_base.copy_(self.next_uid + prefix)
            self.next_uid.add_(self.rank_totals.sum().to(torch.int64))
            a.uid_base = _p(self.uid_base)
            _lib.run(_lib.OP_RESPAWN, spec, a, cfg)
            self.gen_dev.add_(1)
            self.dist.all_gather_rows(self.table, self.next_rows, self.n_total)
        else:
            a.uid_base = _p(self.next_uid)  # updated in place, gen_dev advanced by the kernel
            a.counts = _p(self.counts)       # zeroed by the kernel for the census below
            _lib.run(_lib.OP_RESPAWN_SEQ, spec, a, cfg)
            self._p = 1 - self._p
        if self.stats:
            # per-generation fixpoint-fraction statistics (reference Soup.count, code/soup.py:89-103)
            self.classify_local(self.stats_with_sec, zero=self.dist.enabled)
            self.dist.all_reduce_sum(self.counts)

    def classify_local(self, with_sec: bool = True, zero: bool = True):
        if zero:
            self.counts.zero_()
        cls, _ = K.classify(self.spec, self.local_rows(), self.eps, with_sec, uid=self.uid, seed=self.seed,
                            ctr=0x7FFFFFF0, counts=self.counts)
        return cls

    def count(self, with_sec: bool = True) -> Dict[str, int]:
        """Global class histogram of the current particles (all-reduced)."""
        self.classify_local(with_sec)
        self.dist.all_reduce_sum(self.counts)
        return counts_dict(self.counts.cpu())

    def evolve(self, iterations: int = 1, record: bool = False):
        for _ in range(iterations):
            self.time += 1
            if record and self.recorder is not None:
                slot_uid = self.global_uids()  # uid of every slot at generation start
                self._generation(record=True)
                self.recorder.on_generation_end(self, self.time, slot_uid)
            elif self._graphs is not None:
                self._graphs[self._p].replay()
                self._p = 1 - self._p
            else:
                self._generation()
        return self

    def global_uids(self):
        """uid of every global slot (host numpy); all-gathered when sharded."""
        if not self.dist.enabled:
            return self.uid.cpu().numpy().copy()
        out = torch.zeros(self.n_total, dtype=torch.int64, device=self.device)
        self.dist.all_gather_rows(out, self.uid, self.n_total)
        return out.cpu().numpy()

    # ------------------------------------------------------------------ HIP graphs
    def capture(self, warmup: int = 1) -> bool:
        """Capture the generation for both ping-pong parities in two hipGraphs (single
        rank, ROCm device).  Everything that changes per generation lives in device
        memory (generation counter, next uid), so replays advance the soup exactly like
        the eager path."""
        if self.device.type != "cuda" or self.dist.enabled:
            return False
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(max(warmup, 0)):
                self.time += 1
                self._generation()
        torch.cuda.current_stream(self.device).wait_stream(s)
        graphs = []
        p0 = self._p
        for _ in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._generation()  # flips self._p during capture (nothing ran)
            graphs.append(g)
        self._p = p0
        # graphs[k] was captured with parity p0 ^ k; index them by parity
        self._graphs = graphs if p0 == 0 else graphs[::-1]
        return True
