"""Device soup engine: one fused generation pipeline over a (sharded) population.

Replaces the per-particle Python loop of ``Soup.evolve`` (reference code/soup.py:51-87)
with a *synchronous* (Jacobi) generation computed for every particle at once.

Single rank (4 kernels, captured as hipGraphs):

1. ``decide`` -- every global slot draws its decisions from Philox keyed by
   (seed, slot, generation); attacks on local victims are linked into per-victim lists.
2. ``evolve`` (fused, lane per particle) -- received attacks in ascending attacker-slot
   order with generation-start attacker weights, ``learn_from_severity`` epochs on the
   teacher's generation-start samples, ``train`` self-train epochs, divergence / zero
   respawn flags (reference :77-86); each wave publishes a 64-bit respawn ballot.
3. ``respawn`` (one workgroup) -- scans the ballots, assigns globally sequential uids
   (reference S13), re-initialises the rows (init keyed by (generation, slot)), advances
   next_uid and the generation counter.
4. ``classify`` -- the per-generation census (reference code/soup.py:89-103).

Sharded over R ranks (one process per GPU, RCCL over xGMI): every rank recomputes every
slot's decisions, so it knows which of its rows other ranks need (attackers of their
victims, teachers of their learners): those rows -- ~(attack+learn rate)/R of a shard per
peer -- go through ONE fixed-capacity all-to-all; the census plus each rank's respawn
count go through ONE 48-byte all-gather, from which the uid prefix is computed on device.
No weight table is replicated.  Results are bitwise independent of R
(tests/test_dist_gloo.py).  ``exchange="allgather"`` instead all-gathers every rank's rows
each generation (the X01 pattern of SURVEY §2.5: one collective, no decide-dependent
packing, but every rank holds the whole table) -- same results, bitwise.

``dtype`` selects the storage of the weight tables and exchange rows (fp32, bf16, fp16;
arithmetic is fp32 -- SURVEY §7.7).

Differences from the sequential reference (tested statistically): particle k does not see
the effects of particles < k within the same generation; every read is from the
generation-start weights.  ``Soup(mode="sequential")`` keeps the exact reference order.
"""
from __future__ import annotations

import ctypes
import os
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


MAX_SLOTS = 2 ** 31 - 2  # soup slots are int32 on the device


def plan_population(spec: ArchSpec, dtype=torch.float32, exchange: str = "alltoall", world: int = 1,
                    hbm_bytes: int = 288 * 10 ** 9, fill: float = 0.9, attacking_rate: float = 0.1,
                    learn_from_rate: float = 0.1) -> Dict:
    """Device bytes per particle of a SoupEngine and the largest population that fits
    ``fill`` of each GPU's HBM (288 GB HBM3E per MI355X).  Per local row: two ping-pong
    table rows + uid/flags/action/counterpart/loss/respawn (34 B); per global slot: the
    attacker link (+ the received-row map for all-to-all); exchange: the gathered table
    (all-gather) or the capacity-bounded send/recv rows (all-to-all)."""
    rb = spec.PP * torch.empty((), dtype=dtype).element_size()
    per_local = 2 * rb + 34
    if exchange == "allgather":
        per_slot = 4 + (rb if world > 1 else 0)
        per_local_x = 0.0
    else:
        per_slot = 4 + (4 if world > 1 else 0)
        per_local_x = (2 * 1.2 * min(attacking_rate + learn_from_rate, 2.0) * (rb + 16)) if world > 1 else 0.0
    per_particle = per_slot + (per_local + per_local_x) / world  # bytes per GPU per global particle
    n_fit = int(fill * hbm_bytes / per_particle)
    return dict(row_bytes=rb, bytes_per_particle_per_gpu=per_particle, n_total_fit=n_fit,
                n_total=min(n_fit, MAX_SLOTS), limited_by="hbm" if n_fit <= MAX_SLOTS else "int32 slots",
                world=world, exchange=exchange, dtype=str(dtype).replace("torch.", ""))


class SoupEngine:
    """Population-sharded soup on one device per rank."""

    def __init__(self, spec: ArchSpec, n_total: int, params: Dict, device="cpu", seed: int = 0,
                 lr: float = 0.01, shuffle: bool = True, dist: Optional[Dist] = None, weights=None,
                 dtype: torch.dtype = torch.float32, exchange: str = "alltoall", local_weights=None,
                 init: bool = True):
        """``weights``: the whole population's initial rows [n_total, >= P] (every rank
        takes its slice); ``local_weights``: only this rank's rows [hi - lo, >= P];
        ``init=False``: leave the rows for the caller to fill (the streaming checkpoint
        loader writes them straight into the device table)."""
        self.spec = spec
        self.n_total = int(n_total)
        self.params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, learn_from_severity=1)
        self.params.update(params or {})
        self.device = torch.device(device)
        self.seed = int(seed)
        self.lr = float(lr)
        self.shuffle = bool(shuffle)
        self.dist = dist or Dist()
        if self.device.type == "cuda" and self.dist.enabled:
            # the soup's own RCCL communicator: its collectives can live inside hipGraphs
            self.dist.enable_native_comm(self.device)
        self.lo, self.hi = self.dist.shard(self.n_total)
        self.n = self.hi - self.lo
        if self.n_total > MAX_SLOTS:
            raise ValueError("soup slots are int32 on device")
        seg = int(self.params.get("segment", 0) or 0)
        if seg and self.n_total % seg:
            raise ValueError("population size must be a multiple of the sub-soup segment")
        if exchange not in ("alltoall", "allgather"):
            raise ValueError(f"exchange must be 'alltoall' or 'allgather', got {exchange!r}")
        self.exchange = exchange
        self.dtype = dtype
        self.dtype_code = K.dtype_code(dtype)
        dev, PP = self.device, spec.PP
        i32 = dict(dtype=torch.int32, device=dev)
        # this rank's rows, ping-pong: generation t reads buf[p], writes buf[1-p]
        self._bufs = [torch.zeros((self.n, PP), dtype=dtype, device=dev) for _ in range(2)]
        self._p = 0
        if self.dist.enabled and exchange == "allgather":
            # every rank's generation-start rows, gathered each generation
            self.full = torch.zeros((self.n_total, PP), dtype=dtype, device=dev)
            self.stats_all = torch.zeros(self.dist.world * 6, dtype=torch.int64, device=dev)
            self.census = torch.zeros(5, dtype=torch.int64, device=dev)
        elif self.dist.enabled:
            # exchange of the generation-start rows that other ranks need (attackers of
            # their victims, teachers of their learners): fixed-capacity all-to-all
            R = self.dist.world
            if R > 31:
                # need masks are one int32 bit per destination rank (srnn_kernels.h link_decision)
                raise ValueError("exchange='alltoall' supports at most 31 ranks; use exchange='allgather'")
            n_max = -(-self.n_total // R)  # identical on every rank (buffers must match)
            mean = self._expected_peer_rows()
            xw = PP * self._bufs[0].element_size() // 4 + 4  # row bytes + 16 tag bytes, in fp32 units
            # the first `stat_rows` rows of each destination block carry the sender's
            # int64[6] stats (previous census + respawns): one collective per generation
            self.stat_rows = -(-48 // (4 * xw))
            self.cap = self.stat_rows + int(min(max(mean * 1.2 + 6.0 * mean ** 0.5 + 32, 32), max(n_max, 32)))
            self.need = torch.zeros(self.n, **i32)
            self.sendcnt = torch.full((R,), self.stat_rows, **i32)
            self.rmap = torch.zeros(self.n_total, **i32)
            self.ovf = torch.zeros(1, **i32)
            self.sendbuf = torch.full((R * self.cap, xw), -1, **i32).view(torch.float32)
            self.recvbuf = torch.full((R * self.cap, xw), -1, **i32).view(torch.float32)
            self.stats_all = torch.zeros(R * 6, dtype=torch.int64, device=dev)
            self.census = torch.zeros(5, dtype=torch.int64, device=dev)
        self.uid = torch.arange(self.lo, self.hi, dtype=torch.int64, device=dev)
        self.next_uid = torch.full((1,), self.n_total, dtype=torch.int64, device=dev)
        self.uid_base = torch.zeros(1, dtype=torch.int64, device=dev)
        # generation counter as a 2-slot ring indexed by the ping-pong parity: a launch
        # reads slot _p and the generation-closing kernel writes slot 1-_p, so blocks of
        # one launch never race on it (gen_dev is the current slot)
        self._gen_ring = torch.ones(2, dtype=torch.int32, device=dev)
        self.time = 0
        # attack lists, one buffer per ping-pong parity: the fused single-rank generation
        # links the NEXT generation's attacks into the other parity's buffer
        self.heads = [torch.full((self.n,), -1, **i32) for _ in range(2)]       # first attacker of each local victim
        self.nexts = [torch.full((self.n_total,), -1, **i32) for _ in range(2)]  # attacker -> next attacker
        self._lists_ready = False   # heads[_p] already holds this generation's attacks
        # one launch (+ a one-workgroup finish) per generation: OP_SOUP_GEN; sharded engines
        # with the all-to-all exchange fuse the evolve, census and next decisions too
        # shapes without a templated kernel run on the runtime-shape engine: unfused
        # generation pipeline (decide -> evolve -> respawn -> census), per-lane scratch
        self.generic = _lib.is_generic(spec, _lib.OP_SOUP_GEN, self.dtype_code)
        self.fused = (not self.dist.enabled or exchange == "alltoall") and not self.generic
        self._scratch = None
        if self.device.type == "cuda" and _lib.is_generic(spec, _lib.OP_SOUP_EVOLVE, self.dtype_code):
            self._scratch = torch.empty(_lib.generic_scratch_bytes(spec, self.n, self.dtype_code),
                                        dtype=torch.uint8, device=dev)
        self._mask_src = "i32c"   # where the pending respawn ballots live ("bs": block stats)
        self._packed = False      # sharded: the coming generation's send buffer is packed
        self._fused_census = False
        self.two_phase = os.environ.get("SRNN_GEN_TWO_PHASE", "1") == "1"  # + a 1-workgroup finish kernel
        nb = -(-self.n // 64)
        self._blockstat = torch.zeros(max(nb, 1) * 8, **i32)
        # single rank on a GPU: the finish kernel of generation g (census reduction + uids
        # of its newborns) runs on a side stream beside generation g + 1; the block stats
        # it reads are double-buffered by ping-pong parity (SRNN_ASYNC_FINISH=0: serial)
        # where the finish of a single-rank fused generation on a GPU runs (census reduction
        # + newborn uids, one workgroup): "batch" -- the generation kernel advances the
        # counter itself, the block stats of up to G generations go to a ring and ONE
        # launch finishes them all (per graph chunk / evolve call); "async" -- per
        # generation on a side stream beside the next one (cross-queue sync per generation:
        # measured slower, profiles/r2b_finish_modes.md); "serial" -- after every generation
        fm = os.environ.get("SRNN_FINISH_MODE", "batch")
        if self.device.type != "cuda" or self.dist.enabled or not self.fused:
            fm = "serial"
        self.finish_mode = fm
        self.async_finish = fm == "async"
        # the ring holds 32 B per 64-row block per pending generation: at HBM-filling sizes
        # (2e9 rows = 1 GB per generation) fewer generations share one finish launch
        self._batch = max(1, min(max(self._chunk_sizes() or [1]), (512 << 20) // (max(nb, 1) * 32)))
        # (+ 8 bytes per generation: its newborn count, accumulated by the generation waves)
        self._bs_ring = torch.zeros((self._batch, max(nb, 1) * 8 + 2), **i32) if fm == "batch" else None
        self._pending_fin = 0  # batch mode: generations whose finish is still due
        self._blockstats = [self._blockstat, torch.zeros_like(self._blockstat)] if self.async_finish else None
        # sharded fused generations fold the post-exchange launch (previous generation's
        # uids + received-row index) into the generation launch: block stats by parity (the
        # launch reads the previous generation's ballots while writing its own) and the
        # unpack-done counter its generation waves wait on (SRNN_POST_IN_GEN=0: separate
        # post-exchange launch, round-1 pipeline)
        self.post_in_gen = (self.dist.enabled and exchange == "alltoall" and self.fused
                            and os.environ.get("SRNN_POST_IN_GEN", "1") == "1")
        self._bs2 = [self._blockstat, torch.zeros_like(self._blockstat)] if self.post_in_gen else None
        self._xdone = torch.zeros(1, **i32) if self.post_in_gen else None
        self._side = torch.cuda.Stream(self.device) if self.async_finish else None
        self._fin_ev = [None, None]  # finish events of the generations that wrote each block-stats buffer
        # SGD permutations precomputed by helper waves of the previous generation
        # (Weightwise nets with <= 16 weights, shuffled): [parity][epoch][row] nibble words
        E = int(self.params.get("train", 0)) + (max(int(self.params.get("learn_from_severity", 1)), 0)
                                                 if float(self.params.get("learn_from_rate", 0.1)) > 0 else 0)
        self._perm_e = E
        self._perms = None
        self._perms_ready = False
        if (self.async_finish and self.shuffle and spec.kind == "weightwise" and spec.P <= 16 and 0 < E <= 256
                and 2 * E * 8 * self.n <= 8 * 2 ** 30 and os.environ.get("SRNN_PRE_PERMS", "0") == "1"):
            self._perms = [torch.zeros((E, self.n), dtype=torch.int64, device=dev) for _ in range(2)]
            self._helper_ctl = [torch.zeros(_lib.HELPER_CTL, dtype=torch.int32, device=dev) for _ in range(2)]
            nb = -(-self.n // 64)
            # helper workgroups: enough to give every SIMD with one generation wave a partner
            self._helpers = int(os.environ.get("SRNN_PERM_HELPERS", max(0, 2 * 1024 - nb)))
        self._done = torch.zeros(1, **i32)
        # per-row respawn flags (host) or 64-bit respawn ballots per 64-row wave (device)
        self.flags32 = torch.zeros(max(self.n, 2 * (-(-self.n // 64))), **i32)
        self._pending = False  # sharded: uids of the last generation's newborns not yet assigned
        self.off = torch.zeros(self.n + 1, **i32)
        self.action = torch.zeros(self.n, dtype=torch.int8, device=dev)
        self.counterpart = torch.full((self.n,), -1, dtype=torch.int64, device=dev)
        self.loss = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.respawn = torch.zeros(self.n, dtype=torch.int8, device=dev)
        self.counts = torch.zeros(6, dtype=torch.int64, device=dev)  # classes[5] + respawns
        self.cfg = _lib.make_cfg(spec, self.dtype_code)
        self.recorder = None        # full reference-schema state recorder (compat Soup)
        self.trajectory = None      # sampled TrajectoryRecorder (large soups)
        self.metrics = None         # MetricsWriter (JSONL per-generation metrics)
        self._metrics_uid = None
        self.stats = False          # classify + all-reduce every generation
        self.stats_with_sec = True
        self._graphs = None
        self._chunk = None          # (graph of G generations, start parity, G): the largest
        self._chunks = []           # every captured multi-generation graph, largest first
        self._arg_cache = {}
        # initial particles: uids 0..n_total-1, keyed init (identical for any rank count)
        local = self.local_rows()
        if weights is not None or local_weights is not None:
            if local_weights is not None:
                w = torch.as_tensor(local_weights, dtype=torch.float32)
                if w.shape[0] != self.n:
                    raise ValueError(f"local_weights has {w.shape[0]} rows, this rank owns {self.n}")
            else:
                w = torch.as_tensor(weights, dtype=torch.float32)[self.lo:self.hi]
            local.zero_()
            local[:, : w.shape[1]] = w.to(dev, dtype)
        elif init:
            K.init_rows(spec, local, self.uid, self.seed)

    def _expected_peer_rows(self) -> float:
        """Largest expected number of rows one rank ships to one peer per generation.

        Row i of rank r goes to rank q when i attacks a victim owned by q, or when a
        learner owned by q picks i as teacher.  Partners are uniform over the slot's
        sub-soup (``segment``) or the whole population, so the load of a (r, q) pair is
        sum over r's slots of ar * |S_i n shard_q| / |S_i| plus sum over q's slots of
        lr * |S_j n shard_r| / |S_j|.  Segments spanning several shards concentrate the
        traffic on neighbouring ranks, which a uniform estimate would underestimate."""
        R = self.dist.world
        ar = max(float(self.params.get("attacking_rate", 0.1)), 0.0)
        lr_ = max(float(self.params.get("learn_from_rate", 0.1)), 0.0)
        seg = int(self.params.get("segment", 0) or 0) or self.n_total
        bounds = [self.dist.shard_of_rank(r, self.n_total) for r in range(R)]
        # overlap[r][q] = sum over slots i of shard r of |S_i n shard_q| / |S_i|; a segment
        # inside one shard only adds to the diagonal, so only the (at most R - 1) segments
        # holding a shard boundary are visited
        overlap = [[0.0] * R for _ in range(R)]
        starts = sorted({(lo // seg) * seg for lo, _ in bounds[1:]})
        for s0 in starts:
            s1 = min(s0 + seg, self.n_total)
            inter = [max(0, min(hi, s1) - max(lo, s0)) for lo, hi in bounds]
            for r in range(R):
                if inter[r]:
                    for q in range(R):
                        overlap[r][q] += inter[r] * inter[q] / (s1 - s0)
        worst = 0.0
        for r in range(R):
            for q in range(R):
                if q != r:
                    worst = max(worst, ar * overlap[r][q] + lr_ * overlap[q][r])
        return worst

    # ------------------------------------------------------------------ views
    @property
    def gen_dev(self) -> torch.Tensor:
        """Device scalar (1-element view): the generation about to run."""
        return self._gen_ring[self._p:self._p + 1]

    @property
    def table_in(self) -> torch.Tensor:
        """This rank's generation-start rows read by the next generation."""
        return self._bufs[self._p]

    @property
    def rows_out(self) -> torch.Tensor:
        return self._bufs[1 - self._p]

    def local_rows(self) -> torch.Tensor:
        """Current weights of this rank's particles ([n, PP])."""
        return self._bufs[self._p]

    @property
    def eps(self) -> float:
        # reference default epsilon 1e-14 (code/network.py:78); 0 / None fall back to it
        return float(self.params.get("epsilon") or 1e-14)

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
        a.gen_out = _p(self._gen_ring[1 - self._p:2 - self._p])
        a.segment = int(self.params.get("segment", 0) or 0)
        if self.device.type == "cuda":
            a.dev = 1
            a.stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            if self._scratch is not None:
                a.scratch, a.scratch_bytes = _p(self._scratch), self._scratch.numel()
        return a

    # ------------------------------------------------------------------ one generation
    def _gen_args(self):
        """Populated argument blocks of one generation (cached per parity / stream /
        params: building ctypes structs every generation costs host time)."""
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        key = (self._p, stream, tuple(sorted((k, str(v)) for k, v in self.params.items())), self.stats_with_sec,
               self.lr, self.shuffle, self.stats, self.two_phase, self.finish_mode, self._pending_fin)
        hit = self._arg_cache.get(key)
        if hit is not None:
            return hit
        a = self._args()
        a.W2 = _p(self.table_in)
        a.W = _p(self.rows_out)
        a.uid = _p(self.uid)
        a.i32e, a.i32f = _p(self.heads[self._p]), _p(self.nexts[self._p])
        a.i32c = _p(self.flags32)
        a.action, a.counterpart, a.loss, a.respawn = _p(self.action), _p(self.counterpart), _p(self.loss), _p(self.respawn)
        a.uid_out = _p(self.uid)
        a.counts, a.uid_base = _p(self.counts), _p(self.next_uid)
        ca = None
        if self.dist.enabled:
            d = self.dist
            a.world, a.rank = d.world, d.rank
            if self.exchange == "allgather":
                a.recvbuf = _p(self.full)
                a.flags |= _lib.FLAG_FULL_TABLE
            else:
                a.cap = self.cap
                a.need, a.sendcnt, a.rmap, a.ovf = _p(self.need), _p(self.sendcnt), _p(self.rmap), _p(self.ovf)
                a.sendbuf, a.recvbuf = _p(self.sendbuf), _p(self.recvbuf)
            a.stats, a.census = _p(self.stats_all), _p(self.census)
            ca = self._args()
            ca.n, ca.eps = self.n, self.eps
            ca.flags = ((_lib.FLAG_FIX_SEC if self.stats_with_sec else 0) | _lib.FLAG_COUNT_RESPAWNS
                        | _lib.FLAG_GEN_ADVANCE)
            ca.W, ca.counts, ca.respawn, ca.uid = _p(self.rows_out), _p(self.counts), _p(self.respawn), None
            ca.ctr = 0x7FFFFFF0
        if not self.dist.enabled or self.exchange == "alltoall":
            # fused generation: next generation's lists, block stats, done counter, census
            fa = self._args()
            ctypes.pointer(fa)[0] = a
            fa.i32a, fa.i32b = _p(self.heads[1 - self._p]), _p(self.nexts[1 - self._p])
            fa.i32c = None
            fa.temp, fa.temp_bytes = _p(self._blockstat), self._blockstat.numel() * 4
            fa.i32d = _p(self._done)
            fa.flags = a.flags | _lib.FLAG_RESPAWN_INLINE | (_lib.FLAG_TWO_PHASE if self.two_phase else 0)
            if self.finish_mode == "batch":
                bs = self._bs_ring[self._pending_fin]
                fa.temp, fa.temp_bytes = _p(bs), bs.numel() * 4
                fa.flags |= _lib.FLAG_TWO_PHASE | _lib.FLAG_ASYNC_FINISH | _lib.FLAG_BORN_TOTAL
            if self.async_finish:
                bs = self._blockstats[self._p]
                fa.temp, fa.temp_bytes = _p(bs), bs.numel() * 4
                fa.flags |= _lib.FLAG_TWO_PHASE | _lib.FLAG_ASYNC_FINISH
                if self._perms is not None:
                    fa.flags |= _lib.FLAG_PRE_PERMS
                    fa.perm_cur, fa.perm_next = _p(self._perms[self._p]), _p(self._perms[1 - self._p])
                    fa.helper_ctl, fa.perm_e, fa.helpers = _p(self._helper_ctl[self._p]), self._perm_e, self._helpers
            census = self.stats and self.spec.shuffler == "none"
            if self.dist.enabled:
                # sharded: every global slot's next decisions; counts feed the next pack
                fa.flags |= _lib.FLAG_TWO_PHASE | _lib.FLAG_SHARDED_DECIDE | _lib.FLAG_FINISH_PACK
                census = self.spec.shuffler == "none"
                if self.post_in_gen:
                    bs, prev = self._bs2[self._p], self._bs2[1 - self._p]
                    fa.temp, fa.temp_bytes = _p(bs), bs.numel() * 4
                    fa.temp2, fa.xdone = _p(prev), _p(self._xdone)
                    fa.flags |= _lib.FLAG_GEN_POST | _lib.FLAG_STATS_X
            if census:
                fa.flags |= _lib.FLAG_FUSED_CENSUS | (_lib.FLAG_FIX_SEC if self.stats_with_sec else 0)
            if self.dist.enabled:
                self._fused_census = census
                ca = (ca, fa)
            elif self.async_finish:
                fin = self._args()
                ctypes.pointer(fin)[0] = fa
                fin.stream = ctypes.c_void_p(self._side.cuda_stream)
                ca = (fa, fin)
            else:
                ca = fa
        self._arg_cache[key] = (a, ca, a.flags)
        return self._arg_cache[key]

    def _ballots(self) -> torch.Tensor:
        """Block stats holding the pending respawn ballots: the last generation's parity
        buffer when it was a post-in-gen fused generation, else the single buffer."""
        if self.post_in_gen and self._mask_src == "bs":
            return self._bs2[1 - self._p]
        return self._blockstat

    def _uid_flags(self, flags: int) -> int:
        """uid assignment reads the respawn ballots where the producing generation left
        them: the fused generation's block stats or the evolve kernel's i32c ballots."""
        return flags | (_lib.FLAG_MASKS_BS if self._mask_src == "bs" else 0)

    def _generation(self, record: bool = False):
        spec, cfg = self.spec, self.cfg
        a, ca, flags = self._gen_args()
        a.flags = flags
        # head[] is -1 on entry: set at construction, reset by the evolve kernel after use
        if not self.dist.enabled:
            if self.fused and not (record and self.recorder is not None):
                # ONE launch: evolve + next generation's attack lists + census + uids
                if not self._lists_ready:
                    _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
                if self.finish_mode == "batch":
                    _lib.run(_lib.OP_SOUP_GEN, spec, ca, cfg)  # advances the counter, no finish
                    self._fin_flags = ca.flags
                    self._pending_fin += 1
                    self._lists_ready = True
                    self._p = 1 - self._p
                    if self._pending_fin == self._batch:
                        self._finish_pending()
                    return
                if self.async_finish:
                    # generation on the main stream; its finish on the side stream, beside
                    # the next generation (which only needs the counter it advances itself)
                    fa, fin = ca
                    main = torch.cuda.current_stream(self.device)
                    if self._perms is not None and not self._perms_ready:
                        # first precomputed generation: its permutations by a plain launch
                        pa = self._args()
                        pa.perm_next, pa.perm_e = _p(self._perms[self._p]), self._perm_e
                        _lib.run(_lib.OP_SOUP_PERMS, spec, pa, cfg)
                        self._perms_ready = True
                    ev = self._fin_ev[self._p]
                    if ev is not None:  # this parity's block stats are free again
                        main.wait_event(ev)
                    _lib.run(_lib.OP_SOUP_GEN, spec, fa, cfg)
                    self._side.wait_stream(main)
                    _lib.run(_lib.OP_GEN_FINISH, spec, fin, cfg)
                    ev = torch.cuda.Event()
                    ev.record(self._side)
                    self._fin_ev[self._p] = ev
                    self._lists_ready = True
                    self._p = 1 - self._p
                    return
                _lib.run(_lib.OP_SOUP_GEN, spec, ca, cfg)
                self._lists_ready = True
                self._p = 1 - self._p
                if self.stats and not (ca.flags & _lib.FLAG_FUSED_CENSUS):
                    self.classify_local(self.stats_with_sec, zero=False)
                return
            if not self._lists_ready:
                _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
            # newborn rows are re-initialised by the (parallel) evolve kernel unless the
            # recorder needs the dead particles' final rows first; the one-workgroup
            # respawn scan then only assigns the uids
            inline = not (record and self.recorder is not None)
            a.flags = flags | (_lib.FLAG_RESPAWN_INLINE if inline else 0)
            _lib.run(_lib.OP_SOUP_EVOLVE, spec, a, cfg)
            self._lists_ready = False
            self._perms_ready = False  # the next generation's permutations were not precomputed
            if record and self.recorder is not None:
                self.recorder.on_evolved(self)
            # uids from next_uid (advanced in place), generation counter, census histogram zeroed
            _lib.run(_lib.OP_RESPAWN_SEQ, spec, a, cfg)
            a.flags = flags
            self._p = 1 - self._p
            if self.stats:
                # per-generation fixpoint-fraction statistics (reference Soup.count, code/soup.py:89-103)
                self.classify_local(self.stats_with_sec, zero=False)
            return
        # ---- sharded (all-to-all, ONE collective per generation), fused:
        #   pack (stats rows of the previous generation + rows other ranks need)
        #   -> all-to-all -> unpack -> uids of the previous generation's newborns
        #   -> OP_SOUP_GEN: evolve + census + next generation's decisions of every global
        #      slot (lists + need masks) -> finish (counts, generation counter)
        # ---- sharded, unfused / recording: decide -> pack -> all-to-all -> unpack -> uids
        #   -> evolve -> census + respawn count (+ generation counter)
        # ---- sharded (all-gather): decide -> all-gather rows -> evolve -> census
        #   -> all-gather stats -> uids
        d = self.dist
        if self.exchange == "alltoall" and self.fused and not (record and self.recorder is not None):
            ca0, fa = ca
            if not self._lists_ready:
                _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
            if not self._packed:
                _lib.run(_lib.OP_SOUP_PACK, spec, a, cfg)
            d.all_to_all(self.recvbuf, self.sendbuf)
            if not self.post_in_gen:
                # post-exchange launch: block 0 assigns the uids of the previous generation's
                # newborns (stats rows of the exchange), the other blocks index the received rows
                a.flags = self._uid_flags(flags | _lib.FLAG_STATS_X | _lib.FLAG_POST_UNPACK)
                a.temp, a.temp_bytes = _p(self._blockstat), self._blockstat.numel() * 4
                _lib.run(_lib.OP_UID_ASSIGN, spec, a, cfg)
                a.flags = flags
            # generation (evolve + census + next decisions of every slot); finish launch:
            # block 0 closes the generation, the other blocks pack the next exchange
            _lib.run(_lib.OP_SOUP_GEN, spec, fa, cfg)
            self._packed = True
            if not self._fused_census:
                # random shuffler: census by the classify kernel (adds to counts[0..4])
                cflags = ca0.flags
                ca0.flags = _lib.FLAG_FIX_SEC if self.stats_with_sec else 0
                _lib.run(_lib.OP_CLASSIFY, spec, ca0, cfg)
                ca0.flags = cflags
            self._lists_ready = True
            self._mask_src = "bs"
            self._p = 1 - self._p
            self._pending = True
            return
        if isinstance(ca, tuple):
            ca = ca[0]
        if not self._lists_ready:
            _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
        packed, self._packed = self._packed, False
        if self.exchange == "allgather":
            # raw 32-bit view: the collective moves bytes whatever the storage dtype
            d.all_gather_rows(self.full.view(torch.int32), self.table_in.view(torch.int32), self.n_total)
        else:
            if not packed:
                _lib.run(_lib.OP_SOUP_PACK, spec, a, cfg)
            d.all_to_all(self.recvbuf, self.sendbuf)
            _lib.run(_lib.OP_SOUP_UNPACK, spec, a, cfg)
            a.flags = self._uid_flags(flags | _lib.FLAG_STATS_X)
            bs = self._ballots()
            a.temp, a.temp_bytes = _p(bs), bs.numel() * 4
            _lib.run(_lib.OP_UID_ASSIGN, spec, a, cfg)
        self._lists_ready = False
        self._mask_src = "i32c"
        inline = not (record and self.recorder is not None)
        a.flags = flags | (_lib.FLAG_RESPAWN_INLINE if inline else 0)
        _lib.run(_lib.OP_SOUP_EVOLVE, spec, a, cfg)
        a.flags = flags
        if not inline:
            self.recorder.on_evolved(self)
            _lib.run(_lib.OP_RESPAWN, spec, a, cfg)
        # census of the new generation + this rank's respawn count; advances the generation
        _lib.run(_lib.OP_CLASSIFY, spec, ca, cfg)
        self._p = 1 - self._p
        if self.exchange == "allgather":
            self._pending = True
            self._flush()
        else:
            self._pending = True

    def _finish_pending(self):
        """Batch mode: ONE finish launch for the generations whose block stats wait in the
        ring (in generation order: census of each, newborn uids, next_uid)."""
        m = self._pending_fin
        if m == 0:
            return
        a = self._args()
        a.n = self.n
        a.steps = m
        a.flags = (self._fin_flags & (_lib.FLAG_FUSED_CENSUS | _lib.FLAG_BORN_TOTAL)) | _lib.FLAG_FINISH_BATCH
        a.temp, a.temp_bytes = _p(self._bs_ring), self._bs_ring.stride(0) * 4
        a.uid_out, a.uid_base, a.counts = _p(self.uid), _p(self.next_uid), _p(self.counts)
        if os.environ.get("SRNN_FINISH_PAR", "1") == "1":
            a.i32d = _p(self._done)  # done counter: one finish workgroup per generation
        _lib.run(_lib.OP_GEN_FINISH, self.spec, a, self.cfg)
        self._pending_fin = 0

    def _join_side(self):
        """Make the current stream wait for the side-stream finish kernels (uids, census,
        next_uid are final after this) and run any batched finish still due."""
        if self._side is not None and any(e is not None for e in self._fin_ev):
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._fin_ev = [None, None]
        if self._pending_fin:
            self._finish_pending()

    def _flush(self):
        """Sharded: assign the uids of the last generation's newborns now (all-gather of
        the per-rank stats) instead of with the next generation's row exchange."""
        if not (self.dist.enabled and self._pending):
            return
        a, _, flags = self._gen_args()
        a.flags = self._uid_flags(flags)
        bs = self._ballots()
        a.temp, a.temp_bytes = _p(bs), bs.numel() * 4
        self.dist.all_gather_into(self.stats_all, self.counts)
        _lib.run(_lib.OP_UID_ASSIGN, self.spec, a, self.cfg)
        a.flags = flags
        self._pending = False
        if self._packed:
            # the packed send buffer carries these stats too: they are settled now
            self.sendbuf.view(self.dist.world, -1)[:, :12].zero_()

    def exchange_overflowed(self) -> bool:
        return bool(self.dist.enabled and self.exchange == "alltoall" and int(self.ovf.item()) != 0)

    def classify_local(self, with_sec: bool = True, zero: bool = True):
        if zero:
            self.counts.zero_()
        # census streams (shuffle_random nets) keyed by global slot, like the fused census
        cls, _ = K.classify(self.spec, self.local_rows(), self.eps, with_sec, uid=None, seed=self.seed,
                            scratch=self._scratch, ctr=0x7FFFFFF0, counts=self.counts, key_offset=self.lo)
        return cls

    def count(self, with_sec: bool = True) -> Dict[str, int]:
        """Global class histogram of the current particles (all-reduced)."""
        if self.exchange_overflowed():
            raise RuntimeError("soup row exchange overflowed its capacity: results are invalid")
        self.classify_local(with_sec)
        c = self.counts[:5].clone()
        self.dist.all_reduce_sum(c)
        return counts_dict(c.cpu())

    def last_census(self) -> Dict[str, int]:
        """Census recorded by the last generation (stats / sharded path)."""
        c = self.census if self.dist.enabled else self.counts[:5]
        return counts_dict(c.cpu())

    def evolve(self, iterations: int = 1, record: bool = False):
        left = int(iterations)
        while left > 0:
            # the largest captured multi-generation graph that fits what is left
            ch = next((c for c in self._chunks if c[2] <= left), None)
            if (ch is not None and not (record and self.recorder is not None)
                    and self._p == ch[1] and self.trajectory is None and self.metrics is None):
                # G generations in one graph launch (no inter-graph gaps)
                self._join_side()
                ch[0].replay()
                self.time += ch[2]
                left -= ch[2]
                self._pending = self.dist.enabled
                continue
            left -= 1
            self.time += 1
            if record and self.recorder is not None:
                self._join_side()
                slot_uid = self.global_uids()  # uid of every slot at generation start
                self._generation(record=True)
                self._flush()
                self.recorder.on_generation_end(self, self.time, slot_uid)
            elif self._graphs is not None:
                self._join_side()
                self._graphs[self._p].replay()
                self._p = 1 - self._p
                self._pending = self.dist.enabled
            else:
                self._generation()
            self._hooks()
        self._join_side()
        self._flush()  # uids / census consistent between evolve calls
        if self.dist.native is not None:
            self.dist.native.check()  # RCCL asynchronous errors (peer failure) surface here
        return self

    def _hooks(self):
        """Per-generation observers (host work only when one is due)."""
        t = self.time
        if (self.trajectory is not None and self.trajectory.due(t)) or (self.metrics is not None and self.metrics.due(t)):
            self._join_side()
        if self.trajectory is not None and self.trajectory.due(t):
            self._flush()
            self.trajectory.snapshot(self, t)
        if self.metrics is not None and self.metrics.due(t):
            self._flush()
            census = self.last_census() if (self.stats or self.dist.enabled) else self.count()
            nu = int(self.next_uid.item())
            resp = None if self._metrics_uid is None else nu - self._metrics_uid
            self._metrics_uid = nu
            ls = torch.stack([torch.nan_to_num(self.loss.double(), nan=0.0).sum(),
                              torch.tensor(float(self.n), dtype=torch.float64, device=self.device)])
            self.dist.all_reduce_sum(ls)
            self.metrics.log(t, census, self.n_total, respawns=resp, mean_loss=float(ls[0] / ls[1]), next_uid=nu)

    # ------------------------------------------------------------------ fault injection
    def inject_nan(self, rows) -> None:
        """Fault injection: poison local rows with NaN so the divergence
        test / respawn path runs on them (reference code/network.py:44-52, soup.py:77-86)."""
        rows = torch.as_tensor(rows, dtype=torch.int64, device=self.device)
        if rows.numel() and (int(rows.min()) < 0 or int(rows.max()) >= self.n):
            raise IndexError("inject_nan rows out of this rank's range")
        self.local_rows()[rows, 0] = float("nan")

    def global_uids(self):
        """uid of every global slot (host numpy); all-gathered when sharded."""
        if not self.dist.enabled:
            return self.uid.cpu().numpy().copy()
        out = torch.zeros(self.n_total, dtype=torch.int64, device=self.device)
        self.dist.all_gather_rows(out, self.uid, self.n_total)
        return out.cpu().numpy()

    # ------------------------------------------------------------------ HIP graphs
    def _state(self):
        """Every device tensor a generation reads or writes (graph validation)."""
        names = ["_bufs", "uid", "next_uid", "_gen_ring", "heads", "nexts", "flags32", "action", "counterpart",
                 "loss", "respawn", "counts", "census", "need", "sendcnt", "rmap", "ovf", "sendbuf", "recvbuf",
                 "full", "stats_all", "_blockstats" if self._blockstats else ("_bs2" if self._bs2 else "_blockstat"),
                 "_done", "_perms", "_helper_ctl", "_bs_ring", "_xdone"]
        out = []
        for k in names:
            v = getattr(self, k, None)
            if isinstance(v, list):
                out.extend(v)
            elif isinstance(v, torch.Tensor):
                out.append(v)
        return out

    def capture(self, warmup: int = 1, validate: bool = True) -> bool:
        """Capture the generation for both ping-pong parities in two hipGraphs (ROCm
        device).  Everything that changes per generation lives in device memory
        (generation counter, next uid), so replays advance the soup exactly like the
        eager path.  Sharded engines capture their RCCL collective inside the graph (one
        all-to-all per generation, exchange="alltoall" only); ``validate`` then replays
        two generations from a saved state, compares them bitwise with the eager path on
        every rank and keeps the graphs only if all ranks agree."""
        if self.device.type != "cuda":
            return False
        if self.dist.enabled and self.exchange != "alltoall":
            return False
        if self.dist.enabled and self.dist.native is None:
            # torch's process-group collectives are not captured: their watchdog thread
            # queries events recorded by the capturing stream
            return False
        if self.dist.world > 1 and os.environ.get("SRNN_SHARDED_GRAPH", "1") != "1":
            # SRNN_SHARDED_GRAPH=0: multi-GPU generations run eagerly (RCCL all-to-all
            # enqueued per generation from the host).  By default the all-to-all is captured
            # with the kernels; the replay is validated bitwise against eager generations on
            # every rank and all ranks fall back to eager unless every rank agrees
            return False
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(max(warmup, 1 if (self.dist.enabled or self.fused) else 0)):
                self.time += 1
                self._generation()
            self._join_side()
        torch.cuda.current_stream(self.device).wait_stream(s)
        graphs = []
        p0 = self._p
        pend0 = self._pending
        ok = True
        try:
            for _ in range(2):
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's watchdog thread keeps querying events
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._generation()  # flips self._p during capture (nothing ran)
                    self._join_side()   # the side-stream finish joins inside the graph
                graphs.append(g)
        except Exception as e:  # noqa: BLE001 -- any capture failure -> eager generations
            import sys
            print(f"soup graph capture failed ({type(e).__name__}: {e}); running eagerly", file=sys.stderr)
            ok = False
        self._p = p0
        self._pending = pend0
        if ok and self.dist.enabled and validate:
            ok = self._validate_graphs(graphs if p0 == 0 else graphs[::-1])
        if self.dist.enabled:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            ok = bool(flag.item())
        if not ok:
            self._graphs = None
            return False
        # graphs[k] was captured with parity p0 ^ k; index them by parity
        self._graphs = graphs if p0 == 0 else graphs[::-1]
        self._capture_chunk(s, p0, pend0)
        return True

    @staticmethod
    def _chunk_sizes():
        """Generations per multi-generation graph (SRNN_GRAPH_CHUNKS, even sizes): an evolve
        of K generations replays the largest that fit, so a short timed region pays few
        launches and few finish launches (16 + 4 for K = 20 instead of 8 + 8 + 4 singles)."""
        v = os.environ.get("SRNN_GRAPH_CHUNKS") or os.environ.get("SRNN_GRAPH_CHUNK") or "16,8,4,2"
        return sorted({int(x) for x in v.split(",") if int(x) >= 2 and int(x) % 2 == 0}, reverse=True)

    def _capture_chunk(self, s, p0, pend0):
        self._chunks = []
        for G in self._chunk_sizes():
            ch = self._capture_chunk_g(s, p0, pend0, G)
            if ch is None:
                break
            self._chunks.append(ch)
        self._chunk = self._chunks[0] if self._chunks else None

    def _capture_chunk_g(self, s, p0, pend0, G):
        """A graph of G consecutive generations (G even: it starts and ends at parity
        p0) replayed as one launch, removing the per-generation graph-launch gap;
        validated bitwise against G eager generations (all ranks agree or none use it)."""
        ok = True
        gc = torch.cuda.CUDAGraph()
        flags0 = (self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin)
        try:
            with torch.cuda.graph(gc, stream=s, capture_error_mode="thread_local"):
                for _ in range(G):
                    self._generation()
                self._join_side()
        except Exception as e:  # noqa: BLE001
            import sys
            print(f"multi-generation graph capture failed ({type(e).__name__}: {e})", file=sys.stderr)
            ok = False
        self._p, self._pending = p0, pend0
        self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin = flags0
        if ok:
            ok = self._validate_replay(lambda: gc.replay(), G, parity_after=p0)
        if self.dist.enabled:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            ok = bool(flag.item())
        return (gc, p0, G) if ok else None

    def release_graphs(self):
        """Drop the captured graphs (before tearing down the process group: an RCCL
        communicator must not be destroyed while graph executables still reference it)."""
        if self._graphs is not None or self._chunks:
            torch.cuda.synchronize(self.device)
            for g in (self._graphs or []) + [c[0] for c in self._chunks]:
                g.reset()
            self._graphs = None
            self._chunk = None
            self._chunks = []

    def _validate_graphs(self, graphs) -> bool:
        def replay():
            for _ in range(2):
                graphs[self._p].replay()
                self._p = 1 - self._p
        return self._validate_replay(replay, 2)

    def _validate_replay(self, replay, gens: int, parity_after=None) -> bool:
        """Run ``gens`` eager generations from the current state, restore it, run
        ``replay`` (the captured equivalent), compare bitwise, restore again."""
        state = self._state()
        saved = [t.clone() for t in state]
        p0, pend0, t0 = self._p, self._pending, self.time
        flags0 = (self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin)
        for _ in range(gens):
            self._generation()
        self._join_side()
        torch.cuda.synchronize(self.device)
        flags1 = (self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin)
        eager = [t.clone() for t in state]
        for t, v in zip(state, saved):
            t.copy_(v)
        self._p, self._pending = p0, pend0
        self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin = flags0
        replay()
        if parity_after is not None:
            self._p = parity_after
        self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin = flags1
        torch.cuda.synchronize(self.device)
        # compare the semantic state only: exchange-buffer row order and the attack
        # lists' link order follow atomics and legitimately differ between runs
        keep = {id(t) for t in self._bufs} | {id(getattr(self, k)) for k in (
            "uid", "next_uid", "_gen_ring", "counts", "census", "loss", "respawn", "action", "counterpart",
            "flags32", "ovf") if isinstance(getattr(self, k, None), torch.Tensor)}
        same = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8))
                   for x, y in zip(state, eager) if id(x) in keep)
        for t, v in zip(state, saved):
            t.copy_(v)
        self._p, self._pending, self.time = p0, pend0, t0
        self._lists_ready, self._mask_src, self._packed, self._perms_ready, self._pending_fin = flags0
        torch.cuda.synchronize(self.device)
        return same
