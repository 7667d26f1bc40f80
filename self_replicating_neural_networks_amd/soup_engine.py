"""Device soup engine: one fused generation pipeline over a (sharded) population.

Replaces the per-particle Python loop of ``Soup.evolve`` (reference code/soup.py:51-87)
with a *synchronous* (Jacobi) generation computed for every particle at once.

Single rank (one launch per generation, captured as hipGraphs of 16/8/4/2 generations):
``OP_SOUP_GEN`` evolves every particle (attacks received in ascending attacker-slot order
with generation-start attacker weights, ``learn_from_severity`` epochs on the teacher's
generation-start samples, ``train`` self-train epochs, divergence / zero respawn with the
newborn re-initialised in place -- reference :77-86), links the NEXT generation's attacks
(decisions are a pure function of (seed, slot, generation)) and classifies the stored row
(the census, reference code/soup.py:89-103); one finish launch per graph numbers the
newborns with globally sequential uids (reference S13).

Sharded over R ranks (one process per GPU, RCCL over xGMI), ``exchange="alltoall"``
(csrc/srnn_shard.hip): every rank decides only its OWN slots, one generation ahead, and
tells the owners of its remote victims (notices) and of its remote teachers (requests);
int64 slots, O(local) memory and work, so a soup can fill every GPU's HBM.  The shipped
schedule (``ExecConfig.x2_schedule = "serial"``) runs a generation on ONE stream:

    pack_t        finish of t-1 (census partials, newborn counts) + decisions of t+1
                  (links, notices, requests) + the rows of exchange t
    all-to-all_t  one RCCL all-to-all of fixed-size blocks on the soup's own communicator
    evolve_t      ONE launch: post_t's workgroups first (uids of t-1's newborns, global
                  census, received notices / requests of t+1), then n/64 evolve waves in
                  which the lanes of remote-dependent slots take the remote list's entries

Each cross-queue dependency inside a hipGraph costs ~10 us (profiles/r3b), which is why the
alternative ``"overlap"`` schedule (local slots on a side stream beside pack ->
all-to-all -> remote evolve, post on a third stream) measured slower and is opt-in.
``exchange="allgather"`` instead all-gathers every rank's rows each generation (the X01
pattern of SURVEY §2.5: one collective, every rank holds the whole table and recomputes
every slot's decisions; populations < 2^32).  Results are bitwise independent of R for
both (tests/test_dist_gloo.py).

``dtype`` selects the storage of the weight tables and exchange rows (fp32, bf16, fp16;
arithmetic is fp32 -- SURVEY §7.7).

Differences from the sequential reference (tested statistically): particle k does not see
the effects of particles < k within the same generation; every read is from the
generation-start weights.  ``Soup(mode="sequential")`` / ``SequentialSoupEngine`` keep the
exact reference order.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, Optional

import torch

from .arch import ArchSpec
from .config import ExecConfig
from .ops import _lib
from .ops import kernels as K
from .parallel.dist import Dist
from .population import counts_dict

ACTION_NAMES = {0: None, 1: "attacking", 2: "learn_from", 3: "train_self"}
RESPAWN_NAMES = {1: "divergent_dead", 2: "zweo_dead"}  # sic, reference code/soup.py:84

# list entries are uint32 (csrc/srnn_abi.h): a single-rank or all-gather soup addresses its
# slots directly; a sharded all-to-all soup addresses local rows + received rows per rank
MAX_SLOTS_DIRECT = 2 ** 32 - 2
# rows of a reference-order generation per rank (int32 version codes 2j / 2j+1, csrc/srnn_ordered.h)
ORDERED_MAX_ROWS = 2 ** 30 - 1
X2_ERRORS = {1: "exchange capacity overflow (rows, notices or requests dropped)",
             4: "exchange protocol mismatch (row tag / slot range)"}
# reference-order error bits (csrc/srnn_ordered.h ord::ERR_*), sticky over an engine's life
ORD_ERRORS = {2: "an attack output past the recompute depth left unstored (marking bug)",
              4: "a turn that never ran (scheduling bug)",
              8: "a ready-queue entry never written (scheduling bug)",
              16: "a level's exchange records overflowed the send buffer (sharded; sizing bug)",
              32: "a one-rank timing model of a sharded generation (SRNN_ORDSH_EMULATE) ran only 1/R of the turns",
              64: "an in-run plan workgroup gave up at a phase barrier (scheduling bug)",
              128: "a counter-ordered graph waited > 2 s for the other stream (SRNN_F_ORD_SYNC)"}
ORD_ERR_EMULATED = 32


def describe_ordered_error(bits: int) -> str:
    return "; ".join(f"{b}: {msg}" for b, msg in ORD_ERRORS.items() if bits & b) or f"error bits {bits}"


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _cap(mean: float) -> int:
    """Per-peer capacity of an exchange section for a Poisson-ish load of this mean."""
    return int(mean * 1.2 + 6.0 * math.sqrt(max(mean, 0.0)) + 32)


def x2_capacities(n_total: int, world: int, attacking_rate: float, learn_from_rate: float,
                  segment: int = 0):
    """(rows, notices, requests) per peer block of the sharded exchange: worst (r, q) pair of
    the expected loads.  Row i of rank r goes to rank q when i attacks a victim owned by q
    (notice one generation ahead) or a learner of q picked i as teacher (request).  Partners
    are uniform over the slot's sub-soup (``segment``) or the whole population, so segments
    spanning several shards concentrate the traffic on neighbouring ranks."""
    R = world
    ar, lr_ = max(attacking_rate, 0.0), max(learn_from_rate, 0.0)
    seg = int(segment or 0) or n_total
    bounds = [((r * n_total) // R, ((r + 1) * n_total) // R) for r in range(R)]
    overlap = [[0.0] * R for _ in range(R)]  # sum over slots i of shard r of |S_i n shard_q| / |S_i|
    starts = sorted({(lo // seg) * seg for lo, _ in bounds[1:]}) if seg < n_total else [0]
    for s0 in starts:
        s1 = min(s0 + seg, n_total)
        inter = [max(0, min(hi, s1) - max(lo, s0)) for lo, hi in bounds]
        for r in range(R):
            if inter[r]:
                for q in range(R):
                    overlap[r][q] += inter[r] * inter[q] / (s1 - s0)
    notices = requests = 0.0
    for r in range(R):
        for q in range(R):
            if q != r:
                notices = max(notices, ar * overlap[r][q])
                requests = max(requests, lr_ * overlap[r][q])
    n_max = -(-n_total // R)
    cn, cq = min(_cap(notices), n_max + 32), min(_cap(requests), n_max + 32)
    # a block's rows are the replies (<= cq) then the noticed attackers (<= cn): never more
    return cq + cn, cn, cq


def _finish_batch(nb: int, chunks) -> int:
    """Generations whose block stats share one batched-finish ring (single rank): the largest
    graph chunk, fewer when one generation's stats (32 B per 64-row block) pass 512 MB."""
    return max(1, min(max(list(chunks) or [1]), (512 << 20) // (nb * 32)))


def ordered_bytes(spec: ArchSpec, n: int, dtype=torch.float32, epochs: int = 0, plan_sets: int = 1) -> int:
    """Device bytes of the reference-order generation's buffers for ``n`` planned turns
    (SoupEngine._init_ordered): the stored attack outputs W3 (n rows of the table), and per plan
    set the turns' source codes + levels, the stored flags and the pending records (csrc/srnn_ordered.h
    o_src), the turns' record list, the control words, and -- nibble Weightwise nets with shuffled
    SGD on the device -- the pending records' epoch permutations (``epochs`` = train +
    learn_from_severity; 0: no table).  ``plan_sets``: 2 for a pipelined single-rank engine (the
    next generation's plan is built while this one runs)."""
    n1 = max(int(n), 1)
    rb = spec.PP * torch.empty((), dtype=dtype).element_size()
    rec = _lib.ord_rec_total(n1)
    per_set = 4 * _lib.ord_src_words(n1) + 4 * n1 + 4 * _lib.ORD_CTL_WORDS
    if spec.kind == "weightwise" and spec.P <= 16 and epochs > 0 and (n + 4096) * epochs * 8 <= (2 << 30):
        per_set += 2 * rec * epochs * 8  # permutation table: pending records + critical roots
    return int(n * rb + plan_sets * per_set)


def sharded_ordered_bytes(spec: ArchSpec, n_total: int, world: int, dtype=torch.float32) -> int:
    """Device bytes one rank adds for a reference-order soup sharded over ``world`` ranks
    (csrc/srnn_ordered_sh.h, SoupEngine._init_ordered): every rank plans ALL n_total turns and holds
    the version tables of all rows -- W3 and the E versions (_fw) -- plus the replicated attack lists
    of both parities and one level's exchange records (send: its own turns, receive: every rank's).
    No permutation table (the level launches draw inline)."""
    rb = spec.PP * torch.empty((), dtype=dtype).element_size()
    N = max(int(n_total), 1)
    cap = max(-(-N // world), 1)
    recb = 16 + 2 * rb  # csrc ordsh::rec_bytes
    b = ordered_bytes(spec, N, dtype, epochs=0, plan_sets=1)
    b += N * rb                      # _fw: the E version of every row
    b += 2 * 2 * N * 4 + 16          # replicated heads + nexts of both parities, level-pack counters
    b += (1 + world) * cap * recb    # send + receive records of one level
    return int(b)


def engine_bytes(spec: ArchSpec, n_total: int, world: int = 1, dtype=torch.float32, exchange: str = "alltoall",
                 attacking_rate: float = 0.1, learn_from_rate: float = 0.1, segment: int = 0,
                 diagnostics: bool = True, order: str = "synchronous", epochs: int = 0,
                 ord_pipeline: bool = True) -> int:
    """Device bytes one rank of a SoupEngine allocates (the tensors of ``__init__``);
    ``order="sequential"`` adds the reference-order generation's buffers (``ordered_bytes``,
    ``epochs`` = train + learn_from_severity for its permutation table; two plan sets with
    ``ord_pipeline``).  A sharded reference-order soup runs on the all-gather layout whatever
    ``exchange`` says, with the replicated plan of ``sharded_ordered_bytes``."""
    R = world
    n = -(-n_total // R)
    rb = spec.PP * torch.empty((), dtype=dtype).element_size()
    nb = max(-(-n // 64), 1)
    b = 2 * n * rb + n * 8 + n * 1 + 2 * n * 4 + nb * 8 + 8 * 4  # tables, uid, respawn, heads, ballots
    if diagnostics:
        b += n * (1 + 8 + 4)  # action, counterpart, loss
    if R > 1 and exchange == "alltoall" and order != "sequential":
        cr, cn, cq = x2_capacities(n_total, R, attacking_rate, learn_from_rate, segment)
        xb = rb + 16
        blk = -(-(_lib.X2_HDR * 8 + cr * xb + cn * 16 + cq * 8) // 16) * 16
        nr = max(min(n, R * (cn + cq)), 1)
        b += 2 * (n + R * cr) * 4            # links of local + received rows
        b += 2 * max(-(-n // 32), 1) * 4     # remote-dependent bits
        b += 2 * 2 * nr * 4                  # remote lists
        b += 2 * R * cr * 8 + 2 * R * cn * 4 + R * cq * 4  # received-row slots, notice / request lists
        b += 2 * nb * 32                     # block stats of two generations
        b += 2 * R * blk                     # send + receive buffers
    elif R > 1:
        b += 2 * n_total * 4 + n_total * rb + n * 4 + nb * 32  # links per global slot, gathered table, row flags
    else:
        b += 2 * n * 4 + nb * 32  # links, block stats
        # the batched-finish ring, sized as SoupEngine._init_single_or_allgather sizes it
        b += _finish_batch(nb, ExecConfig().resolved().graph_chunks) * (nb * 8 + 2) * 4
    if order == "sequential":
        if R > 1:
            b += sharded_ordered_bytes(spec, n_total, R, dtype)
        else:
            b += ordered_bytes(spec, n, dtype, epochs, plan_sets=2 if ord_pipeline else 1)
    return int(b)


def plan_population(spec: ArchSpec, dtype=torch.float32, exchange: str = "alltoall", world: int = 1,
                    hbm_bytes: int = 288 * 10 ** 9, fill: float = 0.9, attacking_rate: float = 0.1,
                    learn_from_rate: float = 0.1, diagnostics: bool = False, segment: int = 0,
                    order: str = "synchronous", epochs: int = 0) -> Dict:
    """The largest population whose per-rank engine (``engine_bytes``) fits ``fill`` of each
    GPU's HBM (288 GB HBM3E per MI355X), and what limits it: the HBM, or the uint32 attack-list
    entries (single-rank / all-gather soups address < 2^32 slots; a sharded all-to-all soup
    < 2^32 local + received rows per rank).  HBM-filling soups run without the per-row
    diagnostics columns (``diagnostics=False``, 13 B per row); the returned ``engine_kwargs``
    are what the planned ``SoupEngine`` must be built with for the plan to hold."""
    kw = dict(world=world, dtype=dtype, exchange=exchange, attacking_rate=attacking_rate,
              learn_from_rate=learn_from_rate, diagnostics=diagnostics, segment=segment, order=order, epochs=epochs)
    budget = fill * hbm_bytes
    lo, hi = 1, 1 << 50
    while lo < hi:  # largest n_total with engine_bytes <= budget
        mid = (lo + hi + 1) // 2
        if engine_bytes(spec, mid, **kw) <= budget:
            lo = mid
        else:
            hi = mid - 1
    n_fit = lo
    if world > 1 and exchange == "alltoall" and order != "sequential":
        # local rows + received rows of a rank stay below 2^32 - 1 (capacities as _init_x2
        # computes them, segment included)
        lo2, hi2 = 1, 1 << 50
        while lo2 < hi2:
            mid = (lo2 + hi2 + 1) // 2
            cr = x2_capacities(mid, world, attacking_rate, learn_from_rate, segment)[0]
            if -(-mid // world) + world * cr < _lib.NIL:
                lo2 = mid
            else:
                hi2 = mid - 1
        limit = lo2
    else:
        limit = MAX_SLOTS_DIRECT
    why = "uint32 list entries"
    # (every rank of a sharded reference-order soup plans all n_total turns: the int32 version
    # codes bound the whole soup, not a shard)
    if order == "sequential" and ORDERED_MAX_ROWS < limit:
        limit, why = ORDERED_MAX_ROWS, "ordered version codes (int32)"
    n_total = min(n_fit, limit)
    return dict(n_total=n_total, n_total_fit=n_fit, limited_by="hbm" if n_fit <= limit else why,
                bytes_per_gpu=engine_bytes(spec, n_total, **kw),
                bytes_per_particle_per_gpu=engine_bytes(spec, n_total, **kw) / max(n_total, 1),
                world=world, exchange=exchange, dtype=str(dtype).replace("torch.", ""),
                engine_kwargs=dict(dtype=dtype, exchange=exchange, diagnostics=diagnostics, order=order))


class SoupEngine:
    """Population-sharded soup on one device per rank."""

    def __init__(self, spec: ArchSpec, n_total: int, params: Dict, device="cpu", seed: int = 0,
                 lr: float = 0.01, shuffle: bool = True, dist: Optional[Dist] = None, weights=None,
                 dtype: torch.dtype = torch.float32, exchange: str = "alltoall", local_weights=None,
                 init: bool = True, diagnostics: bool = True, execution: Optional[ExecConfig] = None,
                 order: str = "synchronous"):
        """``weights``: the whole population's initial rows [n_total, >= P] (every rank
        takes its slice); ``local_weights``: only this rank's rows [hi - lo, >= P];
        ``init=False``: leave the rows for the caller to fill (the streaming checkpoint
        loader writes them straight into the device table); ``diagnostics=False``: no
        per-row action / counterpart / loss columns (HBM-filling soups); ``execution``: schedules
        and kernel families (config.ExecConfig; its environment variables override it);
        ``order``: ``"sequential"`` -- the reference's in-place, index-ordered generation
        (code/soup.py:51-87) scheduled by dependency level on the device (OP_SOUP_ORDERED,
        bitwise the serial loop; single rank, lane-template shapes) -- or ``"synchronous"``
        (Jacobi: every read from the generation-start table; any shape, sharded)."""
        if order not in ("synchronous", "sequential"):
            raise ValueError(f"order must be 'synchronous' or 'sequential', got {order!r}")
        self.order = order
        self.execution = (execution or ExecConfig()).resolved()
        self.spec = spec
        self.n_total = int(n_total)
        self.params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=0, learn_from_severity=1)
        self.params.update(params or {})
        self.device = torch.device(device)
        self.seed = int(seed)
        self.lr = float(lr)
        self.shuffle = bool(shuffle)
        self.dist = dist or Dist()
        if exchange not in ("alltoall", "allgather"):
            raise ValueError(f"exchange must be 'alltoall' or 'allgather', got {exchange!r}")
        self.exchange = exchange
        if self.device.type == "cuda" and self.dist.enabled:
            # the soup's own RCCL communicator: its collectives can live inside hipGraphs
            self.dist.enable_native_comm(self.device)
        self.lo, self.hi = self.dist.shard(self.n_total)
        self.n = self.hi - self.lo
        # the reference order shards by replicated plan + per-level all-gathers (srnn_ordered_sh.h),
        # on the all-gather exchange's buffers
        self.x2 = self.dist.enabled and exchange == "alltoall" and order != "sequential"
        if not self.x2 and self.n_total > MAX_SLOTS_DIRECT:
            raise ValueError(f"a single-rank or all-gather soup addresses at most {MAX_SLOTS_DIRECT} slots "
                             "(uint32 attack-list entries); shard it with exchange='alltoall'")
        seg = int(self.params.get("segment", 0) or 0)
        if seg and self.n_total % seg:
            raise ValueError("population size must be a multiple of the sub-soup segment")
        self.dtype = dtype
        self.dtype_code = K.dtype_code(dtype)
        dev, PP = self.device, spec.PP
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        # this rank's rows, ping-pong: generation t reads buf[p], writes buf[1-p]
        self._bufs = [torch.zeros((self.n, PP), dtype=dtype, device=dev) for _ in range(2)]
        self._p = 0
        nb = max(-(-self.n // 64), 1)
        self.uid = torch.arange(self.lo, self.hi, dtype=torch.int64, device=dev)
        self.next_uid = torch.full((1,), self.n_total, dtype=torch.int64, device=dev)
        # generation counter as a 2-slot ring indexed by the ping-pong parity: a launch
        # reads slot _p and the generation-closing kernel writes slot 1-_p, so blocks of
        # one launch never race on it (gen_dev is the current slot)
        self._gen_ring = torch.ones(2, dtype=torch.int32, device=dev)
        self.time = 0
        self.census = torch.zeros(5, dtype=torch.int64, device=dev)
        self.counts = torch.zeros(6, dtype=torch.int64, device=dev)  # classes[5] + respawns
        self.respawn = torch.zeros(self.n, dtype=torch.int8, device=dev)
        if diagnostics:
            self.action = torch.zeros(self.n, dtype=torch.int8, device=dev)
            self.counterpart = torch.full((self.n,), -1, dtype=torch.int64, device=dev)
            self.loss = torch.zeros(self.n, dtype=torch.float32, device=dev)
        else:
            self.action = self.counterpart = self.loss = None
        # attack lists, one buffer per parity (entries: csrc/srnn_abi.h); links of an
        # all-gather soup are indexed by global slot, of an all-to-all soup by local row +
        # received row
        self.generic = _lib.is_generic(spec, _lib.OP_SOUP_GEN, self.dtype_code)
        n_links = self.n_total if (self.dist.enabled and not self.x2) else self.n
        self.heads = [torch.full((self.n,), -1, **i32) for _ in range(2)]
        self._lists_ready = False   # heads[_p] already holds this generation's attacks
        self._scratch = None
        if self.device.type == "cuda" and _lib.is_generic(spec, _lib.OP_SOUP_EVOLVE, self.dtype_code):
            self._scratch = torch.empty(_lib.generic_scratch_bytes(spec, self.n, self.dtype_code),
                                        dtype=torch.uint8, device=dev)
        self.ballots = torch.zeros(nb, **i64)       # respawn ballot per 64-row block (unfused evolve)
        self.rowflags = None                          # per-row respawn flags (all-gather exchange)
        self.err = torch.zeros(1, **i32)              # exchange error bits (X2_ERRORS)
        self.stats = False          # census every generation
        self.stats_with_sec = True
        self.recorder = None        # full reference-schema state recorder (compat Soup)
        self.trajectory = None      # sampled TrajectoryRecorder (large soups)
        self.metrics = None         # MetricsWriter (JSONL per-generation metrics)
        self._metrics_uid = None
        self._graphs = None
        self._chunk = None          # (graph of G generations, start parity, G): the largest
        self._chunks = []           # every captured multi-generation graph, largest first
        self._arg_cache = {}
        self._pending = False       # sharded: uids of the last generation's newborns not yet assigned
        self.overlap = False        # sharded all-to-all: the exchange runs beside the local evolve
        if self.x2:
            self._init_x2(n_links)
        else:
            self.nexts = [torch.full((n_links,), -1, **i32) for _ in range(2)]
            self._init_single_or_allgather(nb)
        self.cfg = _lib.make_cfg(spec, self.dtype_code)
        self._ord_pipe = False      # reference order: plan built one generation ahead (_init_ordered)
        self._ord_side = None       # ... on this side stream (device, mode "stream")
        self._ord_mode = "off"      # ... by the run launch ("kernel") or the side stream ("stream")
        self._ord_census_side = False  # ... with the census of each generation beside the next one
        self._census_due = None
        self._ord_decouple = False  # ... multi-generation graphs as two counter-ordered graphs (SRNN_F_ORD_SYNC)
        self._osync = None
        self._sync = False
        if order == "sequential":
            self._init_ordered()
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
        self._perm_table()  # allocated here, never inside a graph capture
        if self._ord_pipe:
            self._perm_table(1)

    # ------------------------------------------------------------------ state
    def _init_single_or_allgather(self, nb):
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        # one launch (+ a one-workgroup finish) per generation: OP_SOUP_GEN; shapes without a
        # templated kernel run on the runtime-shape engine: decide -> evolve -> respawn -> census
        self.fused = not self.dist.enabled and not self.generic
        self._blockstat = torch.zeros(nb * 8, **i32)  # u64[4] per 64-row block
        self._done = torch.zeros(1, **i32)
        # where the finish of a single-rank fused generation on a GPU runs (census reduction +
        # newborn uids): "batch" -- the generation kernel advances the counter itself, the
        # block stats of up to G generations go to a ring and ONE launch finishes them all
        # (per graph chunk / evolve call); "serial" -- a finish launch after every generation
        fm = self.execution.finish_mode
        if self.device.type != "cuda" or self.dist.enabled or not self.fused:
            fm = "serial"
        self.finish_mode = fm
        # the ring holds 32 B per 64-row block per pending generation: at HBM-filling sizes
        # (2e9 rows = 1 GB per generation) fewer generations share one finish launch
        self._batch = _finish_batch(nb, self._chunk_sizes())
        # (+ 8 bytes per generation: its newborn count, accumulated by the generation waves)
        self._bs_ring = torch.zeros((self._batch, nb * 8 + 2), **i32) if fm == "batch" else None
        self._pending_fin = 0  # batch mode: generations whose finish is still due
        if self.dist.enabled:  # all-gather exchange
            self.full = torch.zeros((self.n_total, self.spec.PP), dtype=self.dtype, device=dev)
            self.stats_all = torch.zeros(self.dist.world * 6, dtype=torch.int64, device=dev)
            self.rowflags = torch.zeros(max(self.n, 1), **i32)

    # synchronous generations up to this many slots per launch draw their SGD permutations in a
    # launch of their own (profiles/r5a_*: 12.5k 0.0397 vs 0.0426 ms, 25k 0.0432 vs 0.0444)
    PERM_TABLE_MAX_N = 32768

    def _use_perm_table(self) -> bool:
        """ExecConfig.perm_table, auto (None): the reference order's critical-path turns (pending
        records and the roots with consumers, k_ord_ptab: ~10 % of the slots), and synchronous
        generations of at most PERM_TABLE_MAX_N slots per launch -- latency-bound, where the lone
        chains gain more from a permutation-free SGD loop than the table launch (k_perm_table)
        costs; above that the launch costs more than it removes (MI355X, profiles/r4b_*, r5a_*)."""
        pt = self.execution.perm_table
        if pt is not None:
            return bool(pt)
        return self.order == "sequential" or self.n <= self.PERM_TABLE_MAX_N

    def _perm_table(self, q: int = 0):
        """The generation's SGD epoch permutations, precomputed by one launch before the
        generation kernel (k_perm_table; nibble Weightwise nets with shuffle, on the device):
        [severity + train][n] uint64, reallocated when the epoch count grows.  None where the
        kernels draw them inline (host, other shapes, > 2 GB of table).  ``q``: the plan set of a
        pipelined reference-order engine (the next generation's table is drawn while this one
        runs)."""
        if (self.device.type != "cuda" or self.spec.kind != "weightwise" or self.spec.P > 16 or not self.shuffle
                or self.generic or not self._use_perm_table()):
            return None
        if self.order == "sequential" and self.dist.enabled:
            return None  # (the sharded reference order's level launches draw their permutations inline)
        E = max(int(self.params.get("train", 0)), 0) + max(int(self.params.get("learn_from_severity", 1)), 0)
        if E <= 0 or (self.n + 4096) * E * 8 > (2 << 30):
            return None
        # (reference order: the pending records' rows and the critical roots' rows, csrc k_ord_ptab)
        rows = 2 * _lib.ord_rec_total(self.n) if self.order == "sequential" else self.n
        name = "_ptab1" if q else "_ptab"
        t = getattr(self, name, None)
        if t is None or t.numel() < rows * E:
            t = torch.zeros(rows * E, dtype=torch.int64, device=self.device)
            setattr(self, name, t)
        return t

    def _init_ordered(self):
        """Buffers of the reference-order generation (csrc/srnn_ordered.h): attack outputs,
        per-turn source versions + level, consumer lists and records, control words.  Sharded
        (srnn_ordered_sh.h): every rank plans all n_total turns and keeps the version tables of
        all rows (E rows, stored attack outputs) next to the gathered generation-start table."""
        dev_side = self.device.type != "cpu"
        if not _lib.supports(self.spec, _lib.OP_SOUP_ORDERED, dev_side, self.dtype_code):
            raise NotImplementedError(
                f"no scheduled reference-order generation for {self.spec} on {self.device.type}: it exists for "
                "the lane-per-particle template shapes (host and device) and the big aggregating nets (device, "
                "csrc/srnn_bignet.h); SequentialSoupEngine runs the same order for any shape on the host, "
                "SoupEngine(order='synchronous') any shape on the device")
        sharded = self.dist.enabled
        N = self.n_total if sharded else self.n  # turns planned on this rank
        if N > ORDERED_MAX_ROWS:
            raise ValueError("reference-order generations address < 2^30 slots")
        if sharded and not _lib.supports(self.spec, _lib.OP_SOUP_ORDERED_SH, dev_side, self.dtype_code):
            raise NotImplementedError(f"no sharded reference-order generation for {self.spec}")
        dev = self.device
        C = int(self.execution.order_levels)
        self.order_levels = C
        self._ord_n = N
        self._abuf = torch.zeros((N, self.spec.PP), dtype=self.dtype, device=dev)
        # [N][4] source codes + level | [N] stored-attack flags | [N] consumer lists | pending records
        self._osrc = torch.zeros(_lib.ord_src_words(N), dtype=torch.int32, device=dev)
        self._olist = torch.zeros(max(N, 1), dtype=torch.int32, device=dev)  # each turn's record
        if sharded:
            i32 = dict(dtype=torch.int32, device=dev)
            self._fw = torch.zeros((N, self.spec.PP), dtype=self.dtype, device=dev)  # E versions of all rows
            self._sh_heads = [torch.full((N,), -1, **i32) for _ in range(2)]  # replicated attack lists
            self._sh_nexts = [torch.full((N,), -1, **i32) for _ in range(2)]
            self._sh_cnt = torch.zeros(4, **i32)
            rb = self.spec.PP * self._bufs[0].element_size()
            self._sh_recb = 16 + 2 * rb  # csrc ordsh::rec_bytes (16-byte slot header, two rows)
            cap = max(hi - lo for lo, hi in (self.dist.shard_of_rank(r, N) for r in range(self.dist.world)))
            self._sh_send = torch.zeros(max(cap, 1) * self._sh_recb // 8, dtype=torch.int64, device=dev)
            self._sh_recv = torch.zeros(self.dist.world * max(cap, 1) * self._sh_recb // 8, dtype=torch.int64,
                                        device=dev)
        self._octl = torch.zeros(_lib.ORD_CTL_WORDS, dtype=torch.int32, device=dev)
        # single rank: the plan of generation t+1 is built while generation t runs, into the other of
        # two plan sets, indexed like the attack lists by the ping-pong parity (ExecConfig.ord_pipeline):
        # "stream" -- by OP_ORD_PLAN on a side stream, joined before the next run (the join costs ~10 us
        # of idle queue inside a hipGraph, the plan ~40 us of launches: profiles/r6a); "kernel" -- by
        # the last workgroups of generation t's run launch (SRNN_F_ORD_INPLAN; measured slower: grid
        # barriers between the plan phases cost more than the join; the host path plans after the
        # generation)
        mode = self.execution.ord_pipeline
        self._ord_pipe = not sharded and mode != "off"
        self._ord_mode = mode if self._ord_pipe else "off"
        self._osrc1 = self._olist1 = self._octl1 = None
        self._ord_side = None
        if self._ord_pipe:
            self._osrc1 = torch.zeros_like(self._osrc)
            self._olist1 = torch.zeros_like(self._olist)
            self._octl1 = torch.zeros_like(self._octl)
            if mode == "stream" and dev.type == "cuda":
                # (ord_graph_sync: the side stream's multi-generation graphs wait on the main stream's
                # counters and the other way round -- the two streams must not share a hardware queue;
                # the high-priority one is drawn from a queue pool of its own)
                self._ord_decouple = bool(self.execution.ord_graph_sync)
                self._ord_side = torch.cuda.Stream(dev, priority=-1 if self._ord_decouple else 0)
                self._osync = torch.zeros(4, dtype=torch.int32, device=dev)  # csrc ord::SYNC_*
        # (stream mode) the census of a generation's final rows runs on the side stream beside the
        # next generation's run (OP_ORD_CENSUS), leaving the close on the critical path only the
        # final rows, ballots and counter
        self._ord_census_side = (self._ord_side is not None and bool(self.execution.ord_census_side) and
                                 _lib.supports(self.spec, _lib.OP_ORD_CENSUS, True, self.dtype_code))
        self._census_due = None  # the block stats of a generation whose census is still to run
        self._rec_rows = None  # recording: every particle's state before any respawn

    def _ord_set(self, q: int):
        """Plan set q of the reference-order generation: (o_src, o_list, o_ctl)."""
        return (self._osrc, self._olist, self._octl) if q == 0 else (self._osrc1, self._olist1, self._octl1)

    def _ord_last(self) -> int:
        """The plan set of the last generation that ran (pipelined: the other parity's -- this
        parity's holds the next generation's plan, not run yet)."""
        return 1 - self._p if self._ord_pipe else 0

    def ordered_levels(self) -> Dict[str, int]:
        """Dependency levels of the last reference-order generation (a turn's level: 1 + its
        deepest producer's, 0 without one): turns per level for the first ``order_levels``
        levels, the turns deeper than those (``tail``), the deepest level, the turns that had
        producers (``pending``: on the device, run as continuations), the error bits (sticky over
        the engine's life: 2 -- an attack output past the recompute depth left unstored, 4 -- a
        turn that never ran, 8 -- a ready-queue entry never written), and how many attack outputs were stored for later turns (the others
        are recomputed by the turns that read them)."""
        C = self.order_levels
        n = self._ord_n
        osrc, _, octl = self._ord_set(self._ord_last())
        lv = osrc[:4 * n].view(n, 4)[:, 3] if n else osrc[:0]
        hist = torch.bincount(lv.clamp(0, _lib.ORD_MAX_LEVELS).long(), minlength=_lib.ORD_MAX_LEVELS + 1)
        hist = hist.cpu().tolist()
        err = self.ordered_error() | (4 if n and int((lv < 0).sum().item()) else 0)
        stored = int(osrc[4 * n:5 * n].sum().item()) if n else 0
        return dict(levels=hist[:C], tail=sum(hist[C:]), max_level=int(lv.max().item()) if n else 0,
                    pending=n - hist[0], error=err, stored_attacks=stored)

    # phases of a turn in a library built with -DSRNN_ORD_TRACE_FINE (csrc/srnn_ordered.h)
    TRACE_PHASES = ("own row", "attack", "teacher row", "learn_from", "self-train", "stores", "publish")

    def ordered_trace(self, on: bool = True, slots: int = 2) -> None:
        """Record, on the device, when each turn of the next reference-order generations starts
        and ends (s_memrealtime, 100 MHz; debug: a few stores per turn).  Read it with
        ``ordered_timeline()``.  ``slots=10``: a library built with -DSRNN_ORD_TRACE_FINE also stamps
        the phases of every turn (TRACE_PHASES) and the shader clock over its self-train."""
        if self.order != "sequential" or self.device.type != "cuda":
            raise ValueError("the turn trace is a device reference-order generation's")
        self._otrace_slots = int(slots)
        self._otrace = (torch.zeros(self._otrace_slots * max(self.n, 1), dtype=torch.int64, device=self.device)
                        if on else None)
        self._arg_cache.clear()

    def ordered_timeline(self) -> Dict[str, list]:
        """The last traced generation per dependency level: turns, first start and last end (us
        after the generation's first turn started), mean / max turn duration (us), and the hand-off
        of each dependent turn -- its start minus its last producer's end (publish, ready queue,
        claim, acquire, record and level reads) -- mean / max per level.  ``critical``: the chain
        that ends last, turn by turn (start, end, hand-off before it)."""
        n = self.n
        S = getattr(self, "_otrace_slots", 2)
        raw = self._otrace.view(-1, S).cpu().double()[:n]
        t = raw[:, [0, 7 if S >= 8 else S - 1]]
        osrc, _, octl = self._ord_set(self._ord_last())
        src = osrc.cpu()
        lv = src[:4 * n].view(n, 4)[:, 3]
        ok = t[:, 0] > 0
        t0 = t[ok, 0].min()
        us = (t - t0) / 100.0
        # the pending records: turn, producers (csrc/srnn_ordered.h pend / rec_cap)
        rec_total = _lib.ord_rec_total(n)
        cap = rec_total // _lib.ORD_NPART
        base = 6 * n
        ctl = octl.cpu().tolist()
        prods = {}
        for part in range(_lib.ORD_NPART):
            for q in range(part * cap, part * cap + int(ctl[2 * _lib.ORD_MAX_LEVELS + 3 + part])):
                r = src[base + _lib.ORD_REC * q: base + _lib.ORD_REC * (q + 1)].tolist()
                prods[int(r[0])] = [int(x) for x in r[2:2 + int(r[1])]]
        hand = {k: float(us[k, 0] - max(us[p, 1] for p in ps)) for k, ps in prods.items() if ok[k]}
        out = {}
        for L in range(int(lv.max()) + 1):
            m = ok & (lv == L)
            if int(m.sum()) == 0:
                continue
            s, e = us[m, 0], us[m, 1]
            h = [hand[k] for k in torch.nonzero(m).flatten().tolist() if k in hand]
            out[L] = dict(turns=int(m.sum()), first_start=float(s.min()), last_start=float(s.max()),
                          last_end=float(e.max()), mean_us=float((e - s).mean()), max_us=float((e - s).max()),
                          handoff_mean_us=sum(h) / len(h) if h else None, handoff_max_us=max(h) if h else None)
        k = int(torch.argmax(torch.where(ok, us[:, 1], torch.full_like(us[:, 1], -1e30))))
        chain = []
        while True:
            step = dict(turn=k, level=int(lv[k]), start=float(us[k, 0]), end=float(us[k, 1]), handoff=hand.get(k))
            if S >= 8:  # phase durations (us) of the fine trace; the self-train's shader clock (GHz)
                ph = raw[k].tolist()
                step["phases"] = {name: (ph[i + 1] - ph[i]) / 100.0 for i, name in enumerate(self.TRACE_PHASES)}
                if S >= 10 and ph[5] > ph[4]:
                    step["train_clock_ghz"] = (ph[9] - ph[8]) / ((ph[5] - ph[4]) * 10.0)
                if S >= 12:
                    r = int(raw[k, 10].item()) if raw[k, 10] < 2 ** 62 else -1
                    step["ptab_row"] = r
                if S >= 36:  # each self-train epoch's duration (us)
                    ep = [x for x in ph[12:36] if x > 0] + [ph[5]]
                    step["epochs_us"] = [round((b - a) / 100.0, 2) for a, b in zip(ep, ep[1:])]
                    # the other turns that ran on the same SIMD (HW_ID + XCC_ID) during its self-train
                    hw = self._otrace.view(-1, S)[:n, 11].cpu()
                    simd = ((hw >> 32) << 16) | (hw & 0xFF30)  # xcc, se, sh, cu, simd (no wave slot / pipe)
                    mine = int(simd[k])
                    lo_t, hi_t = float(ph[4]), float(ph[5])
                    other = (simd == mine) & ok & (raw[:, 0] < hi_t) & (raw[:, 7] > lo_t)
                    other[k] = False
                    step["simd_neighbours"] = int(other.sum())
            chain.append(step)
            if k not in prods:
                break
            k = max(prods[k], key=lambda p: float(us[p, 1]))
        out["critical"] = chain[::-1]
        return out

    def ordered_error(self) -> int:
        """This rank's reference-order error bits (ORD_ERRORS), sticky over the engine's life (0:
        none); read without communicating (``ordered_error_all``: every rank's)."""
        if self.order != "sequential":
            return 0
        e = int(self._octl[_lib.ORD_ERRW].item())
        if self._octl1 is not None:
            e |= int(self._octl1[_lib.ORD_ERRW].item())
        return e

    def ordered_error_all(self) -> int:
        """The reference-order error bits of ANY rank, OR-ed (a sharded generation sets some bits
        on one rank only: its own rows' close, its own level's pack).  COLLECTIVE: every rank must
        call it, so every rank raises together instead of one leaving the others in a collective."""
        e = self.ordered_error()
        if not self.dist.enabled or self.order != "sequential":
            return e
        out = torch.zeros(self.dist.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into(out, torch.tensor([e], dtype=torch.int64, device=self.device))
        v = 0
        for x in out.cpu().tolist():
            v |= int(x)
        return v

    def _init_x2(self, n_links):
        dev, R = self.device, self.dist.world
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        self.fused = not self.generic
        self.finish_mode = "x2"
        # the big aggregating nets' row kernels evolve without a fused census
        bignet = self.spec.kind == "aggregating" and self.spec.P > 64 and not _lib.is_generic(
            self.spec, _lib.OP_SOUP_EVOLVE, self.dtype_code)
        self._evolve_census = not bignet
        # generation schedule: "serial" -- pack -> all-to-all -> ONE launch: post's workgroups +
        # the evolve of the local and the remote slots, on one stream (no cross-queue dependencies: each costs
        # ~10 us inside a graph, profiles/r3b); "overlap" -- the local slots on a side stream
        # beside pack -> all-to-all -> remote evolve, post on a third stream
        self.schedule = self.execution.x2_schedule
        # the lane kernels evolve both kinds of slot in one launch (bignet / runtime-shape: two)
        self._x2_both = not bignet and not _lib.is_generic(self.spec, _lib.OP_SOUP_EVOLVE, self.dtype_code)
        # single-launch generations: pack leaves, per 64-row block, how many remote-dependent slots
        # come before it (the launch's lanes on those slots take the remote list's entries)
        self.x_hpre = self.x_hgrp = None
        p = self.params
        cr, cn, cq = x2_capacities(self.n_total, R, float(p.get("attacking_rate", 0.1)),
                                   float(p.get("learn_from_rate", 0.1)), int(p.get("segment", 0) or 0))
        self.x_cr, self.x_cn, self.x_cq = cr, cn, cq
        rb = self.spec.PP * self._bufs[0].element_size()
        xb = rb + 16
        blk = _lib.X2_HDR * 8 + cr * xb + cn * 16 + cq * 8
        self.x_blk = -(-blk // 16) * 16
        if self.n + R * cr >= _lib.NIL:
            raise ValueError("local rows + received rows exceed the uint32 list entries: use more ranks")
        nb = max(-(-self.n // 64), 1)
        self.x_groups = int(min(max(-(-nb // 64), 1), 1024))
        self.nexts = [torch.full((self.n + R * cr,), -1, **i32) for _ in range(2)]
        self.x_dep = [torch.zeros(max(-(-self.n // 32), 1), **i32) for _ in range(2)]
        # a slot is remote-dependent through a received notice or one of its requests: at most
        # R * (cn + cq) of them per generation
        nr = max(min(self.n, R * (cn + cq)), 1)
        # timing model of R ranks on one GPU (SRNN_X2_EMULATE_REMOTE=<fraction>, world 1 only):
        # that fraction of the slots runs through the remote list after the exchange, as the
        # remote-dependent slots of a multi-rank soup do (same results: the rows are local)
        fr = self.execution.x2_emulate_remote if R == 1 else 0.0
        self.x_emul = int(min(max(fr, 0.0), 1.0) * 0xFFFFFFFF)
        if self.x_emul:
            nr = max(self.n, 1)
        self.x_rlist = [torch.zeros(2 * nr, **i32) for _ in range(2)]
        self.x_rcount = [torch.zeros(1, **i32) for _ in range(2)]
        self.x_rslot = [torch.zeros(R * cr, **i64) for _ in range(2)]
        self.x_satt = [torch.zeros(R * cn, **i32) for _ in range(2)]
        self.x_cno = [torch.zeros(R, **i32) for _ in range(2)]
        self.x_crq = [torch.zeros(R, **i32) for _ in range(2)]
        self.x_srep = torch.zeros(R * cq, **i32)
        self.x_nsrep = torch.zeros(R, **i32)
        self.x_part = torch.zeros(self.x_groups * 6, **i64)
        if self.schedule == "serial" and self._x2_both:
            self.x_hpre = torch.zeros(nb, **i32)
            self.x_hgrp = torch.zeros(self.x_groups, **i32)
        self.x_ctl = torch.zeros(8, **i32)
        self.x_bstat = [torch.zeros(nb * 4, **i64) for _ in range(2)]  # u64[4] per 64-row block
        # notice / request areas are -1 terminated (csrc/srnn_shard.hip): start all -1
        self.sendbuf = torch.full((R * self.x_blk,), 255, dtype=torch.uint8, device=dev)
        self.recvbuf = torch.zeros(R * self.x_blk, dtype=torch.uint8, device=dev)
        self.stats_all = torch.zeros(R * 6, **i64)
        self._primed = False
        self._xs = torch.cuda.Stream(dev) if dev.type == "cuda" else None  # local evolve
        self._xp = torch.cuda.Stream(dev) if dev.type == "cuda" else None  # post
        self.overlap = self._xs is not None and self.schedule == "overlap"

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

    def _stream(self, s=None):
        if self.device.type != "cuda":
            return None
        return ctypes.c_void_p((s or torch.cuda.current_stream(self.device)).cuda_stream)

    def _args(self, stream=None) -> _lib.SrnnArgs:
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
        a.world, a.rank = self.dist.world, self.dist.rank
        a.err = _p(self.err)
        if self.device.type == "cuda":
            a.dev = 1
            a.stream = self._stream(stream)
            if self._scratch is not None:
                a.scratch, a.scratch_bytes = _p(self._scratch), self._scratch.numel()
        return a

    def _census_fused(self) -> bool:
        return self.stats and self.spec.shuffler == "none"

    def _cache_key(self, *extra):
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        return (self._p, stream, tuple(sorted((k, str(v)) for k, v in self.params.items())), self.stats,
                self.stats_with_sec, self.lr, self.shuffle, self._pending_fin if not self.x2 else 0,
                self._sync) + extra

    # ------------------------------------------------------------------ single rank / all-gather
    def _gen_args(self):
        """Populated argument blocks of one generation (cached per parity / stream /
        params: building ctypes structs every generation costs host time)."""
        key = self._cache_key("gen")
        hit = self._arg_cache.get(key)
        if hit is not None:
            return hit
        a = self._args()
        a.W2 = _p(self.table_in)
        a.W = _p(self.rows_out)
        a.uid = _p(self.uid)
        a.ptab = _p(self._perm_table())
        a.heads, a.nexts = _p(self.heads[self._p]), _p(self.nexts[self._p])
        a.ballots = _p(self.ballots)
        a.action, a.counterpart, a.loss, a.respawn = _p(self.action), _p(self.counterpart), _p(self.loss), _p(self.respawn)
        a.uid_out = _p(self.uid)
        a.counts, a.uid_base = _p(self.counts), _p(self.next_uid)
        ca = None
        if self.dist.enabled:  # all-gather exchange
            a.recvbuf = _p(self.full)
            a.flags |= _lib.FLAG_FULL_TABLE | _lib.FLAG_ROW_FLAGS
            a.rowflags = _p(self.rowflags)
            a.stats, a.census = _p(self.stats_all), _p(self.census)
            ca = self._args()
            ca.flags = ((_lib.FLAG_FIX_SEC if self.stats_with_sec else 0) | _lib.FLAG_COUNT_RESPAWNS
                        | _lib.FLAG_GEN_ADVANCE)
            ca.W, ca.counts, ca.respawn = _p(self.rows_out), _p(self.counts), _p(self.respawn)
        else:
            # fused generation: next generation's lists, block stats, done counter, census
            fa = self._args()
            ctypes.pointer(fa)[0] = a
            fa.heads_next, fa.nexts_next = _p(self.heads[1 - self._p]), _p(self.nexts[1 - self._p])
            fa.ballots = None
            fa.temp, fa.temp_bytes = _p(self._blockstat), self._blockstat.numel() * 4
            fa.done = _p(self._done)
            fa.flags = a.flags | _lib.FLAG_RESPAWN_INLINE
            if self.finish_mode == "batch":
                bs = self._bs_ring[self._pending_fin]
                fa.temp, fa.temp_bytes = _p(bs), bs.numel() * 4
                fa.flags |= _lib.FLAG_TWO_PHASE | _lib.FLAG_GEN_COUNTS | _lib.FLAG_BORN_TOTAL
            elif self.device.type == "cuda":
                fa.flags |= _lib.FLAG_TWO_PHASE
            if self._census_fused():
                fa.flags |= _lib.FLAG_FUSED_CENSUS | (_lib.FLAG_FIX_SEC if self.stats_with_sec else 0)
            if self.order == "sequential":
                q = self._p if self._ord_pipe else 0
                osrc, olist, octl = self._ord_set(q)
                fa.W3, fa.o_src, fa.o_list, fa.o_ctl = _p(self._abuf), _p(osrc), _p(olist), _p(octl)
                fa.ptab = _p(self._perm_table(q))
                if self._ord_pipe:
                    fa.flags |= _lib.FLAG_ORD_PLANNED
                if self._sync:  # (two counter-ordered graphs)
                    fa.flags |= _lib.FLAG_ORD_SYNC
                    fa.o_sync = _p(self._osync)
                if self._ord_census_side and (fa.flags & _lib.FLAG_FUSED_CENSUS):
                    # the census of the final rows after the close: on the side stream beside the
                    # next run, or (two-graph chunks) by extra workgroups of the next run launch
                    fa.flags |= _lib.FLAG_ORD_CENSUS_LATER
                if self._ord_mode == "kernel":  # the run launch also builds the next generation's plan
                    nsrc, nlist, nctl = self._ord_set(1 - q)
                    fa.flags |= _lib.FLAG_ORD_INPLAN
                    fa.o_src_next, fa.o_list_next, fa.o_ctl_next = _p(nsrc), _p(nlist), _p(nctl)
                    fa.ptab_next = _p(self._perm_table(1 - q))
                    fa.o_plan_groups = self.plan_groups(self.n)
                fa.o_levels = self.order_levels
                fa.o_trace = _p(getattr(self, "_otrace", None))
            ca = fa
        self._arg_cache[key] = (a, ca, a.flags)
        return self._arg_cache[key]

    def _generation(self, record: bool = False):
        if self.x2:
            return self._x2_generation(record)
        spec, cfg = self.spec, self.cfg
        a, ca, flags = self._gen_args()
        a.flags = flags
        if not self.dist.enabled:
            if self.order == "sequential":
                return self._ordered_generation(a, ca, record)
            if self.fused and not (record and self.recorder is not None):
                # ONE launch: evolve + next generation's attack lists + census + uids
                if not self._lists_ready:
                    _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
                _lib.run(_lib.OP_SOUP_GEN, spec, ca, cfg)
                self._lists_ready = True
                self._p = 1 - self._p
                if self.finish_mode == "batch":
                    self._fin_flags = ca.flags
                    self._pending_fin += 1
                    if self._pending_fin == self._batch:
                        self._finish_pending()
                elif self.stats and not (ca.flags & _lib.FLAG_FUSED_CENSUS):
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
        if self.order == "sequential":
            return self._ordered_sharded_generation(a, ca, record)
        # ---- sharded, all-gather: decide -> all-gather rows -> evolve -> census + respawn
        #      count (+ generation counter) -> all-gather stats -> uids
        d = self.dist
        if not self._lists_ready:
            _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
        # raw 32-bit view: the collective moves bytes whatever the storage dtype
        d.all_gather_rows(self.full.view(torch.int32), self.table_in.view(torch.int32), self.n_total)
        self._lists_ready = False
        inline = not (record and self.recorder is not None)
        a.flags = flags | (_lib.FLAG_RESPAWN_INLINE if inline else 0)
        _lib.run(_lib.OP_SOUP_EVOLVE, spec, a, cfg)
        a.flags = flags
        if not inline:
            self.recorder.on_evolved(self)
            _lib.run(_lib.OP_RESPAWN, spec, a, cfg)
        _lib.run(_lib.OP_CLASSIFY, spec, ca, cfg)
        self._p = 1 - self._p
        self._pending = True
        self._flush()

    def _ordered_generation(self, a, ca, record: bool):
        """One reference-order generation (OP_SOUP_ORDERED: plan -> levels -> level launches ->
        tail -> close; the newborns' uids by the finish, batched like the fused generation's).
        Recording keeps every particle's pre-respawn row and counterparts as slots; the
        recorder maps them to uids as of each turn (a counterpart slot < k that respawned at
        its own turn is already the newborn)."""
        spec, cfg = self.spec, self.cfg
        side = main = None
        if self._sync:  # (a two-graph chunk: the plans are the side graph's, _capture_side)
            assert self._lists_ready and record is False
        elif self._ord_pipe:
            if not self._lists_ready:  # the first generation's plan (later ones: planned ahead)
                _lib.run(_lib.OP_ORD_PLAN, spec, self._plan_args(False), cfg)
            if self._ord_mode == "stream":
                # the next generation's plan beside this one (weight independent); it overwrites the
                # plan set and attack lists the previous generation's close finished with; first the
                # previous generation's census, if its close left it
                if self._ord_side is not None:
                    side, main = self._ord_side, torch.cuda.current_stream(self.device)
                    side.wait_stream(main)
                with torch.cuda.stream(side) if side is not None else _nullcontext():
                    self._run_census_due()
                _lib.run(_lib.OP_ORD_PLAN, spec, self._plan_args(True), cfg)
        elif not self._lists_ready:
            _lib.run(_lib.OP_SOUP_DECIDE, spec, a, cfg)
        rec = record and self.recorder is not None
        if rec:
            if self._rec_rows is None:
                self._rec_rows = torch.zeros_like(self._abuf)
            ca.traj = _p(self._rec_rows)
            uid0 = self.uid.clone()
        if self._sync and self._census_due is not None:
            # the previous close's census by this run launch (its final rows are this generation's W2)
            W, temp, _, _ = self._census_due
            assert W == ca.W2, "census rows are the next generation's start rows"
            ca.o_census_temp = temp
            self._census_due = None
        try:
            _lib.run(_lib.OP_SOUP_ORDERED, spec, ca, cfg)
        finally:
            ca.traj = None
            ca.o_census_temp = None
            if side is not None:
                main.wait_stream(side)  # the next generation starts on a complete plan
        if ca.flags & _lib.FLAG_ORD_CENSUS_LATER:
            self._census_due = (ca.W, ca.temp, ca.temp_bytes, ca.flags)
        self._lists_ready = True
        self._p = 1 - self._p
        if self.finish_mode == "batch":
            self._fin_flags = ca.flags
            self._pending_fin += 1
            if self._pending_fin == self._batch or rec:
                self._finish_pending()
        elif self.stats and not (ca.flags & _lib.FLAG_FUSED_CENSUS):
            self.classify_local(self.stats_with_sec, zero=False)
        if rec:
            self.recorder.on_evolved(self, rows=self._rec_rows, old_uid=uid0, ordered=True)

    @staticmethod
    def plan_groups(n: int) -> int:
        """Workgroups of a run launch that build the next generation's plan (ord_pipeline "kernel"):
        one per 64-turn chunk up to 512 -- each plan phase then takes a few chunks per workgroup, well
        inside the run's dependent tail (csrc/srnn_ordered.h ord::plan_group)."""
        return max(1, min(512, -(-int(n) // 64)))

    def _plan_args(self, nxt: bool) -> _lib.SrnnArgs:
        """OP_ORD_PLAN arguments: the plan of the generation about to run (``nxt`` False: the
        first one, on the current stream, into this parity's plan set and lists) or of the one
        after it (into the other parity's, on the side stream)."""
        key = self._cache_key("plan", nxt)
        a = self._arg_cache.get(key)
        if a is None:
            q = 1 - self._p if nxt else self._p
            a = self._args(self._ord_side if nxt else None)
            osrc, olist, octl = self._ord_set(q)
            a.o_src, a.o_list, a.o_ctl = _p(osrc), _p(olist), _p(octl)
            a.heads, a.nexts = _p(self.heads[q]), _p(self.nexts[q])
            a.ptab = _p(self._perm_table(q))
            a.o_levels = self.order_levels
            if nxt:
                a.flags |= _lib.FLAG_ORD_NEXT
                if self._sync:
                    a.flags |= _lib.FLAG_ORD_SYNC
                    a.o_sync = _p(self._osync)
            self._arg_cache[key] = a
        return a

    def _sh_args(self, phase: int, level: int = 0) -> _lib.SrnnArgs:
        """Argument block of a sharded reference-order phase, in the global view (csrc
        srnn_ordered_sh.h): all n_total turns planned, this rank's [lo, hi) run; per-row columns
        addressed by global slot through pointers offset by -lo."""
        key = self._cache_key("ordsh", phase)
        a = self._arg_cache.get(key)
        if a is None:
            N, lo = self.n_total, self.lo

            def shifted(t):
                return ctypes.c_void_p(t.data_ptr() - lo * t.element_size()) if t is not None else None

            a = self._args()
            a.n, a.n_total, a.lo = N, N, 0
            a.o_lo, a.o_hi = self.lo, self.hi
            em = int(self.execution.ordsh_emulate)
            if self.dist.world == 1 and em > 1:  # timing model of `em` ranks: this one runs 1/em of the turns
                a.o_hi = a.o_lo + -(-N // em)
                # the other turns never run: the rows are invalid -- a sticky error bit, so count()
                # and checkpoints refuse them (an environment variable left over from profiling
                # must not pass for a soup)
                self._octl[_lib.ORD_ERRW] |= ORD_ERR_EMULATED
            a.W2, a.W, a.W3 = _p(self.full), _p(self._fw), _p(self._abuf)
            a.o_src, a.o_list, a.o_ctl = _p(self._osrc), _p(self._olist), _p(self._octl)
            a.heads, a.nexts = _p(self._sh_heads[self._p]), _p(self._sh_nexts[self._p])
            a.heads_next, a.nexts_next = _p(self._sh_heads[1 - self._p]), _p(self._sh_nexts[1 - self._p])
            a.action, a.counterpart, a.loss = shifted(self.action), shifted(self.counterpart), shifted(self.loss)
            a.respawn, a.rowflags = shifted(self.respawn), shifted(self.rowflags)
            a.sendbuf, a.recvbuf, a.x_ctl = _p(self._sh_send), _p(self._sh_recv), _p(self._sh_cnt)
            a.steps = phase
            self._arg_cache[key] = a
        a.o_levels = level if phase in (_lib.ORDSH_LEVEL, _lib.ORDSH_PACK) else self.order_levels
        return a

    def _ordered_sharded_generation(self, a, ca, record: bool):
        """One reference-order generation sharded over the ranks (csrc/srnn_ordered_sh.h):
        all-gather of the generation-start rows -> replicated plan + levels -> per level: this
        rank's turns, their outputs all-gathered -> close of this rank's rows -> the next
        generation's lists -> census + respawn count (OP_CLASSIFY) -> uids (flush).  Bitwise the
        single-rank generation (tests/test_ordered_sharded.py).  Eager: the number of levels is
        read back every generation."""
        if record and self.recorder is not None:
            raise NotImplementedError("recording states of a sharded reference-order soup")
        spec, cfg, d = self.spec, self.cfg, self.dist
        N, R = self.n_total, d.world

        def run(phase, level=0, **fields):
            sa = self._sh_args(phase, level)
            for k, v in fields.items():
                setattr(sa, k, v)
            _lib.run(_lib.OP_SOUP_ORDERED_SH, spec, sa, cfg)

        if not self._lists_ready:  # this generation's attack lists, every slot (the global view)
            self._sh_heads[self._p].fill_(-1)
            _lib.run(_lib.OP_SOUP_DECIDE, spec, self._sh_args(_lib.ORDSH_PLAN), cfg)
        d.all_gather_rows(self.full.view(torch.int32), self.table_in.view(torch.int32), N)
        run(_lib.ORDSH_PLAN)
        caps, maxl = self._sh_level_caps(N, R)  # records per rank and level: the same on every rank
        recw = self._sh_recb // 8
        for L in range(maxl + 1):
            run(_lib.ORDSH_LEVEL, L)
            cap = int(caps[L])
            if cap == 0:
                continue
            send = self._sh_send[:cap * recw]
            send.view(cap, recw)[:, 0].fill_(-1)
            run(_lib.ORDSH_PACK, L, x_blk=cap)
            d.all_gather_into(self._sh_recv[:R * cap * recw], send)
            run(_lib.ORDSH_UNPACK, x_blk=cap)
        run(_lib.ORDSH_CLOSE)
        self.rows_out.copy_(self._fw[self.lo:self.hi])
        run(_lib.ORDSH_LINK)
        self._lists_ready = True
        _lib.run(_lib.OP_CLASSIFY, spec, ca, cfg)  # census + respawn count + the generation counter
        self._p = 1 - self._p
        self._pending = True
        self._flush()

    _SH_LEVEL_BINS = 64

    def _sh_level_caps(self, N: int, R: int):
        """The largest count of one rank's turns at each dependency level (every rank plans the
        whole generation, so every rank computes the same numbers) and the deepest level, read back
        in ONE device-to-host copy: turns binned by (rank of the slot, level) with a scatter-add --
        the rank of slot k is ((k + 1) R - 1) // N for the shards [r N / R, (r + 1) N / R) -- instead
        of a bincount per rank (each one a host synchronisation)."""
        B = self._SH_LEVEL_BINS
        lv = self._osrc[:4 * N].view(N, 4)[:, 3]
        if N <= (1 << 24):
            if getattr(self, "_sh_key", None) is None or self._sh_key.numel() != N:
                k = torch.arange(N, dtype=torch.int64, device=self.device)
                self._sh_key = ((k + 1) * R - 1) // N * B
                self._sh_one = torch.ones(N, dtype=torch.int64, device=self.device)
            key = self._sh_key + lv.clamp(0, B - 1).long()
            cnt = torch.zeros(R * B, dtype=torch.int64, device=self.device).scatter_add_(0, key, self._sh_one)
            info = torch.cat([cnt.view(R, B).max(dim=0).values,
                              self._octl[_lib.ORD_MAXLW:_lib.ORD_MAXLW + 1].long()]).cpu().tolist()
            maxl = int(info[-1])
            if maxl < B:
                return info[:maxl + 1], maxl
        maxl = int(self._octl[_lib.ORD_MAXLW].item())
        counts = torch.stack([torch.bincount(lv[lo:hi].clamp(min=0).long(), minlength=maxl + 1)[:maxl + 1]
                              for lo, hi in (self.dist.shard_of_rank(r, N) for r in range(R))])
        return counts.max(dim=0).values.cpu().tolist(), maxl

    def _finish_pending(self):
        """Batch mode: ONE finish launch for the generations whose block stats wait in the
        ring (in generation order: census of each, newborn uids, next_uid)."""
        m = self._pending_fin
        if m == 0:
            return
        self._run_census_due()  # (the last generation's class counts complete its block stats)
        a = self._args()
        a.n = self.n
        a.steps = m
        a.flags = (self._fin_flags & (_lib.FLAG_FUSED_CENSUS | _lib.FLAG_BORN_TOTAL)) | _lib.FLAG_FINISH_BATCH
        a.temp, a.temp_bytes = _p(self._bs_ring), self._bs_ring.stride(0) * 4
        a.uid_out, a.uid_base, a.counts = _p(self.uid), _p(self.next_uid), _p(self.counts)
        if self.execution.finish_par:
            a.done = _p(self._done)  # done counter: one finish workgroup per generation
        _lib.run(_lib.OP_GEN_FINISH, self.spec, a, self.cfg)
        self._pending_fin = 0

    def _run_census_due(self):
        """The census a reference-order close left (FLAG_ORD_CENSUS_LATER), on the current stream."""
        if self._census_due is None:
            return
        W, temp, temp_bytes, flags = self._census_due
        key = ("census", W, temp, self._stream_key())
        a = self._arg_cache.get(key)
        if a is None:
            a = self._args()
            a.W, a.temp, a.temp_bytes = W, temp, temp_bytes
            a.flags = flags & (_lib.FLAG_FIX_SEC | _lib.FLAG_FUSED_CENSUS)
            self._arg_cache[key] = a
        _lib.run(_lib.OP_ORD_CENSUS, self.spec, a, self.cfg)
        self._census_due = None

    def _stream_key(self):
        return torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0

    def _join_side(self):
        """Run any census and batched finish still due (uids, census, next_uid are final after this)."""
        if self._census_due is not None:
            self._run_census_due()  # (on the main stream: it reads the rows the close just wrote)
        if not self.x2 and self._pending_fin:
            self._finish_pending()

    # ------------------------------------------------------------------ sharded all-to-all (X2)
    def _x2_base(self, p: int, stream=None) -> _lib.SrnnArgs:
        """Fields shared by the X2 launches of a generation of parity p ("this" = p,
        "next" = 1 - p)."""
        a = self._args(stream)
        a.x_cr, a.x_cn, a.x_cq, a.x_blk = self.x_cr, self.x_cn, self.x_cq, self.x_blk
        a.x_emul = self.x_emul
        if self.device.type == "cuda" and self.execution.x2_prio:
            a.flags |= _lib.FLAG_X2_PRIO  # pack / post / remote evolve win the shared SIMDs
        a.sendbuf, a.recvbuf = _p(self.sendbuf), _p(self.recvbuf)
        a.census = _p(self.census)
        q = 1 - p
        a.heads, a.nexts = _p(self.heads[p]), _p(self.nexts[p])
        a.heads_next, a.nexts_next = _p(self.heads[q]), _p(self.nexts[q])
        a.x_dep, a.x_dep_next = _p(self.x_dep[p]), _p(self.x_dep[q])
        a.x_rlist, a.x_rlist_next = _p(self.x_rlist[p]), _p(self.x_rlist[q])
        a.x_rcount, a.x_rcount_next = _p(self.x_rcount[p]), _p(self.x_rcount[q])
        a.x_rslot, a.x_rslot_next = _p(self.x_rslot[p]), _p(self.x_rslot[q])
        a.x_satt, a.x_satt_next = _p(self.x_satt[p]), _p(self.x_satt[q])
        a.x_cno, a.x_cno_next = _p(self.x_cno[p]), _p(self.x_cno[q])
        a.x_crq, a.x_crq_next = _p(self.x_crq[p]), _p(self.x_crq[q])
        a.x_srep, a.x_nsrep = _p(self.x_srep), _p(self.x_nsrep)
        a.x_part, a.x_ctl, a.x_groups = _p(self.x_part), _p(self.x_ctl), self.x_groups
        a.x_hpre, a.x_hgrp = _p(self.x_hpre), _p(self.x_hgrp)
        a.uid_out, a.uid_base, a.counts = _p(self.uid), _p(self.next_uid), _p(self.counts)
        return a

    def _x2_args(self, record: bool = False):
        """(pack, post, remote evolve, local evolve) argument blocks of a generation of the
        current parity (cached)."""
        key = self._cache_key("x2", record)
        hit = self._arg_cache.get(key)
        if hit is not None:
            return hit
        p = self._p
        xs = self._xs
        # the census of the stored rows inside the evolve (templated and runtime-shape nets),
        # else a classify launch adding to counts; the finish sums both
        # (always on for the sharded exchange, as the census rides on it: shuffle_random nets
        # classify in a separate launch)
        census = self.spec.shuffler == "none" and not record and self._evolve_census
        pa = self._x2_base(p)
        pa.W2 = _p(self.table_in)
        pa.temp = _p(self.x_bstat[1 - p])  # the finished generation's block stats
        po = self._x2_base(p, self._xp)  # post runs beside the remote evolve
        po.temp = _p(self.x_bstat[1 - p])
        ev = self._x2_base(p)
        ev.W2, ev.W = _p(self.table_in), _p(self.rows_out)
        ev.temp = _p(self.x_bstat[p])
        ev.action, ev.counterpart, ev.loss, ev.respawn = (_p(self.action), _p(self.counterpart), _p(self.loss),
                                                           _p(self.respawn))
        ev.flags |= _lib.FLAG_X2 | (0 if record else _lib.FLAG_RESPAWN_INLINE)
        if census:
            ev.flags |= _lib.FLAG_FUSED_CENSUS | (_lib.FLAG_FIX_SEC if self.stats_with_sec else 0)
        rem = self._x2_base(p)
        ctypes.pointer(rem)[0] = ev
        rem.flags = ev.flags | _lib.FLAG_X2_REMOTE
        loc = self._x2_base(p, xs)
        ctypes.pointer(loc)[0] = ev
        loc.stream = self._stream(xs)
        if self.schedule == "serial":
            po = self._x2_base(p)  # everything on the current stream
            po.temp = _p(self.x_bstat[1 - p])
            loc = self._x2_base(p)
            ctypes.pointer(loc)[0] = ev
            if self._x2_both:
                # ONE launch: post's workgroups first, then n/64 waves evolving every slot
                rem.flags |= _lib.FLAG_X2_BOTH | _lib.FLAG_X2_POST_FUSED
                rem.temp2 = _p(self.x_bstat[1 - p])
                rem.ptab = _p(self._perm_table())  # the generation's permutations, ahead of it
                if rem.ptab:  # built by pack's extra workgroups (no table launch on the critical path)
                    pa.ptab = rem.ptab
                    rem.flags |= _lib.FLAG_PTAB_READY
                loc = None
                po = None
        self._arg_cache[key] = (pa, po, rem, loc, census)
        return self._arg_cache[key]

    def _x2_exchange(self, post: _lib.SrnnArgs, remote: Optional[_lib.SrnnArgs] = None):
        """all-to-all -> remote evolve on the current stream (RCCL inside a hipGraph is
        captured from the origin stream), post beside the remote evolve on its own stream:
        the remote-dependent slots of this generation need only the received rows, post
        prepares the next generation (nothing of this one reads what it writes)."""
        self.dist.all_to_all(self.recvbuf, self.sendbuf)
        xp = self._xp if remote is not None else None
        if xp is None:
            _lib.run(_lib.OP_X2_POST, self.spec, post, self.cfg)
            if remote is not None:
                _lib.run(_lib.OP_SOUP_EVOLVE, self.spec, remote, self.cfg)
            return
        main = torch.cuda.current_stream(self.device)
        xp.wait_stream(main)
        with torch.cuda.stream(xp):
            _lib.run(_lib.OP_X2_POST, self.spec, post, self.cfg)
        _lib.run(_lib.OP_SOUP_EVOLVE, self.spec, remote, self.cfg)
        main.wait_stream(xp)

    def _x2_prime(self):
        """First exchange of a (re)started soup: the decisions of THIS generation go out as
        notices / requests (no rows, no stats); afterwards every generation's pack prepares
        the next one."""
        p = self._p
        gen = int(self.gen_dev.item())
        pa = self._x2_base(p)
        q = 1 - p
        # "next" = this generation's structures, "this" = the other parity's (empty) counters
        for f, lst in (("heads", self.heads), ("nexts", self.nexts), ("x_dep", self.x_dep),
                       ("x_rlist", self.x_rlist), ("x_rcount", self.x_rcount), ("x_rslot", self.x_rslot),
                       ("x_satt", self.x_satt), ("x_cno", self.x_cno), ("x_crq", self.x_crq)):
            setattr(pa, f + "_next", _p(lst[p]))
            setattr(pa, f, _p(lst[q]))
        pa.gen_ptr, pa.gen = None, gen
        pa.W2 = _p(self.table_in)
        pa.temp = _p(self.x_bstat[q])
        pa.flags |= _lib.FLAG_X2_PRIME
        po = self._x2_base(p)
        ctypes.pointer(po)[0] = pa
        _lib.run(_lib.OP_X2_PACK, self.spec, pa, self.cfg)
        self._x2_exchange(po)
        self._primed = True

    def _x2_generation(self, record: bool = False):
        spec, cfg = self.spec, self.cfg
        if not self._primed:
            self._x2_prime()
        pa, po, rem, loc, census = self._x2_args(record)
        if self.schedule == "serial":
            _lib.run(_lib.OP_X2_PACK, spec, pa, cfg)
            self.dist.all_to_all(self.recvbuf, self.sendbuf)
            if po is not None:  # (else fused into the evolve launch)
                _lib.run(_lib.OP_X2_POST, spec, po, cfg)
            if loc is not None:
                _lib.run(_lib.OP_SOUP_EVOLVE, spec, loc, cfg)
            _lib.run(_lib.OP_SOUP_EVOLVE, spec, rem, cfg)  # (with FLAG_X2_BOTH: the local slots too)
            self._x2_close(record, census)
            return
        # the local slots need nothing of this generation's exchange: they start at once on
        # the side stream, beside pack -> all-to-all -> post -> remote-dependent slots
        side = self._xs
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                _lib.run(_lib.OP_SOUP_EVOLVE, spec, loc, cfg)
        _lib.run(_lib.OP_X2_PACK, spec, pa, cfg)
        self._x2_exchange(po, rem)
        if side is not None:
            torch.cuda.current_stream(self.device).wait_stream(side)
        else:
            _lib.run(_lib.OP_SOUP_EVOLVE, spec, loc, cfg)
        self._x2_close(record, census)

    def _x2_close(self, record: bool, census: bool):
        spec, cfg = self.spec, self.cfg
        if record and self.recorder is not None:
            self.recorder.on_evolved(self)
            ra = self._args()
            ra.W, ra.respawn = _p(self.rows_out), _p(self.respawn)
            _lib.run(_lib.OP_RESPAWN, spec, ra, cfg)
        if not census:
            # census of the stored rows (classify -> counts, read by the next finish)
            cls, _ = K.classify(self.spec, self.rows_out, self.eps, self.stats_with_sec, uid=None, seed=self.seed,
                                scratch=self._scratch, ctr=0x7FFFFFF0, counts=self.counts, key_offset=self.lo)
        self._p = 1 - self._p  # (post_t advanced the generation counter)
        self._pending = True

    def _x2_flush(self):
        """Finish of the last generation now: this rank's stats (finish-only pack) ->
        all-gather -> uids of its newborns, global census."""
        p = self._p
        key = self._cache_key("x2flush")
        hit = self._arg_cache.get(key)
        if hit is None:
            pa = self._x2_base(p)
            pa.temp = _p(self.x_bstat[1 - p])
            pa.flags |= _lib.FLAG_X2_FINISH_ONLY
            po = self._x2_base(p)
            po.temp = _p(self.x_bstat[1 - p])
            po.stats = _p(self.stats_all)
            po.flags |= _lib.FLAG_X2_FINISH_ONLY
            hit = self._arg_cache[key] = (pa, po)
        pa, po = hit
        _lib.run(_lib.OP_X2_PACK, self.spec, pa, self.cfg)
        hdr = self.sendbuf[:48].view(torch.int64)  # this rank's stats (header words 0..5 of block 0)
        self.dist.all_gather_into(self.stats_all, hdr)
        _lib.run(_lib.OP_X2_POST, self.spec, po, self.cfg)

    # ------------------------------------------------------------------ finish / flush
    def _flush(self):
        """Sharded: assign the uids of the last generation's newborns now."""
        if not (self.dist.enabled and self._pending):
            return
        if self.x2:
            self._x2_flush()
        else:
            a, _, flags = self._gen_args()
            self.dist.all_gather_into(self.stats_all, self.counts)
            if self.device.type == "cuda":
                # the grid-wide assignment's scratch (csrc uid_temp_bytes: a count per 4096-row
                # chunk + this rank's first uid); allocated once, outside graph captures
                nb = (-(-self.n // 4096) * 4 + 7) // 8 * 8 + 8
                t = getattr(self, "_uid_tmp", None)
                if t is None or t.numel() * 8 < nb:
                    self._uid_tmp = t = torch.zeros(nb // 8, dtype=torch.int64, device=self.device)
                ua = self._args()
                ctypes.pointer(ua)[0] = a
                ua.temp, ua.temp_bytes = _p(t), t.numel() * 8
                a = ua
            _lib.run(_lib.OP_UID_ASSIGN, self.spec, a, self.cfg)
        self._pending = False

    def local_exchange_error(self) -> int:
        """This rank's exchange error bits (X2_ERRORS), read without communicating."""
        return int(self.err.item()) if self.dist.enabled else 0

    def exchange_error(self) -> Optional[str]:
        """Description of any exchange error of this soup on ANY rank (the flags are
        all-gathered so every rank stops together), or None.  COLLECTIVE: every rank must
        call it (``local_exchange_error`` reads this rank's bits alone)."""
        if not self.dist.enabled:
            return None
        out = torch.zeros(self.dist.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into(out, self.err.to(torch.int64))
        v = 0
        for x in out.cpu().tolist():
            v |= int(x)
        if not v:
            return None
        return "; ".join(msg for bit, msg in X2_ERRORS.items() if v & bit) or f"error bits {v}"

    def exchange_overflowed(self) -> bool:
        """Collective, like ``exchange_error``: every rank must call it."""
        return self.exchange_error() is not None

    def classify_local(self, with_sec: bool = True, zero: bool = True):
        if zero:
            self.counts.zero_()
        # census streams (shuffle_random nets) keyed by global slot, like the fused census
        cls, _ = K.classify(self.spec, self.local_rows(), self.eps, with_sec, uid=None, seed=self.seed,
                            scratch=self._scratch, ctr=0x7FFFFFF0, counts=self.counts, key_offset=self.lo)
        return cls

    def count(self, with_sec: bool = True) -> Dict[str, int]:
        """Global class histogram of the current particles (all-reduced)."""
        err = self.exchange_error()
        if err:
            raise RuntimeError(f"soup row exchange failed ({err}): results are invalid")
        e = self.ordered_error_all()
        if e:
            raise RuntimeError(f"reference-order generation: error bits {e} ({describe_ordered_error(e)}); results are "
                               "invalid")
        c = torch.zeros(6, dtype=torch.int64, device=self.device)
        cls, _ = K.classify(self.spec, self.local_rows(), self.eps, with_sec, uid=None, seed=self.seed,
                            scratch=self._scratch, ctr=0x7FFFFFF0, counts=c, key_offset=self.lo)
        c = c[:5].clone()
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
            ch = next((c for c in self._chunks if c[2] <= left and c[1] == self._p), None)
            if (ch is not None and not (record and self.recorder is not None)
                    and self.trajectory is None and self.metrics is None):
                # G generations in one graph launch (no inter-graph gaps)
                self._join_side()
                self._replay_chunk(ch)
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
            loss = self.loss if self.loss is not None else torch.zeros(1, device=self.device)
            ls = torch.stack([torch.nan_to_num(loss.double(), nan=0.0).sum(),
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
        self._flush()
        out = torch.zeros(self.n_total, dtype=torch.int64, device=self.device)
        self.dist.all_gather_rows(out, self.uid, self.n_total)
        return out.cpu().numpy()

    # ------------------------------------------------------------------ HIP graphs
    def _state(self):
        """Every device tensor a generation reads or writes (graph validation)."""
        names = ["_bufs", "uid", "next_uid", "_gen_ring", "heads", "nexts", "ballots", "rowflags", "action",
                 "counterpart", "loss", "respawn", "counts", "census", "err", "full", "stats_all", "_blockstat",
                 "_done", "_bs_ring", "x_dep", "x_rlist", "x_rcount", "x_rslot", "x_satt", "x_cno", "x_crq",
                 "x_srep", "x_nsrep", "x_part", "x_ctl", "x_bstat", "x_hpre", "x_hgrp", "sendbuf", "recvbuf",
                 "_abuf", "_osrc", "_olist", "_octl", "_ptab", "_osrc1", "_olist1", "_octl1", "_ptab1", "_osync",
                 "_fw", "_sh_heads", "_sh_nexts", "_sh_cnt", "_sh_send", "_sh_recv"]
        out = []
        for k in names:
            v = getattr(self, k, None)
            if isinstance(v, list):
                out.extend(v)
            elif isinstance(v, torch.Tensor):
                out.append(v)
        return out

    def _agree(self, ok: bool) -> bool:
        """All ranks agree (MIN) before anything collective depends on a local outcome."""
        if not self.dist.enabled:
            return ok
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
        return bool(flag.item())

    def capture(self, warmup: int = 1, validate: bool = True) -> bool:
        """Capture the generation for both ping-pong parities in two hipGraphs (ROCm
        device).  Everything that changes per generation lives in device memory
        (generation counter, next uid), so replays advance the soup exactly like the
        eager path.  Sharded engines capture their RCCL collective inside the graph (one
        all-to-all per generation on the comm stream, joined back); ``validate`` then
        replays generations from a saved state, compares them bitwise with the eager path
        on every rank and keeps the graphs only if all ranks agree.  Every rank first agrees
        that capture succeeded everywhere, so a rank whose capture failed never leaves the
        others waiting inside a collective."""
        if self.device.type != "cuda":
            return False
        if self.dist.enabled and not self.x2:
            return False
        if self.dist.enabled and self.dist.native is None:
            # torch's process-group collectives are not captured: their watchdog thread
            # queries events recorded by the capturing stream
            return False
        if self.dist.world > 1 and not self.execution.sharded_graph:
            return False
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        # max(warmup, 1) eager generations in all: the last one runs between the capture of the
        # multi-generation graphs of the two parities (below)
        with torch.cuda.stream(s):
            for _ in range(max(warmup, 1) - 1):
                self.time += 1
                self._generation()
            self._join_side()
            self._prepare_capture()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        graphs = []
        p0 = self._p
        pend0 = self._pending
        flags0 = self._flags_state()
        ok = True
        try:
            for _ in range(2):
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's watchdog thread keeps querying events
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._generation()  # flips self._p during capture (nothing ran)
                    self._join_side()
                graphs.append(g)
        except Exception as e:  # noqa: BLE001 -- any capture failure -> eager generations
            import sys
            print(f"soup graph capture failed ({type(e).__name__}: {e}); running eagerly", file=sys.stderr)
            ok = False
        self._p = p0
        self._pending = pend0
        self._set_flags_state(flags0)  # a capture that failed midway may have advanced them
        ok = self._agree(ok)
        if ok and validate:
            ok = self._agree(self._validate_graphs(graphs if p0 == 0 else graphs[::-1]))
        if not ok:
            self._graphs = None
            self.time += 1  # the last warmup generation, eagerly
            self._generation()
            self._join_side()
            return False
        # graphs[k] was captured with parity p0 ^ k; index them by parity
        self._graphs = graphs if p0 == 0 else graphs[::-1]
        self._chunks = []
        self._capture_chunk(s, p0, pend0)
        # the last warmup generation (eager), then the same chunks from the other parity: an
        # evolve replays multi-generation graphs whatever parity it starts at (an odd
        # warmup would otherwise leave every later generation on single-generation graphs)
        with torch.cuda.stream(s):
            self.time += 1
            self._generation()
            self._join_side()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        if self._chunks:
            self._capture_chunk(s, self._p, self._pending)
        return True

    def _prepare_capture(self):
        """The one-time work a first generation does before its graph-captured steady state:
        this generation's attack lists (fused single rank) or the first exchange (sharded)."""
        if self.x2:
            if not self._primed:
                self._x2_prime()
        elif self.fused and not self._lists_ready and not self.dist.enabled:
            if self._ord_pipe:
                _lib.run(_lib.OP_ORD_PLAN, self.spec, self._plan_args(False), self.cfg)
            else:
                a, _, _ = self._gen_args()
                _lib.run(_lib.OP_SOUP_DECIDE, self.spec, a, self.cfg)
            self._lists_ready = True

    def _chunk_sizes(self):
        """Generations per multi-generation graph (ExecConfig.graph_chunks, even sizes): an
        evolve of K generations replays the largest that fit, so a short timed region pays few
        launches and few finish launches (one 20-generation graph for K = 20, 20 + 20 + 8 + 2
        for K = 50)."""
        return sorted({int(x) for x in self.execution.graph_chunks}, reverse=True)

    def _capture_chunk(self, s, p0, pend0):
        """Multi-generation graphs starting (and ending) at parity p0, added to _chunks
        (largest first)."""
        for G in self._chunk_sizes():
            ch = self._capture_chunk_g(s, p0, pend0, G)
            if ch is None:
                break
            self._chunks.append(ch)
        self._chunks.sort(key=lambda c: -c[2])
        self._chunk = self._chunks[0] if self._chunks else None

    def _flags_state(self):
        return (self._lists_ready, self._pending_fin if not self.x2 else 0, self._census_due)

    def _set_flags_state(self, st):
        self._lists_ready = st[0]
        if not self.x2:
            self._pending_fin = st[1]
        self._census_due = st[2]

    def _capture_chunk_g(self, s, p0, pend0, G):
        """A graph of G consecutive generations (G even: it starts and ends at parity
        p0) replayed as one launch, removing the per-generation graph-launch gap;
        validated bitwise against G eager generations (all ranks agree or none use it).
        Reference order with the side-stream plan (ExecConfig.ord_graph_sync): first as TWO
        graphs -- the G runs + closes, and on the side stream the G plans of the generations
        after them -- ordered by device counters (SRNN_F_ORD_SYNC) instead of a cross-queue join
        per generation (~10 us of idle queue each, profiles/r6a); the one-graph form if that
        capture or its validation fails."""
        if self._ord_decouple and self._lists_ready and self._streams_concurrent():
            ch = self._capture_chunk_sync(s, p0, pend0, G)
            if ch is not None:
                return ch
        ok = True
        gc = torch.cuda.CUDAGraph()
        flags0 = self._flags_state()
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
        self._set_flags_state(flags0)
        ok = self._agree(ok)
        if ok:
            ok = self._agree(self._validate_replay(lambda: gc.replay(), G, parity_after=p0))
        return (gc, p0, G, None) if ok else None

    def _streams_concurrent(self) -> bool:
        """(once per engine) whether kernels on the side stream and the current one run at the same
        time -- a two-graph chunk's counters need it: under a profiler that serialises kernels
        (rocprofv3 --pmc) or on a shared hardware queue every wait would run into its timeout.
        Agreed over the ranks."""
        if getattr(self, "_conc", None) is None:
            ok = _lib.streams_concurrent(self._ord_side, torch.cuda.current_stream(self.device), self.device)
            if not ok:
                import sys
                print("side stream does not run beside the current one (serialising profiler?): "
                      "one-graph chunks", file=sys.stderr)
            self._conc = self._agree(ok)
        return self._conc

    def _capture_chunk_sync(self, s, p0, pend0, G):
        """The two-graph form of a G-generation chunk (see _capture_chunk_g): main graph = G x
        (run + close, the close waiting for the next plan) + the batched finish; side graph = G x
        (gate on the run counter, plan of the next generation, done count)."""
        gc, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        flags0 = self._flags_state()
        ok = True
        self._sync = True
        try:
            with torch.cuda.graph(gc, stream=s, capture_error_mode="thread_local"):
                for _ in range(G):
                    self._generation()
                self._join_side()
            self._p = p0
            with torch.cuda.graph(gs, stream=self._ord_side, capture_error_mode="thread_local"):
                for g in range(G):
                    self._p = p0 ^ (g & 1)
                    _lib.run(_lib.OP_ORD_PLAN, self.spec, self._plan_args(True), self.cfg)
        except Exception as e:  # noqa: BLE001
            import sys
            print(f"two-graph capture failed ({type(e).__name__}: {e}); one graph", file=sys.stderr)
            ok = False
        finally:
            self._sync = False
        self._p, self._pending = p0, pend0
        self._set_flags_state(flags0)
        ch = (gc, p0, G, gs)
        ok = self._agree(ok)
        if ok:
            ok = self._agree(self._validate_replay(lambda: self._replay_chunk(ch), G, parity_after=p0,
                                                   ring=self.finish_mode == "batch"))
        return ch if ok else None

    def _replay_chunk(self, ch):
        """Replay a multi-generation chunk; a two-graph chunk's side graph first, on the side stream
        (after the work already queued on this one: its first plan overwrites the set of the
        generation before the chunk), the two then run on their own, ordered by the counters."""
        if ch[3] is not None:
            main = torch.cuda.current_stream(self.device)
            self._ord_side.wait_stream(main)
            with torch.cuda.stream(self._ord_side):
                ch[3].replay()
        ch[0].replay()

    def release_graphs(self):
        """Drop the captured graphs (before tearing down the process group: an RCCL
        communicator must not be destroyed while graph executables still reference it)."""
        if self._graphs is not None or self._chunks:
            torch.cuda.synchronize(self.device)
            for g in (self._graphs or []) + [c[0] for c in self._chunks] + [c[3] for c in self._chunks if c[3]]:
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

    def _validate_replay(self, replay, gens: int, parity_after=None, ring: bool = False) -> bool:
        """Run ``gens`` eager generations from the current state, restore it, run
        ``replay`` (the captured equivalent), compare bitwise, restore again."""
        state = self._state()
        saved = [t.clone() for t in state]
        p0, pend0, t0 = self._p, self._pending, self.time
        flags0 = self._flags_state()
        for _ in range(gens):
            self._generation()
        self._join_side()
        torch.cuda.synchronize(self.device)
        flags1 = self._flags_state()
        eager = [t.clone() for t in state]
        for t, v in zip(state, saved):
            t.copy_(v)
        self._p, self._pending = p0, pend0
        self._set_flags_state(flags0)
        replay()
        if parity_after is not None:
            self._p = parity_after
        self._set_flags_state(flags1)
        torch.cuda.synchronize(self.device)
        # compare the semantic state only: exchange-buffer row order and the attack
        # lists' link order follow atomics and legitimately differ between runs
        keep = {id(t) for t in self._bufs} | {id(getattr(self, k)) for k in (
            "uid", "next_uid", "_gen_ring", "counts", "census", "loss", "respawn", "action", "counterpart", "err")
            if isinstance(getattr(self, k, None), torch.Tensor)}
        if ring and isinstance(getattr(self, "_bs_ring", None), torch.Tensor):
            # (a chunk batches its finishes like the eager generations: every generation's census and
            # ballots, wherever they ran, compared too)
            keep.add(id(self._bs_ring))
        same = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8))
                   for x, y in zip(state, eager) if id(x) in keep)
        # (reference order: and no error bit the eager generations did not raise either)
        for ctl in (self._octl, self._octl1) if self.order == "sequential" else ():
            if ctl is not None:
                i = next(k for k, x in enumerate(state) if x is ctl)
                same = same and int(ctl[_lib.ORD_ERRW]) == int(eager[i][_lib.ORD_ERRW])
        for t, v in zip(state, saved):
            t.copy_(v)
        self._p, self._pending, self.time = p0, pend0, t0
        self._set_flags_state(flags0)
        torch.cuda.synchronize(self.device)
        return same
