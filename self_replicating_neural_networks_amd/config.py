"""Typed configuration.

The reference configures everything through mutable kwargs dicts (``with_params``,
``Soup.with_params``, ad-hoc experiment attributes; code/network.py:92-98,
code/soup.py:17-18, :33-35).  Here the same knobs are frozen dataclasses that serialise
to JSON, are stored in checkpoints and drive the command-line runner
(``python -m self_replicating_neural_networks_amd.run``).  The fluent ``with_params``
API stays on the compat facades.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Any, Dict, Optional, Tuple

from .arch import ArchSpec

_DTYPES = ("float32", "bfloat16", "float16")


@dataclasses.dataclass(frozen=True)
class SoupConfig:
    """``Soup.params`` of the reference (code/soup.py:17-18), same names and defaults."""
    attacking_rate: float = 0.1
    learn_from_rate: float = 0.1
    train: int = 0
    learn_from_severity: int = 1
    remove_divergent: bool = False
    remove_zero: bool = False
    epsilon: float = 1e-4
    segment: int = 0  # >0: independent sub-soups of this many particles (setups at population scale)

    def params(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def validate(self):
        if self.train < 0 or self.learn_from_severity < 0:
            raise ValueError("train and learn_from_severity must be >= 0")
        if self.epsilon <= 0:
            raise ValueError("epsilon must be > 0")
        if self.segment < 0:
            raise ValueError("segment must be >= 0")
        return self


@dataclasses.dataclass(frozen=True)
class RecorderConfig:
    """Trajectory sampling policy: which particles, how often."""
    policy: str = "none"            # none | subset | full
    every: int = 1                  # record every k generations
    subset: int = 0                 # policy "subset": number of slots (evenly spaced)
    capacity: int = 1024            # ring-buffer snapshots kept on the host

    def validate(self):
        if self.policy not in ("none", "subset", "full"):
            raise ValueError(f"unknown recorder policy {self.policy!r}")
        if self.every < 1 or self.capacity < 1:
            raise ValueError("every and capacity must be >= 1")
        if self.policy == "subset" and self.subset < 1:
            raise ValueError("policy 'subset' needs subset >= 1")
        return self


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    return default if v is None or v == "" else v not in ("0", "false", "False", "no")


def _tri_state(v: str) -> Optional[bool]:
    """A tri-state knob's environment value: -1 / auto / none -> None (the built-in choice),
    0 / false / no / off -> False, anything else -> True."""
    t = v.strip().lower()
    if t in ("-1", "auto", "none", "default"):
        return None
    return t not in ("0", "false", "no", "off")


@dataclasses.dataclass(frozen=True)
class ExecConfig:
    """Execution knobs: which schedule / kernel family runs, never what is computed (every
    choice gives bitwise the same soup).  Each field has an environment variable that, when
    set, overrides it (A/B runs on the GPU box); ``resolved()`` applies those overrides and
    is what the engines use and what bench.py prints.

    Engine-level (``SoupEngine``): ``finish_mode``, ``finish_par``, ``graph_chunks``,
    ``x2_schedule``, ``x2_prio``, ``x2_emulate_remote``, ``sharded_graph``; process-level
    (``Dist``): ``native_comm``, ``loopback``; library-level (libsrnn knobs, process wide,
    ``apply_library()``): ``force_generic`` ... ``soup_lanes`` (None: the library's default)."""
    finish_mode: str = "batch"              # SRNN_FINISH_MODE: batch | serial (single-rank generation finish)
    finish_par: bool = True                 # SRNN_FINISH_PAR: one finish workgroup per batched generation
    graph_chunks: Tuple[int, ...] = (20, 16, 8, 4, 2)  # SRNN_GRAPH_CHUNKS: generations per multi-generation graph
    x2_schedule: str = "serial"             # SRNN_X2_SCHEDULE: serial | overlap (sharded generation)
    x2_prio: bool = True                    # SRNN_X2_PRIO: raised wave priority of the exchange chain
    x2_emulate_remote: float = 0.0          # SRNN_X2_EMULATE_REMOTE: one-rank timing model of R ranks
    sharded_graph: bool = True              # SRNN_SHARDED_GRAPH: capture sharded generations (RCCL inside)
    native_comm: bool = True                # SRNN_NATIVE_COMM: the soup's own RCCL communicator
    loopback: bool = False                  # SRNN_LOOPBACK: one-rank all-to-all as a device copy
    force_generic: Optional[bool] = None    # SRNN_FORCE_GENERIC
    ww_wave: Optional[int] = None           # SRNN_WW_WAVE: 0 lane path, 1 waves (register SGD where
                                            # instantiated), 2 waves with the LDS SGD
    rnn_wave: Optional[bool] = None         # SRNN_RNN_WAVE
    rnn_spec: Optional[bool] = None         # SRNN_RNN_SPEC
    rnn_soup: Optional[bool] = None         # SRNN_RNN_SOUP
    big_wave: Optional[bool] = None         # SRNN_BIG_WAVE
    fix_group: Optional[bool] = None        # SRNN_FIX_GROUP (None: by population size)
    soup_lanes: Optional[int] = None        # SRNN_SOUP_LANES (None / 0: by population size)
    ord_crit: Optional[bool] = None         # SRNN_ORD_CRIT: reference-order generations run the producers of
                                            # later turns first, at raised wave priority (None: on)
    ord_queue: Optional[bool] = None        # SRNN_ORD_QUEUE: reference-order continuations through one ready
                                            # queue per generation, or per-wave lists (None: lists, measured
                                            # faster -- 0.173 vs 0.296 ms, profiles/r6a r6q)
    ord_shadow: Optional[int] = None        # SRNN_ORD_SHADOW: a reference-order round of at most this many
                                            # turns in a wave runs each on several lanes (None: 32, measured best
                                            # of 16 / 32 / 63; 0: off)
    ord_bulk_delay: Optional[int] = None    # SRNN_ORD_BULK_DELAY: microseconds a reference-order run's turn
                                            # waves wait before their first turn, the critical chain's root
                                            # ahead of the bulk (None: 12 for the lane nets, first residency
                                            # round only, measured best of 0-35; 0 for the big nets)
    ordsh_emulate: int = 0                  # SRNN_ORDSH_EMULATE: one-rank timing model of R ranks of a sharded
                                            # reference-order generation (the rank runs 1/R of the turns;
                                            # the other turns never run: timing only, results invalid)
    order_levels: int = 4                   # SRNN_ORDER_LEVELS: dependency levels a reference-order generation
                                            # reports one by one (ordered_levels; deeper: the tail bin)
    perm_table: Optional[bool] = None       # SRNN_PERM_TABLE: a generation's SGD permutations precomputed by
                                            # one launch ahead of it (nibble Weightwise nets on the device;
                                            # None: the reference order's pending turns only)
    ord_pipeline: str = "stream"            # SRNN_ORD_PIPELINE: a single-rank reference-order generation's plan
                                            # (lists, versions, records, permutations) is built one generation
                                            # ahead -- "stream": by launches on a side stream (a hipGraph join per
                                            # generation); "kernel": by the last workgroups of the run launch in
                                            # flight (measured slower: 0.288 vs 0.176 ms, profiles/r6a); "off":
                                            # inline, before each run (True / False: stream / off)
    ord_census_side: bool = True            # SRNN_ORD_CENSUS_SIDE: with the side-stream plan, each generation's
                                            # census runs on the side stream beside the next run, the close keeps
                                            # only the final rows, ballots and counter
    ord_graph_sync: bool = True             # SRNN_ORD_GRAPH_SYNC: with the side-stream plan, a multi-generation
                                            # hipGraph is TWO graphs replayed on two streams (the generations on
                                            # the current one, their plans on a high-priority side stream),
                                            # ordered by device counters instead of a cross-queue join per
                                            # generation (SRNN_F_ORD_SYNC; validated bitwise, else not used)

    _ENV = dict(finish_mode="SRNN_FINISH_MODE", finish_par="SRNN_FINISH_PAR", graph_chunks="SRNN_GRAPH_CHUNKS",
                x2_schedule="SRNN_X2_SCHEDULE", x2_prio="SRNN_X2_PRIO", x2_emulate_remote="SRNN_X2_EMULATE_REMOTE",
                sharded_graph="SRNN_SHARDED_GRAPH", native_comm="SRNN_NATIVE_COMM", loopback="SRNN_LOOPBACK",
                force_generic="SRNN_FORCE_GENERIC", ww_wave="SRNN_WW_WAVE", rnn_wave="SRNN_RNN_WAVE",
                rnn_spec="SRNN_RNN_SPEC", rnn_soup="SRNN_RNN_SOUP", big_wave="SRNN_BIG_WAVE",
                fix_group="SRNN_FIX_GROUP", soup_lanes="SRNN_SOUP_LANES", ord_crit="SRNN_ORD_CRIT", ord_queue="SRNN_ORD_QUEUE",
                ord_shadow="SRNN_ORD_SHADOW", ord_bulk_delay="SRNN_ORD_BULK_DELAY",
                ordsh_emulate="SRNN_ORDSH_EMULATE",
                order_levels="SRNN_ORDER_LEVELS",
                perm_table="SRNN_PERM_TABLE", ord_pipeline="SRNN_ORD_PIPELINE",
                ord_census_side="SRNN_ORD_CENSUS_SIDE", ord_graph_sync="SRNN_ORD_GRAPH_SYNC")
    # Optional[bool] knobs whose None means "the built-in choice" (by population size, ...)
    TRI_STATE = ("force_generic", "rnn_wave", "rnn_spec", "rnn_soup", "big_wave", "fix_group", "perm_table",
                 "ord_crit", "ord_queue")
    LIBRARY_KNOBS = ("force_generic", "ww_wave", "rnn_wave", "rnn_spec", "rnn_soup", "big_wave", "fix_group",
                     "soup_lanes", "ord_crit", "ord_queue", "ord_shadow", "ord_bulk_delay")

    def validate(self):
        if self.finish_mode not in ("batch", "serial"):
            raise ValueError("finish_mode must be batch or serial")
        if self.x2_schedule not in ("serial", "overlap"):
            raise ValueError("x2_schedule must be serial or overlap")
        if any(int(g) < 2 or int(g) % 2 for g in self.graph_chunks):
            raise ValueError("graph_chunks must be even sizes >= 2")
        if not 0.0 <= self.x2_emulate_remote <= 1.0:
            raise ValueError("x2_emulate_remote is a fraction in [0, 1]")
        if not 1 <= int(self.order_levels) <= 16:
            raise ValueError("order_levels must be in 1..16")
        if self.ord_pipeline not in ("kernel", "stream", "off"):
            raise ValueError("ord_pipeline must be kernel, stream or off")
        return self

    def __post_init__(self):
        # (booleans of the earlier on/off knob: on = the side-stream form)
        if isinstance(self.ord_pipeline, bool):
            object.__setattr__(self, "ord_pipeline", "stream" if self.ord_pipeline else "off")

    def resolved(self) -> "ExecConfig":
        """This config with every knob whose environment variable is set overridden by it."""
        kw = {}
        for f in dataclasses.fields(self):
            env = self._ENV.get(f.name)
            v = os.environ.get(env) if env else None
            if v is None or v == "":
                continue
            cur = getattr(self, f.name)
            if f.name == "graph_chunks":
                kw[f.name] = tuple(sorted({int(x) for x in v.split(",") if int(x) >= 2 and int(x) % 2 == 0},
                                          reverse=True))
            elif f.name in ("finish_mode", "x2_schedule"):
                kw[f.name] = v
            elif f.name == "ord_pipeline":
                kw[f.name] = {"1": "stream", "true": "stream", "on": "stream", "0": "off", "false": "off"}.get(v.lower(), v)
            elif f.name == "x2_emulate_remote":
                kw[f.name] = float(v)
            elif f.name in ("soup_lanes", "order_levels", "ww_wave", "ordsh_emulate", "ord_shadow", "ord_bulk_delay"):
                kw[f.name] = int(v)
            elif f.name in self.TRI_STATE:
                kw[f.name] = _tri_state(v)
            else:
                kw[f.name] = _env_bool(env, bool(cur))
        return dataclasses.replace(self, **kw).validate() if kw else self.validate()

    def apply_library(self) -> None:
        """Push the library-level knobs that are set (not None) into libsrnn (process wide;
        their environment variables still override inside the library)."""
        from .ops import _lib
        for name in self.LIBRARY_KNOBS:
            v = getattr(self, name)
            if v is not None:
                _lib.set_knob(name, int(v))

    def as_dict(self) -> Dict[str, Any]:
        d = {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}
        d["graph_chunks"] = list(self.graph_chunks)
        return d

    def in_force(self) -> Dict[str, Any]:
        """The resolved knobs plus the library knobs' values in force (env included; -1 =
        the library's built-in default): what a benchmark line records."""
        d = self.resolved().as_dict()
        try:
            from .ops import _lib
            d["library"] = {k: _lib.get_knob(k) for k in self.LIBRARY_KNOBS}
        except Exception:  # noqa: BLE001 -- no library: nothing to report
            pass
        return d


@dataclasses.dataclass(frozen=True)
class RunConfig:
    """How a soup runs: population, precision, parallelism, I/O."""
    n_total: int = 100_000
    generations: int = 100
    seed: int = 0
    lr: float = 0.01
    shuffle: bool = True
    dtype: str = "float32"                 # weight-table storage (arithmetic is fp32)
    exchange: str = "alltoall"             # sharded row exchange: alltoall | allgather
    device: str = "cuda"                   # cuda | cpu
    backend: Optional[str] = None          # torch.distributed backend (nccl = RCCL; gloo on CPU)
    graph: bool = True                     # capture generations in hipGraphs
    census_every: int = 1                  # 1: census every generation, 0: only at the end
    metrics_path: Optional[str] = None     # JSONL stream of per-generation metrics
    metrics_every: int = 1
    checkpoint_dir: Optional[str] = None   # periodic native checkpoints (exact resume)
    checkpoint_every: int = 0
    collective_timeout_s: float = 600.0    # process-group timeout (failure detection)
    # soup semantics: "sequential" -- the reference's in-place, index-order Soup.evolve
    # (code/soup.py:51-87), level-scheduled on the device; "synchronous" -- Jacobi (every read
    # from the generation-start table), the variant for shapes / rank counts the ordered
    # generation does not cover.  A checkpoint records it; resuming with the other order raises.
    order: str = "sequential"
    recorder: RecorderConfig = RecorderConfig()
    execution: ExecConfig = ExecConfig()   # schedules / kernel families (env vars override)

    def validate(self):
        if self.n_total < 1 or self.generations < 0:
            raise ValueError("n_total >= 1 and generations >= 0 required")
        if self.dtype not in _DTYPES:
            raise ValueError(f"dtype must be one of {_DTYPES}")
        if self.exchange not in ("alltoall", "allgather"):
            raise ValueError("exchange must be alltoall or allgather")
        if self.device not in ("cuda", "cpu"):
            raise ValueError("device must be cuda or cpu")
        if self.order not in ("sequential", "synchronous"):
            raise ValueError("order must be sequential (the reference's) or synchronous (Jacobi)")
        if self.census_every not in (0, 1):
            # the census is fused into the generation kernel: on (every generation) or off
            raise ValueError("census_every must be 0 (final census only) or 1 (every generation)")
        self.recorder.validate()
        self.execution.validate()
        return self

    def torch_dtype(self):
        import torch
        return {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}[self.dtype]


@dataclasses.dataclass(frozen=True)
class ExperimentConfig:
    """One soup experiment: architecture + soup parameters + run settings."""
    arch: ArchSpec = ArchSpec.weightwise(2, 2)
    soup: SoupConfig = SoupConfig()
    run: RunConfig = RunConfig()

    def validate(self):
        self.soup.validate()
        self.run.validate()
        return self

    def to_dict(self) -> Dict[str, Any]:
        run = dataclasses.asdict(self.run)
        run["execution"] = self.run.execution.as_dict()
        return dict(arch=json.loads(self.arch.to_json()), soup=dataclasses.asdict(self.soup), run=run)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), indent=1, sort_keys=True)

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "ExperimentConfig":
        run = dict(d.get("run", {}))
        run.pop("reference_compat", None)  # accepted from round-1 config files; quirks live in the compat API
        rec = RecorderConfig(**run.pop("recorder", {}))
        ex = dict(run.pop("execution", {}))
        if "graph_chunks" in ex:
            ex["graph_chunks"] = tuple(ex["graph_chunks"])
        ex = ExecConfig(**ex)
        return ExperimentConfig(arch=ArchSpec.from_json(json.dumps(d["arch"])) if "arch" in d else ArchSpec.weightwise(2, 2),
                                soup=SoupConfig(**d.get("soup", {})),
                                run=RunConfig(recorder=rec, execution=ex, **run)).validate()

    @staticmethod
    def from_json(s: str) -> "ExperimentConfig":
        return ExperimentConfig.from_dict(json.loads(s))

    @staticmethod
    def load(path: str) -> "ExperimentConfig":
        with open(path) as f:
            return ExperimentConfig.from_json(f.read())

    def replace(self, **sections) -> "ExperimentConfig":
        """Copy with section fields overridden: ``cfg.replace(run=dict(n_total=10))``."""
        out = self
        for name, kw in sections.items():
            out = dataclasses.replace(out, **{name: dataclasses.replace(getattr(out, name), **kw)})
        return out.validate()
