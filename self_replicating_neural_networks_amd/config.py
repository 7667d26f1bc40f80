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
from typing import Any, Dict, Optional

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
    recorder: RecorderConfig = RecorderConfig()

    def validate(self):
        if self.n_total < 1 or self.generations < 0:
            raise ValueError("n_total >= 1 and generations >= 0 required")
        if self.dtype not in _DTYPES:
            raise ValueError(f"dtype must be one of {_DTYPES}")
        if self.exchange not in ("alltoall", "allgather"):
            raise ValueError("exchange must be alltoall or allgather")
        if self.device not in ("cuda", "cpu"):
            raise ValueError("device must be cuda or cpu")
        if self.census_every not in (0, 1):
            # the census is fused into the generation kernel: on (every generation) or off
            raise ValueError("census_every must be 0 (final census only) or 1 (every generation)")
        self.recorder.validate()
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
        return dict(arch=json.loads(self.arch.to_json()), soup=dataclasses.asdict(self.soup),
                    run=dataclasses.asdict(self.run))

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), indent=1, sort_keys=True)

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "ExperimentConfig":
        run = dict(d.get("run", {}))
        run.pop("reference_compat", None)  # accepted from round-1 config files; quirks live in the compat API
        rec = RecorderConfig(**run.pop("recorder", {}))
        return ExperimentConfig(arch=ArchSpec.from_json(json.dumps(d["arch"])) if "arch" in d else ArchSpec.weightwise(2, 2),
                                soup=SoupConfig(**d.get("soup", {})), run=RunConfig(recorder=rec, **run)).validate()

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
