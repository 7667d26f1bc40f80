"""Architecture specifications of the particle networks.

A particle is a tiny linear, bias-free network whose flat weight vector is laid out in
Keras ``get_weights()`` order (reference ``code/network.py:100-104``): layer by layer,
each kernel row-major ``(in, out)``; a SimpleRNN layer contributes ``[kernel,
recurrent_kernel]``.  ``ArchSpec`` derives every shape/offset/coordinate the kernels and
the oracle need, so the four reference classes (``code/network.py:213-574``) become one
table-driven description:

=============  ===========================================  =======================
kind           layers                                       reference
=============  ===========================================  =======================
weightwise     (4,w) (w,w)x(d-1) (w,1)                      network.py:213-289
aggregating    (a,w) (w,w)x(d-1) (w,a)                      network.py:292-439
fft            as aggregating                               network.py:442-521
recurrent      [(1,w),(w,w)] [(w,w),(w,w)]x(d-1) [(w,1),(1,1)]  network.py:524-574
=============  ===========================================  =======================
"""
from __future__ import annotations

import dataclasses
import json
from typing import List, Tuple

import numpy as np

KINDS = ("weightwise", "aggregating", "recurrent", "fft")
KIND_ID = {k: i for i, k in enumerate(("weightwise", "aggregating", "recurrent", "fft"))}
AGGREGATORS = {"mean": 0, "max": 1, "max_ref": 2}
SHUFFLERS = {"none": 0, "random": 1}


def normalize_id(value: int, norm: int) -> float:
    """Reference ``WeightwiseNeuralNetwork.normalize_id`` (code/network.py:216-220)."""
    if norm > 1:
        return float(value) / float(norm)
    return float(value)


@dataclasses.dataclass(frozen=True)
class ArchSpec:
    kind: str
    width: int = 2
    depth: int = 2
    aggregates: int = 0
    aggregator: str = "mean"
    shuffler: str = "none"
    activation: str = "linear"
    use_bias: bool = False

    def __post_init__(self):
        if self.kind not in KINDS:
            raise ValueError(f"unknown network kind {self.kind!r}")
        if self.width < 1 or self.depth < 1:
            raise ValueError("width and depth must be >= 1")
        if self.kind in ("aggregating", "fft") and self.aggregates < 1:
            raise ValueError(f"{self.kind} needs aggregates >= 1")
        if self.activation != "linear" or self.use_bias:
            # every network the reference ran is linear and bias-free
            raise NotImplementedError("only linear, bias-free particles are supported")
        if self.aggregator not in AGGREGATORS:
            raise ValueError(f"unknown aggregator {self.aggregator!r}")
        if self.shuffler not in SHUFFLERS:
            raise ValueError(f"unknown shuffler {self.shuffler!r}")
        if self.kind == "aggregating":
            p, a = self.num_weights, self.aggregates
            cs = p // a
            if cs < 1 or p // cs != a:
                raise ValueError(
                    f"aggregating net with {p} weights cannot be cut into {a} chunks "
                    "(reference collect_weights, code/network.py:389-403)")
        if self.kind == "fft" and self.aggregates > self.num_weights:
            raise ValueError("fft aggregates must not exceed the number of weights")

    # -------------------------------------------------------------- constructors
    @staticmethod
    def weightwise(width=2, depth=2) -> "ArchSpec":
        return ArchSpec("weightwise", width, depth)

    @staticmethod
    def aggregating(aggregates=4, width=2, depth=2, aggregator="mean", shuffler="none") -> "ArchSpec":
        return ArchSpec("aggregating", width, depth, aggregates, aggregator, shuffler)

    @staticmethod
    def recurrent(width=2, depth=2) -> "ArchSpec":
        return ArchSpec("recurrent", width, depth)

    @staticmethod
    def fft(aggregates=4, width=2, depth=2, shuffler="none") -> "ArchSpec":
        return ArchSpec("fft", width, depth, aggregates, "mean", shuffler)

    # -------------------------------------------------------------- shapes
    @property
    def layer_shapes(self) -> List[Tuple[int, int]]:
        w, d = self.width, self.depth
        if self.kind == "weightwise":
            return [(4, w)] + [(w, w)] * (d - 1) + [(w, 1)]
        if self.kind in ("aggregating", "fft"):
            a = self.aggregates
            return [(a, w)] + [(w, w)] * (d - 1) + [(w, a)]
        # recurrent: [kernel, recurrent_kernel] per SimpleRNN layer
        shapes = [(1, w), (w, w)]
        for _ in range(d - 1):
            shapes += [(w, w), (w, w)]
        shapes += [(w, 1), (1, 1)]
        return shapes

    @property
    def num_weights(self) -> int:
        return int(sum(r * c for r, c in self.layer_shapes))

    @property
    def P(self) -> int:
        return self.num_weights

    @property
    def PP(self) -> int:
        """Padded row stride in floats (multiple of 4: one dwordx4 per 4 weights)."""
        return (self.P + 3) & ~3

    @property
    def offsets(self) -> List[int]:
        offs, o = [], 0
        for r, c in self.layer_shapes:
            offs.append(o)
            o += r * c
        return offs

    @property
    def chunk_size(self) -> int:
        return self.P // self.aggregates

    @property
    def chunks(self) -> List[Tuple[int, int]]:
        """(start, length) of every aggregation chunk; the last absorbs the leftovers."""
        cs, a = self.chunk_size, self.aggregates
        out = [(k * cs, cs) for k in range(a)]
        s, _ = out[-1]
        out[-1] = (s, self.P - s)
        return out

    def coords(self) -> np.ndarray:
        """(P, 3) normalised (layer, cell, position) coordinates of every weight
        (reference compute_all_duplex_weight_points, code/network.py:240-255)."""
        shapes = self.layer_shapes
        L = len(shapes) - 1
        out = []
        for l, (r, c) in enumerate(shapes):
            for i in range(r):
                for j in range(c):
                    out.append((normalize_id(l, L), normalize_id(i, r - 1), normalize_id(j, c - 1)))
        return np.asarray(out, dtype=np.float32)

    def unflatten(self, flat) -> List[np.ndarray]:
        flat = np.asarray(flat, dtype=np.float32).reshape(-1)[: self.P]
        return [flat[o:o + r * c].reshape(r, c).copy() for (r, c), o in zip(self.layer_shapes, self.offsets)]

    def flatten(self, weights) -> np.ndarray:
        return np.hstack([np.asarray(w, dtype=np.float32).reshape(-1) for w in weights]).astype(np.float32)

    # -------------------------------------------------------------- native config
    def native_cfg_tuple(self):
        return (KIND_ID[self.kind], self.width, self.depth, self.aggregates if self.kind in ("aggregating", "fft") else 0,
                AGGREGATORS[self.aggregator], SHUFFLERS[self.shuffler], self.PP, self.P)

    @property
    def class_name(self) -> str:
        return {"weightwise": "WeightwiseNeuralNetwork", "aggregating": "AggregatingNeuralNetwork",
                "recurrent": "RecurrentNeuralNetwork", "fft": "FFTNeuralNetwork"}[self.kind]

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), sort_keys=True)

    @staticmethod
    def from_json(s: str) -> "ArchSpec":
        return ArchSpec(**json.loads(s))
