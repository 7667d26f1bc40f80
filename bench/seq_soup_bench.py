"""Exact sequential (in-place, index-order) soups on the native host engine: ms per generation.

The reference evolves its soups particle by particle (code/soup.py:51-87); this times
``SequentialSoupEngine`` (OP_SOUP_SEQ, one native call per evolve) on the reference's soup
parameter sets at 1000 particles, and the per-object host loop (``Soup(mode="sequential")``)
at the reference's 20-100 particle sizes for comparison.  CPU only; prints JSON lines.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.models import network as N  # noqa: E402
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine  # noqa: E402
from self_replicating_neural_networks_amd.soup import Soup  # noqa: E402
from self_replicating_neural_networks_amd.utils import rng  # noqa: E402

RESPAWN = dict(remove_divergent=True, remove_zero=True)
CASES = [
    # (name, spec, reference facade, params)
    ("ww22 train=20 (trajectory soup)", ArchSpec.weightwise(2, 2),
     lambda: N.WeightwiseNeuralNetwork(2, 2), dict(attacking_rate=0.1, learn_from_rate=-1, train=20, **RESPAWN)),
    ("ww22 learn_from severity=10", ArchSpec.weightwise(2, 2),
     lambda: N.WeightwiseNeuralNetwork(2, 2), dict(attacking_rate=-1, learn_from_rate=0.1, learn_from_severity=10, **RESPAWN)),
    ("agg422 attack+learn", ArchSpec.aggregating(4, 2, 2),
     lambda: N.AggregatingNeuralNetwork(4, 2, 2), dict(attacking_rate=0.1, learn_from_rate=0.1, **RESPAWN)),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--gens", type=int, default=20)
    ap.add_argument("--host-n", type=int, default=20)
    ap.add_argument("--host-gens", type=int, default=2)
    args = ap.parse_args()
    for name, spec, facade, params in CASES:
        e = SequentialSoupEngine(spec, args.n, dict(params, epsilon=1e-4), seed=1)
        e.evolve(1)
        t = time.perf_counter()
        e.evolve(args.gens)
        native = (time.perf_counter() - t) / args.gens * 1e3
        rng.set_seed(1)
        gen = lambda: N.TrainingNeuralNetworkDecorator(facade()).with_params(epsilon=1e-4)  # noqa: E731
        s = Soup(args.host_n, gen, mode="sequential").with_params(**params)
        s.seed()
        t = time.perf_counter()
        s.evolve(args.host_gens)
        host = (time.perf_counter() - t) / args.host_gens * 1e3
        print(json.dumps({"case": name, "native_n": args.n, "native_ms_per_gen": round(native, 3),
                          "native_us_per_particle_gen": round(native * 1e3 / args.n, 2),
                          "host_loop_n": args.host_n, "host_loop_ms_per_gen": round(host, 1),
                          "host_loop_us_per_particle_gen": round(host * 1e3 / args.host_n, 1),
                          "census": e.count()}), flush=True)


if __name__ == "__main__":
    main()
