#!/usr/bin/env python
"""Timeline of one device reference-order generation by dependency level (SoupEngine.ordered_trace:
s_memrealtime at each turn's start and end), the bench soup by default.

    python bench/ordered_trace.py [--particles N] [--warmup W]
prints one JSON line: per level {turns, first_start, last_start, last_end, mean_us, max_us}
(microseconds after the generation's first turn started)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=100_000)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gens", type=int, default=2)
    ap.add_argument("--slots", type=int, default=2, help="10: per-phase stamps + the self-train clock (library built with -DSRNN_ORD_TRACE_FINE)")
    args = ap.parse_args()
    import torch
    from self_replicating_neural_networks_amd.arch import ArchSpec
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine

    params = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=20,
                  remove_divergent=True, remove_zero=True, epsilon=1e-4)
    eng = SoupEngine(ArchSpec.weightwise(2, 2), args.particles, params, device="cuda", order="sequential")
    eng.evolve(args.warmup)
    eng.ordered_trace(True, slots=args.slots)
    for g in range(args.gens):
        eng.evolve(1)
        torch.cuda.synchronize()
        print(json.dumps({"generation": eng.time, "levels": eng.ordered_levels()["levels"],
                          "timeline": eng.ordered_timeline(),
                          "env": {k: v for k, v in os.environ.items() if k.startswith("SRNN_")}}), flush=True)


if __name__ == "__main__":
    main()
