#!/usr/bin/env python
"""Lanes per particle vs population size for the headline soup (WW(2,2), train 20, attack 0.1,
learn_from 0.1, respawn): ms per generation of the single-rank synchronous generation and of the
reference-order generation, one lane per particle (SRNN_SOUP_LANES=1) vs a lane pair (=2), with
and without the precomputed permutation table.  One JSON line per (order, n, lanes, table).

usage: python bench/pair_sweep.py [--sizes 12500,25000,...] [--gens 20] [--orders synchronous,sequential]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8192,12500,16384,25000,32768,50000,65536,100000")
    ap.add_argument("--gens", type=int, default=20)
    ap.add_argument("--orders", default="synchronous,sequential")
    ap.add_argument("--tables", default="1")
    args = ap.parse_args()
    import torch
    from self_replicating_neural_networks_amd.arch import ArchSpec
    from self_replicating_neural_networks_amd.config import ExecConfig
    from self_replicating_neural_networks_amd.ops import _lib
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine

    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=20, remove_divergent=True, remove_zero=True,
                  epsilon=1e-4)
    dev = torch.device("cuda", 0)
    for order in args.orders.split(","):
        for n in [int(x) for x in args.sizes.split(",")]:
            for table in [int(x) for x in args.tables.split(",")]:
                for lanes in (1, 2):
                    _lib.set_knob("soup_lanes", lanes)
                    e = SoupEngine(spec, n, params, device=dev, seed=0, order=order,
                                   execution=ExecConfig(perm_table=bool(table), graph_chunks=(20,)))
                    e.stats = True
                    e.capture(warmup=1)
                    e.evolve(4)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    e.evolve(args.gens)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / args.gens * 1e3
                    rec = dict(order=order, n=n, lanes=lanes, table=table, ms_per_gen=round(ms, 5),
                               particle_gen_per_s=n / ms * 1e3, census=e.last_census())
                    if order == "sequential":
                        rec["levels"] = e.ordered_levels()
                    print(json.dumps(rec), flush=True)
                    e.release_graphs()
                    del e
    _lib.set_knob("soup_lanes", -1)


if __name__ == "__main__":
    main()
