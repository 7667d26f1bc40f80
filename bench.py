#!/usr/bin/env python
"""Headline benchmark: self-application steps/sec of a soup on 1..8 MI355X GPUs.

Metric (BASELINE.json): "self-application steps/sec (whole node) for 100k-particle soup".
One step = one soup generation (reference ``Soup.evolve``, code/soup.py:51-87) for every
particle: attacks (rate 0.1), learn_from (rate 0.1, severity 1), 20 self-train epochs,
divergent/zero respawn, plus the per-generation fixpoint census (``Soup.count``,
code/soup.py:89-103) all-reduced over ranks.  The soup configuration is the reference's
active soup demo (code/soup.py:127-138: WeightwiseNeuralNetwork(2, 2), train=20,
remove_divergent, remove_zero, epsilon=1e-4) with 100k particles per GPU (weak
scaling: the population is sharded, every rank owns 100k particles; at N=1 this is the
100k-particle soup).  Random-init weights, fp32 (the reference's dtype; bf16 would make
the 1e-4 fixpoint test meaningless).

Multi-GPU (N>1): every rank owns 100k particles; one generation is ONE all-to-all on the
soup's own RCCL communicator (partner rows + per-rank stats rows, over xGMI) -> post-exchange
launch (received-row index + newborn uids) -> generation kernel (evolve + census + the next
generation's decisions of every global slot) -> finish launch (counts + packing the next
exchange).  Single GPU: the generation kernel + finish, 8 generations per hipGraph.

value = particles x generations / second over the whole job (max time over ranks).

Usage: python bench.py --gpus N --steps K --warmup W
       (N>1 is launched by torch.distributed.run, one rank per GPU, RCCL over xGMI)
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.parallel.dist import from_env  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--particles-per-gpu", type=int, default=100_000)
    ap.add_argument("--train", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (rehearsal)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0")
    ap.add_argument("--force-sharded", action="store_true",
                    help="rehearsal: run the multi-GPU generation (RCCL all-to-all) even with one rank")
    args = ap.parse_args()
    if args.force_sharded:
        os.environ["SRNN_FORCE_SHARDED"] = "1"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.share_device:
        os.environ["SRNN_SHARE_DEVICE"] = "1"
    d = from_env(backend=args.backend)
    dev = torch.device("cuda", 0 if args.share_device else d.local_rank)
    torch.cuda.set_device(dev)

    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=args.train,
                  remove_divergent=True, remove_zero=True, epsilon=1e-4)
    n_total = args.particles_per_gpu * d.world
    eng = SoupEngine(spec, n_total, params, device=dev, seed=args.seed, dist=d)
    eng.stats = not args.no_stats
    graphed = False
    if not args.no_graph:
        graphed = eng.capture(warmup=1)
    eng.evolve(args.warmup)
    torch.cuda.synchronize(dev)
    d.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.evolve(args.steps)
    torch.cuda.synchronize(dev)
    d.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if d.enabled:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if eng.exchange_overflowed():
        # rows that did not fit the all-to-all capacity were dropped: the generation is invalid
        raise SystemExit(f"soup row exchange overflowed its capacity (ovf flags {int(eng.ovf.item())}: 1 rows dropped, "
                         "2 a wait timed out): the measured generations are invalid")
    census = eng.count()
    value = n_total * args.steps / dt
    if d.rank == 0:
        print(json.dumps({
            "metric": "self-application steps/sec (whole node) for 100k-particle soup",
            "value": value,
            "unit": "particle-generations/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (random-init particles, Philox seed %d)" % args.seed,
            "config": {"model": "Soup of WeightwiseNeuralNetwork(width=2, depth=2), train=20, attack 0.1, "
                                "learn_from 0.1, remove divergent/zero",
                       "global_batch": n_total, "particles_per_gpu": args.particles_per_gpu, "seq_len": None,
                       "parallelism": f"population-dp{d.world}", "hip_graph": graphed,
                       "multi_generation_graph": eng._chunk is not None,
                       "collectives": ("native RCCL communicator (" + d.native.library + ")") if d.native
                       else ("torch.distributed" if d.enabled else None),
                       "census_every_step": eng.stats, "final_census": census},
        }), flush=True)
    eng.release_graphs()  # graph executables reference the RCCL communicator
    d.close()
    if d.enabled:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
