#!/usr/bin/env python
"""The five BASELINE.json configurations, one JSON line each (rank 0 / one GPU).

  1  single WeightwiseNeuralNetwork(2,2) self-trained to a fixpoint on CPU (plumbing):
     reference-API facade, epochs/s and epochs to fixpoint
  2  10k-particle Weightwise(2,2) self-application population, bf16 table, 1 GPU:
     100 self-applications per launch, self-applications/s
  3  100k-particle soup (the headline metric): see bench.py
  4  Aggregating(4,10,3) (P = 280), 1M particles: self-application / attack / train rates
  5  mixed learn+attack soup with fp16 tables and the all-gather exchange (every rank
     holds the full table each generation), population sized from the HBM budget

The reference publishes no throughput for any of them; the numbers here
are this framework's own baseline.  Synthetic random-init particles throughout.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine, plan_population  # noqa: E402


def timeit(fn, reps=5, warmup=2, pre=None):
    """Median event time of fn(); ``pre`` (untimed) runs before every call, e.g. to restore
    the input table of an in-place operator."""
    for _ in range(warmup):
        if pre is not None:
            pre()
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        if pre is not None:
            pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)  # s
    ts.sort()
    return ts[len(ts) // 2]


def config1(args):
    from self_replicating_neural_networks_amd.models.network import (TrainingNeuralNetworkDecorator,
                                                                     WeightwiseNeuralNetwork)
    net = TrainingNeuralNetworkDecorator(WeightwiseNeuralNetwork(2, 2)).with_params(epsilon=1e-4)
    t0 = time.perf_counter()
    epochs = 0
    while not net.is_fixpoint() and epochs < 5000:
        net.train()
        epochs += 1
    dt = time.perf_counter() - t0
    return dict(config=1, name="single WW(2,2) self-train to fixpoint (CPU facade)", device="cpu",
                epochs_to_fixpoint=epochs, fixpoint=bool(net.is_fixpoint()), seconds=dt,
                epochs_per_s=epochs / dt if dt else None)


def config2(args):
    spec, n, steps = ArchSpec.weightwise(2, 2), args.n2, 100
    dev = torch.device("cuda", 0)
    uid = torch.arange(n, dtype=torch.int64, device=dev)
    res = dict(config=2, name=f"{n} WW(2,2) self-application population", steps_per_launch=steps)
    for dt_name, dtype in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        W0 = torch.zeros(n, spec.PP, dtype=dtype, device=dev)
        K.init_rows(spec, W0, uid, 1)
        W = W0.clone()

        def run():
            K.run_fixpoint(spec, W, steps, 1e-4, early_exit=False, with_sec=False)
        t = timeit(run, args.reps, pre=lambda: W.copy_(W0))
        res[f"{dt_name}_us"] = t * 1e6
        res[f"{dt_name}_self_applications_per_s"] = n * steps / t
    return res


def config4(args):
    spec, n = ArchSpec.aggregating(4, 10, 3), args.n4
    dev = torch.device("cuda", 0)
    uid = torch.arange(n, dtype=torch.int64, device=dev)
    W0 = torch.zeros(n, spec.PP, device=dev)
    K.init_rows(spec, W0, uid, 1)
    W = W0.clone()
    out = torch.empty_like(W)
    idx = torch.roll(torch.arange(n, device=dev), 1).contiguous()
    res = dict(config=4, name=f"{n} Aggregating(4,10,3) particles (P={spec.P})")

    def selfapp():
        K.run_fixpoint(spec, W, 100, 1e-4, early_exit=False, with_sec=False)
    t = timeit(selfapp, args.reps, pre=lambda: W.copy_(W0))
    res["self_apply100_ms"] = t * 1e3
    res["self_applications_per_s"] = n * 100 / t
    t = timeit(lambda: K.apply(spec, W0, out, idx_f=idx), args.reps)
    res["attack_ms"] = t * 1e3
    res["attack_GBps"] = 3 * n * spec.PP * 4 / t / 1e9
    t = timeit(lambda: K.classify(spec, W0, 1e-4), args.reps)
    res["classify_ms"] = t * 1e3
    res["classify_GBps"] = n * spec.PP * 4 / t / 1e9

    def train():
        K.train(spec, W, epochs=1, uid=uid, seed=3)
    t = timeit(train, args.reps, pre=lambda: W.copy_(W0))
    res["train_epoch_ms"] = t * 1e3
    res["train_epoch_GBps"] = 2 * n * spec.PP * 4 / t / 1e9
    res["sgd_steps_per_s"] = n / t
    return res


def config4s(args):
    """The north-star net living in a soup: Aggregating(4,10,3) particles attack, learn
    from and self-train each other (reference code/soup.py:132-134 with the P = 280 net),
    fp32 and bf16 tables, shuffle_not and shuffle_random."""
    n, gens = args.n4s, args.gens4s
    dev = torch.device("cuda", 0)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=args.train4s,
                  remove_divergent=True, remove_zero=True, epsilon=1e-4)
    res = dict(config="4s", name=f"{n} Aggregating(4,10,3) soup", n=n, params=params, gens=gens)
    variants = [(label, shuffler, dtype, "synchronous") for label, shuffler, dtype in (
        ("fp32", "none", torch.float32), ("bf16", "none", torch.bfloat16),
        ("fp32_shuffle_random", "random", torch.float32))]
    # the reference's in-place, index-ordered generation of the same soup (csrc/srnn_bignet.h BigOrd)
    if args.order4s in ("both", "sequential"):
        variants += [("ref_order_" + label, shuffler, dtype, "sequential") for label, shuffler, dtype, _ in variants]
    if args.order4s == "sequential":
        variants = [v for v in variants if v[3] == "sequential"]
    for label, shuffler, dtype, order in variants:
        spec = ArchSpec.aggregating(4, 10, 3, shuffler=shuffler)
        eng = SoupEngine(spec, n, params, device=dev, seed=0, dtype=dtype, order=order)
        eng.stats = True
        graphed = eng.capture(warmup=1)
        eng.evolve(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.evolve(gens)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[f"{label}_ms_per_generation"] = dt / gens * 1e3
        res[f"{label}_particle_generations_per_s"] = n * gens / dt
        res[f"{label}_graph"] = graphed
        res[f"{label}_generic_engine"] = bool(eng.generic)
        res[f"{label}_census"] = eng.count()
        if order == "sequential":
            res[f"{label}_levels"] = eng.ordered_levels()
        del eng
        torch.cuda.empty_cache()
    return res


def config5(args):
    spec = ArchSpec.weightwise(2, 2)
    dev = torch.device("cuda", 0)
    hbm = torch.cuda.get_device_properties(dev).total_memory
    plan = plan_population(spec, torch.float16, "allgather", world=8, hbm_bytes=hbm)
    n = args.n5
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=10,
                  remove_divergent=True, remove_zero=True, epsilon=1e-4)
    res = dict(config=5, name="mixed learn+attack soup, fp16 tables, all-gather exchange", n=n, params=params,
               hbm_bytes=hbm, hbm_plan_8gpu=plan)
    for dt_name, dtype in (("fp16", torch.float16), ("fp32", torch.float32)):
        eng = SoupEngine(spec, n, params, device=dev, seed=0, dtype=dtype, exchange="allgather")
        eng.stats = True
        eng.capture(warmup=1)
        eng.evolve(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.evolve(args.gens5)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[f"{dt_name}_ms_per_generation"] = dt / args.gens5 * 1e3
        res[f"{dt_name}_particle_generations_per_s"] = n * args.gens5 / dt
        res[f"{dt_name}_census"] = eng.last_census()
        del eng
        torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="1,2,4,5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n2", type=int, default=10_000)
    ap.add_argument("--n4", type=int, default=1_000_000)
    ap.add_argument("--n5", type=int, default=10_000_000)
    ap.add_argument("--gens5", type=int, default=10)
    ap.add_argument("--n4s", type=int, default=1_000_000)
    ap.add_argument("--gens4s", type=int, default=5)
    ap.add_argument("--train4s", type=int, default=20)
    ap.add_argument("--order4s", choices=["synchronous", "sequential", "both"], default="both",
                    help="config 4s: the synchronous generation, the reference order, or both")
    args = ap.parse_args()
    for c in args.only.split(","):
        fn = {"1": config1, "2": config2, "4": config4, "4s": config4s, "5": config5}[c.strip()]
        if c.strip() != "1" and not torch.cuda.is_available():
            print(json.dumps(dict(config=int(c), skipped="no GPU")), flush=True)
            continue
        print(json.dumps(fn(args)), flush=True)


if __name__ == "__main__":
    main()
