#!/usr/bin/env python
"""Per-kernel micro-benchmarks on one GPU (hipEvent timing, random-init particles).

Reports, for a population of N particles of each shipped architecture:
  init, self-apply (100 steps, one launch), run_fixpoint (early exit), classify,
  train (E epochs), learn_from, soup generation (fused evolve pipeline).
Derived: particle-ops/s and effective FLOP rate of the compute (VALU fp32).
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
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402


def timeit(fn, reps=5, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)  # us
    ts.sort()
    return ts[len(ts) // 2]


def flops_apply(spec):
    # MACs of one application (layerwise evaluation) x2
    if spec.kind == "weightwise":
        w, d = spec.width, spec.depth
        return 2 * spec.P * (4 * w + (d - 1) * w * w + w)
    return 2 * spec.P  # small MLP on aggregates / rnn scan: ~P MACs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--big-n", type=int, default=1_000_000, help="population of the big aggregating nets")
    ap.add_argument("--wide-n", type=int, default=100_000, help="population of the MFMA weightwise nets")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    specs = [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2),
             ArchSpec.fft(4, 2, 2), ArchSpec.weightwise(4, 3), ArchSpec.aggregating(4, 10, 3),
             ArchSpec.weightwise(16, 2), ArchSpec.weightwise(32, 2)]
    res = []
    for spec in specs:
        name = f"{spec.kind}({spec.aggregates},{spec.width},{spec.depth})"
        if args.only and args.only not in name:
            continue
        n = args.n
        uid = torch.arange(n, dtype=torch.int64, device=dev)
        W = torch.zeros(n, spec.PP, device=dev)
        K.init_rows(spec, W, uid, 1)
        W0 = W.clone()
        out = torch.zeros_like(W)
        big = K.is_wave_per_particle(spec)
        if big and args.big_n:
            if spec.kind == "weightwise":
                args_n = args.wide_n
            else:
                args_n = args.big_n
            n = args_n
            uid = torch.arange(n, dtype=torch.int64, device=dev)
            W = torch.zeros(n, spec.PP, device=dev)
            K.init_rows(spec, W, uid, 1)
            W0 = W.clone()
            out = torch.zeros_like(W)
        r = {"arch": name, "P": spec.P, "n": n}
        r["init_us"] = timeit(lambda: K.init_rows(spec, W, uid, 1), args.reps)

        def selfapply():
            W.copy_(W0)
            K.run_fixpoint(spec, W, 100, 1e-4, early_exit=False, with_sec=False)
        t = timeit(selfapply, args.reps)
        r["self_apply100_us"] = t
        r["self_apply_per_s"] = n * 100 / (t * 1e-6)
        r["self_apply_tflops"] = n * 100 * flops_apply(spec) / (t * 1e-6) / 1e12
        r["apply_attack_us"] = timeit(lambda: K.apply(spec, W0, out, idx_f=torch.roll(uid, 1)), args.reps)
        # HBM traffic of one attack: attacker + target rows read, output row written
        r["apply_attack_GBps"] = 3 * n * spec.PP * 4 / (r["apply_attack_us"] * 1e-6) / 1e9
        r["classify_us"] = timeit(lambda: K.classify(spec, W0, 1e-4), args.reps)

        def train():
            W.copy_(W0)
            K.train(spec, W, epochs=args.epochs, uid=uid, seed=3)
        if spec.kind == "weightwise" and big:
            res.append(r)
            print(json.dumps(r), flush=True)
            continue
        t = timeit(train, args.reps)
        r["train_us"] = t
        steps = spec.P if spec.kind == "weightwise" else 1
        r["sgd_steps_per_s"] = n * args.epochs * steps / (t * 1e-6)
        if big:
            res.append(r)
            print(json.dumps(r), flush=True)
            continue
        eng = SoupEngine(spec, n, dict(train=args.epochs, remove_divergent=True, remove_zero=True, epsilon=1e-4),
                         device=dev, seed=5)
        r["soup_gen_us"] = timeit(lambda: eng.evolve(1), args.reps)
        eng.capture()
        r["soup_gen_graph_us"] = timeit(lambda: eng.evolve(1), args.reps)
        res.append(r)
        print(json.dumps(r), flush=True)
    return res


if __name__ == "__main__":
    main()
