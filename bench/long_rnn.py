#!/usr/bin/env python
"""SURVEY §5.7 analogue of long context: Recurrent nets whose sequence (their own weight
vector, length P) grows with width/depth.  Throughput of self-application and BPTT
self-training on the runtime-shape engine (lane per particle, BPTT states element-major in
device scratch) for P from 17 to ~5000 timesteps.

  python bench/long_rnn.py [--n 20000]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.population import Population  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    args = ap.parse_args()
    for w, d in ((2, 2), (4, 2), (8, 2), (16, 2), (16, 4), (32, 2)):
        spec = ArchSpec.recurrent(w, d)
        n = args.n if spec.P < 1000 else max(args.n // 4, 1024)
        pop = Population(spec, n, device="cuda", seed=1)
        W0 = pop.W.clone()

        def train():
            pop.W.copy_(W0)
            pop.train(1)

        def apply():
            pop.W.copy_(W0)
            pop.self_apply(1)
        tt, ta = timed(train), timed(apply)
        print(json.dumps(dict(arch=f"RecurrentNeuralNetwork({w}, {d})", P=spec.P, n=n,
                              train_epoch_ms=tt * 1e3, bptt_timesteps_per_s=n * spec.P / tt,
                              self_apply_ms=ta * 1e3, rnn_steps_per_s=n * spec.P / ta)), flush=True)
        del pop, W0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
