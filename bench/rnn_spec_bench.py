#!/usr/bin/env python
"""A/B of the width / depth-specialised Recurrent wave kernels (csrc/srnn_generic.hip
k_rnn_wave<OP, W, D>) against the runtime-shape wave kernel: self-train, learn_from and
run_fixpoint + census of RNN(W, D) populations on one GPU, one JSON line per shape.

  python bench/rnn_spec_bench.py [--n 16384] [--epochs 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import _lib  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402


def timeit(fn, reps=3, warmup=1):
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
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16_384)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for w, d in [(8, 2), (16, 2), (32, 2), (8, 3), (16, 3)]:
        spec = ArchSpec.recurrent(w, d)
        n = args.n
        uid = torch.arange(n, dtype=torch.int64, device=dev)
        W = torch.zeros(n, spec.PP, device=dev)
        K.init_rows(spec, W, uid, 1)
        W0 = W.clone()
        r = {"arch": f"recurrent({w},{d})", "P": spec.P, "n": n, "epochs": args.epochs}
        for on in (False, True):
            _lib.set_rnn_spec(on)
            tag = "spec" if on else "runtime"

            def train():
                W.copy_(W0)
                K.train(spec, W, epochs=args.epochs, uid=uid, seed=3)

            def fix():
                W.copy_(W0)
                K.run_fixpoint(spec, W, 4, 1e-4, early_exit=False)

            r[f"train_us_{tag}"] = round(timeit(train, args.reps), 1)
            r[f"fixpoint4_us_{tag}"] = round(timeit(fix, args.reps), 1)
        _lib.set_rnn_spec(True)
        r["train_speedup"] = round(r["train_us_runtime"] / r["train_us_spec"], 2)
        r["fixpoint_speedup"] = round(r["fixpoint4_us_runtime"] / r["fixpoint4_us_spec"], 2)
        print(json.dumps(r), flush=True)
        del W, W0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
