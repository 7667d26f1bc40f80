#!/usr/bin/env python
"""Train and soup-generation timings of the reference's other network shapes on one GPU
(verdict r2 item 5): which engine serves each shape (templated lane kernels, wave kernels or
the runtime-shape engine), SGD steps/s, soup generation time at the headline parameters and
its ratio to WW(2,2) against the ratio of the per-particle FLOPs of one generation.

  python bench/shape_bench.py [--n 100000] [--epochs 20] [--only weightwise(4,3)]

One JSON line per shape."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import _lib  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402

PARAMS = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, remove_divergent=True,
              remove_zero=True, epsilon=1e-4)


def timeit(fn, reps=5, warmup=1):
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
    ts.sort()
    return ts[len(ts) // 2]


def sgd_macs(spec):
    """MACs of one SGD step (forward + input gradients + weight updates) of one particle."""
    if spec.kind == "weightwise":
        shapes = spec.layer_shapes
        fwd = sum(r * c for r, c in shapes)
        bwd = sum(r * c for r, c in shapes[1:])
        return fwd + bwd + fwd, spec.P  # per step, steps per epoch
    if spec.kind == "recurrent":
        fwd = spec.P * spec.P  # P timesteps of a P-weight cell stack (approx.)
        return 3 * fwd, 1
    return 3 * spec.P, 1


def engine_of(spec, op):
    if _lib.is_generic(spec, op):
        if op in (_lib.OP_TRAIN, _lib.OP_LEARN):
            if spec.kind == "weightwise" and spec.P > 16 and 3 <= spec.width <= 64:
                return "runtime-shape, lanes-per-particle waves (k_ww_wave)"
            if spec.kind == "recurrent" and spec.width >= 8:
                spec_wd = (spec.width, spec.depth) in ((8, 2), (16, 2), (32, 2), (8, 3), (16, 3))
                return ("width/depth-specialised" if spec_wd else "runtime-shape") + ", wave per particle (k_rnn_wave)"
        if (op == _lib.OP_SOUP_EVOLVE and spec.kind == "recurrent" and spec.width >= 8
                and os.environ.get("SRNN_RNN_SOUP", "1") != "0"):
            return "runtime-shape, wave per particle (k_rnn_wave_soup)"
        return "runtime-shape, lane per particle"
    return "wave" if K.is_wave_per_particle(spec) else "lane"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--big-n", type=int, default=16_384, help="population of the shapes with P > 100")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--soup-max-p", type=int, default=400,
                    help="time soup generations only up to this P (larger nets' soups run the lane path)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    specs = [ArchSpec.weightwise(2, 2), ArchSpec.weightwise(3, 3), ArchSpec.weightwise(4, 3),
             ArchSpec.weightwise(10, 3), ArchSpec.weightwise(16, 2), ArchSpec.recurrent(2, 2),
             ArchSpec.recurrent(8, 2), ArchSpec.recurrent(16, 2)]
    base = None
    for spec in specs:
        name = f"{spec.kind}({spec.width},{spec.depth})"
        if args.only and args.only != name and name != "weightwise(2,2)":
            continue
        n = args.n if spec.P <= 100 else args.big_n
        uid = torch.arange(n, dtype=torch.int64, device=dev)
        W = torch.zeros(n, spec.PP, device=dev)
        K.init_rows(spec, W, uid, 1)
        W0 = W.clone()
        r = {"arch": name, "P": spec.P, "n": n, "epochs": args.epochs,
             "train_engine": engine_of(spec, _lib.OP_TRAIN), "soup_engine": engine_of(spec, _lib.OP_SOUP_EVOLVE)}

        def train():
            W.copy_(W0)
            K.train(spec, W, epochs=args.epochs, uid=uid, seed=3)
        t = timeit(train, args.reps)
        macs, steps = sgd_macs(spec)
        r["train_us"] = round(t, 1)
        r["sgd_steps_per_s"] = n * args.epochs * steps / (t * 1e-6)
        r["train_tflops"] = n * args.epochs * steps * macs * 2 / (t * 1e-6) / 1e12
        print(json.dumps({"arch": name, "train_us": r["train_us"], "note": "train done"}), flush=True)
        if spec.P > args.soup_max_p:
            print(json.dumps(r), flush=True)
            continue
        eng = SoupEngine(spec, n, dict(PARAMS, train=args.epochs), device=dev, seed=5)
        eng.evolve(1)
        r["soup_gen_us"] = round(timeit(lambda: eng.evolve(1), args.reps), 1)
        if eng.capture():
            r["soup_gen_graph_us"] = round(timeit(lambda: eng.evolve(4), args.reps) / 4, 1)
        gen_flops = (args.epochs + 0.1) * steps * macs * 2  # train + learn_from epochs per particle
        r["gen_flops_per_particle"] = gen_flops
        t_gen = r.get("soup_gen_graph_us", r["soup_gen_us"])
        if base is None:
            base = (t_gen, gen_flops)
        r["time_ratio_vs_ww22"] = round(t_gen / base[0] * args.n / n, 2)  # per particle
        r["flop_ratio_vs_ww22"] = round(gen_flops / base[1], 2)
        print(json.dumps(r), flush=True)
        del eng, W, W0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
