#!/usr/bin/env python
"""Bisection of the Recurrent self-training divergence gap (docs/semantics.md §7):
published 38/50 = 76 % of RecurrentNeuralNetwork(2, 2) nets diverge within 1000 self-train
epochs (code/results/exp-training_fixpoint-*/log.txt), this framework gives ~48 %.

Every variant changes ONE ingredient of the Keras-2.2.4 formulas and reruns the experiment
on the native kernels (host or GPU), N nets each:

* init of the kernels / recurrent kernels (glorot_uniform + orthogonal is Keras' default),
* loss reduction over the 17 timesteps (Keras: mean) -- i.e. the effective step size,
* float64 instead of float32 training (is it rounding?).

  python bench/rnn_divergence_bisect.py [--n 2000] [--epochs 1000] [--device cpu]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.population import Population  # noqa: E402

SPEC = ArchSpec.recurrent(2, 2)


def _haar(n, rng):
    a = rng.standard_normal((n, n))
    u, _, v = np.linalg.svd(a)  # Keras 2.2.4 Orthogonal: SVD of a gaussian matrix
    return u


def init_variant(kind, n, rng):
    w = np.zeros((n, SPEC.P), dtype=np.float32)
    o = 0
    for li, (r, c) in enumerate(SPEC.layer_shapes):
        recurrent = li % 2 == 1
        for i in range(n):
            if recurrent and kind in ("default", "glorot_kernels_normal"):
                m = _haar(r, rng)
            elif recurrent and kind == "recurrent_identity":
                m = np.eye(r)
            elif recurrent and kind == "recurrent_glorot":
                lim = np.sqrt(6.0 / (r + c))
                m = rng.uniform(-lim, lim, (r, c))
            elif kind == "keras_uniform":  # Dense/RNN 'uniform' initializer U(-0.05, 0.05)
                m = rng.uniform(-0.05, 0.05, (r, c)) if not recurrent else _haar(r, rng)
            elif kind == "glorot_kernels_normal":
                m = rng.normal(0, np.sqrt(2.0 / (r + c)), (r, c))
            else:
                lim = np.sqrt(6.0 / (r + c))
                m = rng.uniform(-lim, lim, (r, c))
            w[i, o:o + r * c] = m.reshape(-1)
        o += r * c
    return w


def diverged_fraction(w0, epochs, lr, device, dtype_f64=False):
    if dtype_f64:  # torch autograd in float64 (the kernels are fp32)
        from tests.test_autograd_parity import _rnn_autograd_train  # noqa: E402
        w = _rnn_autograd_train(SPEC, torch.as_tensor(w0), epochs, lr)
        return float((~torch.isfinite(w).all(1)).float().mean())
    pop = Population(SPEC, w0.shape[0], device=device, weights=w0, lr=lr)
    for _ in range(epochs // 100):
        pop.train(100)
    return float((~torch.isfinite(pop.weights().float()).all(1)).float().mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--device", default="cpu")
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    rows = []
    base = init_variant("default", args.n, rng)
    rows.append(("Keras default init (glorot_uniform kernels, orthogonal recurrent), mean over T, lr 0.01",
                 diverged_fraction(base, args.epochs, 0.01, args.device)))
    for kind, label in (("recurrent_glorot", "recurrent kernels glorot_uniform instead of orthogonal"),
                        ("recurrent_identity", "recurrent kernels identity"),
                        ("keras_uniform", "kernels U(-0.05, 0.05) ('uniform')"),
                        ("glorot_kernels_normal", "kernels glorot_normal")):
        rows.append((label, diverged_fraction(init_variant(kind, args.n, rng), args.epochs, 0.01, args.device)))
    for f, label in ((17.0, "loss summed over the 17 timesteps (lr x 17)"), (2.0, "lr x 2"), (0.5, "lr x 0.5")):
        rows.append((label, diverged_fraction(base, args.epochs, 0.01 * f, args.device)))
    small = base[: min(args.n, 500)]
    rows.append(("float64 autograd model of the Keras graph (500 nets)", diverged_fraction(small, args.epochs, 0.01,
                                                                                          args.device, True)))
    for label, frac in rows:
        print(json.dumps(dict(variant=label, diverged=frac)), flush=True)


if __name__ == "__main__":
    main()
