#!/usr/bin/env python
"""Kernel-only durations (run under rocprofv3 --kernel-trace) of the WW(2,2) self-train
kernel at 100k particles for 1, 2, 5, 20 epochs, plus one soup generation: separates the
fixed per-launch cost from the per-epoch SGD chain."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402

dev = torch.device("cuda", 0)
spec = ArchSpec.weightwise(2, 2)
n = 100000
uid = torch.arange(n, dtype=torch.int64, device=dev)
W = torch.zeros(n, spec.PP, device=dev)
K.init_rows(spec, W, uid, 1)
for ep in (1, 2, 5, 20):
    for _ in range(5):
        K.train(spec, W, epochs=ep, uid=uid, seed=2, shuffle=True)
    for _ in range(5):
        K.train(spec, W, epochs=ep, uid=uid, seed=2, shuffle=False)
for train in (0, 1, 20):
    eng = SoupEngine(spec, n, dict(attacking_rate=0.1, learn_from_rate=0.1, train=train, remove_divergent=True,
                                   remove_zero=True, epsilon=1e-4), device=dev, seed=0)
    eng.evolve(5)
torch.cuda.synchronize()
print("done")
