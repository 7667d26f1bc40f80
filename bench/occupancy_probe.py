#!/usr/bin/env python
"""Time of the lane-per-particle kernels vs population size around the 1024-SIMD
boundaries (1024 waves = one per SIMD): shows whether co-resident waves share a SIMD for
free (the 100k-particle soup has 1563 waves)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402


def t_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


spec = ArchSpec.weightwise(2, 2)
dev = torch.device("cuda", 0)
for n in (16384, 32768, 49152, 65536, 81920, 100000, 114688, 131072, 196608, 262144, 524288):
    uid = torch.arange(n, dtype=torch.int64, device=dev)
    W0 = torch.zeros(n, spec.PP, device=dev)
    K.init_rows(spec, W0, uid, 1)
    W = W0.clone()

    def tr():
        W.copy_(W0)
        K.train(spec, W, epochs=20, uid=uid, seed=2)
    train_ms = t_ms(tr)
    eng = SoupEngine(spec, n, dict(attacking_rate=0.1, learn_from_rate=0.1, train=20, remove_divergent=True,
                                   remove_zero=True, epsilon=1e-4), device=dev, seed=0)
    eng.capture(warmup=1)
    gen_ms = t_ms(lambda: eng.evolve(10)) / 10
    print(json.dumps(dict(n=n, waves=-(-n // 64), train20_ms=round(train_ms, 4), soup_gen_ms=round(gen_ms, 4),
                          train_ns_per_particle=round(train_ms * 1e6 / n, 3))), flush=True)
