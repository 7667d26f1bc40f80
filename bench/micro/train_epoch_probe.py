#!/usr/bin/env python
"""Per-epoch vs fixed cost of the lane-per-particle self-train kernel (WW(2,2), one wave per
SIMD and below): time K.train for 1..40 epochs; the slope is the dependent-chain cost of one
epoch (14 SGD steps), the intercept the launch + load/store + first-shuffle cost."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402


def t_ms(fn, reps=7):
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


dev = torch.device("cuda", 0)
for spec in (ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2)):
    for n in (16384, 65536, 100000):
        uid = torch.arange(n, dtype=torch.int64, device=dev)
        W0 = torch.zeros(n, spec.PP, device=dev)
        K.init_rows(spec, W0, uid, 1)
        W = W0.clone()
        for shuffle in (True, False):
            res = {}
            for ep in (1, 5, 20, 40):
                res[ep] = t_ms(lambda: (W.copy_(W0), K.train(spec, W, epochs=ep, uid=uid, seed=2, shuffle=shuffle)))
            slope = (res[40] - res[5]) / 35
            print(json.dumps(dict(arch=spec.class_name, n=n, shuffle=shuffle, ms={k: round(v, 4) for k, v in res.items()},
                                  us_per_epoch=round(slope * 1e3, 3), fixed_us=round((res[5] - 5 * slope) * 1e3, 2),
                                  cycles_per_sgd_step=round(slope * 1e-3 * 2.4e9 / spec.P, 1) if spec.kind == "weightwise" else None)),
                  flush=True)
