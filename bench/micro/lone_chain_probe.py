#!/usr/bin/env python
"""Latency of ONE particle's SGD chain (WW(2,2), lane per particle): K.train of n particles for
E epochs at n = 1 and 8 (one lane / 8 lanes of one wave), 64 (one wave on the whole chip), 64 x 16, 64 x 1024 (one wave per SIMD), with
and without shuffle.  The per-epoch slope at n = 64 is the dependent-chain cost a reference-order
continuation link pays 21 times (profiles/r6*)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.ops import kernels as K  # noqa: E402


def t_ms(fn, reps=9):
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
spec = ArchSpec.weightwise(2, 2)
for n in (1, 8, 64, 1024, 65536):
    uid = torch.arange(n, dtype=torch.int64, device=dev)
    W0 = torch.zeros(n, spec.PP, device=dev)
    K.init_rows(spec, W0, uid, 1)
    W = W0.clone()
    for shuffle in (True, False):
        res = {}
        for ep in (20, 220):
            res[ep] = t_ms(lambda: K.train(spec, W, epochs=ep, uid=uid, seed=2, shuffle=shuffle))
        slope = (res[220] - res[20]) / 200
        print(json.dumps(dict(n=n, shuffle=shuffle, ms={k: round(v, 4) for k, v in res.items()},
                              us_per_epoch=round(slope * 1e3, 4), cycles_per_step_at_2_4GHz=round(slope * 1e-3 * 2.4e9 / spec.P, 1))),
              flush=True)

# the same chain inside a synchronous soup generation (k_soup_gen, lane per particle) and on a
# lane pair per particle (k_soup_gen2, SRNN_SOUP_LANES=2): 64 particles, train 20 vs 220
from self_replicating_neural_networks_amd.ops import _lib  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402

for lanes, npart in ((1, 1), (1, 8), (1, 64), (2, 64)):
    _lib.set_knob("soup_lanes", lanes)
    res = {}
    for tr in (20, 220):
        p = dict(attacking_rate=0.0, learn_from_rate=0.0, train=tr, remove_divergent=True, remove_zero=True,
                 epsilon=1e-4)
        eng = SoupEngine(spec, npart, p, device=dev, seed=0)
        eng.evolve(2)
        res[tr] = t_ms(lambda: eng.evolve(1))
    slope = (res[220] - res[20]) / 200
    print(json.dumps(dict(soup_lanes=lanes, n=npart, ms={k: round(v, 4) for k, v in res.items()},
                          us_per_epoch=round(slope * 1e3, 4), cycles_per_step_at_2_4GHz=round(slope * 1e-3 * 2.4e9 / 14, 1))),
          flush=True)
_lib.set_knob("soup_lanes", -1)
