#!/usr/bin/env python
"""Per-generation time of the single-rank soup pipeline variants (100k WW(2,2), train=20):
unfused (decide -> evolve -> respawn [-> classify]), fused one-phase (last-wave hand-off)
and fused two-phase (+ a one-workgroup finish kernel), census on/off, hipGraph replay."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402

P = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=20, remove_divergent=True,
         remove_zero=True, epsilon=1e-4)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
dev = torch.device("cuda", 0)
ref = None
for name, fused, two in (("unfused", False, False), ("fused_1phase", True, False), ("fused_2phase", True, True)):
    for stats in (False, True):
        eng = SoupEngine(ArchSpec.weightwise(2, 2), n, P, device=dev, seed=0)
        eng.fused, eng.two_phase, eng.stats = fused, two, stats
        eng.capture(warmup=1)
        eng.evolve(5)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.evolve(50)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 50
        if stats:
            c = eng.last_census()
            same = None if ref is None else (c == ref[0] and torch.equal(eng.local_rows(), ref[1]))
            if ref is None:
                ref = (c, eng.local_rows().clone())
        print(json.dumps(dict(variant=name, census=stats, n=n, ms_per_generation=round(ms, 4),
                              **({"equal_to_unfused": same} if stats else {}))), flush=True)
        eng.release_graphs()
        del eng
