"""Sequential soup: one GPU lane (k_soup_seq) vs the host loop, ms per generation."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.seq_soup import SequentialSoupEngine  # noqa: E402

R = dict(remove_divergent=True, remove_zero=True, epsilon=1e-4)
for name, spec, prm, n in [("ww22 train=20", ArchSpec.weightwise(2, 2), dict(attacking_rate=0.1, learn_from_rate=-1, train=20), 200),
                           ("agg422 attack+learn", ArchSpec.aggregating(4, 2, 2), dict(attacking_rate=0.1, learn_from_rate=0.1), 1000)]:
    out = {"case": name, "n": n}
    for dev in ("cpu", "cuda"):
        e = SequentialSoupEngine(spec, n, dict(prm, **R), seed=1, device=dev)
        e.evolve(1)
        torch.cuda.synchronize()
        t = time.perf_counter()
        e.evolve(2)
        torch.cuda.synchronize()
        out[f"{dev}_ms_per_gen"] = round((time.perf_counter() - t) / 2 * 1e3, 3)
    print(json.dumps(out), flush=True)
