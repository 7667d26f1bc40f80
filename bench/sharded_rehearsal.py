#!/usr/bin/env python
"""Rehearse the sharded soup generation on ONE GPU: a one-rank RCCL group runs the full
multi-GPU code path (decide -> pack -> all-to-all -> unpack/uids -> evolve -> census),
eagerly and captured in hipGraphs with the collective inside, and both are compared
bitwise with the unsharded engine.  Prints one JSON line with per-generation times.

    SRNN_FORCE_SHARDED=1 python bench/sharded_rehearsal.py [--n 100000] [--gens 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.parallel.dist import from_env  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402

PARAMS = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=20,
              remove_divergent=True, remove_zero=True, epsilon=1e-4)


def stage(msg):
    print(f"[rehearsal] {msg}", file=sys.stderr, flush=True)


def timed(eng, gens):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.evolve(gens)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / gens * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--gens", type=int, default=20)
    args = ap.parse_args()
    os.environ["SRNN_FORCE_SHARDED"] = "1"
    stage("init process group")
    d = from_env(backend="nccl")
    stage("process group up")
    assert d.enabled and d.world == 1
    dev = torch.device("cuda", 0)
    spec = ArchSpec.weightwise(2, 2)
    res = dict(n=args.n, gens=args.gens)

    ref = SoupEngine(spec, args.n, PARAMS, device=dev, seed=3)
    ref.stats = True
    ref.capture(warmup=1)
    res["unsharded_graph_ms"] = timed(ref, args.gens)

    stage("unsharded done")
    eager = SoupEngine(spec, args.n, PARAMS, device=dev, seed=3, dist=d)
    eager.evolve(1)
    torch.cuda.synchronize()
    stage("first sharded generation done")
    res["sharded_eager_ms"] = timed(eager, args.gens)
    stage("sharded eager done")
    if os.environ.get("SRNN_REHEARSAL_NO_GRAPH") == "1":
        print(json.dumps(res), flush=True)
        return
    g = SoupEngine(spec, args.n, PARAMS, device=dev, seed=3, dist=d)
    res["sharded_graph_captured"] = g.capture(warmup=1)
    stage(f"capture returned {res['sharded_graph_captured']}")
    res["sharded_graph_ms"] = timed(g, args.gens)
    stage("sharded graph done")

    for name, e in (("eager", eager), ("graph", g)):
        res[f"{name}_bitwise_equal"] = bool(
            torch.equal(e.local_rows(), ref.local_rows()) and torch.equal(e.uid, ref.uid)
            and int(e.next_uid.item()) == int(ref.next_uid.item()))
    res["census_equal"] = g.last_census() == ref.last_census()
    print(json.dumps(res), flush=True)
    mode = os.environ.get("SRNN_REHEARSAL_EXIT", "release_destroy")
    if mode.startswith("release"):
        g.release_graphs()
        del g
        import gc
        gc.collect()
        torch.cuda.synchronize()
        stage("graphs released")
    if mode.endswith("destroy"):
        d.close()
        torch.distributed.destroy_process_group()
        stage("process group destroyed")
    ok = res["eager_bitwise_equal"] and res["graph_bitwise_equal"] and res["census_equal"]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
