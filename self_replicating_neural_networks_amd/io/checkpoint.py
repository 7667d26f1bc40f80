"""Native checkpoints with exact resume (the reference could not resume).

Layout of a checkpoint directory::

    manifest.json        spec, population size, params, seed, lr, generation, next uid, ...
    shard-<lo>-<hi>.pt   {"W": float32[hi-lo, P], "uid": int64[hi-lo]}  (one per writing rank)

16-bit tables (bf16 / fp16) are written widened to fp32 (exact) and narrowed again on load;
the manifest records the storage dtype.

Every random stream of the engine is a pure function of (seed, slot/uid, generation), so a
resumed soup continues bit-for-bit.  Shards are keyed by their global row range, so a
checkpoint written by R ranks can be loaded by any number of ranks (re-sharding).  Files
are read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Optional

import numpy as np
import torch

from ..arch import ArchSpec
from ..parallel.dist import Dist

FORMAT = "srnn-checkpoint-v1"
_DTYPE_NAMES = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float16: "float16"}
_DTYPES = {v: k for k, v in _DTYPE_NAMES.items()}


def save_engine(eng, path: str) -> str:
    """Write this rank's shard (+ the manifest on rank 0). Collective when sharded."""
    os.makedirs(path, exist_ok=True)
    P = eng.spec.P
    torch.save({"W": eng.local_rows()[:, :P].detach().float().cpu().contiguous(), "uid": eng.uid.detach().cpu().clone()},
               os.path.join(path, f"shard-{eng.lo:012d}-{eng.hi:012d}.pt"))
    if eng.dist.rank == 0:
        manifest = dict(format=FORMAT, kind="soup", spec=json.loads(eng.spec.to_json()), n_total=eng.n_total,
                        params={k: v for k, v in eng.params.items()}, seed=eng.seed, lr=eng.lr, shuffle=eng.shuffle,
                        time=eng.time, gen=int(eng.gen_dev.item()), next_uid=int(eng.next_uid.item()),
                        world=eng.dist.world, dtype=_DTYPE_NAMES[eng.dtype], exchange=eng.exchange)
        with open(os.path.join(path, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
    eng.dist.barrier()
    return path


def _read_rows(path: str, lo: int, hi: int, P: int):
    W = np.zeros((hi - lo, P), dtype=np.float32)
    uid = np.zeros(hi - lo, dtype=np.int64)
    covered = 0
    for f in sorted(glob.glob(os.path.join(path, "shard-*.pt"))):
        a, b = (int(x) for x in os.path.basename(f)[6:-3].split("-"))
        s, e = max(a, lo), min(b, hi)
        if s >= e:
            continue
        d = torch.load(f, weights_only=True)
        W[s - lo:e - lo] = d["W"][s - a:e - a].numpy()
        uid[s - lo:e - lo] = d["uid"][s - a:e - a].numpy()
        covered += e - s
    if covered != hi - lo:
        raise ValueError(f"checkpoint {path} does not cover rows [{lo}, {hi})")
    return W, uid


def load_engine(path: str, device="cpu", dist: Optional[Dist] = None):
    """Rebuild a SoupEngine from a checkpoint (any rank count)."""
    from ..soup_engine import SoupEngine

    with open(os.path.join(path, "manifest.json")) as f:
        m = json.load(f)
    if m.get("format") != FORMAT or m.get("kind") != "soup":
        raise ValueError(f"{path}: not a soup checkpoint")
    spec = ArchSpec(**m["spec"])
    d = dist or Dist()
    lo, hi = d.shard(m["n_total"])
    W, uid = _read_rows(path, lo, hi, spec.P)  # this rank's rows only: host memory O(shard)
    eng = SoupEngine(spec, m["n_total"], m["params"], device=device, seed=m["seed"], lr=m["lr"],
                     shuffle=m["shuffle"], dist=d, local_weights=W, dtype=_DTYPES[m.get("dtype", "float32")],
                     exchange=m.get("exchange", "alltoall"))
    eng.uid.copy_(torch.from_numpy(uid))
    eng.next_uid.fill_(m["next_uid"])
    eng.gen_dev.fill_(m["gen"])
    eng.time = m["time"]
    return eng


def save_population(pop, path: str) -> str:
    os.makedirs(path, exist_ok=True)
    torch.save({"W": pop.weights().detach().float().cpu().contiguous(), "uid": pop.uid.detach().cpu().clone()},
               os.path.join(path, f"shard-{0:012d}-{pop.n:012d}.pt"))
    with open(os.path.join(path, "manifest.json"), "w") as f:
        json.dump(dict(format=FORMAT, kind="population", spec=json.loads(pop.spec.to_json()), n_total=pop.n,
                       seed=pop.seed, lr=pop.lr, ctr=pop.ctr, dtype=_DTYPE_NAMES[pop.W.dtype]), f, indent=1,
                  sort_keys=True)
    return path


def load_population(path: str, device="cpu"):
    from ..population import Population

    with open(os.path.join(path, "manifest.json")) as f:
        m = json.load(f)
    if m.get("format") != FORMAT or m.get("kind") != "population":
        raise ValueError(f"{path}: not a population checkpoint")
    spec = ArchSpec(**m["spec"])
    W, uid = _read_rows(path, 0, m["n_total"], spec.P)
    pop = Population(spec, m["n_total"], device=device, seed=m["seed"], weights=W, lr=m["lr"],
                     dtype=_DTYPES[m.get("dtype", "float32")])
    pop.uid.copy_(torch.from_numpy(uid))
    pop.ctr = m["ctr"]
    return pop
