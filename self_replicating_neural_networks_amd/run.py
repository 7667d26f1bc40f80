"""Production soup runner: config file -> sharded soup on every GPU of the node, with
per-generation metrics, sampled trajectories, periodic checkpoints and restart.

    python -m self_replicating_neural_networks_amd.run --config soup.json
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m self_replicating_neural_networks_amd.run \\
        --config soup.json --resume

The reference runs soups in a script loop (code/soup.py:111-147, code/setups/*.py) with
no restart capability.  Here:

* checkpoints are written every ``run.checkpoint_every`` generations to
  ``<checkpoint_dir>/gen-<t>`` via a temporary directory renamed into place, then a
  ``LATEST`` pointer -- a crash mid-write never leaves a half checkpoint as the latest;
* ``--resume`` continues from ``LATEST`` bit-for-bit (every random stream is keyed by
  (seed, slot/uid, generation)) with any number of ranks (re-sharding);
* the process group has a timeout (``run.collective_timeout_s``): a rank that dies or
  hangs makes the others fail instead of waiting forever; restart with ``--resume``;
* the row-exchange capacity is checked after every segment (overflow aborts the run).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import torch

from .config import ExperimentConfig
from .io.checkpoint import load_engine, save_engine
from .parallel.dist import from_env
from .recorder import TrajectoryRecorder
from .soup_engine import SoupEngine
from .utils.metrics import MetricsWriter


def latest_checkpoint(ckpt_dir: str):
    p = os.path.join(ckpt_dir, "LATEST")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    path = os.path.join(ckpt_dir, name)
    return path if os.path.exists(os.path.join(path, "manifest.json")) else None


def write_checkpoint(eng, ckpt_dir: str) -> str:
    name = f"gen-{eng.time:09d}"
    final = os.path.join(ckpt_dir, name)
    tmp = final + ".tmp"
    if eng.dist.rank == 0:
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp, exist_ok=True)
    eng.dist.barrier()
    save_engine(eng, tmp)  # collective (barrier inside)
    if eng.dist.rank == 0:
        shutil.rmtree(final, ignore_errors=True)
        os.replace(tmp, final)
        with open(os.path.join(ckpt_dir, "LATEST.tmp"), "w") as f:
            f.write(name)
        os.replace(os.path.join(ckpt_dir, "LATEST.tmp"), os.path.join(ckpt_dir, "LATEST"))
    eng.dist.barrier()
    return final


def build_engine(cfg: ExperimentConfig, dist, device, resume: bool = False):
    """The configured soup (``run.order``: the reference's sequential order or Jacobi), or the
    latest checkpoint's with ``resume`` -- which must have been written in the same order."""
    r = cfg.run
    execution = r.execution.resolved()
    execution.apply_library()
    if resume and r.checkpoint_dir:
        path = latest_checkpoint(r.checkpoint_dir)
        if path is not None:
            eng = load_engine(path, device=device, dist=dist, order=r.order, execution=execution)
            return eng, path
    eng = SoupEngine(cfg.arch, r.n_total, cfg.soup.params(), device=device, seed=r.seed, lr=r.lr,
                     shuffle=r.shuffle, dist=dist, dtype=r.torch_dtype(), exchange=r.exchange,
                     execution=execution, order=r.order)
    return eng, None


def run(cfg: ExperimentConfig, resume: bool = False, log=print):
    cfg.validate()
    r = cfg.run
    backend = r.backend or ("nccl" if r.device == "cuda" else "gloo")
    d = from_env(backend=backend, device_type=r.device, timeout_s=r.collective_timeout_s)
    device = torch.device("cuda", d.local_rank) if r.device == "cuda" else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    eng, resumed = build_engine(cfg, d, device, resume)
    eng.stats = r.census_every == 1
    if r.metrics_path:
        eng.metrics = MetricsWriter(r.metrics_path, every=r.metrics_every, rank=d.rank,
                                    extra=dict(world=d.world))
    if r.recorder.policy != "none":
        eng.trajectory = TrajectoryRecorder(eng, r.recorder)
    if r.graph and device.type == "cuda":
        eng.capture(warmup=1 if d.enabled else 0)  # a sharded warmup initialises the communicator
    if d.rank == 0:
        log(json.dumps(dict(event="start", resumed_from=resumed, time=eng.time, world=d.world,
                            n_total=eng.n_total, order=eng.order, graph=eng._graphs is not None)))
    t0 = time.perf_counter()
    start = eng.time
    seg = r.checkpoint_every if (r.checkpoint_dir and r.checkpoint_every > 0) else max(r.generations - eng.time, 0)
    while eng.time < r.generations:
        k = min(seg or 1, r.generations - eng.time)
        eng.evolve(k)
        err = eng.exchange_error()  # all-reduced: every rank stops together
        if err:
            raise RuntimeError(f"soup row exchange failed: {err}")
        if r.checkpoint_dir and r.checkpoint_every > 0:
            path = write_checkpoint(eng, r.checkpoint_dir)
            if d.rank == 0:
                log(json.dumps(dict(event="checkpoint", time=eng.time, path=path)))
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    census = eng.count()
    gens = eng.time - start
    out = dict(event="done", time=eng.time, order=eng.order, census=census, seconds=dt,
               particle_generations_per_s=(eng.n_total * gens / dt) if dt > 0 and gens else None)
    if eng.trajectory is not None and r.checkpoint_dir:
        eng.trajectory.save(os.path.join(r.checkpoint_dir, "trajectories"), d.rank)
    if eng.metrics is not None:
        eng.metrics.close()
    if d.rank == 0:
        log(json.dumps(out))
    eng.release_graphs()
    d.close()
    return eng, out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--config", help="ExperimentConfig JSON (defaults otherwise)")
    ap.add_argument("--resume", action="store_true", help="continue from <checkpoint_dir>/LATEST")
    ap.add_argument("--set", action="append", default=[], metavar="SECTION.KEY=VALUE",
                    help="override a field, e.g. --set run.n_total=1000000 --set soup.train=20")
    ap.add_argument("--print-config", action="store_true")
    args = ap.parse_args(argv)
    cfg = ExperimentConfig.load(args.config) if args.config else ExperimentConfig()
    over = {}
    for kv in args.set:
        key, val = kv.split("=", 1)
        sec, field = key.split(".", 1)
        try:
            v = json.loads(val)
        except json.JSONDecodeError:
            v = val
        over.setdefault(sec, {})[field] = v
    d = cfg.to_dict()
    for sec, kw in over.items():
        d.setdefault(sec, {}).update(kw)
    cfg = ExperimentConfig.from_dict(d)
    if args.print_config:
        print(cfg.to_json())
        return 0
    run(cfg, resume=args.resume)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
