#!/usr/bin/env python
"""Headline benchmark: self-application steps/sec of a soup on 1..8 MI355X GPUs.

Metric (BASELINE.json): "self-application steps/sec (whole node) for 100k-particle soup".
One step = one soup generation (reference ``Soup.evolve``, code/soup.py:51-87) for every
particle: attacks (rate 0.1), learn_from (rate 0.1, severity 1), 20 self-train epochs,
divergent/zero respawn, plus the per-generation fixpoint census (``Soup.count``,
code/soup.py:89-103).  The soup configuration is the reference's active soup demo
(code/soup.py:127-138: WeightwiseNeuralNetwork(2, 2), train=20, remove_divergent, remove_zero,
epsilon=1e-4).  Random-init weights, fp32 (the reference's dtype; bf16 would make the 1e-4
fixpoint test meaningless).

Semantics (``--order``): ``sequential`` (default) is the reference's own generation -- in
place, in index order: particle k sees every change made by particles < k in the same
generation -- computed on the device by its dependency DAG, bitwise the serial loop
(csrc/srnn_ordered.h).  ``synchronous`` is the Jacobi variant (every read from the
generation-start table): different dynamics, reported only as a side number
(``config.jacobi``) next to the reference-order headline on one GPU.

Scaling (``--scaling``): ``strong`` (default) is the metric as BASELINE.json writes it -- ONE
100k-particle soup at any GPU count (100k / N particles per rank); ``weak`` keeps
``--particles-per-gpu`` per rank (an N x 100k soup).

Multi-GPU (N>1): one process per GPU, each rank owns a contiguous shard of ONE global soup
(partners uniform over all slots).  The reference order shards by a replicated plan and one
all-gather of each dependency level's outputs (csrc/srnn_ordered_sh.h); the Jacobi variant by
ONE all-to-all per generation on the soup's own RCCL communicator over xGMI
(csrc/srnn_shard.hip).

value = particles x generations / second over the whole job (max time over ranks).

Usage: python bench.py --gpus N --steps K --warmup W
       N > 1 without torchrun's env: bench.py launches torch.distributed.run itself (one rank
       per GPU, RCCL over xGMI) as a child process and relays rank 0's JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: one --particles soup at any GPU count (the BASELINE metric); "
                         "weak: --particles-per-gpu on every rank")
    ap.add_argument("--particles", type=int, default=100_000, help="soup size (strong scaling)")
    ap.add_argument("--particles-per-gpu", type=int, default=100_000, help="per-rank soup size (weak scaling)")
    ap.add_argument("--order", choices=["sequential", "synchronous"], default="sequential",
                    help="sequential (default): the reference's in-place, index-ordered generation (DAG-scheduled, "
                         "bitwise the serial loop; sharded by replicated plan + per-level all-gathers); synchronous: "
                         "the Jacobi variant, every read from the generation-start table")
    ap.add_argument("--side-steps", "--reference-order-steps", dest="side_steps", type=int, default=None,
                    help="ALSO time this many generations of the same soup in the OTHER order on the same ranks "
                         "(config.jacobi beside a reference-order headline, config.reference_order beside a Jacobi "
                         "one); -1: --steps; default: --steps on one GPU, off on several; 0: off")
    ap.add_argument("--train", type=int, default=20)
    ap.add_argument("--attacking-rate", type=float, default=0.1)
    ap.add_argument("--learn-from-rate", type=float, default=0.1)
    ap.add_argument("--severity", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (rehearsal)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: host rehearsal of the same engine (gloo backend)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0")
    ap.add_argument("--force-sharded", action="store_true",
                    help="rehearsal: run the multi-GPU generation (RCCL all-to-all) even with one rank")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """--gpus N > 1 outside torchrun: start torch.distributed.run as a CHILD process (nothing
    here has touched the GPU) and relay its output; the exit code is the child's."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def model_string(args) -> str:
    parts = [f"train={args.train}"]
    parts.append(f"attack {args.attacking_rate:g}" if args.attacking_rate > 0 else "no attacks")
    if args.learn_from_rate > 0:
        parts.append(f"learn_from {args.learn_from_rate:g}" + (f" x{args.severity}" if args.severity != 1 else ""))
    else:
        parts.append("no learn_from")
    parts.append("remove divergent/zero")
    parts.append("reference (sequential) order" if args.order == "sequential" else "synchronous order")
    return "Soup of WeightwiseNeuralNetwork(width=2, depth=2), " + ", ".join(parts)


def _agree(d, ok: bool, dev, backend) -> bool:
    """Every rank's verdict (MIN) before anything collective depends on a local outcome."""
    if not d.enabled:
        return ok
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _side(args, order, spec, n_total, params, dev, d, execution, k_side, sync, backend):
    """The same soup in the other order on the same ranks, timed after the headline's region (a
    second number, never part of the headline value).  A failure is reported in the line instead
    of costing the headline: the ranks agree after every step that can fail locally (the engine's
    allocations, the graph capture) before any of them enters a collective of the measurement."""
    import torch
    import torch.distributed as dist
    from self_replicating_neural_networks_amd.soup_engine import SoupEngine

    label = "reference-order" if order == "sequential" else "jacobi"
    eng, err = None, None
    try:
        eng = SoupEngine(spec, n_total, params, device=dev, seed=args.seed, dist=d, execution=execution,
                         order=order)
        eng.stats = not args.no_stats
    except Exception as e:  # noqa: BLE001
        err = e
    if not _agree(d, err is None, dev, backend):
        return {"semantics": label, "error": f"{type(err).__name__}: {err}"[:500] if err else "failed on another rank"}
    try:
        if dev.type == "cuda" and not args.no_graph:
            eng.capture(warmup=1)  # (collective and agreed inside; sharded reference order: eager)
        eng.evolve(args.warmup)
        sync()
        d.barrier()
        sync()
        t1 = time.perf_counter()
        eng.evolve(k_side)
        sync()
        d.barrier()
        sync()
        tr = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        if d.enabled:
            dist.all_reduce(tr, op=dist.ReduceOp.MAX)
        dt = float(tr.item())
        out = {"semantics": label, "steps": k_side, "warmup": args.warmup, "ms_per_step": dt / k_side * 1e3,
               "value": n_total * k_side / dt, "unit": "particle-generations/s", "final_census": eng.count()}
        if order == "sequential":
            out["levels"] = eng.ordered_levels()
        eng.release_graphs()
        return out
    except Exception as e:  # noqa: BLE001 -- the headline line must still be printed
        return {"semantics": label, "error": f"{type(e).__name__}: {e}"[:500]}


def main(argv=None):
    args = parse_args(argv)
    in_launcher = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not in_launcher:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a number for a "
              "different GPU count", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist
    from self_replicating_neural_networks_amd.arch import ArchSpec
    from self_replicating_neural_networks_amd.config import ExecConfig
    from self_replicating_neural_networks_amd.parallel.dist import from_env
    from self_replicating_neural_networks_amd.soup_engine import ORD_ERR_EMULATED, SoupEngine

    if args.force_sharded:
        os.environ["SRNN_FORCE_SHARDED"] = "1"
    if args.share_device:
        os.environ["SRNN_SHARE_DEVICE"] = "1"
    on_gpu = args.device == "cuda"
    backend = args.backend if on_gpu else "gloo"
    d = from_env(backend=backend, device_type=args.device)
    if on_gpu:
        dev = torch.device("cuda", 0 if args.share_device else d.local_rank)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=args.attacking_rate, learn_from_rate=args.learn_from_rate,
                  learn_from_severity=args.severity, train=args.train,
                  remove_divergent=True, remove_zero=True, epsilon=1e-4)
    n_total = args.particles if args.scaling == "strong" else args.particles_per_gpu * d.world
    execution = ExecConfig().resolved()
    execution.apply_library()
    eng = SoupEngine(spec, n_total, params, device=dev, seed=args.seed, dist=d, execution=execution,
                     order=args.order)
    eng.stats = not args.no_stats
    graphed = False
    if on_gpu and not args.no_graph:
        graphed = eng.capture(warmup=1)
    eng.evolve(args.warmup)
    sync()
    d.barrier()
    sync()
    t0 = time.perf_counter()
    eng.evolve(args.steps)
    sync()
    d.barrier()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if d.enabled:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    err = eng.exchange_error()
    if err:
        # rows that did not fit the exchange capacity were dropped: the generations are invalid
        raise SystemExit(f"soup row exchange failed ({err}): the measured generations are invalid")
    oerr = eng.ordered_error_all()
    if oerr & ~ORD_ERR_EMULATED:
        raise SystemExit(f"reference-order generation failed (error bits {oerr}): the measured generations are invalid")
    # (a one-rank timing model of a sharded reference order -- SRNN_ORDSH_EMULATE -- runs 1/R of the
    # turns: a timing, not a soup; its census is not taken)
    census = eng.count() if not oerr else "invalid: one-rank timing model (SRNN_ORDSH_EMULATE)"
    value = n_total * args.steps / dt
    # what RCCL itself reports about the soup's communicator on every rank (ncclCommCount /
    # ncclCommUserRank): the line shows that the collective really spanned N ranks
    comm = None
    if d.native is not None:
        mine = torch.tensor([d.native.nranks, d.native.comm_rank], dtype=torch.int64, device=dev)
        allr = torch.zeros(2 * d.world, dtype=torch.int64, device=dev)
        d.all_gather_into(allr, mine)
        allr = allr.view(d.world, 2).cpu().tolist()
        comm = {"library": d.native.library, "rccl_nranks": [r[0] for r in allr],
                "rccl_user_ranks": [r[1] for r in allr]}
    # the same soup in the other order, timed after the headline's region: a second number, never
    # part of the headline value
    side = None
    k_side = args.side_steps
    if k_side is None:
        k_side = -1 if d.world == 1 else 0
    k_side = args.steps if k_side < 0 else k_side
    other = "synchronous" if args.order == "sequential" else "sequential"
    if k_side > 0:
        eng.release_graphs()
        side = _side(args, other, spec, n_total, params, dev, d, execution, k_side, sync, backend)
    if d.rank == 0:
        print(json.dumps({
            "metric": "self-application steps/sec (whole node) for 100k-particle soup",
            "value": value,
            "unit": "particle-generations/s",
            # which soup semantics `value` measures: "reference-order" (code/soup.py:51-87, in place,
            # index order: the reference's own) or "jacobi" (the synchronous variant: every read from
            # the generation-start table); the other order's number rides along as config.jacobi /
            # config.reference_order
            "semantics": "reference-order" if args.order == "sequential" else "jacobi",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (random-init particles, Philox seed %d)" % args.seed,
            "config": {"model": model_string(args),
                       "global_batch": n_total, "particles_per_gpu": n_total / d.world, "seq_len": None,
                       "parallelism": f"population-dp{d.world}", "device": args.device, "hip_graph": graphed,
                       "multi_generation_graph": eng._chunk is not None,
                       "two_graph_chunks": any(c[3] is not None for c in eng._chunks),
                       "collectives": comm if comm is not None
                       else (f"torch.distributed ({backend})" if d.enabled else None),
                       "world_size": d.world, "execution": execution.in_force(),
                       "perm_table_in_use": eng._perm_table() is not None,
                       "overlap": getattr(eng, "overlap", False),
                       "sharded_schedule": getattr(eng, "schedule", None) if getattr(eng, "x2", False) else None,
                       "census_every_step": eng.stats, "final_census": census, "order": args.order,
                       "ordered_levels": eng.ordered_levels() if args.order == "sequential" else None,
                       "ord_pipeline": eng._ord_mode, "ord_census_side": eng._ord_census_side,
                       "jacobi": side if other == "synchronous" else None,
                       "reference_order": side if other == "sequential" else None},
        }), flush=True)
    eng.release_graphs()  # graph executables reference the RCCL communicator
    d.close()
    if d.enabled:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
