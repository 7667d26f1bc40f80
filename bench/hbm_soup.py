#!/usr/bin/env python
"""BASELINE config 5 at HBM scale on one MI355X: a mixed learn+attack soup with fp16 weight
tables, population sized to fill the GPU's 288 GB of HBM3E, timed per generation, plus an
optional streaming checkpoint -> resume round trip at that size (io/checkpoint.py format v2)
checked bit-exactly.  ``--sharded`` runs the multi-GPU layout (the all-to-all exchange
protocol of csrc/srnn_shard.hip: int64 slots, O(local) lists) forced at one rank, without the
per-row diagnostic columns -- the configuration each of 8 ranks runs when the node's soup
fills every GPU.

  python bench/hbm_soup.py [--n N] [--gens G] [--fill 0.92] [--sharded] [--checkpoint DIR]

One JSON line: particles, bytes per particle (measured), device memory in use (torch and
rocm-smi), ms per generation, particle-generations/s, census, checkpoint timings."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.io import checkpoint as C  # noqa: E402
from self_replicating_neural_networks_amd.parallel.dist import Dist  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import MAX_SLOTS_DIRECT, SoupEngine  # noqa: E402

PARAMS = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=10, remove_divergent=True,
              remove_zero=True, epsilon=1e-4)


def smi_vram_used():
    try:
        out = subprocess.run(["rocm-smi", "--showmeminfo", "vram", "--json"], capture_output=True, text=True,
                             timeout=30).stdout
        d = json.loads(out)
        card = next(iter(d.values()))
        return int(card.get("VRAM Total Used Memory (B)", 0))
    except Exception:  # noqa: BLE001 -- informational only
        return None


def fingerprint(eng, chunk=1 << 22):
    """Order-sensitive digest of rows + uids (chunked on the device: no full-size temporaries)."""
    rows = eng.local_rows().view(torch.int16)
    acc = torch.zeros((), dtype=torch.int64, device=rows.device)
    for s in range(0, rows.shape[0], chunk):
        e = min(rows.shape[0], s + chunk)
        r = rows[s:e].to(torch.int64)
        mix = (torch.arange(s, e, device=rows.device, dtype=torch.int64) * 2654435761) % 2147483647 + 1
        acc += (r.sum(1) * mix).sum() + (eng.uid[s:e] * mix).sum()
    return int(acc.item())


def heartbeat(period=30.0):
    """A line on stderr every `period` s (long checkpoint I/O must not look hung)."""
    import threading

    t0 = time.perf_counter()
    stop = threading.Event()

    def run():
        while not stop.wait(period):
            print(f"[hbm_soup] ... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()
    return stop


def main():
    hb = heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0, help="particles (0: size from free HBM)")
    ap.add_argument("--gens", type=int, default=3)
    ap.add_argument("--fill", type=float, default=0.92)
    ap.add_argument("--checkpoint", default="")
    ap.add_argument("--sharded", action="store_true", help="all-to-all layout forced at one rank")
    args = ap.parse_args()
    if args.sharded:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        dist.init_process_group("gloo", rank=0, world_size=1)
    d = Dist(0, 1, 0, None, force=True) if args.sharded else None
    kw = dict(dist=d, diagnostics=not args.sharded)
    dev = torch.device("cuda", 0)
    spec = ArchSpec.weightwise(2, 2)
    dtype = torch.float16
    # measured bytes per particle of the engine (tables, lists, uids, per-row state)
    probe_n = 1 << 20
    base = torch.cuda.memory_allocated(dev)
    p = SoupEngine(spec, probe_n, PARAMS, device=dev, seed=0, dtype=dtype, **kw)
    bpp = (torch.cuda.memory_allocated(dev) - base) / probe_n
    del p
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info(dev)
    n = args.n or int(min(MAX_SLOTS_DIRECT if not args.sharded else 2 ** 32 - 2 ** 26, args.fill * free / bpp))
    t0 = time.perf_counter()
    eng = SoupEngine(spec, n, PARAMS, device=dev, seed=0, dtype=dtype, **kw)
    eng.stats = True
    torch.cuda.synchronize(dev)
    t_init = time.perf_counter() - t0
    mem_torch = torch.cuda.memory_allocated(dev)
    eng.evolve(1)  # warmup
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.evolve(args.gens)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    res = dict(config=5, name="mixed learn+attack soup, fp16 tables, HBM-filling population (one MI355X)",
               layout="sharded all-to-all (forced, 1 rank)" if args.sharded else "single rank", particles=n,
               above_2_31=n > 2 ** 31, params=PARAMS, dtype="float16", bytes_per_particle=bpp, hbm_total_bytes=total,
               device_bytes_torch=mem_torch, device_bytes_peak=torch.cuda.max_memory_allocated(dev),
               vram_used_rocm_smi=smi_vram_used(), init_s=t_init, gens=args.gens,
               ms_per_generation=dt / args.gens * 1e3, particle_generations_per_s=n * args.gens / dt,
               census=eng.last_census())
    print(json.dumps(res), flush=True)
    if args.checkpoint:
        ck = args.checkpoint
        shutil.rmtree(ck, ignore_errors=True)
        du = shutil.disk_usage(os.path.dirname(os.path.abspath(ck)) or ".")
        need = n * (spec.P * 2 + 8)
        if du.free < need * 1.02:
            print(json.dumps(dict(checkpoint="skipped", reason=f"{du.free / 1e9:.1f} GB free on disk, "
                                                                   f"{need / 1e9:.1f} GB needed")), flush=True)
            return
        t0 = time.perf_counter()
        C.save_engine(eng, ck)
        t_save = time.perf_counter() - t0
        eng.evolve(1)
        torch.cuda.synchronize(dev)
        want = fingerprint(eng)
        del eng
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        r = C.load_engine(ck, device=dev, dist=d, diagnostics=not args.sharded)
        r.stats = True
        torch.cuda.synchronize(dev)
        t_load = time.perf_counter() - t0
        r.evolve(1)
        torch.cuda.synchronize(dev)
        got = fingerprint(r)
        print(json.dumps(dict(checkpoint=ck, bytes_on_disk=sum(os.path.getsize(os.path.join(ck, f))
                                                               for f in os.listdir(ck)),
                              save_s=t_save, load_s=t_load, resume_bit_exact=bool(got == want))), flush=True)
        shutil.rmtree(ck, ignore_errors=True)
    hb.set()


if __name__ == "__main__":
    main()
