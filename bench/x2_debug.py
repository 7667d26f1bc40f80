"""Stage-by-stage run of the sharded (all-to-all) soup forced at one rank, printing after each
stage (locates a failure of the multi-GPU pipeline on a one-GPU box)."""
import faulthandler
import os
import sys
import time

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29571")
os.environ["SRNN_FORCE_SHARDED"] = "1"

import torch  # noqa: E402

from self_replicating_neural_networks_amd.arch import ArchSpec  # noqa: E402
from self_replicating_neural_networks_amd.parallel.dist import from_env  # noqa: E402
from self_replicating_neural_networks_amd.soup_engine import SoupEngine  # noqa: E402


def say(*a):
    print(f"[{time.perf_counter() - T0:7.2f}s]", *a, flush=True)


T0 = time.perf_counter()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
graph = "--graph" in sys.argv
d = from_env(backend="nccl")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
say("dist", d.world, d.enabled, "native", d.native is not None)
P = dict(attacking_rate=0.1, learn_from_rate=0.1, learn_from_severity=1, train=20, remove_divergent=True,
         remove_zero=True, epsilon=1e-4)
e = SoupEngine(ArchSpec.weightwise(2, 2), n, P, device=dev, seed=0, dist=d)
e.stats = True
say("engine x2", e.x2, "caps", e.x_cr, e.x_cn, e.x_cq, "blk", e.x_blk, "groups", e.x_groups)
e._x2_prime()
torch.cuda.synchronize()
say("primed; rcount", e.x_rcount[e._p].item(), "err", e.err.item())
e.time += 1
e._generation()
torch.cuda.synchronize()
say("generation 1; err", e.err.item(), "gen", e.gen_dev.item())
e._flush()
torch.cuda.synchronize()
say("flushed; census", e.last_census(), "next_uid", int(e.next_uid.item()))
e.evolve(3)
torch.cuda.synchronize()
say("evolve(3) eager; census", e.last_census(), "err", e.exchange_error())
if graph:
    ok = e.capture(warmup=1)
    torch.cuda.synchronize()
    say("captured", ok, "chunks", [c[2] for c in e._chunks])
    e.evolve(20)
    torch.cuda.synchronize()
    say("evolve(20) graphs; census", e.last_census(), "err", e.exchange_error())
ref = SoupEngine(ArchSpec.weightwise(2, 2), n, P, device=dev, seed=0)
ref.evolve(e.time)
torch.cuda.synchronize()
same = torch.equal(ref.local_rows(), e.local_rows()) and torch.equal(ref.uid, e.uid)
say("equal to the single-rank soup after", e.time, "generations:", same)
e.release_graphs()
d.close()
