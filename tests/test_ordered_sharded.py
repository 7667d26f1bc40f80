"""The reference's in-place, index-order soup (code/soup.py:51-87) sharded over ranks
(SoupEngine(order="sequential") with a process group; csrc/srnn_ordered_sh.h): every rank plans
the whole generation, runs its own turns level by level, and all-gathers each level's outputs.
The result must be BITWISE the single-rank reference-order engine -- rows, uids, actions, losses,
census -- for any rank count (gloo on CPU here; device ranks: tests/test_ordered_sharded_gpu.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.parallel.dist import Dist
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

HOT = dict(attacking_rate=0.3, learn_from_rate=0.3, train=2, learn_from_severity=2, remove_divergent=True,
           remove_zero=True, epsilon=1e-4)
BENCH = dict(attacking_rate=0.1, learn_from_rate=0.1, train=3, learn_from_severity=1, remove_divergent=True,
             remove_zero=True, epsilon=1e-4)
N_TOTAL, GENS = 307, 4  # uneven shards on purpose
DTYPES = {"float32": torch.float32, "bfloat16": torch.bfloat16}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, spec_json, out_dir, params, dtype, chunks):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = Dist(rank, world, 0, None, force=world == 1)
        e = SoupEngine(ArchSpec.from_json(spec_json), N_TOTAL, params, device="cpu", seed=13, dist=d,
                       dtype=DTYPES[dtype], order="sequential")
        e.stats = True
        for k in chunks:
            e.evolve(k)
        counts = e.count()
        lv = e.ordered_levels()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=e.local_rows().float().numpy(), uid=e.uid.numpy(),
                 next_uid=e.next_uid.numpy(), action=e.action.numpy(), loss=e.loss.numpy(),
                 respawn=e.respawn.numpy(), counts=np.array([counts[k] for k in sorted(counts)]),
                 max_level=np.array([lv["max_level"], lv["error"]]))
    finally:
        dist.destroy_process_group()


def _run(tmp_path, spec, world, params=HOT, dtype="float32", chunks=(GENS,)):
    ref = SoupEngine(spec, N_TOTAL, params, device="cpu", seed=13, dtype=DTYPES[dtype], order="sequential")
    ref.evolve(sum(chunks))
    ref_counts = ref.count()
    mp.start_processes(_worker, args=(world, _free_port(), spec.to_json(), str(tmp_path), params, dtype, chunks),
                       nprocs=world, start_method="spawn", join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    cat = {k: np.concatenate([p[k] for p in parts]) for k in ("W", "uid", "action", "loss", "respawn")}
    assert np.array_equal(cat["uid"], ref.uid.numpy())
    assert np.array_equal(cat["W"].view(np.int32), ref.local_rows().float().numpy().view(np.int32))
    assert np.array_equal(cat["action"], ref.action.numpy()) and np.array_equal(cat["respawn"], ref.respawn.numpy())
    assert np.array_equal(cat["loss"].view(np.int32), ref.loss.numpy().view(np.int32))
    for p in parts:
        assert int(p["next_uid"][0]) == int(ref.next_uid[0])
        assert list(p["counts"]) == [ref_counts[k] for k in sorted(ref_counts)]
        assert int(p["max_level"][1]) == 0 and int(p["max_level"][0]) >= 1


@pytest.mark.parametrize("world,chunks", [(2, (GENS,)), (3, (1, 3)), (4, (2, 2)), (8, (GENS,)), (1, (1, 2, 1))])
def test_sharded_reference_order_equals_single_rank(tmp_path, world, chunks):
    """1-8 ranks (world 1: the sharded path over a one-rank group)"""
    _run(tmp_path, ArchSpec.weightwise(2, 2), world, chunks=chunks)


@pytest.mark.parametrize("spec,world", [(ArchSpec.aggregating(4, 2, 2), 3), (ArchSpec.recurrent(2, 2), 2)],
                         ids=["agg-4-2-2", "rnn-2-2"])
def test_sharded_reference_order_other_nets(tmp_path, spec, world):
    _run(tmp_path, spec, world)


def test_sharded_reference_order_bench_params_bf16(tmp_path):
    _run(tmp_path, ArchSpec.weightwise(2, 2), 2, params=BENCH, dtype="bfloat16")
