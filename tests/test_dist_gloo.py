"""Population sharding over a process group (gloo on CPU): results are independent of the
number of ranks (R-invariance)."""
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

PARAMS = dict(attacking_rate=0.2, learn_from_rate=0.2, train=2, learn_from_severity=1, remove_divergent=True,
              remove_zero=True, epsilon=1e-4)
N_TOTAL, GENS = 203, 6  # uneven shards on purpose


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


DTYPES = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}


def _worker(rank, world, port, spec_json, out_dir, dtype="float32", exchange="alltoall", chunks=(GENS,), params=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = Dist(rank, world, 0, None, force=world == 1)
        spec = ArchSpec.from_json(spec_json)
        e = SoupEngine(spec, N_TOTAL, params or PARAMS, device="cpu", seed=21, dist=d, dtype=DTYPES[dtype],
                       exchange=exchange)
        e.stats = True
        for k in chunks:  # uids of the newborns are settled between evolve calls
            e.evolve(k)
        counts = e.count()
        assert not e.exchange_overflowed()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=e.local_rows().float().numpy(), uid=e.uid.numpy(),
                 next_uid=e.next_uid.numpy(), counts=np.array([counts[k] for k in sorted(counts)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dtype,exchange,chunks", [
    (2, "float32", "alltoall", (GENS,)), (3, "float32", "alltoall", (1, 2, 3)), (4, "float32", "alltoall", (GENS,)),
    (2, "float32", "allgather", (2, 4)), (2, "bfloat16", "alltoall", (GENS,)), (3, "float16", "allgather", (GENS,)),
    (1, "float32", "alltoall", (2, 1, 3)),
    (8, "float32", "alltoall", (4, 2))])  # the node's rank count (bench.py --gpus 8)
def test_sharded_soup_equals_single_rank(tmp_path, world, dtype, exchange, chunks):
    """world 1 = the forced sharded path (collectives over a one-rank group)."""
    spec = ArchSpec.weightwise(2, 2)
    ref = SoupEngine(spec, N_TOTAL, PARAMS, device="cpu", seed=21, dtype=DTYPES[dtype])
    ref.evolve(GENS)
    ref_counts = ref.count()
    mp.start_processes(_worker, args=(world, _free_port(), spec.to_json(), str(tmp_path), dtype, exchange, chunks),
                       nprocs=world, start_method="spawn", join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    W = np.concatenate([p["W"] for p in parts])
    uid = np.concatenate([p["uid"] for p in parts])
    assert np.array_equal(uid, ref.uid.numpy())
    assert np.array_equal(W, ref.local_rows().float().numpy(), equal_nan=True)  # bitwise: per-row math is identical
    for p in parts:
        assert int(p["next_uid"][0]) == int(ref.next_uid[0])
        assert list(p["counts"]) == [ref_counts[k] for k in sorted(ref_counts)]


@pytest.mark.parametrize("spec,world,exchange", [
    (ArchSpec.recurrent(3, 2), 2, "alltoall"), (ArchSpec.aggregating(4, 3, 2), 3, "allgather"),
    (ArchSpec.weightwise(3, 3), 3, "alltoall")], ids=["rnn-3-2", "agg-4-3-2", "ww-3-3"])
def test_sharded_generic_shapes(tmp_path, spec, world, exchange):
    """shapes on the runtime-shape engine (unfused generation) shard bitwise too"""
    ref = SoupEngine(spec, N_TOTAL, PARAMS, device="cpu", seed=21)
    assert ref.generic
    ref.evolve(GENS)
    mp.start_processes(_worker, args=(world, _free_port(), spec.to_json(), str(tmp_path), "float32", exchange, (GENS,)),
                       nprocs=world, start_method="spawn", join=True)
    W = np.concatenate([np.load(os.path.join(tmp_path, f"r{r}.npz"))["W"] for r in range(world)])
    uid = np.concatenate([np.load(os.path.join(tmp_path, f"r{r}.npz"))["uid"] for r in range(world)])
    assert np.array_equal(W, ref.local_rows().float().numpy(), equal_nan=True)
    assert np.array_equal(uid, ref.uid.numpy())


def test_sharded_segments_spanning_shards(tmp_path):
    """sub-soups larger than a shard concentrate the row traffic on neighbouring ranks: the
    exchange capacity is sized from the segment span, so nothing overflows"""
    p = dict(PARAMS, attacking_rate=0.5, learn_from_rate=0.5)
    for seg in (29, 203):
        p["segment"] = seg
        ref = SoupEngine(ArchSpec.weightwise(2, 2), N_TOTAL, p, device="cpu", seed=21)
        ref.evolve(GENS)
        mp.start_processes(_worker, args=(4, _free_port(), ArchSpec.weightwise(2, 2).to_json(), str(tmp_path),
                                          "float32", "alltoall", (GENS,), dict(p)),
                           nprocs=4, start_method="spawn", join=True)
        W = np.concatenate([np.load(os.path.join(tmp_path, f"r{r}.npz"))["W"] for r in range(4)])
        assert np.array_equal(W, ref.local_rows().float().numpy(), equal_nan=True)


def _worker_hi(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = dict(PARAMS, attacking_rate=0.9, learn_from_rate=0.9, learn_from_severity=2)
        e = SoupEngine(ArchSpec.aggregating(4, 2, 2), 160, p, device="cpu", seed=5, dist=Dist(rank, world, 0, None))
        e.evolve(4)
        assert not e.exchange_overflowed()
        np.save(os.path.join(out_dir, f"h{rank}.npy"), e.local_rows().numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_high_rates_aggregating(tmp_path):
    p = dict(PARAMS, attacking_rate=0.9, learn_from_rate=0.9, learn_from_severity=2)
    ref = SoupEngine(ArchSpec.aggregating(4, 2, 2), 160, p, device="cpu", seed=5)
    ref.evolve(4)
    mp.start_processes(_worker_hi, args=(4, _free_port(), str(tmp_path)), nprocs=4, start_method="spawn", join=True)
    W = np.concatenate([np.load(os.path.join(tmp_path, f"h{r}.npy")) for r in range(4)])
    assert np.array_equal(W, ref.local_rows().numpy(), equal_nan=True)


def _worker_emul(rank, world, port, out_dir, frac):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SRNN_X2_EMULATE_REMOTE=str(frac))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e = SoupEngine(ArchSpec.weightwise(2, 2), N_TOTAL, PARAMS, device="cpu", seed=21,
                       dist=Dist(rank, world, 0, None, force=True))
        assert e.x_emul > 0
        e.evolve(GENS)
        assert not e.exchange_overflowed()
        np.savez(os.path.join(out_dir, "emul.npz"), W=e.local_rows().numpy(), uid=e.uid.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("frac", [0.2, 1.0])
def test_emulated_remote_slots_change_nothing(tmp_path, frac):
    """the one-rank timing model of R ranks (SRNN_X2_EMULATE_REMOTE) sends a fraction of the
    slots through the remote list: the soup is bitwise the single-rank one"""
    ref = SoupEngine(ArchSpec.weightwise(2, 2), N_TOTAL, PARAMS, device="cpu", seed=21)
    ref.evolve(GENS)
    mp.start_processes(_worker_emul, args=(1, _free_port(), str(tmp_path), frac), nprocs=1, start_method="spawn",
                       join=True)
    got = np.load(os.path.join(tmp_path, "emul.npz"))
    assert np.array_equal(got["W"], ref.local_rows().numpy(), equal_nan=True)
    assert np.array_equal(got["uid"], ref.uid.numpy())
