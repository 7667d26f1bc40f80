"""The multi-GPU generation pipeline with real remote rows, on the one-GPU box: 2 and 3 ranks
(gloo process group, every rank on cuda:0, all-to-all staged through the host) run the sharded
fused device pipeline -- decisions of every global slot, need masks, pack of the rows other
ranks need, all-to-all, received-row index, uids of the newborns from the exchanged stats rows,
census -- and must reproduce the single-rank device soup bitwise (the device counterpart of
tests/test_dist_gloo.py; at one rank the forced sharded path never packs a remote row)."""
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

pytestmark = pytest.mark.gpu

PARAMS = dict(attacking_rate=0.2, learn_from_rate=0.2, train=3, learn_from_severity=1, remove_divergent=True,
              remove_zero=True, epsilon=1e-4)
N_TOTAL = 1003  # uneven shards, partial last wave on every rank
DTYPES = {"float32": torch.float32, "bfloat16": torch.bfloat16}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, spec_json, out_dir, dtype, chunks, schedule):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SRNN_SHARE_DEVICE="1",
                      SRNN_X2_SCHEDULE=schedule)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        d = Dist(rank, world, 0, None)
        e = SoupEngine(ArchSpec.from_json(spec_json), N_TOTAL, PARAMS, device=dev, seed=21, dist=d,
                       dtype=DTYPES[dtype])
        assert e.fused and e.x2 and e.overlap == (schedule == "overlap") and e.schedule == schedule
        e.stats = True
        for k in chunks:
            e.evolve(k)
        counts = e.count()
        torch.cuda.synchronize()
        assert not e.exchange_overflowed()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=e.local_rows().float().cpu().numpy(),
                 uid=e.uid.cpu().numpy(), next_uid=e.next_uid.cpu().numpy(),
                 counts=np.array([counts[k] for k in sorted(counts)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dtype,chunks,schedule,shape", [
    (2, "float32", (2, 4), "serial", (2, 2)), (3, "float32", (6,), "serial", (2, 2)),
    (2, "bfloat16", (3, 3), "serial", (2, 2)), (2, "float32", (2, 4), "overlap", (2, 2)),
    (3, "float32", (6,), "overlap", (2, 2)), (2, "float32", (3,), "serial", (2, 1)), (2, "float32", (3,), "serial", (1, 1))])
def test_multirank_device_soup_equals_single_rank(cuda, tmp_path, world, dtype, chunks, schedule, shape):
    """both generation schedules: one stream, or the local slots beside the exchange; WW(2,1) /
    WW(1,1): the permutation table built by pack for other nibble shapes (runtime P)"""
    spec = ArchSpec.weightwise(*shape)
    ref = SoupEngine(spec, N_TOTAL, PARAMS, device=cuda, seed=21, dtype=DTYPES[dtype])
    ref.stats = True
    ref.evolve(sum(chunks))
    ref_counts = ref.count()
    torch.cuda.synchronize()
    mp.start_processes(_worker, args=(world, _free_port(), spec.to_json(), str(tmp_path), dtype, chunks, schedule),
                       nprocs=world, start_method="spawn", join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    W = np.concatenate([p["W"] for p in parts])
    uid = np.concatenate([p["uid"] for p in parts])
    assert np.array_equal(uid, ref.uid.cpu().numpy())
    assert np.array_equal(W, ref.local_rows().float().cpu().numpy(), equal_nan=True)
    for p in parts:
        assert int(p["next_uid"][0]) == int(ref.next_uid[0])
        assert list(p["counts"]) == [ref_counts[k] for k in sorted(ref_counts)]
