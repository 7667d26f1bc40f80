"""The sharded reference-order generation (csrc/srnn_ordered_sh.h) on the device: 2 and 3 ranks
on the one-GPU box (gloo process group, every rank on cuda:0, the all-gathers staged through the
host) must reproduce the single-rank device reference-order soup -- which itself is the serial
loop and the exact fp32 oracle -- bitwise (the device counterpart of tests/test_ordered_sharded.py)."""
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
N_TOTAL = 1003
DTYPES = {"float32": torch.float32, "bfloat16": torch.bfloat16}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, dtype, chunks, n_total=N_TOTAL):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SRNN_SHARE_DEVICE="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        d = Dist(rank, world, 0, None)
        e = SoupEngine(ArchSpec.weightwise(2, 2), n_total, PARAMS, device=dev, seed=21, dist=d, dtype=DTYPES[dtype],
                       order="sequential")
        e.stats = True
        for k in chunks:
            e.evolve(k)
        counts = e.count()
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=e.local_rows().float().cpu().numpy(),
                 uid=e.uid.cpu().numpy(), next_uid=e.next_uid.cpu().numpy(), loss=e.loss.cpu().numpy(),
                 counts=np.array([counts[k] for k in sorted(counts)]), err=np.array([e.ordered_error()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dtype,chunks,n_total", [(2, "float32", (3,), N_TOTAL), (3, "float32", (1, 2), N_TOTAL),
                                                       (2, "bfloat16", (3,), N_TOTAL), (2, "float32", (2,), 20011)])
def test_device_sharded_reference_order_equals_single_rank(tmp_path, world, dtype, chunks, n_total):
    """(20,011 particles: > 8192 rows per rank, the uid assignment's multi-tile path)"""
    ref = SoupEngine(ArchSpec.weightwise(2, 2), n_total, PARAMS, device="cuda", seed=21, dtype=DTYPES[dtype],
                     order="sequential")
    ref.evolve(sum(chunks))
    ref_counts = ref.count()
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), dtype, chunks, n_total), nprocs=world,
                       start_method="spawn", join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    W = np.concatenate([p["W"] for p in parts])
    assert np.array_equal(np.concatenate([p["uid"] for p in parts]), ref.uid.cpu().numpy())
    assert np.array_equal(W.view(np.int32), ref.local_rows().float().cpu().numpy().view(np.int32))
    assert np.array_equal(np.concatenate([p["loss"] for p in parts]).view(np.int32),
                          ref.loss.cpu().numpy().view(np.int32))
    for p in parts:
        assert int(p["next_uid"][0]) == int(ref.next_uid[0]) and int(p["err"][0]) == 0
        assert list(p["counts"]) == [ref_counts[k] for k in sorted(ref_counts)]
