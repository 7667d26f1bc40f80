"""Native checkpoint / exact resume / re-sharding."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.io import checkpoint as C
from self_replicating_neural_networks_amd.parallel.dist import Dist
from self_replicating_neural_networks_amd.population import Population
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

PARAMS = dict(attacking_rate=0.2, learn_from_rate=0.2, train=2, remove_divergent=True, remove_zero=True, epsilon=1e-4)


def test_soup_resume_is_exact(tmp_path):
    spec = ArchSpec.weightwise(2, 2)
    a = SoupEngine(spec, 300, PARAMS, seed=9)
    a.evolve(6)
    b = SoupEngine(spec, 300, PARAMS, seed=9)
    b.evolve(3)
    C.save_engine(b, str(tmp_path / "ck"))
    c = C.load_engine(str(tmp_path / "ck"))
    c.evolve(3)
    assert torch.equal(a.uid, c.uid) and int(a.next_uid) == int(c.next_uid)
    assert torch.equal(a.local_rows(), c.local_rows())
    assert c.time == 6


def test_population_roundtrip(tmp_path):
    p = Population(ArchSpec.recurrent(2, 2), 50, seed=3)
    p.train(3)
    C.save_population(p, str(tmp_path / "p"))
    q = C.load_population(str(tmp_path / "p"))
    assert np.array_equal(p.W.numpy(), q.W.numpy(), equal_nan=True)  # diverged rows hold NaN
    assert torch.equal(p.uid, q.uid) and q.ctr == p.ctr


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _resume_worker(rank, world, port, ck, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e = C.load_engine(ck, dist=Dist(rank, world, 0, None))
        e.evolve(3)
        np.save(os.path.join(out, f"r{rank}.npy"), e.local_rows().numpy())
    finally:
        dist.destroy_process_group()


def test_checkpoint_reshards_1_to_2(tmp_path):
    spec = ArchSpec.weightwise(2, 2)
    a = SoupEngine(spec, 201, PARAMS, seed=4)
    a.evolve(6)
    b = SoupEngine(spec, 201, PARAMS, seed=4)
    b.evolve(3)
    ck = str(tmp_path / "ck")
    C.save_engine(b, ck)
    mp.start_processes(_resume_worker, args=(2, _port(), ck, str(tmp_path)), nprocs=2, start_method="spawn", join=True)
    W = np.concatenate([np.load(os.path.join(tmp_path, f"r{r}.npy")) for r in range(2)])
    assert np.array_equal(W, a.local_rows().numpy(), equal_nan=True)


def test_streaming_checkpoint_16bit_chunks_and_v1_compat(tmp_path):
    """v2 shards keep the storage format (bf16 as raw bits), stream in chunks smaller than a
    shard, resume bit-exactly; a v1 (torch .pt, fp32) directory still loads."""
    spec = ArchSpec.weightwise(2, 2)
    for dt in (torch.bfloat16, torch.float16):
        a = SoupEngine(spec, 257, PARAMS, seed=5, dtype=dt)
        a.evolve(4)
        b = SoupEngine(spec, 257, PARAMS, seed=5, dtype=dt)
        b.evolve(2)
        ck = str(tmp_path / f"ck{dt}")
        C.save_engine(b, ck, chunk_bytes=1000)  # ~35 rows per chunk
        r = np.load(os.path.join(ck, f"rows-{0:012d}-{257:012d}.npy"), mmap_mode="r")
        assert r.dtype == (np.uint16 if dt == torch.bfloat16 else np.float16) and r.shape == (257, spec.P)
        c = C.load_engine(ck, chunk_bytes=700)
        c.evolve(2)
        assert c.dtype == dt and torch.equal(a.local_rows().view(torch.int16), c.local_rows().view(torch.int16))
        assert torch.equal(a.uid, c.uid)
    # v1 layout written by the round-1 writer
    e = SoupEngine(spec, 40, PARAMS, seed=1)
    e.evolve(2)
    v1 = tmp_path / "v1"
    v1.mkdir()
    torch.save({"W": e.local_rows()[:, :spec.P].clone(), "uid": e.uid.clone()}, str(v1 / f"shard-{0:012d}-{40:012d}.pt"))
    import json
    m = dict(format="srnn-checkpoint-v1", kind="soup", spec=json.loads(spec.to_json()), n_total=40, params=PARAMS,
             seed=1, lr=0.01, shuffle=True, time=2, gen=int(e.gen_dev.item()), next_uid=int(e.next_uid.item()),
             world=1, dtype="float32", exchange="alltoall")
    (v1 / "manifest.json").write_text(json.dumps(m))
    f = C.load_engine(str(v1))
    assert torch.equal(f.local_rows(), e.local_rows()) and torch.equal(f.uid, e.uid)


def test_reference_order_resume_is_exact_and_order_checked(tmp_path):
    """an ordered (reference-order) soup checkpointed mid-run resumes in the SAME order, bitwise
    equal to the uninterrupted run; resuming it as another order raises instead of silently
    switching to Jacobi dynamics"""
    import pytest

    spec = ArchSpec.weightwise(2, 2)
    a = SoupEngine(spec, 300, PARAMS, seed=9, order="sequential")
    a.evolve(5)
    b = SoupEngine(spec, 300, PARAMS, seed=9, order="sequential")
    b.evolve(2)
    C.save_engine(b, str(tmp_path / "ck"))
    assert C.checkpoint_order(str(tmp_path / "ck")) == "sequential"
    c = C.load_engine(str(tmp_path / "ck"))
    assert c.order == "sequential"
    c.evolve(3)
    assert torch.equal(a.uid, c.uid) and int(a.next_uid) == int(c.next_uid) and c.time == 5
    assert torch.equal(a.local_rows(), c.local_rows())
    assert torch.equal(a.action, c.action) and torch.equal(a.loss.view(torch.int32), c.loss.view(torch.int32))
    with pytest.raises(ValueError, match="change its dynamics"):
        C.load_engine(str(tmp_path / "ck"), order="synchronous")
    s = SoupEngine(spec, 300, PARAMS, seed=9)
    C.save_engine(s, str(tmp_path / "cs"))
    with pytest.raises(ValueError, match="change its dynamics"):
        C.load_engine(str(tmp_path / "cs"), order="sequential")
