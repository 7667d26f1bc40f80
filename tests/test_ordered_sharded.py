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


def _error_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from self_replicating_neural_networks_amd.io.checkpoint import save_engine
        from self_replicating_neural_networks_amd.ops import _lib
        d = Dist(rank, world, 0, None)
        e = SoupEngine(ArchSpec.weightwise(2, 2), 101, HOT, device="cpu", seed=3, dist=d, order="sequential")
        e.evolve(1)
        if rank == world - 1:  # a bit only this rank's kernels could have set (its own rows' close)
            e._octl[_lib.ORD_ERRW] |= 4
        msgs = []
        for call in (e.count, lambda: save_engine(e, os.path.join(out_dir, "ckpt"))):
            try:
                call()
                msgs.append("ok")
            except RuntimeError as err:
                msgs.append(str(err))
        dist.barrier()  # every rank got here: none of them was left inside a collective
        with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
            f.write("\n".join(msgs))
    finally:
        dist.destroy_process_group()


def test_an_error_bit_on_one_rank_raises_on_every_rank(tmp_path):
    """count() and save_engine() OR the reference-order error word over the ranks before raising:
    an error set on one rank alone makes every rank raise together (no rank waits in a collective
    the raising rank never enters), and the message names the bit"""
    world = 3
    mp.start_processes(_error_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    for r in range(world):
        msgs = open(os.path.join(tmp_path, f"err{r}.txt")).read().split("\n")
        assert len(msgs) == 2 and all("error bits 4" in m and "never ran" in m for m in msgs), msgs
    assert not os.path.exists(os.path.join(tmp_path, "ckpt"))


def _emulate_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from self_replicating_neural_networks_amd.config import ExecConfig
        d = Dist(0, 1, 0, None, force=True)
        e = SoupEngine(ArchSpec.weightwise(2, 2), 200, HOT, device="cpu", seed=3, dist=d, order="sequential",
                       execution=ExecConfig(ordsh_emulate=4))
        e.evolve(2)
        bits = e.ordered_error()
        try:
            e.count()
            msg = "ok"
        except RuntimeError as err:
            msg = str(err)
        with open(os.path.join(out_dir, "emu.txt"), "w") as f:
            f.write(f"{bits}\n{msg}")
    finally:
        dist.destroy_process_group()


def test_one_rank_timing_model_marks_its_rows_invalid(tmp_path):
    """SRNN_ORDSH_EMULATE > 1 (a one-rank timing model of R ranks) runs 1/R of the turns: a sticky
    error bit makes count() (and checkpoints) refuse the rows instead of passing them for a soup"""
    mp.start_processes(_emulate_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, start_method="spawn",
                       join=True)
    bits, msg = open(os.path.join(tmp_path, "emu.txt")).read().split("\n", 1)
    assert int(bits) & 32 and "SRNN_ORDSH_EMULATE" in msg
