"""Process-group plumbing for population sharding (one process per GPU).

The reference is single-process; here a population of ``n_total`` particles
is sharded contiguously over the ranks of a ``torch.distributed`` group.  On ROCm the
``"nccl"`` backend is RCCL, whose collectives run over the xGMI links of an MI355X node;
CPU tests use ``"gloo"``.  Only three collective shapes are needed:

* all-gather of weight rows (cross-shard attacks / learn_from partners),
* all-reduce of int64 class histograms (fixpoint-fraction statistics),
* all-gather of per-rank respawn counts (globally sequential uids).
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class Dist:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    group: Optional[object] = None
    # run the sharded code path (collectives included) even with one rank: rehearses the
    # multi-GPU generation -- and its hipGraph capture with RCCL -- on a one-GPU box
    force: bool = False
    _pad_bufs: dict = dataclasses.field(default_factory=dict, repr=False)

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.force

    def shard(self, n_total: int):
        """Contiguous [lo, hi) rows of this rank (sizes differ by at most one)."""
        lo = (self.rank * n_total) // self.world
        hi = ((self.rank + 1) * n_total) // self.world
        return lo, hi

    def shard_sizes(self, n_total: int):
        return [((r + 1) * n_total) // self.world - (r * n_total) // self.world for r in range(self.world)]

    # ---------------------------------------------------------------- collectives
    def all_gather_rows(self, out: torch.Tensor, local: torch.Tensor, n_total: int):
        """out[n_total, PP] <- concatenation of every rank's local rows."""
        if not self.enabled:
            if out.data_ptr() != local.data_ptr():
                out.copy_(local)
            return out
        sizes = self.shard_sizes(n_total)
        if len(set(sizes)) == 1:
            dist.all_gather_into_tensor(out, local, group=self.group)
        else:
            # uneven shards: gather max-size padded blocks, then compact
            m = max(sizes)
            key = (tuple(local.shape[1:]), local.dtype, local.device, m)
            buf = self._pad_bufs.get(key)
            if buf is None:
                buf = (torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device),
                       torch.zeros((self.world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device))
                self._pad_bufs[key] = buf
            send, recv = buf
            send[: local.shape[0]].copy_(local)
            dist.all_gather_into_tensor(recv, send, group=self.group)
            o = 0
            for r, sz in enumerate(sizes):
                out[o:o + sz].copy_(recv[r * m:r * m + sz])
                o += sz
        return out

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        """Equal-split all-to-all (RCCL over xGMI for nccl: direct peer links)."""
        if self.enabled:
            dist.all_to_all_single(out, inp, group=self.group)
        else:
            out.copy_(inp)
        return out

    def all_gather_into(self, out: torch.Tensor, local: torch.Tensor):
        if self.enabled:
            dist.all_gather_into_tensor(out, local, group=self.group)
        else:
            out.copy_(local)
        return out

    def all_reduce_sum(self, t: torch.Tensor):
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def all_gather_scalar(self, out: torch.Tensor, local: torch.Tensor):
        """out[world] <- every rank's 1-element ``local``."""
        if self.enabled:
            dist.all_gather_into_tensor(out, local.reshape(1), group=self.group)
        else:
            out.copy_(local.reshape(1))
        return out

    def barrier(self):
        if self.enabled:
            dist.barrier(group=self.group)


def from_env(backend: Optional[str] = None, device_type: str = "cuda", timeout_s: Optional[float] = None) -> Dist:
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/...).
    ``timeout_s`` bounds every collective: a dead or hung peer makes the others raise
    instead of waiting forever (failure detection)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    force = os.environ.get("SRNN_FORCE_SHARDED") == "1"
    if world <= 1 and not force:
        return Dist(0, 1, 0, None)
    if world <= 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if device_type == "cuda" else "gloo"
        kw = {}
        if timeout_s:
            import datetime
            kw["timeout"] = datetime.timedelta(seconds=float(timeout_s))
        if backend == "nccl":
            dev_idx = 0 if os.environ.get("SRNN_SHARE_DEVICE") == "1" else local_rank
            torch.cuda.set_device(dev_idx)
            kw["device_id"] = torch.device("cuda", dev_idx)
        dist.init_process_group(backend=backend, **kw)
    return Dist(dist.get_rank(), dist.get_world_size(), local_rank, None, force=force)


def current() -> Dist:
    if dist.is_available() and dist.is_initialized():
        return Dist(dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0")), None)
    return Dist()
