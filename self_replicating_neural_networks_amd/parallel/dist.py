"""Process-group plumbing for population sharding (one process per GPU).

The reference is single-process; here a population of ``n_total`` particles
is sharded contiguously over the ranks of a ``torch.distributed`` group.  On ROCm the
``"nccl"`` backend is RCCL, whose collectives run over the xGMI links of an MI355X node;
CPU tests use ``"gloo"``.  The collective shapes:

* all-to-all of fixed-size exchange blocks (``all_to_all``): the row path of a sharded soup
  (``SoupEngine(exchange="alltoall")``, the default): each rank ships only the rows its
  peers' attacks and learn_from requests need, plus notices / requests / stats headers;
* all-gather of weight rows (``all_gather_rows``): the optional ``exchange="allgather"``
  soup (every rank holds the whole table) and the trajectory / uid gathers;
* all-reduce of int64 class histograms (fixpoint-fraction statistics) and all-gather of
  per-rank stats (globally sequential uids).

The device collectives go through the soup's own RCCL communicator (``NativeComm``,
csrc/srnn_comm.cpp) so they can be captured in hipGraphs; torch.distributed carries the
rendezvous and the CPU (gloo) rehearsals.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import torch
import torch.distributed as dist


def _torch_rccl_path() -> Optional[str]:
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


class NativeComm:
    """The soup's own RCCL communicator (csrc/srnn_comm.cpp): collectives are
    enqueued on the caller's HIP stream straight into RCCL, so they can be captured in a
    hipGraph with the kernels of a generation.  torch.distributed only carries rank 0's
    ncclUniqueId to the other ranks (rendezvous)."""

    def __init__(self, world: int, rank: int, device: "torch.device"):
        import ctypes
        from ..ops import _lib
        self._ct = ctypes
        self.L = _lib.lib()
        self.hint = (_torch_rccl_path() or "").encode()
        self.world, self.rank, self.device = world, rank, device
        if not self.L.srnn_comm_available(self.hint):
            raise RuntimeError("RCCL not available: " + _lib.last_error())
        buf = ctypes.create_string_buffer(256)
        uid = None
        if rank == 0:
            n = self.L.srnn_comm_unique_id(self.hint, buf, 256)
            if n <= 0:
                raise RuntimeError("ncclGetUniqueId failed: " + _lib.last_error())
            uid = bytes(buf.raw[:n])
        if world > 1 or dist.is_initialized():
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]
        h = ctypes.c_void_p()
        r = self.L.srnn_comm_init(self.hint, ctypes.create_string_buffer(uid, len(uid)), world, rank,
                                  device.index or 0, ctypes.byref(h))
        if r != 0:
            raise RuntimeError(f"ncclCommInitRank failed ({r}): " + _lib.last_error())
        self.comm = h
        self.library = self.L.srnn_comm_library().decode()

    @property
    def nranks(self) -> int:
        """Ranks of the communicator as RCCL reports them (ncclCommCount; -1 if unavailable)."""
        return int(self.L.srnn_comm_count(self.comm)) if self.comm else -1

    @property
    def comm_rank(self) -> int:
        """This process's rank in the communicator (ncclCommUserRank; -1 if unavailable)."""
        return int(self.L.srnn_comm_user_rank(self.comm)) if self.comm else -1

    def _stream(self):
        return self._ct.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _ok(self, r, what):
        if r != 0:
            from ..ops import _lib
            raise RuntimeError(f"{what} failed ({r}): " + _lib.last_error())

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        nb = inp.numel() * inp.element_size()
        if nb % self.world or out.numel() * out.element_size() != nb:
            raise ValueError("all-to-all buffers must split evenly over the ranks")
        self._ok(self.L.srnn_comm_all_to_all(self.comm, inp.data_ptr(), out.data_ptr(), nb // self.world,
                                             self._stream()), "all-to-all")

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        nb = inp.numel() * inp.element_size()
        if out.numel() * out.element_size() != nb * self.world:
            raise ValueError("all-gather output must be world x input")
        self._ok(self.L.srnn_comm_all_gather(self.comm, inp.data_ptr(), out.data_ptr(), nb, self._stream()),
                 "all-gather")

    def all_reduce_sum_i64(self, t: torch.Tensor):
        if t.dtype != torch.int64:
            raise TypeError("int64 only")
        self._ok(self.L.srnn_comm_all_reduce_i64(self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._stream()),
                 "all-reduce")

    def check(self):
        """Raise if RCCL reported an asynchronous error (peer died, network failure)."""
        self._ok(self.L.srnn_comm_async_error(self.comm), "RCCL async error")

    def close(self, abort: bool = False):
        if self.comm:
            self.L.srnn_comm_destroy(self.comm, 1 if abort else 0)
            self.comm = None


@dataclasses.dataclass
class Dist:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    group: Optional[object] = None
    # run the sharded code path (collectives included) even with one rank: rehearses the
    # multi-GPU generation -- and its hipGraph capture with RCCL -- on a one-GPU box
    force: bool = False
    native: Optional[NativeComm] = None   # own RCCL communicator (device collectives)
    # ExecConfig (native_comm, loopback); None: the defaults, environment variables override
    execution: Optional[object] = None
    _pad_bufs: dict = dataclasses.field(default_factory=dict, repr=False)
    _resolved: Optional[object] = dataclasses.field(default=None, repr=False)

    def _exec(self):
        """The ExecConfig in force, resolved (environment overrides) once per Dist: the
        per-generation collectives read it without re-parsing the environment."""
        if self._resolved is None:
            from ..config import ExecConfig
            self._resolved = (self.execution or ExecConfig()).resolved()
        return self._resolved

    def enable_native_comm(self, device) -> bool:
        """Create the soup's own RCCL communicator on ``device`` (collective over all
        ranks).  No-op on CPU, without the nccl backend or with SRNN_NATIVE_COMM=0."""
        if self.native is not None:
            return True
        device = torch.device(device)
        if (not self.enabled or device.type != "cuda" or not self._exec().native_comm
                or dist.get_backend(self.group) != "nccl"):
            return False
        try:
            self.native = NativeComm(self.world, self.rank, device)
        except (RuntimeError, OSError) as e:  # symmetric failures: every rank falls back
            import sys
            print(f"native RCCL communicator unavailable ({e}); using torch.distributed collectives",
                  file=sys.stderr)
            self.native = None
            return False
        return True

    def close(self):
        if self.native is not None:
            self.native.close()
            self.native = None

    def _use_native(self, *ts) -> bool:
        return self.native is not None and all(t.is_cuda for t in ts)

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.force

    def shard(self, n_total: int):
        """Contiguous [lo, hi) rows of this rank (sizes differ by at most one)."""
        lo = (self.rank * n_total) // self.world
        hi = ((self.rank + 1) * n_total) // self.world
        return lo, hi

    def shard_of_rank(self, rank: int, n_total: int):
        """[lo, hi) rows of ``rank``."""
        return (rank * n_total) // self.world, ((rank + 1) * n_total) // self.world

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
        if len(set(sizes)) == 1 and self._use_native(out, local):
            self.native.all_gather(out, local)
        elif len(set(sizes)) == 1:
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
        """Equal-split all-to-all (RCCL over xGMI for nccl: direct peer links).  One rank with
        ExecConfig.loopback: a device copy instead of the collective (rehearsal timing without
        RCCL's own latency)."""
        if self.world == 1 and self._exec().loopback:
            out.copy_(inp)
            return out
        if self._use_native(out, inp):
            self.native.all_to_all(out, inp)
        elif self.enabled and inp.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo rehearsal of device tensors (e.g. ranks sharing one GPU): stage on the host
            o = torch.empty_like(out, device="cpu")
            dist.all_to_all_single(o, inp.cpu(), group=self.group)
            out.copy_(o)
        elif self.enabled:
            dist.all_to_all_single(out, inp, group=self.group)
        else:
            out.copy_(inp)
        return out

    def all_gather_into(self, out: torch.Tensor, local: torch.Tensor):
        if self._use_native(out, local):
            self.native.all_gather(out, local)
        elif self.enabled:
            dist.all_gather_into_tensor(out, local, group=self.group)
        else:
            out.copy_(local)
        return out

    def all_reduce_sum(self, t: torch.Tensor):
        if self._use_native(t) and t.dtype == torch.int64:
            self.native.all_reduce_sum_i64(t)
        elif self.enabled:
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
