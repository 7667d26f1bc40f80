"""Native checkpoints with exact resume (the reference could not resume).

Layout of a checkpoint directory (format v2)::

    manifest.json            spec, population size, params, seed, lr, generation, next uid, ...
    rows-<lo>-<hi>.npy       the rows [lo, hi) in the table's OWN storage format: float32,
                             float16, or bfloat16 as raw uint16 bits ([hi - lo, P], no padding)
    uid-<lo>-<hi>.npy        int64[hi - lo]

One (rows, uid) pair per writing rank.  Both sides stream: a shard is written and read in
chunks of ``chunk_bytes`` through numpy memory maps (``np.load(mmap_mode="r")``, no pickle),
so host memory stays O(chunk) whatever the population -- a 2-billion-particle HBM-filling
soup (BASELINE config 5) checkpoints and resumes with a few hundred MB of host buffers.
Files are keyed by their global row range, so a checkpoint written by R ranks loads on any
number of ranks (re-sharding); each rank reads only the ranges overlapping its own rows.

Every random stream of the engine is a pure function of (seed, slot/uid, generation), so a
resumed soup continues bit-for-bit.  Format v1 directories (``shard-<lo>-<hi>.pt`` torch
files of fp32 rows, read with ``torch.load(weights_only=True)``) still load.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from ..arch import ArchSpec
from ..parallel.dist import Dist

FORMAT = "srnn-checkpoint-v2"
FORMATS = ("srnn-checkpoint-v1", FORMAT)
_DTYPE_NAMES = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float16: "float16"}
_DTYPES = {v: k for k, v in _DTYPE_NAMES.items()}
_NP = {torch.float32: np.float32, torch.float16: np.float16, torch.bfloat16: np.uint16}
CHUNK_BYTES = 256 << 20


def _chunks(n: int, row_bytes: int, chunk_bytes: int) -> Iterator[Tuple[int, int]]:
    step = max(1, chunk_bytes // max(row_bytes, 1))
    for s in range(0, n, step):
        yield s, min(n, s + step)


def _to_numpy(t: torch.Tensor) -> np.ndarray:
    """Host copy in the storage format (bf16 as its raw bits)."""
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _from_numpy(a: np.ndarray, dtype: torch.dtype) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:
        a = a.copy()
    if dtype == torch.bfloat16:
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(a)


class _NpyWriter:
    """A .npy file written sequentially in chunks with plain file I/O; written pages are
    synced and dropped from the page cache as it goes (a 70 GB shard must not pile up as
    dirty page cache on the host)."""

    def __init__(self, fn: str, dtype, shape):
        self.f = open(fn, "wb")
        np.lib.format.write_array_header_1_0(self.f, dict(descr=np.lib.format.dtype_to_descr(np.dtype(dtype)),
                                                          fortran_order=False, shape=tuple(shape)))
        self.done = 0

    def write(self, a: np.ndarray):
        self.f.write(np.ascontiguousarray(a).tobytes())
        self.done += a.nbytes
        if self.done >= (1 << 30):
            self._drop()

    def _drop(self):
        self.f.flush()
        os.fsync(self.f.fileno())
        if hasattr(os, "posix_fadvise"):
            os.posix_fadvise(self.f.fileno(), 0, 0, os.POSIX_FADV_DONTNEED)
        self.done = 0

    def close(self):
        self._drop()
        self.f.close()


def _write_shard(path: str, lo: int, hi: int, rows: torch.Tensor, uid: torch.Tensor, P: int,
                 chunk_bytes: int) -> None:
    """rows-<lo>-<hi>.npy / uid-<lo>-<hi>.npy, streamed chunk by chunk from the device."""
    n = hi - lo
    tag = f"{lo:012d}-{hi:012d}"
    tmp_r, tmp_u = os.path.join(path, f".rows-{tag}.npy"), os.path.join(path, f".uid-{tag}.npy")
    R = _NpyWriter(tmp_r, _NP[rows.dtype], (n, P))
    for s, e in _chunks(n, P * rows.element_size(), chunk_bytes):
        R.write(_to_numpy(rows[s:e, :P]))
    R.close()
    U = _NpyWriter(tmp_u, np.int64, (n,))
    for s, e in _chunks(n, 8, chunk_bytes):
        U.write(uid[s:e].detach().cpu().numpy())
    U.close()
    # atomic publish: a crash mid-write never leaves a truncated shard under the real name
    os.replace(tmp_r, os.path.join(path, f"rows-{tag}.npy"))
    os.replace(tmp_u, os.path.join(path, f"uid-{tag}.npy"))


def _shard_files(path: str):
    """[(lo, hi, rows_file, uid_file or None, version)] of a checkpoint directory."""
    out = []
    for f in sorted(glob.glob(os.path.join(path, "rows-*.npy"))):
        a, b = (int(x) for x in os.path.basename(f)[5:-4].split("-"))
        out.append((a, b, f, os.path.join(path, f"uid-{a:012d}-{b:012d}.npy"), 2))
    for f in sorted(glob.glob(os.path.join(path, "shard-*.pt"))):
        a, b = (int(x) for x in os.path.basename(f)[6:-3].split("-"))
        out.append((a, b, f, None, 1))
    return out


def _fill_rows(path: str, lo: int, hi: int, P: int, rows: torch.Tensor, uid: torch.Tensor,
               chunk_bytes: int = CHUNK_BYTES) -> None:
    """Stream rows [lo, hi) of the checkpoint into ``rows[:, :P]`` / ``uid`` (any device)."""
    covered = 0
    for a, b, f, fu, ver in _shard_files(path):
        s, e = max(a, lo), min(b, hi)
        if s >= e:
            continue
        if ver == 1:
            d = torch.load(f, weights_only=True)
            rows[s - lo:e - lo, :P] = d["W"][s - a:e - a].to(rows.device, rows.dtype)
            uid[s - lo:e - lo] = d["uid"][s - a:e - a].to(uid.device)
        else:
            R = np.load(f, mmap_mode="r")
            U = np.load(fu, mmap_mode="r")
            if R.dtype != _NP[rows.dtype] or R.shape[1] != P:
                raise ValueError(f"{f}: stored {R.dtype}[{R.shape[1]}] does not match {rows.dtype}[{P}]")
            fds = [os.open(f, os.O_RDONLY), os.open(fu, os.O_RDONLY)]
            try:
                for cs, ce in _chunks(e - s, P * rows.element_size(), chunk_bytes):
                    r0, r1 = s - a + cs, s - a + ce
                    rows[s - lo + cs:s - lo + ce, :P] = _from_numpy(R[r0:r1], rows.dtype).to(rows.device)
                    uid[s - lo + cs:s - lo + ce] = _from_numpy(U[r0:r1], torch.int64).to(uid.device)
                    if hasattr(os, "posix_fadvise"):  # read pages are not needed again
                        for fd in fds:
                            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            finally:
                for fd in fds:
                    os.close(fd)
            del R, U
        covered += e - s
    if covered != hi - lo:
        raise ValueError(f"checkpoint {path} does not cover rows [{lo}, {hi})")


def save_engine(eng, path: str, chunk_bytes: int = CHUNK_BYTES) -> str:
    """Write this rank's shard (+ the manifest on rank 0). Collective when sharded.  An engine
    whose rows are invalid (exchange or reference-order error bits on any rank) is refused on
    every rank before anything is written."""
    err = eng.exchange_error()
    oerr = eng.ordered_error_all()
    if err or oerr:
        from ..soup_engine import describe_ordered_error
        why = err or f"reference-order error bits {oerr} ({describe_ordered_error(oerr)})"
        raise RuntimeError(f"refusing to checkpoint a soup with invalid rows: {why}")
    os.makedirs(path, exist_ok=True)
    _write_shard(path, eng.lo, eng.hi, eng.local_rows(), eng.uid, eng.spec.P, chunk_bytes)
    if eng.dist.rank == 0:
        manifest = dict(format=FORMAT, kind="soup", spec=json.loads(eng.spec.to_json()), n_total=eng.n_total,
                        params={k: v for k, v in eng.params.items()}, seed=eng.seed, lr=eng.lr, shuffle=eng.shuffle,
                        time=eng.time, gen=int(eng.gen_dev.item()), next_uid=int(eng.next_uid.item()),
                        world=eng.dist.world, dtype=_DTYPE_NAMES[eng.dtype], exchange=eng.exchange,
                        order=eng.order)
        tmp = os.path.join(path, ".manifest.json")
        with open(tmp, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        os.replace(tmp, os.path.join(path, "manifest.json"))
    eng.dist.barrier()
    return path


def _manifest(path: str, kind: str):
    with open(os.path.join(path, "manifest.json")) as f:
        m = json.load(f)
    if m.get("format") not in FORMATS or m.get("kind") != kind:
        raise ValueError(f"{path}: not a {kind} checkpoint")
    return m


def checkpoint_order(path: str) -> str:
    """The soup order a checkpoint was written in (manifests before the field existed were
    written by synchronous engines: the runner had no other)."""
    return _manifest(path, "soup").get("order", "synchronous")


def load_engine(path: str, device="cpu", dist: Optional[Dist] = None, chunk_bytes: int = CHUNK_BYTES,
                diagnostics: bool = True, order: Optional[str] = None, execution=None):
    """Rebuild a SoupEngine from a checkpoint (any rank count), in the order it was written
    in.  ``order``: the order the caller expects -- a different one raises (resuming a
    reference-order soup with Jacobi generations, or the reverse, would silently change its
    dynamics).  Each rank streams only its own rows straight into its device table: host
    memory O(chunk), not O(shard)."""
    from ..soup_engine import SoupEngine

    m = _manifest(path, "soup")
    written = m.get("order", "synchronous")
    if order is not None and order != written:
        raise ValueError(f"{path}: checkpoint of a {written!r}-order soup; resuming it with order={order!r} would "
                         "change its dynamics")
    spec = ArchSpec(**m["spec"])
    d = dist or Dist()
    eng = SoupEngine(spec, m["n_total"], m["params"], device=device, seed=m["seed"], lr=m["lr"],
                     shuffle=m["shuffle"], dist=d, dtype=_DTYPES[m.get("dtype", "float32")],
                     exchange=m.get("exchange", "alltoall"), init=False, diagnostics=diagnostics,
                     order=written, execution=execution)
    rows = eng.local_rows()
    rows.zero_()
    _fill_rows(path, eng.lo, eng.hi, spec.P, rows, eng.uid, chunk_bytes)
    eng.next_uid.fill_(m["next_uid"])
    eng.gen_dev.fill_(m["gen"])
    eng.time = m["time"]
    return eng


def save_population(pop, path: str, chunk_bytes: int = CHUNK_BYTES) -> str:
    os.makedirs(path, exist_ok=True)
    _write_shard(path, 0, pop.n, pop.W, pop.uid, pop.spec.P, chunk_bytes)
    with open(os.path.join(path, "manifest.json"), "w") as f:
        json.dump(dict(format=FORMAT, kind="population", spec=json.loads(pop.spec.to_json()), n_total=pop.n,
                       seed=pop.seed, lr=pop.lr, ctr=pop.ctr, dtype=_DTYPE_NAMES[pop.W.dtype]), f, indent=1,
                  sort_keys=True)
    return path


def load_population(path: str, device="cpu"):
    from ..population import Population

    m = _manifest(path, "population")
    spec = ArchSpec(**m["spec"])
    pop = Population(spec, m["n_total"], device=device, seed=m["seed"], lr=m["lr"],
                     dtype=_DTYPES[m.get("dtype", "float32")], init=False)
    pop.W.zero_()
    _fill_rows(path, 0, m["n_total"], spec.P, pop.W, pop.uid)
    pop.ctr = m["ctr"]
    return pop
