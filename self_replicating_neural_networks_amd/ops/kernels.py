"""Population operators on torch tensors, executed by libsrnn.so.

Every function takes a weight table ``W`` of shape ``[N, spec.PP]`` (float32, contiguous)
on either the CPU (host thread-pool path of the native library) or a ROCm device (HIP
kernels for gfx950, lane-per-particle).  Both paths run the *same* C++ per-particle code
(csrc/srnn_kernels.h); the numpy oracle in ``..oracle`` is the independent reference.

Shapes are checked on the host before anything is launched.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import SrnnArgs

_CHECKED = os.environ.get("SRNN_CHECKED", "0") == "1"


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


# weight-table storage formats; arithmetic is fp32 in registers for all of them
TABLE_DTYPES = {torch.float32: _lib.DTYPE_FP32, torch.bfloat16: _lib.DTYPE_BF16, torch.float16: _lib.DTYPE_FP16}


def dtype_code(dtype: torch.dtype) -> int:
    if dtype not in TABLE_DTYPES:
        raise TypeError(f"weight tables must be float32, bfloat16 or float16, got {dtype}")
    return TABLE_DTYPES[dtype]


def _check_table(spec, W: torch.Tensor, name="W", like: Optional[torch.Tensor] = None) -> int:
    code = dtype_code(W.dtype)
    if like is not None and W.dtype != like.dtype:
        raise TypeError(f"{name} has dtype {W.dtype}, expected {like.dtype} (same storage as W)")
    if W.dim() != 2 or W.shape[1] != spec.PP:
        raise ValueError(f"{name} must have shape [N, {spec.PP}] for {spec}, got {tuple(W.shape)}")
    if not W.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return code


def _check_idx(idx: Optional[torch.Tensor], n_items: int, n_rows: int, dev, name: str):
    if idx is None:
        if n_items > n_rows:
            raise ValueError(f"{name}: {n_items} items but only {n_rows} rows")
        return
    if idx.dtype != torch.int64 or idx.dim() != 1 or idx.numel() != n_items or not idx.is_contiguous():
        raise ValueError(f"{name} must be a contiguous int64 vector of length {n_items}")
    if idx.device != dev:
        raise ValueError(f"{name} is on {idx.device}, expected {dev}")
    if n_items and (idx.device.type == "cpu" or _CHECKED):
        lo, hi = int(idx.min()), int(idx.max())
        if lo < 0 or hi >= n_rows:
            raise IndexError(f"{name} out of range [0, {n_rows}): min {lo} max {hi}")


def is_wave_per_particle(spec) -> bool:
    """Nets too large for the register kernels run wave-per-particle: aggregating nets
    (csrc/srnn_bignet.hip, chunk-state multi-step) and width >= 16 weightwise nets
    (csrc/srnn_wide.hip, MFMA) -- for the shapes those files instantiate; every other
    shape runs on the runtime-shape engine (csrc/srnn_generic.hip)."""
    return (((spec.kind == "aggregating" and spec.P > 64) or (spec.kind == "weightwise" and spec.width >= 16))
            and not _lib.is_generic(spec, _lib.OP_RUN_FIXPOINT))


def needs_chunk_state_temp(spec) -> bool:
    return spec.kind == "aggregating" and spec.P > 64 and not _lib.is_generic(spec, _lib.OP_RUN_FIXPOINT)


def _base_args(W: torch.Tensor, seed: int = 0, ctr: int = 0, scratch: Optional[torch.Tensor] = None) -> SrnnArgs:
    """``scratch``: device bytes for the runtime-shape engine (csrc/srnn_generic.hip); when
    omitted the library uses its own cached buffer (not allowed inside a graph capture)."""
    a = SrnnArgs()
    a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    a.ctr = int(ctr) & 0xFFFFFFFF
    if W.device.type == "cuda":
        a.dev = 1
        a.stream = ctypes.c_void_p(torch.cuda.current_stream(W.device).cuda_stream)
        if scratch is not None:
            a.scratch, a.scratch_bytes = _p(scratch), scratch.numel() * scratch.element_size()
    else:
        a.dev = 0
    return a


def _uid(uid: Optional[torch.Tensor], n: int, dev):
    if uid is None:
        return None
    if uid.dtype != torch.int64 or uid.numel() < n or uid.device != dev or not uid.is_contiguous():
        raise ValueError("uid must be a contiguous int64 tensor on the table's device covering every row")
    return uid


def init_rows(spec, W: torch.Tensor, uid: torch.Tensor, seed: int) -> torch.Tensor:
    """W[i] = fresh particle (glorot kernels, orthogonal recurrent kernels) keyed by uid[i]."""
    dt = _check_table(spec, W)
    n = W.shape[0]
    a = _base_args(W, seed)
    a.n = n
    a.W = _p(W)
    a.uid = _p(_uid(uid, n, W.device))
    _lib.run(_lib.OP_INIT, spec, a, dtype=dt)
    return W


def apply(spec, W: torch.Tensor, out: torch.Tensor, idx_f=None, idx_t=None, idx_o=None, n=None,
          uid=None, seed=0, ctr=0) -> torch.Tensor:
    """out[idx_o[i]] = f_{W[idx_f[i]]}(W[idx_t[i]])  (attack; reference code/network.py:112-118)."""
    dt = _check_table(spec, W)
    _check_table(spec, out, "out", like=W)
    if n is None:
        n = (idx_t if idx_t is not None else idx_f if idx_f is not None else W).shape[0]
    for nm, ix, rows in (("idx_f", idx_f, W.shape[0]), ("idx_t", idx_t, W.shape[0]), ("idx_o", idx_o, out.shape[0])):
        _check_idx(ix, n, rows, W.device, nm)
    a = _base_args(W, seed, ctr)
    a.n = n
    a.W, a.W2 = _p(W), _p(out)
    a.idx_f, a.idx_t, a.idx_o = _p(idx_f), _p(idx_t), _p(idx_o)
    a.uid = _p(_uid(uid, W.shape[0], W.device))
    _lib.run(_lib.OP_APPLY, spec, a, dtype=dt)
    return out


def run_fixpoint(spec, W: torch.Tensor, steps: int, eps: float, early_exit: bool = True, with_sec: bool = True,
                 record: bool = False, uid=None, seed=0, ctr=0) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """Per-row ``FixpointExperiment.run_net`` (code/experiment.py:70-91), in place.

    Returns (class int8[N], steps int32[N], trajectory [(steps+1), N, PP] or None)."""
    dt = _check_table(spec, W)
    n = W.shape[0]
    cls = torch.empty(n, dtype=torch.int8, device=W.device)
    nsteps = torch.empty(n, dtype=torch.int32, device=W.device)
    traj = torch.zeros((steps + 1, n, spec.PP), dtype=W.dtype, device=W.device) if record else None
    a = _base_args(W, seed, ctr)
    a.n, a.steps, a.eps, a.early_exit = n, int(steps), float(eps), int(bool(early_exit))
    a.flags = _lib.FLAG_FIX_SEC if with_sec else 0
    a.W, a.cls, a.nsteps, a.traj = _p(W), _p(cls), _p(nsteps), _p(traj)
    a.uid = _p(_uid(uid, n, W.device))
    temp = None
    if is_wave_per_particle(spec) and record:
        raise NotImplementedError("trajectory recording is not supported for wave-per-particle nets")
    if needs_chunk_state_temp(spec):
        if record:
            raise NotImplementedError("trajectory recording is not supported for wave-per-particle nets")
        temp = torch.empty(n * (4 * spec.aggregates + 1), dtype=torch.uint8, device=W.device)
        a.temp, a.temp_bytes = _p(temp), temp.numel()
    _lib.run(_lib.OP_RUN_FIXPOINT, spec, a, dtype=dt)
    return cls, nsteps, traj


def vary_run(spec, W: torch.Tensor, steps: int, eps: float, uid=None, seed=0, ctr=0):
    """Known-fixpoint-variation dynamics (code/setups/known-fixpoint-variation.py:66-83).
    Returns (time_to_vergence int32[N], time_as_fixpoint float32[N])."""
    dt = _check_table(spec, W)
    n = W.shape[0]
    tts = torch.empty(n, dtype=torch.int32, device=W.device)
    taf = torch.empty(n, dtype=torch.float32, device=W.device)
    a = _base_args(W, seed, ctr)
    a.n, a.steps, a.eps = n, int(steps), float(eps)
    a.W, a.nsteps, a.loss = _p(W), _p(tts), _p(taf)
    a.uid = _p(_uid(uid, n, W.device))
    _lib.run(_lib.OP_VARY_RUN, spec, a, dtype=dt)
    return tts, taf


def perturb(spec, W: torch.Tensor, e: float, uid=None, seed=0, ctr=0) -> torch.Tensor:
    """w +-= U(0,1)*e with p=1/2 per weight (reference ``vary``, known-fixpoint-variation.py:37-46)."""
    dt = _check_table(spec, W)
    a = _base_args(W, seed, ctr)
    a.n, a.eps = W.shape[0], float(e)
    a.W = _p(W)
    a.uid = _p(_uid(uid, W.shape[0], W.device))
    _lib.run(_lib.OP_PERTURB, spec, a, dtype=dt)
    return W


def train(spec, W: torch.Tensor, epochs: int = 1, lr: float = 0.01, shuffle: bool = True, uid=None, seed=0,
          ctr=0, rows: Optional[int] = None) -> torch.Tensor:
    """``epochs`` self-train epochs per row, in place (code/network.py:613-618). Returns last loss [N]."""
    dt = _check_table(spec, W)
    n = W.shape[0] if rows is None else rows
    loss = torch.empty(n, dtype=torch.float32, device=W.device)
    a = _base_args(W, seed, ctr)
    a.n, a.epochs, a.lr = n, int(epochs), float(lr)
    a.flags = _lib.FLAG_SHUFFLE if shuffle else 0
    a.W, a.loss = _p(W), _p(loss)
    a.uid = _p(_uid(uid, n, W.device))
    _lib.run(_lib.OP_TRAIN, spec, a, dtype=dt)
    return loss


def learn_from(spec, W: torch.Tensor, teachers: torch.Tensor, idx_t=None, epochs: int = 1, lr: float = 0.01,
               shuffle: bool = True, uid=None, seed=0, ctr=0) -> torch.Tensor:
    """Row i trains ``epochs`` epochs on the samples of teachers[idx_t[i]] (code/network.py:620-626)."""
    dt = _check_table(spec, W)
    _check_table(spec, teachers, "teachers", like=W)
    n = W.shape[0]
    _check_idx(idx_t, n, teachers.shape[0], W.device, "idx_t")
    loss = torch.empty(n, dtype=torch.float32, device=W.device)
    a = _base_args(W, seed, ctr)
    a.n, a.epochs, a.lr = n, int(epochs), float(lr)
    a.flags = _lib.FLAG_SHUFFLE if shuffle else 0
    a.W, a.W2, a.idx_t, a.loss = _p(W), _p(teachers), _p(idx_t), _p(loss)
    a.uid = _p(_uid(uid, n, W.device))
    _lib.run(_lib.OP_LEARN, spec, a, dtype=dt)
    return loss


def classify(spec, W: torch.Tensor, eps: float, with_sec: bool = True, uid=None, seed=0, ctr=0,
             counts: Optional[torch.Tensor] = None, scratch: Optional[torch.Tensor] = None, key_offset: int = 0):
    """Per-row class (0 divergent, 1 fix_zero, 2 fix_other, 3 fix_sec, 4 other) and the
    5-bin histogram (reference code/experiment.py:79-91, code/soup.py:89-103)."""
    dt = _check_table(spec, W)
    n = W.shape[0]
    cls = torch.empty(n, dtype=torch.int8, device=W.device)
    if counts is None:
        counts = torch.zeros(5, dtype=torch.int64, device=W.device)
    a = _base_args(W, seed, ctr, scratch)
    a.n, a.eps = n, float(eps)
    a.lo = int(key_offset)  # without uids, row i's random streams are keyed by key_offset + i
    a.flags = _lib.FLAG_FIX_SEC if with_sec else 0
    a.W, a.cls, a.counts = _p(W), _p(cls), _p(counts)
    a.uid = _p(_uid(uid, n, W.device))
    _lib.run(_lib.OP_CLASSIFY, spec, a, dtype=dt)
    return cls, counts
