"""Float32 numpy oracle of the engine's EXACT arithmetic for Weightwise nets.

``oracle.core`` states the reference semantics with numpy's own
rounding: every product rounded, then added.  The native code (csrc/srnn_core.h), built
with ``-ffp-contract=on`` for the device and ``-Xarch_host -mfma`` for the host, FUSES the
multiply-adds its source writes as ``fmaf`` or as one ``a*b + c`` expression -- one
rounding instead of two -- in a fixed order.  Chaotic particle dynamics amplify that 1-ulp
difference, so ``core`` can pin the engine only loosely over many SGD steps.

This module replays the engine's operation sequence step for step:

* ``dense_fwd``         acc = x0*k0, then acc = fma(x_i, k_i, acc)       (csrc dense_fwd)
* folded SGD step       so = -(2 lr) * err; si = K . so (pre-update K, the same chain);
                        K[i, j] = fma(x_i, so_j, K[i, j])                (MLP::backward_update)
* epoch loss            acc = fma(err, err, acc); loss = acc / P        (train_epochs)
* glorot init           w = fma(2 lim, u, -lim)                          (glorot_fill)

A fused multiply-add of float32 operands is emulated in float64: the product is exact
(48 significant bits), the sum is rounded to 53 bits, then to 24.  That double rounding
differs from a true fma only when the 53-bit sum lands exactly on a float32 tie (about
one operation in 2^29), so the oracle equals the host and device engines bitwise in
practice -- ``tests/test_exact_oracle.py`` checks it at zero tolerance on the host, and
the GPU tests / ``smoke()`` check a device generation against it.

The reference's sequential soup (code/soup.py:51-87) is ``seq_generation``; the native
serial loop is csrc Item::soup_seq_one and the level-scheduled GPU generation
csrc/srnn_ordered.h, both bitwise equal to it.
"""
from __future__ import annotations

import numpy as np

from ..arch import ArchSpec
from . import core as C

F32 = np.float32
F64 = np.float64


def fma(a, b, c):
    """float32 fma(a, b, c) (see the module docstring for the double-rounding caveat)."""
    return (np.asarray(a, F32).astype(F64) * np.asarray(b, F32).astype(F64)
            + np.asarray(c, F32).astype(F64)).astype(F32)


def _check(spec: ArchSpec):
    if spec.kind != "weightwise":
        raise NotImplementedError("the exact oracle covers Weightwise nets (the soup benchmark's net)")


# ------------------------------------------------------------------------------ init
def init(spec: ArchSpec, uids, seed) -> np.ndarray:
    """glorot_fill with the device's fused ``-lim + (2 lim) * u``."""
    _check(spec)
    uids = np.asarray(uids, dtype=np.uint64).reshape(-1)
    w = np.zeros((uids.shape[0], spec.P), dtype=F32)
    for (r, c), off in zip(spec.layer_shapes, spec.offsets):
        lim = F32(np.sqrt(F32(6.0) / F32(r + c)))
        n = r * c
        for b in range((n + 3) // 4):
            words = C.draw(seed, uids, off * 1024 + b, C.P_INIT)
            for q in range(4):
                k = b * 4 + q
                if k < n:
                    w[:, off + k] = fma(F32(2.0) * lim, C.u01(words[q]), -lim)
    return w


# ------------------------------------------------------------------------------ layers
def _mats(spec, w):
    """Per-layer kernels as lists of columns: k[l][i][j] is an (n,) float32 array."""
    out = []
    for (r, c), o in zip(spec.layer_shapes, spec.offsets):
        out.append([[w[:, o + i * c + j].copy() for j in range(c)] for i in range(r)])
    return out


def _flat(spec, mats, n):
    w = np.empty((n, spec.P), dtype=F32)
    for ((r, c), o), k in zip(zip(spec.layer_shapes, spec.offsets), mats):
        for i in range(r):
            for j in range(c):
                w[:, o + i * c + j] = k[i][j]
    return w


def _dense(k, x):
    """csrc dense_fwd: y_j = x0 * k[0][j], then fma(x_i, k[i][j], y_j) for i = 1.."""
    r, c = len(k), len(k[0])
    y = []
    for j in range(c):
        acc = (x[0] * k[0][j]).astype(F32)
        for i in range(1, r):
            acc = fma(x[i], k[i][j], acc)
        y.append(acc)
    return y


def _forward(mats, x):
    acts = [x]
    h = x
    for k in mats:
        h = _dense(k, h)
        acts.append(h)
    return h, acts


def _step(mats, acts, err, lr2):
    """MLP::backward_update in folded form with dL/dy = err and lr = 2 lr (train_epochs)."""
    so = [(F32(-lr2) * err).astype(F32)]
    for l in range(len(mats) - 1, -1, -1):
        k, x = mats[l], acts[l]
        r, c = len(k), len(k[0])
        si = None
        if l > 0:  # si = K . so with the pre-update kernel, the same fma chain
            si = []
            for i in range(r):
                acc = (k[i][0] * so[0]).astype(F32)
                for j in range(1, c):
                    acc = fma(k[i][j], so[j], acc)
                si.append(acc)
        for i in range(r):
            for j in range(c):
                k[i][j] = fma(x[i], so[j], k[i][j])
        so = si


# ------------------------------------------------------------------------------ ops
def apply(spec: ArchSpec, a, t) -> np.ndarray:
    """f_a(t) per row (Weightwise::apply: every target weight -> the net's output at its point)."""
    _check(spec)
    a = np.asarray(a, dtype=F32)
    t = np.asarray(t, dtype=F32)
    n = a.shape[0]
    mats = _mats(spec, a)
    co = spec.coords().astype(F32)
    out = np.empty((n, spec.P), dtype=F32)
    with np.errstate(over="ignore", invalid="ignore"):
        for k in range(spec.P):
            x = [t[:, k]] + [np.full(n, co[k, q], dtype=F32) for q in range(3)]
            y, _ = _forward(mats, x)
            out[:, k] = y[0]
    return out


def _perm(spec, n, shuffle, seed, uids, ctr):
    if not shuffle:
        return np.tile(np.arange(spec.P), (n, 1))
    if spec.P <= 16:
        return C.shuffle16(spec.P, seed, uids, ctr, C.P_SHUFFLE)
    return C.fisher_yates(spec.P, seed, uids, ctr, C.P_SHUFFLE)


def train_epochs(spec: ArchSpec, w, t, epochs: int, self_train: bool, lr=0.01, shuffle=True, seed=0, uids=None,
                 ctr=0):
    """``epochs`` Keras epochs (batch 1) in the engine's order: samples = the weights at each
    epoch start (``self_train``) or the fixed rows ``t`` (learn_from); epoch e permuted with
    counter ``ctr + e``.  Returns (w', last epoch's mean loss)."""
    _check(spec)
    w = np.array(w, dtype=F32, copy=True)
    n = w.shape[0]
    if uids is None:
        uids = np.arange(n, dtype=np.uint64)
    if epochs <= 0:
        return w, np.zeros(n, dtype=F32)
    co = spec.coords().astype(F32)
    rows = np.arange(n)
    lr2 = F32(2.0) * F32(lr)
    mats = _mats(spec, w)
    loss = np.zeros(n, dtype=F32)
    with np.errstate(over="ignore", invalid="ignore"):
        src = None if self_train else np.asarray(t, dtype=F32)
        for e in range(epochs):
            s = _flat(spec, mats, n) if self_train else src  # samples frozen at epoch start
            perm = _perm(spec, n, shuffle, seed, uids, ctr + e)
            acc = np.zeros(n, dtype=F32)
            for q in range(spec.P):
                idx = perm[:, q]
                x0 = s[rows, idx]
                x = [x0] + [co[idx, c].astype(F32) for c in range(3)]
                y, acts = _forward(mats, x)
                err = (y[0] - x0).astype(F32)
                acc = fma(err, err, acc)
                _step(mats, acts, err, lr2)
            loss = (acc / F32(spec.P)).astype(F32)
    return _flat(spec, mats, n), loss


# ------------------------------------------------------------------------------ soups
def seq_generation(spec: ArchSpec, W0, gen: int, seed: int, params, lr=0.01, shuffle=True, record_turns=False):
    """One sequential (reference-order, in place) soup generation with the engine's keys
    (csrc Item::soup_seq_one / Ord::turn): slot j in index order attacks att[j] (W[v] =
    f_{W[j]}(W[v])), learns ``learn_from_severity`` epochs from te[j]'s current row, self-trains
    ``train`` epochs, and is re-initialised with respawn_key(gen, j) when divergent / zero.
    Returns (W1, action, counterpart, loss, respawn[, turns]) -- ``turns[j]`` is slot j's row at
    the end of its own turn before any respawn (the per-turn output the tests compare)."""
    _check(spec)
    n = W0.shape[0]
    att, te = C.soup_decisions(seed, gen, n, params["attacking_rate"], params["learn_from_rate"],
                               int(params.get("segment", 0) or 0))
    W = np.array(W0, dtype=F32, copy=True)
    keys = np.arange(n, dtype=np.uint64)
    action = np.zeros(n, dtype=np.int8)
    cp = np.full(n, -1, dtype=np.int64)
    loss = np.zeros(n, dtype=F32)
    respawn = np.zeros(n, dtype=np.int8)
    turns = np.zeros((n, spec.P), dtype=F32) if record_turns else None
    eps = params.get("epsilon") or 1e-14
    sev = int(params.get("learn_from_severity", 1))
    epochs = int(params.get("train", 0))
    with np.errstate(over="ignore", invalid="ignore"):
        for j in range(n):
            v = att[j]
            if v >= 0:
                W[v:v + 1] = apply(spec, W[j:j + 1], W[v:v + 1])
                action[j], cp[j] = 1, v
            c = (gen * 1024 + 512) & C.M32
            if te[j] >= 0:
                if sev > 0:
                    W[j:j + 1], l = train_epochs(spec, W[j:j + 1], W[te[j]:te[j] + 1], sev, False, lr, shuffle, seed,
                                                 keys[j:j + 1], c)
                    loss[j] = l[0]
                c += sev
                action[j], cp[j] = 2, te[j]
            if epochs > 0:
                W[j:j + 1], l = train_epochs(spec, W[j:j + 1], None, epochs, True, lr, shuffle, seed, keys[j:j + 1], c)
                loss[j] = l[0]
                action[j], cp[j] = 3, -1
            if turns is not None:
                turns[j] = W[j]
            rs = 0
            if params.get("remove_divergent") and C.is_diverged(W[j:j + 1])[0]:
                rs = 1
            elif params.get("remove_zero") and C.is_zero(W[j:j + 1], eps)[0]:
                rs = 2
            if rs:
                W[j] = init(spec, np.array([C.respawn_key(gen, j)], dtype=np.uint64), seed)[0]
            respawn[j] = rs
    out = (W, action, cp, loss, respawn)
    return out + (turns,) if record_turns else out


def max_row_error(a, b) -> float:
    """max over rows of max|a - b| / max(max|b|, 1) (non-finite entries must match)."""
    a = np.asarray(a, dtype=F64)
    b = np.asarray(b, dtype=F64)
    fa, fb = np.isfinite(a), np.isfinite(b)
    if not np.array_equal(fa, fb):
        return float("inf")
    d = np.where(fa, np.abs(np.where(fa, a, 0) - np.where(fb, b, 0)), 0.0)
    scale = np.maximum(np.max(np.where(fb, np.abs(b), 0.0), axis=1), 1.0)
    return float(np.max(np.max(d, axis=1) / scale)) if a.size else 0.0
