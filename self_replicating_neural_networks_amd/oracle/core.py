"""Float32 numpy oracle of the particle semantics.

Independent of the native library: used by the tests as the reference every HIP/host
kernel is compared against, and by the exact *sequential* soup mode (reference
``Soup.evolve`` order, code/soup.py:51-87) for small populations.

All functions are vectorised over a leading particle axis ``n``.  Random streams use the
same Philox4x32-10 counters as csrc/srnn_core.h so that inits, shuffles and soup
decisions agree with the kernels.
"""
from __future__ import annotations

import numpy as np

from ..arch import ArchSpec, AGGREGATORS, SHUFFLERS

U32 = np.uint32
M32 = 0xFFFFFFFF

P_INIT, P_NORMAL, P_SHUFFLE, P_AGGSHUF, P_SOUP, P_PERTURB = 1, 2, 3, 4, 5, 6
C_DIVERGENT, C_FIX_ZERO, C_FIX_OTHER, C_FIX_SEC, C_OTHER = 0, 1, 2, 3, 4
CLASS_NAMES = ("divergent", "fix_zero", "fix_other", "fix_sec", "other")


# ------------------------------------------------------------------------------ RNG
def philox(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & M32 for x in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(int(k0) & M32)
    k1 = np.uint64(int(k1) & M32)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(M32)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(M32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & np.uint64(M32)
        k1 = (k1 + np.uint64(0xBB67AE85)) & np.uint64(M32)
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def draw(seed, ident, step, purpose):
    ident = np.asarray(ident, dtype=np.uint64)
    return philox(ident & np.uint64(M32), ident >> np.uint64(32), np.asarray(step, dtype=np.uint64),
                  np.uint64(purpose), int(seed) & M32, (int(seed) >> 32) & M32)


def u01(x):
    return (np.asarray(x, dtype=np.uint32) >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)


def u01_open0(x):
    return ((np.asarray(x, dtype=np.uint32) >> 8) + 1).astype(np.float32) * np.float32(1.0 / 16777216.0)


def fisher_yates(n_items, seed, ids, step, purpose):
    """Per-particle permutation of range(n_items) (same stream as csrc fisher_yates)."""
    ids = np.asarray(ids, dtype=np.uint64).reshape(-1)
    n = ids.shape[0]
    perm = np.tile(np.arange(n_items, dtype=np.int64), (n, 1))
    rows = np.arange(n)
    words = None
    used, blk = 4, 0
    for i in range(n_items - 1, 0, -1):
        if used == 4:
            # block index in the purpose word's high bits (csrc fisher_yates)
            words = draw(seed, ids, np.uint64(int(step) & M32), (int(purpose) + (blk << 8)) & M32)
            blk += 1
            used = 0
        x = words[used]
        used += 1
        j = (u01(x) * np.float32(i + 1)).astype(np.int64)
        j = np.minimum(j, i)
        a = perm[rows, i].copy()
        perm[rows, i] = perm[rows, j]
        perm[rows, j] = a
    return perm


def shuffle16(n_items, seed, ids, step, purpose):
    """Nibble-register Fisher-Yates of csrc shuffle16 (n <= 16): the swap indices are the
    mixed-radix digits of one uniform 64-bit value (j = hi64(u * (i+1)), u = lo64(...)),
    taken from half of the Philox draw (step >> 1) (one draw per two epochs)."""
    ids = np.asarray(ids, dtype=np.uint64).reshape(-1)
    n = ids.shape[0]
    perm = np.tile(np.arange(n_items, dtype=np.int64), (n, 1))
    rows = np.arange(n)
    step = int(step)
    r = draw(seed, ids, np.uint64(((step >> 1) * 64) & M32), purpose)
    lo_w, hi_w = (r[2], r[3]) if step & 1 else (r[0], r[1])
    ul = lo_w.astype(np.uint64)
    uh = hi_w.astype(np.uint64)
    m32 = np.uint64(0xFFFFFFFF)
    for i in range(n_items - 1, 0, -1):
        k = np.uint64(i + 1)
        lo = ul * k
        hi = uh * k + (lo >> np.uint64(32))
        j = (hi >> np.uint64(32)).astype(np.int64)
        ul = lo & m32
        uh = hi & m32
        a = perm[rows, i].copy()
        perm[rows, i] = perm[rows, j]
        perm[rows, j] = a
    return perm


# ------------------------------------------------------------------------------ init
def _glorot(w, off, r, c, seed, uids):
    lim = np.sqrt(np.float32(6.0) / np.float32(r + c)).astype(np.float32)
    n = r * c
    for b in range((n + 3) // 4):
        words = draw(seed, uids, off * 1024 + b, P_INIT)
        for q in range(4):
            k = b * 4 + q
            if k < n:
                w[:, off + k] = -lim + np.float32(2.0) * lim * u01(words[q])


def _orthogonal(w, off, N, seed, uids):
    n = uids.shape[0]
    vals = []
    blk = 0
    while len(vals) < N * N:
        u = draw(seed, uids, off * 1024 + blk, P_NORMAL)
        blk += 1
        r1 = np.sqrt(np.float32(-2.0) * np.log(u01_open0(u[0])))
        t1 = np.float32(6.283185307179586) * u01(u[1])
        r2 = np.sqrt(np.float32(-2.0) * np.log(u01_open0(u[2])))
        t2 = np.float32(6.283185307179586) * u01(u[3])
        vals += [r1 * np.cos(t1), r1 * np.sin(t1), r2 * np.cos(t2), r2 * np.sin(t2)]
    a = np.stack(vals[:N * N], axis=1).astype(np.float32).astype(np.float64).reshape(n, N, N)
    if N == 2:
        # Keras 2.2.4 Orthogonal = U of numpy.linalg.svd (LAPACK dgesdd): for 2x2 always a
        # reflection with a biased angle -- not Haar (csrc/srnn_core.h lapack_u2)
        w[:, off:off + 4] = np.linalg.svd(a)[0].astype(np.float32).reshape(n, 4)
        return
    # modified Gram-Schmidt in float64 (N = 1: sign(a) = LAPACK's U; N >= 3: Haar)
    for j in range(N):
        for p in range(j):
            d = np.sum(a[:, :, p] * a[:, :, j], axis=1)
            a[:, :, j] -= d[:, None] * a[:, :, p]
        s = np.sum(a[:, :, j] * a[:, :, j], axis=1)
        a[:, :, j] *= (1.0 / np.sqrt(s))[:, None]
    w[:, off:off + N * N] = a.astype(np.float32).reshape(n, N * N)


def init(spec: ArchSpec, uids, seed) -> np.ndarray:
    uids = np.asarray(uids, dtype=np.uint64).reshape(-1)
    w = np.zeros((uids.shape[0], spec.P), dtype=np.float32)
    shapes, offs = spec.layer_shapes, spec.offsets
    for l, ((r, c), o) in enumerate(zip(shapes, offs)):
        if spec.kind == "recurrent" and l % 2 == 1:
            _orthogonal(w, o, r, seed, uids)
        else:
            _glorot(w, o, r, c, seed, uids)
    return w


# ------------------------------------------------------------------------------ dense
def _dense(x, k):
    """y = x . k with the kernels' accumulation order (per output: sum over i ascending)."""
    # x: (n, IN), k: (n, IN, OUT)
    y = x[:, 0:1] * k[:, 0, :]
    for i in range(1, k.shape[1]):
        y = y + x[:, i:i + 1] * k[:, i, :]
    return y.astype(np.float32)


def _mats(spec, w):
    return [w[:, o:o + r * c].reshape(-1, r, c) for (r, c), o in zip(spec.layer_shapes, spec.offsets)]


def _mlp_forward(mats, x):
    acts = [x]
    h = x
    for m in mats:
        h = _dense(h, m)
        acts.append(h)
    return h, acts


def _mlp_backward_update(mats, acts, gy, lr):
    """Folded SGD step (csrc MLP::backward_update): st = -lr*dL/dout propagated with the
    pre-update kernels; every weight gets K += x (x) st."""
    st = (np.float32(-lr) * gy).astype(np.float32)
    for l in range(len(mats) - 1, -1, -1):
        m = mats[l]
        nxt = np.einsum("nij,nj->ni", m, st).astype(np.float32) if l > 0 else None
        m += acts[l][:, :, None] * st[:, None, :]
        st = nxt


# ------------------------------------------------------------------------------ aggregation
def aggregate(spec, t, aggregator="mean"):
    g = np.empty((t.shape[0], spec.aggregates), dtype=np.float32)
    for k, (s, L) in enumerate(spec.chunks):
        ch = t[:, s:s + L]
        if aggregator == "mean":
            g[:, k] = (np.sum(ch.astype(np.float64), axis=1) / L).astype(np.float32)
        elif aggregator == "max":
            m = ch[:, 0].copy()
            for i in range(L):
                v = ch[:, i]
                m = np.where(v > m, v, m)
            g[:, k] = m
        else:  # reference `weight > max_found and weight or max_found`
            m = ch[:, 0].copy()
            for i in range(L):
                v = ch[:, i]
                m = np.where((v > m) & (v != 0.0), v, m)
            g[:, k] = m
    return g


def fft_reduce(spec, t):
    a = spec.aggregates
    g = np.zeros((t.shape[0], a), dtype=np.float32)
    for k in range(a):
        for n_ in range(a):
            cs = np.cos(np.float32(6.283185307179586) * np.float32((k * n_) % a) / np.float32(a)).astype(np.float32)
            g[:, k] = g[:, k] + t[:, n_] * cs
    return g


def _shuffle(spec, out, seed, uids, ctr):
    if spec.shuffler != "random":
        return out
    perm = fisher_yates(spec.P, seed, uids, ctr, P_AGGSHUF)
    return np.take_along_axis(out, perm, axis=1)


# ------------------------------------------------------------------------------ apply
def apply(spec: ArchSpec, a, t, seed=0, uids=None, ctr=0):
    """f_a(t) for every particle: the applying nets ``a`` rewrite targets ``t``."""
    a = np.asarray(a, dtype=np.float32)
    t = np.asarray(t, dtype=np.float32)
    n = a.shape[0]
    if uids is None:
        uids = np.arange(n, dtype=np.uint64)
    mats = _mats(spec, a)
    if spec.kind == "weightwise":
        co = spec.coords()
        out = np.empty((n, spec.P), dtype=np.float32)
        for k in range(spec.P):
            x = np.empty((n, 4), dtype=np.float32)
            x[:, 0] = t[:, k]
            x[:, 1:] = co[k]
            y, _ = _mlp_forward(mats, x)
            out[:, k] = y[:, 0]
        return out
    if spec.kind in ("aggregating", "fft"):
        g = aggregate(spec, t, spec.aggregator) if spec.kind == "aggregating" else fft_reduce(spec, t)
        h, _ = _mlp_forward(mats, g)
        out = np.empty((n, spec.P), dtype=np.float32)
        if spec.kind == "aggregating":
            for k, (s, L) in enumerate(spec.chunks):
                out[:, s:s + L] = h[:, k:k + 1]
        else:
            P = spec.P
            out[:] = 0.0
            for m in range(P):
                acc = np.zeros(n, dtype=np.float32)
                for k in range(spec.aggregates):
                    cs = np.cos(np.float32(6.283185307179586) * np.float32((k * m) % P) / np.float32(P)).astype(np.float32)
                    acc = acc + h[:, k] * cs
                out[:, m] = acc / np.float32(P)
        return _shuffle(spec, out, seed, uids, ctr)
    # recurrent
    return _rnn_forward(spec, mats, t)[0]


def _rnn_layers(spec):
    w, d = spec.width, spec.depth
    return [(1 if l == 0 else w, 1 if l == d else w) for l in range(d + 1)]


def _rnn_forward(spec, mats, s):
    n, T = s.shape
    layers = _rnn_layers(spec)
    hs = [np.zeros((n, u), dtype=np.float32) for _, u in layers]
    hist = []
    out = np.empty((n, T), dtype=np.float32)
    for t in range(T):
        x = s[:, t:t + 1]
        step = []
        for l, (i_, u) in enumerate(layers):
            K, R = mats[2 * l], mats[2 * l + 1]
            h = (_dense(x, K) + _dense(hs[l], R)).astype(np.float32)
            hs[l] = h
            step.append(h)
            x = h
        hist.append(step)
        out[:, t] = x[:, 0]
    return out, hist


# ------------------------------------------------------------------------------ train
def samples(spec, w):
    """Reference ``compute_samples`` (x, y) for one particle set (weightwise only)."""
    co = spec.coords()
    n = w.shape[0]
    x = np.empty((n, spec.P, 4), dtype=np.float32)
    x[:, :, 0] = w[:, :spec.P]
    x[:, :, 1:] = co[None]
    return x, x[:, :, 0].copy()


def train_epoch(spec: ArchSpec, w, s, lr=0.01, shuffle=True, seed=0, uids=None, ctr=0):
    """One Keras epoch (batch 1, SGD) on the samples of ``s``; returns (w', mean loss)."""
    w = np.array(w, dtype=np.float32, copy=True)
    s = np.asarray(s, dtype=np.float32)
    n = w.shape[0]
    if uids is None:
        uids = np.arange(n, dtype=np.uint64)
    mats = _mats(spec, w)
    if spec.kind == "weightwise":
        x, y = samples(spec, s)
        if not shuffle:
            perm = np.tile(np.arange(spec.P), (n, 1))
        elif spec.P <= 16:
            perm = shuffle16(spec.P, seed, uids, ctr, P_SHUFFLE)
        else:
            perm = fisher_yates(spec.P, seed, uids, ctr, P_SHUFFLE)
        loss = np.zeros(n, dtype=np.float32)
        rows = np.arange(n)
        for q in range(spec.P):
            idx = perm[:, q]
            xs = x[rows, idx]
            ys = y[rows, idx]
            out, acts = _mlp_forward(mats, xs)
            e = out[:, 0] - ys
            loss += e * e
            # dL/dy = 2e, folded step -(2 lr) * e (csrc Weightwise::train_epoch)
            _mlp_backward_update(mats, acts, e[:, None], 2 * lr)
        return _flat(spec, mats), loss / np.float32(spec.P)
    if spec.kind in ("aggregating", "fft"):
        g = aggregate(spec, s, spec.aggregator) if spec.kind == "aggregating" else fft_reduce(spec, s)
        h, acts = _mlp_forward(mats, g)
        e = h - g
        loss = np.sum(e * e, axis=1) / np.float32(spec.aggregates)
        _mlp_backward_update(mats, acts, np.float32(2.0) * e / np.float32(spec.aggregates), lr)
        return _flat(spec, mats), loss.astype(np.float32)
    # recurrent: BPTT over the single (1, P, 1) sample
    T = spec.P
    out, hist = _rnn_forward(spec, mats, s)
    layers = _rnn_layers(spec)
    grads = [np.zeros_like(m) for m in mats]
    carry = [np.zeros((n, u), dtype=np.float32) for _, u in layers]
    loss = np.zeros(n, dtype=np.float32)
    for t in range(T - 1, -1, -1):
        e = out[:, t] - s[:, t]
        loss += e * e
        dtop = (np.float32(2.0) * e / np.float32(T))[:, None]
        for l in range(len(layers) - 1, -1, -1):
            K, R = mats[2 * l], mats[2 * l + 1]
            dh = dtop + carry[l]
            xin = s[:, t:t + 1] if l == 0 else hist[t][l - 1]
            hp = hist[t - 1][l] if t > 0 else np.zeros_like(hist[t][l])
            grads[2 * l] += xin[:, :, None] * dh[:, None, :]
            grads[2 * l + 1] += hp[:, :, None] * dh[:, None, :]
            dx = np.einsum("nij,nj->ni", K, dh).astype(np.float32)
            carry[l] = np.einsum("nij,nj->ni", R, dh).astype(np.float32)
            dtop = dx
    for m, g in zip(mats, grads):
        m += g * np.float32(-lr)
    return _flat(spec, mats), loss / np.float32(T)


def _flat(spec, mats):
    return np.concatenate([m.reshape(m.shape[0], -1) for m in mats], axis=1).astype(np.float32)


# ------------------------------------------------------------------------------ predicates
def is_diverged(w):
    return ~np.all(np.isfinite(w), axis=1)


def is_zero(w, eps):
    with np.errstate(invalid="ignore"):
        return np.all((-eps <= w) & (w <= eps), axis=1)


def is_fixpoint(spec, w, eps, degree=1, **kw):
    nw = w
    for _ in range(degree):
        nw = apply(spec, w, nw, **kw)
    with np.errstate(invalid="ignore"):
        close = ~np.any(np.abs(nw - w) >= eps, axis=1)
    return ~is_diverged(nw) & close


def classify(spec, w, eps, with_sec=True, **kw):
    with np.errstate(over="ignore", invalid="ignore"):
        w = np.asarray(w, dtype=np.float32)
        cls = np.full(w.shape[0], C_OTHER, dtype=np.int8)
        div = is_diverged(w)
        fix1 = is_fixpoint(spec, w, eps, 1, **kw)
        zero = is_zero(w, eps)
        sec = is_fixpoint(spec, w, eps, 2, **kw) if with_sec else np.zeros_like(div)
        cls[sec] = C_FIX_SEC
        cls[fix1 & ~zero] = C_FIX_OTHER
        cls[fix1 & zero] = C_FIX_ZERO
        cls[div] = C_DIVERGENT
    return cls


def counts_of(cls):
    return {name: int(np.sum(cls == i)) for i, name in enumerate(CLASS_NAMES)}


def run_fixpoint(spec, w, steps, eps, early_exit=True, with_sec=True):
    """Per-row ``FixpointExperiment.run_net`` (code/experiment.py:70-77)."""
    with np.errstate(over="ignore", invalid="ignore"):
        w = np.array(w, dtype=np.float32, copy=True)
        n = w.shape[0]
        active = np.ones(n, dtype=bool)
        nsteps = np.zeros(n, dtype=np.int32)
        for _ in range(steps):
            if early_exit:
                nw = apply(spec, w, w)
                fix = ~is_diverged(nw) & ~np.any(np.abs(nw - w) >= eps, axis=1)
                active &= ~is_diverged(w) & ~fix
            else:
                nw = apply(spec, w, w)
            if not active.any():
                break
            w[active] = nw[active]
            nsteps[active] += 1
        return w, nsteps, classify(spec, w, eps, with_sec)


def perturb(w, e, seed, uids, ctr):
    w = np.array(w, dtype=np.float32, copy=True)
    for k in range(w.shape[1]):
        u = draw(seed, uids, (int(ctr) * 1024 + k) & M32, P_PERTURB)
        mag = u01(u[1]).astype(np.float64) * float(np.float32(e))  # kernel argument is fp32
        up = u01(u[0]) < np.float32(0.5)
        w[:, k] = np.where(up, (w[:, k].astype(np.float64) + mag), (w[:, k].astype(np.float64) - mag)).astype(np.float32)
    return w


# ------------------------------------------------------------------------------ soup (synchronous)
def soup_decisions(seed, gen, n_total, attacking_rate, learn_from_rate, segment=0):
    slots = np.arange(n_total, dtype=np.uint64)
    d = draw(seed, slots, gen, P_SOUP)
    span = np.uint64(segment if segment > 0 else n_total)
    base = (np.arange(n_total) // segment * segment) if segment > 0 else np.zeros(n_total, dtype=np.int64)
    att = np.where(u01(d[0]) < np.float32(attacking_rate),
                   base + ((d[1].astype(np.uint64) * span) >> np.uint64(32)).astype(np.int64), -1)
    te = np.where(u01(d[2]) < np.float32(learn_from_rate),
                  base + ((d[3].astype(np.uint64) * span) >> np.uint64(32)).astype(np.int64), -1)
    return att, te


def soup_generation_sync(spec, W0, uids, gen, seed, params, lr=0.01, shuffle=True):
    """Synchronous (Jacobi) soup generation — the semantics of the fused kernel
    (csrc Item::soup_evolve).  ``uids`` are the random-stream keys of the slots: the engine
    keys soup streams by global slot (``np.arange(n)``).  Returns (W1, action, counterpart,
    loss, respawn)."""
    n = W0.shape[0]
    att, te = soup_decisions(seed, gen, n, params["attacking_rate"], params["learn_from_rate"],
                             int(params.get("segment", 0)))
    W = np.array(W0, dtype=np.float32, copy=True)
    ctr = np.full(n, (gen * 1024) & M32, dtype=np.int64)
    with np.errstate(over="ignore", invalid="ignore"):
        for i in range(n):  # ascending attacker slot per victim
            j = att[i]
            if j < 0:
                continue
            W[j:j + 1] = apply(spec, W0[i:i + 1], W[j:j + 1], seed=seed, uids=uids[j:j + 1], ctr=int(ctr[j]))
            ctr[j] += 1
        action = np.where(att >= 0, 1, 0).astype(np.int8)
        cp = np.where(att >= 0, att, -1).astype(np.int64)
        loss = np.zeros(n, dtype=np.float32)
        tctr = (gen * 1024 + 512) & M32
        sev = int(params.get("learn_from_severity", 1))
        for i in range(n):
            c = tctr
            if te[i] >= 0:
                for _ in range(sev):
                    W[i:i + 1], l = train_epoch(spec, W[i:i + 1], W0[te[i]:te[i] + 1], lr, shuffle, seed, uids[i:i + 1], c)
                    loss[i] = l[0]
                    c += 1
                action[i] = 2
                cp[i] = te[i]
            for _ in range(int(params.get("train", 0))):
                W[i:i + 1], l = train_epoch(spec, W[i:i + 1], W[i:i + 1].copy(), lr, shuffle, seed, uids[i:i + 1], c)
                loss[i] = l[0]
                c += 1
                action[i] = 3
                cp[i] = -1
        respawn = np.zeros(n, dtype=np.int8)
        eps = params.get("epsilon", 1e-14)
        if params.get("remove_divergent"):
            respawn[is_diverged(W)] = 1
        if params.get("remove_zero"):
            respawn[(respawn == 0) & is_zero(W, eps)] = 2
    return W, action, cp, loss, respawn


def respawn_key(gen, slot):
    """csrc respawn_key: init key of the particle born in `slot` at generation `gen`."""
    return (1 << 62) | ((int(gen) & M32) << 32) | int(slot)


def soup_generation_seq(spec, W0, gen, seed, params, lr=0.01, shuffle=True):
    """Sequential (Gauss-Seidel) soup generation -- the reference order (code/soup.py:51-87,
    S11) with the native engine's keys (csrc Item::soup_seq_one): particles in index order,
    the table updated in place; j attacks att[j] (shuffle_random keyed by the attacker),
    learns from te[j]'s current weights, self-trains, and is re-initialised with
    respawn_key(gen, j) when divergent / zero.  Returns (W1, action, counterpart, loss,
    respawn)."""
    n = W0.shape[0]
    att, te = soup_decisions(seed, gen, n, params["attacking_rate"], params["learn_from_rate"],
                             int(params.get("segment", 0)))
    W = np.array(W0, dtype=np.float32, copy=True)
    keys = np.arange(n, dtype=np.uint64)
    action = np.zeros(n, dtype=np.int8)
    cp = np.full(n, -1, dtype=np.int64)
    loss = np.zeros(n, dtype=np.float32)
    respawn = np.zeros(n, dtype=np.int8)
    eps = params.get("epsilon", 1e-14)
    sev = int(params.get("learn_from_severity", 1))
    with np.errstate(over="ignore", invalid="ignore"):
        for j in range(n):
            v = att[j]
            if v >= 0:
                W[v:v + 1] = apply(spec, W[j:j + 1].copy(), W[v:v + 1].copy(), seed=seed, uids=keys[j:j + 1],
                                   ctr=(gen * 1024 + 1) & M32)
                action[j], cp[j] = 1, v
            c = (gen * 1024 + 512) & M32
            if te[j] >= 0:
                for _ in range(sev):
                    W[j:j + 1], l = train_epoch(spec, W[j:j + 1], W[te[j]:te[j] + 1].copy(), lr, shuffle, seed,
                                                keys[j:j + 1], c)
                    loss[j] = l[0]
                    c += 1
                action[j], cp[j] = 2, te[j]
            for _ in range(int(params.get("train", 0))):
                W[j:j + 1], l = train_epoch(spec, W[j:j + 1], W[j:j + 1].copy(), lr, shuffle, seed, keys[j:j + 1], c)
                loss[j] = l[0]
                c += 1
                action[j], cp[j] = 3, -1
            rs = 0
            if params.get("remove_divergent") and is_diverged(W[j:j + 1])[0]:
                rs = 1
            elif params.get("remove_zero") and is_zero(W[j:j + 1], eps)[0]:
                rs = 2
            if rs:
                W[j] = init(spec, np.array([respawn_key(gen, j)], dtype=np.uint64), seed)[0]
            respawn[j] = rs
    return W, action, cp, loss, respawn
