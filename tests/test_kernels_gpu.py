"""HIP kernels (gfx950) vs the float32 numpy oracle, and vs the host path of the
same C++ code.  Every test here needs a ROCm device and the native library: the HIP
path must be the one that runs (no eager fallback exists)."""
import numpy as np
import pytest
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import kernels as K
from self_replicating_neural_networks_amd.oracle import core as O
from self_replicating_neural_networks_amd.soup_engine import SoupEngine

pytestmark = pytest.mark.gpu

SPECS = [ArchSpec.weightwise(2, 2), ArchSpec.weightwise(4, 3), ArchSpec.aggregating(4, 2, 2),
         ArchSpec.aggregating(4, 2, 2, shuffler="random"), ArchSpec.recurrent(2, 2), ArchSpec.fft(4, 2, 2)]


def _rel(a, b):
    """max over rows of |a-b| / (row scale of b): robust to cancellation in single entries."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if a.ndim == 1:
        a, b = a[:, None], b[:, None]
    ok = np.all(np.isfinite(a), axis=1) & np.all(np.isfinite(b), axis=1)
    if not ok.any():
        return 0.0
    a, b = a[ok], b[ok]
    scale = np.max(np.abs(b), axis=1, keepdims=True) + 1e-6
    return float(np.max(np.abs(a - b) / scale))


@pytest.mark.parametrize("spec", SPECS, ids=lambda s: f"{s.kind}-{s.width}-{s.depth}-{s.shuffler}")
def test_init_apply_train_classify_vs_oracle(cuda, spec):
    n, seed = 2048, 11
    uid = torch.arange(n, dtype=torch.int64, device=cuda) + 5
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, uid, seed)
    ow = O.init(spec, uid.cpu().numpy(), seed)
    # orthogonal init goes through logf/cosf/sqrtf: device libm differs by a few ulp
    assert _rel(W[:, :spec.P].cpu().numpy(), ow) < (2e-3 if spec.kind == "recurrent" else 1e-4)
    # padding stays zero
    assert torch.all(W[:, spec.P:] == 0)
    # one step of each op from the SAME inputs (the device's rows): fp32 differences are
    # rounding only -- fma contraction and summation order.  1e-5 of the row scale for the
    # feed-forward nets (measured host path vs oracle: <= 4e-6); the recurrent BPTT sums 17
    # timestep products in another association (host path vs oracle: 1.4e-5) -> 5e-5.
    tol = 5e-5 if spec.kind == "recurrent" else 1e-5
    w0 = W[:, :spec.P].cpu().numpy()
    # attack: row i attacked by row i-1
    out = torch.zeros_like(W)
    idx_f = torch.roll(torch.arange(n, device=cuda), 1).contiguous()
    K.apply(spec, W, out, idx_f=idx_f, uid=uid, seed=seed, ctr=3)
    oo = O.apply(spec, np.roll(w0, 1, axis=0), w0, seed=seed, uids=uid.cpu().numpy(), ctr=3)
    assert _rel(out[:, :spec.P].cpu().numpy(), oo) < tol
    # self-train epoch
    W2 = W.clone()
    loss = K.train(spec, W2, epochs=1, lr=0.01, uid=uid, seed=seed, ctr=9)
    tw, tl = O.train_epoch(spec, w0, w0, 0.01, True, seed, uid.cpu().numpy(), 9)
    assert _rel(W2[:, :spec.P].cpu().numpy(), tw) < tol
    assert _rel(loss.cpu().numpy(), tl) < tol
    # classification
    cls, counts = K.classify(spec, W, 1e-4, uid=uid, seed=seed)
    ocls = O.classify(spec, ow, 1e-4)
    assert (cls.cpu().numpy() == ocls).mean() > 0.99
    assert int(counts.sum()) == n


@pytest.mark.parametrize("spec", SPECS[:3] + SPECS[4:5], ids=lambda s: f"{s.kind}-{s.width}-{s.depth}")
def test_device_matches_host_path(cuda, spec):
    """Same C++ per-particle code on CPU threads and on the GPU."""
    n, seed = 1000, 5
    uid = torch.arange(n, dtype=torch.int64)
    Wc = torch.zeros(n, spec.PP)
    K.init_rows(spec, Wc, uid, seed)
    Wg = Wc.to(cuda)
    K.train(spec, Wc, epochs=3, uid=uid, seed=seed)
    K.train(spec, Wg, epochs=3, uid=uid.to(cuda), seed=seed)
    # same C++ code; fma contraction differs host/device: BPTT amplifies the last ulps
    assert _rel(Wg.cpu().numpy(), Wc.numpy()) < (5e-3 if spec.kind == "recurrent" else 1e-4)
    cc, _ = K.run_fixpoint(spec, Wc, 5, 1e-4)[:2]
    cg, _ = K.run_fixpoint(spec, Wg, 5, 1e-4)[:2]
    assert (cc.numpy() == cg.cpu().numpy()).mean() > 0.99


def test_run_fixpoint_statistics_weightwise(cuda):
    """applying-fixpoints (code/setups/applying-fixpoints.py): 100 self-applications of
    WW(2,2); published 23/50 divergent, 27/50 fix_zero (log.txt:1-2)."""
    spec = ArchSpec.weightwise(2, 2)
    n = 20000
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, uid, 2024)
    cls, _, _ = K.run_fixpoint(spec, W, 100, 1e-4, early_exit=False)
    c = np.bincount(cls.cpu().numpy(), minlength=5)
    p_div = c[0] / n
    assert abs(p_div - 0.46) < 0.05, c
    assert c[0] + c[1] > 0.97 * n, c


def test_soup_engine_gpu_vs_oracle(cuda):
    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=3, remove_divergent=True, remove_zero=True,
                  epsilon=1e-4)
    e = SoupEngine(spec, 3000, params, device=cuda, seed=7)
    W0 = e.local_rows()[:, :spec.P].cpu().numpy().copy()
    uids = np.arange(3000, dtype=np.uint64)  # soup streams are keyed by slot, not uid
    e.evolve(1)
    W1, act, cp, loss, resp = O.soup_generation_sync(spec, W0, uids, 1, 7, params)
    keep = resp == 0
    # a generation = attacks + learn_from + 3 epochs of SGD (~60 dependent steps per particle)
    assert _rel(e.local_rows()[:, :spec.P].cpu().numpy()[keep], W1[keep]) < 1e-5
    assert (e.action.cpu().numpy() == act).all()
    assert (e.counterpart.cpu().numpy() == cp).all()
    assert (e.respawn.cpu().numpy() == resp).mean() > 0.999


def test_soup_graph_replay_matches_eager(cuda):
    spec = ArchSpec.weightwise(2, 2)
    params = dict(train=2, remove_divergent=True, remove_zero=True, epsilon=1e-4)
    a = SoupEngine(spec, 4096, params, device=cuda, seed=3)
    b = SoupEngine(spec, 4096, params, device=cuda, seed=3)
    assert b.capture(warmup=1)
    a.evolve(1 + 5)  # capture() ran one eager warmup generation and captured (not ran) one
    b.evolve(5)
    torch.cuda.synchronize()
    assert torch.equal(a.uid, b.uid)
    assert torch.allclose(a.local_rows(), b.local_rows(), equal_nan=True)


BIG = [ArchSpec.aggregating(4, 10, 3), ArchSpec.aggregating(4, 8, 2, aggregator="max")]


@pytest.mark.parametrize("spec", BIG, ids=lambda s: f"agg-{s.aggregates}-{s.width}-{s.depth}-{s.aggregator}")
def test_wave_per_particle_aggregating_vs_oracle(cuda, spec):
    """Aggregating(4, 10, 3) (P = 280, north-star config) runs wave-per-particle."""
    n, seed = 3000, 21
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, uid, seed)
    ow = O.init(spec, uid.cpu().numpy(), seed)
    assert _rel(W[:, :spec.P].cpu().numpy(), ow) < 1e-5
    out = torch.zeros_like(W)
    idx_f = torch.roll(torch.arange(n, device=cuda), 1).contiguous()
    K.apply(spec, W, out, idx_f=idx_f)
    oo = O.apply(spec, np.roll(ow, 1, axis=0), ow)
    assert _rel(out[:, :spec.P].cpu().numpy(), oo) < 1e-5
    # multi-step self-application on the chunk state == step-by-step oracle
    W5 = W.clone()
    cls, nsteps, _ = K.run_fixpoint(spec, W5, 5, 1e-4, early_exit=False)
    w = ow.copy()
    with np.errstate(all="ignore"):
        for _ in range(5):
            w = O.apply(spec, w, w)
    # five chained degree-(D+1) polynomial maps amplify fma-order ulps: compare loosely
    assert _rel(W5[:, :spec.P].cpu().numpy(), w) < 1e-2
    assert (cls.cpu().numpy() == O.classify(spec, w, 1e-4)).mean() > 0.99
    c2, counts = K.classify(spec, W, 1e-4)
    assert (c2.cpu().numpy() == O.classify(spec, ow, 1e-4)).mean() > 0.99 and int(counts.sum()) == n
    W2 = W.clone()
    loss = K.train(spec, W2, epochs=3, lr=0.01)
    tw = ow.copy()
    for _ in range(3):
        tw, tl = O.train_epoch(spec, tw, tw, 0.01, False)
    assert _rel(W2[:, :spec.P].cpu().numpy(), tw) < 1e-4
    assert _rel(loss.cpu().numpy(), tl) < 1e-4


def test_big_aggregating_applying_statistics(cuda):
    """applying-fixpoints on the north-star shape: the chunk-state kernel runs 100 steps."""
    spec = ArchSpec.aggregating(4, 10, 3)
    n = 100_000
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, torch.arange(n, dtype=torch.int64, device=cuda), 3)
    cls, _, _ = K.run_fixpoint(spec, W, 100, 1e-4, early_exit=False)
    c = np.bincount(cls.cpu().numpy(), minlength=5)
    assert c.sum() == n and c[0] + c[1] > 0.9 * n  # divergent or collapsed to zero


WIDE = [ArchSpec.weightwise(16, 2), ArchSpec.weightwise(16, 3), ArchSpec.weightwise(32, 2)]


@pytest.mark.parametrize("spec", WIDE, ids=lambda s: f"ww-{s.width}-{s.depth}")
def test_mfma_weightwise_vs_oracle(cuda, spec):
    """Wide Weightwise nets: all P weight-points of a target through one MLP = a GEMM
    chain on v_mfma_f32_16x16x4_f32 (wave per particle)."""
    n, seed = 512, 8
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, uid, seed)
    ow = O.init(spec, uid.cpu().numpy(), seed)
    assert _rel(W[:, :spec.P].cpu().numpy(), ow) < 1e-5
    assert torch.all(W[:, spec.P:] == 0)
    out = torch.zeros_like(W)
    idx_f = torch.roll(torch.arange(n, device=cuda), 1).contiguous()
    K.apply(spec, W, out, idx_f=idx_f)
    oo = O.apply(spec, np.roll(ow, 1, axis=0), ow)
    assert _rel(out[:, :spec.P].cpu().numpy(), oo) < 1e-4
    W3 = W.clone()
    cls, nsteps, _ = K.run_fixpoint(spec, W3, 3, 1e-4, early_exit=False)
    w = ow.copy()
    with np.errstate(all="ignore"):
        for _ in range(3):
            w = O.apply(spec, w, w)
    assert _rel(W3[:, :spec.P].cpu().numpy(), w) < 1e-2
    assert (cls.cpu().numpy() == O.classify(spec, w, 1e-4)).mean() > 0.98
    c0, counts = K.classify(spec, W, 1e-4)
    assert (c0.cpu().numpy() == O.classify(spec, ow, 1e-4)).mean() > 0.99 and int(counts.sum()) == n


def test_mfma_weightwise_identity_fixpoint(cuda):
    """The identity fixpoint generalises to any width: f(x) = x[0] stays put exactly."""
    spec = ArchSpec.weightwise(16, 2)
    W = torch.zeros(4, spec.PP, device=cuda)
    W[:, 0] = 1.0                      # A0[0][0]
    W[:, spec.offsets[1]] = 1.0        # A1[0][0]
    W[:, spec.offsets[2]] = 1.0        # A2[0][0]
    before = W.clone()
    cls, _, _ = K.run_fixpoint(spec, W, 5, 1e-4, early_exit=False)
    assert torch.equal(W, before) and cls.tolist() == [O.C_FIX_OTHER] * 4


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("spec", [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2)], ids=["ww", "agg"])
def test_lowp_device_equals_rounded_fp32(cuda, spec, dtype):
    """16-bit tables on the GPU: K fused self-applications == K rounded fp32 steps (bitwise)."""
    n = 5000
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W = torch.zeros(n, spec.PP, dtype=dtype, device=cuda)
    K.init_rows(spec, W, uid, 2)
    W32 = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W32, uid, 2)
    assert torch.equal(W, W32.to(dtype))
    Wk = W.clone()
    K.run_fixpoint(spec, Wk, 4, 1e-4, early_exit=False)
    ref = W.clone()
    for _ in range(4):
        r = ref.float()
        K.run_fixpoint(spec, r, 1, 1e-4, early_exit=False)
        ref = r.to(dtype)
    nan = lambda t: t.float().nan_to_num(7.0, 9.0, -9.0)
    assert torch.equal(nan(Wk), nan(ref))
    Wt, Wt32 = W.clone(), W.float()
    K.train(spec, Wt, epochs=2, uid=uid, seed=1)
    K.train(spec, Wt32, epochs=2, uid=uid, seed=1)
    assert torch.equal(nan(Wt), nan(Wt32.to(dtype)))
    # device == host path of the same 16-bit kernels
    Wc = W.cpu()
    K.run_fixpoint(spec, Wc, 4, 1e-4, early_exit=False)
    assert (nan(Wc) == nan(Wk.cpu())).float().mean() > 0.999


def test_lowp_soup_graph_on_device(cuda):
    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=5, remove_divergent=True, remove_zero=True)
    a = SoupEngine(spec, 20_000, params, device=cuda, seed=4, dtype=torch.float16, exchange="allgather")
    b = SoupEngine(spec, 20_000, params, device=cuda, seed=4, dtype=torch.float16)
    assert a.capture(warmup=1)
    b.evolve(1)
    a.evolve(5)
    b.evolve(5)
    assert torch.equal(a.local_rows(), b.local_rows()) and torch.equal(a.uid, b.uid)
    c = a.count()
    assert sum(c.values()) == 20_000


@pytest.mark.parametrize("spec", [ArchSpec.weightwise(2, 2), ArchSpec.aggregating(4, 2, 2), ArchSpec.recurrent(2, 2)],
                         ids=lambda s: s.kind)
def test_fused_generation_equals_unfused(cuda, spec):
    """OP_SOUP_GEN (one launch: evolve + next attack lists + census + last-wave uid scan
    across all XCDs) == decide -> evolve -> respawn -> classify, bitwise, every generation;
    n not a multiple of 64 and enough waves to span every XCD."""
    params = dict(attacking_rate=0.2, learn_from_rate=0.2, train=3, remove_divergent=True, remove_zero=True,
                  epsilon=1e-4)
    n = 70001
    a = SoupEngine(spec, n, params, device=cuda, seed=13)
    b = SoupEngine(spec, n, params, device=cuda, seed=13)
    b.fused = False
    a.stats = b.stats = True
    for g in range(6):
        a.evolve(1)
        b.evolve(1)
        assert torch.equal(a.local_rows(), b.local_rows()), g
        assert torch.equal(a.uid, b.uid), g
        assert int(a.next_uid) == int(b.next_uid), g
        assert a.last_census() == b.last_census(), g
    assert int(a.gen_dev) == int(b.gen_dev)
    assert int(a._done) == 0
    a.capture(warmup=1)
    b.evolve(1)
    a.evolve(3)
    b.evolve(3)
    assert torch.equal(a.local_rows(), b.local_rows())
    assert a.last_census() == b.last_census()


def test_multi_generation_graph_equals_eager(cuda):
    """capture() also records graphs of 20, 16, 8, 4 and 2 consecutive generations for both
    start parities (one launch each): 21 and then 23 generations through them (20 + a
    single-generation graph, then 20 + 2 + 1 from the other parity) == eager."""
    spec = ArchSpec.weightwise(2, 2)
    params = dict(attacking_rate=0.1, learn_from_rate=0.1, train=4, remove_divergent=True, remove_zero=True,
                  epsilon=1e-4)
    a = SoupEngine(spec, 30000, params, device=cuda, seed=21)
    b = SoupEngine(spec, 30000, params, device=cuda, seed=21)
    a.stats = b.stats = True
    assert a.capture(warmup=1)
    assert a._chunk is not None and [c[2] for c in a._chunks] == [20, 20, 16, 16, 8, 8, 4, 4, 2, 2]
    assert sorted({c[1] for c in a._chunks}) == [0, 1]
    b.evolve(1)
    a.evolve(21)
    b.evolve(21)
    a.evolve(23)
    b.evolve(23)
    assert a.time == b.time == 45
    assert torch.equal(a.local_rows(), b.local_rows())
    assert torch.equal(a.uid, b.uid)
    assert a.last_census() == b.last_census()
    a.release_graphs()


def test_soup_is_deterministic_run_to_run(cuda):
    """Race detector for the atomics of the generation (attack-list links, need masks,
    block stats): two identical soups stay bitwise equal."""
    params = dict(attacking_rate=0.5, learn_from_rate=0.5, train=2, remove_divergent=True, remove_zero=True,
                  epsilon=1e-4)
    runs = []
    for _ in range(2):
        e = SoupEngine(ArchSpec.weightwise(2, 2), 50000, params, device=cuda, seed=77)
        e.stats = True
        e.capture(warmup=1)
        e.evolve(12)
        runs.append((e.local_rows().clone(), e.uid.clone(), e.last_census()))
        e.release_graphs()
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert runs[0][2] == runs[1][2]


@pytest.mark.parametrize("aggregator", ["mean", "max"])
def test_big_aggregating_row_kernels_match_wave_kernels(cuda, aggregator, monkeypatch):
    """Lane-per-particle row kernels (row in VGPRs, default) vs the wave-per-particle
    kernels (SRNN_BIG_WAVE=1) for the P = 280 north-star net: attack, classify, train,
    learn_from."""
    spec = ArchSpec.aggregating(4, 10, 3, aggregator=aggregator)
    n = 5000
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W = torch.zeros(n, spec.PP, device=cuda)
    K.init_rows(spec, W, uid, 4)
    idx = torch.roll(torch.arange(n, device=cuda), 3).contiguous()
    res = {}
    for mode in ("wave", "row"):
        if mode == "wave":
            monkeypatch.setenv("SRNN_BIG_WAVE", "1")
        else:
            monkeypatch.delenv("SRNN_BIG_WAVE", raising=False)
        out = torch.zeros_like(W)
        K.apply(spec, W, out, idx_f=idx)
        cls, counts = K.classify(spec, W, 1e-4)
        Wt = W.clone()
        lt = K.train(spec, Wt, epochs=3, uid=uid, seed=5)
        Wl = W.clone()
        ll = K.learn_from(spec, Wl, W, idx_t=idx, epochs=2, uid=uid, seed=5)
        Wf = W.clone()
        fc, fs, _ = K.run_fixpoint(spec, Wf, 30, 1e-4)
        res[mode] = (out, cls, counts, Wt, lt, Wl, ll, Wf, fc, fs)
    a, b = res["wave"], res["row"]
    assert _rel(a[0][:, :spec.P].cpu().numpy(), b[0][:, :spec.P].cpu().numpy()) < 1e-5
    assert (a[1] == b[1]).float().mean() > 0.999
    assert torch.equal(a[2], b[2]) or (a[2] - b[2]).abs().sum() <= 2
    for i in (3, 5):
        assert _rel(a[i][:, :spec.P].cpu().numpy(), b[i][:, :spec.P].cpu().numpy()) < 1e-5
    for i in (4, 6):
        assert _rel(a[i].cpu().numpy(), b[i].cpu().numpy()) < 1e-4
    assert torch.equal(a[7], b[7]) and torch.equal(a[8], b[8]) and torch.equal(a[9], b[9])  # run_fixpoint


@pytest.mark.parametrize("width,depth,dtype", [(2, 2, torch.float32), (2, 2, torch.bfloat16),
                                               (2, 1, torch.float32), (1, 1, torch.float32)])
def test_group_fixpoint_kernel_matches_lane_kernel(cuda, dtype, width, depth, monkeypatch):
    """Small-population run_fixpoint (16 lanes per particle, SRNN_FIX_GROUP=1) vs the
    lane-per-particle kernel (SRNN_FIX_GROUP=0): bitwise equal weights, classes, step
    counts and trajectories."""
    spec = ArchSpec.weightwise(width, depth)
    n = 3001
    uid = torch.arange(n, dtype=torch.int64, device=cuda)
    W0 = torch.zeros(n, spec.PP, dtype=dtype, device=cuda)
    K.init_rows(spec, W0, uid, 7)
    W0[:50] *= 40.0  # divergent
    W0[50:100] *= 1e-3  # towards zero
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("SRNN_FIX_GROUP", mode)
        out = []
        for early, sec, rec, steps in ((True, True, False, 100), (False, False, False, 37), (True, True, True, 12)):
            W = W0.clone()
            cls, ns, traj = K.run_fixpoint(spec, W, steps, 1e-4, early_exit=early, with_sec=sec, record=rec)
            out.append((W, cls, ns, traj))
        res[mode] = out
    bits = torch.int32 if dtype == torch.float32 else torch.int16

    def same(x, y):  # bitwise, so NaN rows compare equal
        return torch.equal(x.contiguous().view(bits), y.contiguous().view(bits))

    for a, b in zip(res["0"], res["1"]):
        assert same(a[0][:, :spec.P], b[0][:, :spec.P])
        assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
        if a[3] is not None:
            assert same(a[3][..., :spec.P], b[3][..., :spec.P])
    cls = res["1"][0][1].cpu()
    assert len(torch.unique(cls)) >= 2  # a mixture of outcomes was exercised


def _bf16_host(u32: np.ndarray) -> np.ndarray:
    """The host form of StBF16::enc (csrc/srnn_kernels.h): RNE, NaN kept quiet."""
    u = u32.astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    return np.where(nan, ((u >> 16) | 0x40) & 0xFFFF, r).astype(np.uint16)


def test_bf16_encode_matches_host_rounding(cuda):
    """The device bf16 storage rounding (gfx950 v_cvt_pk_bf16_f32) equals the host formula
    bit for bit: ties, denormals, infinities and NaN payloads of both signs."""
    import ctypes
    from self_replicating_neural_networks_amd.ops import _lib
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2 ** 32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    special = np.array([0, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0xFFC00000, 0x7F800001, 0xFF800001,
                        0x7FBFFFFF, 0x7F808000, 0x00000001, 0x807FFFFF, 0x00018000, 0x00008000, 0x3F808000,
                        0x3F818000, 0x3F80FFFF, 0x7F7FFFFF, 0x7F7F8000, 0xFF7F8000], dtype=np.uint32)
    ties = (rng.integers(0, 2 ** 16, size=4096, dtype=np.uint64).astype(np.uint32) << 16) | 0x8000
    u = np.concatenate([special, ties, bits])
    x = torch.from_numpy(u.view(np.float32).copy()).to(cuda)
    out = torch.empty(x.numel(), dtype=torch.int16, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    r = _lib.lib().srnn_storage_encode(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                       x.numel(), 1, ctypes.c_void_p(st))
    assert r == 0
    got = out.cpu().numpy().view(np.uint16)
    want = _bf16_host(u)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(hex(u[i]), hex(got[i]), hex(want[i])) for i in bad[:8]]
    # fp16: IEEE RNE for every non-NaN value
    r = _lib.lib().srnn_storage_encode(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                       x.numel(), 2, ctypes.c_void_p(st))
    assert r == 0
    f = u.view(np.float32)
    ok = ~np.isnan(f)
    with np.errstate(over="ignore"):
        want16 = f.astype(np.float16).view(np.uint16)
    assert np.array_equal(out.cpu().numpy().view(np.uint16)[ok], want16[ok])
