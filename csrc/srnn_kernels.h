// srnn_kernels.h — population-batched operators, instantiated per architecture.
//
// Each operator is written once as a per-item function `Item<Net>::op(args, i, scratch)`
// (host + device).  `k_op<Net, OP>` runs it lane-per-particle on the GPU (one wave per
// 64 particles, the particle's weights in VGPRs, lane-private sample / permutation
// scratch in LDS); `host_op<Net, OP>` runs the identical code over a host thread pool for
// CPU tensors.  Reference hot loops replaced here: the per-weight `model.predict` of
// code/network.py:265-279, the Keras `fit` epochs of :613-626, the run_net loop of
// code/experiment.py:70-91 and the per-particle soup loop of code/soup.py:51-103.
#pragma once
#include "srnn_core.h"
#include "srnn_abi.h"
#include <thread>
#include <vector>
#include <algorithm>
#include <climits>
#include <cstdlib>

namespace srnn {

void set_error(const char* msg);

constexpr int TB = 64;  // threads per block: one wave; lane-private LDS scratch per thread

enum Action : int8_t { A_NONE = 0, A_ATTACKING = 1, A_LEARN_FROM = 2, A_TRAIN_SELF = 3 };

template <class F>
void host_parallel(int64_t n, F&& f) {
  unsigned hw = std::thread::hardware_concurrency();
  int64_t nt = std::min<int64_t>(hw ? hw : 1, 16);
  if (n < 256 || nt <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  nt = std::min<int64_t>(nt, (n + 127) / 128);
  std::vector<std::thread> th;
  int64_t chunk = (n + nt - 1) / nt;
  for (int64_t t = 0; t < nt; ++t) {
    int64_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    th.emplace_back([b, e, &f]() {
      for (int64_t i = b; i < e; ++i) f(i);
    });
  }
  for (auto& x : th) x.join();
}

SRNN_HD int32_t atomic_add_i32(int32_t* p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}

// stride (in float4) between the sample slots of one lane: TB in LDS on the device,
// 1 in the host scratch array
#if defined(__HIP_DEVICE_COMPILE__)
#define SAMP_STRIDE TB
#else
#define SAMP_STRIDE 1
#endif

SRNN_HD int32_t atomic_or_i32(int32_t* p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicOr(p, v);
#else
  return __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}

// rank owning global slot g under the contiguous sharding lo_r = floor(r * N / R)
SRNN_HD int32_t shard_of(int64_t g, int64_t n_total, int32_t world) {
  int32_t r = (int32_t)((g * world) / n_total);
  while (r + 1 < world && ((int64_t)(r + 1) * n_total) / world <= g) ++r;
  while (r > 0 && ((int64_t)r * n_total) / world > g) --r;
  return r;
}

// init key of the particle born in slot g at generation `gen` (rank-count invariant)
SRNN_HD uint64_t respawn_key(int32_t gen, int64_t g) {
  return (1ull << 62) | ((uint64_t)(uint32_t)gen << 32) | (uint64_t)g;
}

// ----------------------------------------------------------------------------------
// Storage precision of the weight tables.  Arithmetic is always fp32 in
// registers; a 16-bit table holds every *stored* weight state in that format, and the
// multi-step operators round after each application (so a K-step launch equals K
// one-step launches and fixpoint tests compare what would be stored).
// ----------------------------------------------------------------------------------
SRNN_HD float bits_f(uint32_t u) {
  union { uint32_t u; float f; } x;
  x.u = u;
  return x.f;
}
SRNN_HD uint32_t f_bits(float f) {
  union { uint32_t u; float f; } x;
  x.f = f;
  return x.u;
}
struct StF32 {
  static constexpr int ID = 0, BYTES = 4;
  SRNN_HD static float q(float x) { return x; }
};
struct StBF16 {  // round-to-nearest-even, NaN kept quiet
  static constexpr int ID = 1, BYTES = 2;
  SRNN_HD static uint16_t enc(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    // gfx950 v_cvt_pk_bf16_f32: the same RNE rounding and NaN quieting as the host form
    // (tests/test_kernels_gpu.py::test_bf16_encode_matches_host_rounding).  The barrier keeps
    // the fp32 rounding of the producing fma: without it the backend may fold
    // fptrunc(fma) into one bf16-rounded fma (as for fp16 below), so a kernel that rounds a
    // freshly trained weight would differ from one that rounds it after a store
    asm volatile("" : "+v"(x));
    return __builtin_bit_cast(uint16_t, (__bf16)x);
#else
    uint32_t u = f_bits(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
#endif
  }
  SRNN_HD static float dec(uint16_t h) { return bits_f((uint32_t)h << 16); }
  SRNN_HD static float q(float x) { return dec(enc(x)); }
};
struct StF16 {  // IEEE binary16, round-to-nearest-even (overflow -> inf = divergent)
  static constexpr int ID = 2, BYTES = 2;
  SRNN_HD static uint16_t enc(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    // keep the fp32 rounding of the producing fma: without the barrier the backend folds
    // fptrunc(fma) into v_fma_mixlo_f16 (one rounding instead of fp32-then-fp16)
    asm volatile("" : "+v"(x));
#endif
    _Float16 h = (_Float16)x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    return u;
  }
  SRNN_HD static float dec(uint16_t u) {
    _Float16 h;
    __builtin_memcpy(&h, &u, 2);
    return (float)h;
  }
  SRNN_HD static float q(float x) { return dec(enc(x)); }
};

template <class Net, class S = StF32>
struct Item {
  static constexpr int P = Net::P;
  static constexpr int PP = Net::PP;
  static constexpr int RB = PP * S::BYTES;  // bytes per table row
  static constexpr int XB = RB + 16;        // exchange row: weights + (slot, gen, -, -) int32 tags
  // the first SR rows of every destination block of the all-to-all carry the sender's
  // int64[6] stats (census of its previous generation + respawn count): the per-rank
  // stats all-gather rides on the row exchange (one collective per generation)
  static constexpr int SR = (48 + XB - 1) / XB;

  // stats word q of rank r: from the exchange receive buffer (flag 256) or the gathered
  // [world][6] array
  SRNN_HD static int64_t stat(const SrnnArgs& a, int r, int q) {
    if (a.flags & 256)
      return reinterpret_cast<const int64_t*>(reinterpret_cast<const char*>(a.recvbuf) + (int64_t)r * a.cap * XB)[q];
    return a.stats[r * 6 + q];
  }
  SRNN_HD static void pack_stats(const SrnnArgs& a) {
    for (int r = 0; r < a.world; ++r) {
      int64_t* d = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(a.sendbuf) + (int64_t)r * a.cap * XB);
      for (int q = 0; q < 6; ++q) d[q] = (int64_t)a.counts[q];
    }
  }

  SRNN_HD static char* rowp(float* base, int64_t i) { return reinterpret_cast<char*>(base) + i * RB; }
  SRNN_HD static const char* rowp(const float* base, int64_t i) { return reinterpret_cast<const char*>(base) + i * RB; }

  // generation-start row of global slot g: local table (W2, this rank's rows) or the
  // exchange receive buffer for slots of other ranks
  // (flag 128: recvbuf is the all-gathered [n_total] table of every rank's rows)
  SRNN_HD static const char* row_of(const SrnnArgs& a, int64_t g) {
    if (a.world <= 1 || (g >= a.lo && g < a.lo + a.n)) return rowp(a.W2, g - a.lo);
    if (a.flags & 128) return rowp(a.recvbuf, g);
#if defined(__HIP_DEVICE_COMPILE__)
    if (a.flags & 524288)  // indexed by unpack workgroups of this same launch: memory-side read
      return reinterpret_cast<const char*>(a.recvbuf) +
             (int64_t)__hip_atomic_load(a.rmap + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * XB;
#endif
    return reinterpret_cast<const char*>(a.recvbuf) + (int64_t)a.rmap[g] * XB;
  }

  SRNN_HD static void q(float* w) {
    if constexpr (S::ID != 0) {
#pragma unroll
      for (int k = 0; k < P; ++k) w[k] = S::q(w[k]);
    }
  }

  SRNN_HD static void load(const char* __restrict__ row, float* __restrict__ w) {
    if constexpr (S::ID == 0) {
      const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll
      for (int q = 0; q < PP / 4; ++q) {
        float4 v = r4[q];
        if (4 * q + 0 < P) w[4 * q + 0] = v.x;
        if (4 * q + 1 < P) w[4 * q + 1] = v.y;
        if (4 * q + 2 < P) w[4 * q + 2] = v.z;
        if (4 * q + 3 < P) w[4 * q + 3] = v.w;
      }
    } else {
      const uint2* r2 = reinterpret_cast<const uint2*>(row);  // 4 x 16 bit
#pragma unroll
      for (int q = 0; q < PP / 4; ++q) {
        uint2 v = r2[q];
        if (4 * q + 0 < P) w[4 * q + 0] = S::dec((uint16_t)(v.x & 0xffffu));
        if (4 * q + 1 < P) w[4 * q + 1] = S::dec((uint16_t)(v.x >> 16));
        if (4 * q + 2 < P) w[4 * q + 2] = S::dec((uint16_t)(v.y & 0xffffu));
        if (4 * q + 3 < P) w[4 * q + 3] = S::dec((uint16_t)(v.y >> 16));
      }
    }
  }
  SRNN_HD static void store(char* __restrict__ row, const float* __restrict__ w) {
    if constexpr (S::ID == 0) {
      float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
      for (int q = 0; q < PP / 4; ++q) {
        float4 v;
        v.x = 4 * q + 0 < P ? w[4 * q + 0] : 0.f;
        v.y = 4 * q + 1 < P ? w[4 * q + 1] : 0.f;
        v.z = 4 * q + 2 < P ? w[4 * q + 2] : 0.f;
        v.w = 4 * q + 3 < P ? w[4 * q + 3] : 0.f;
        r4[q] = v;
      }
    } else {
      uint2* r2 = reinterpret_cast<uint2*>(row);
#pragma unroll
      for (int q = 0; q < PP / 4; ++q) {
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = 4 * q + k < P ? S::enc(w[4 * q + k]) : 0u;
        r2[q] = make_uint2(e[0] | (e[1] << 16), e[2] | (e[3] << 16));
      }
    }
  }
  SRNN_HD static void copy(float* __restrict__ d, const float* __restrict__ s) {
#pragma unroll
    for (int k = 0; k < P; ++k) d[k] = s[k];
  }
  SRNN_HD static Rng rng(const SrnnArgs& a) { return Rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)}; }
  // stream key of row i: its uid, or without a uid column its global slot lo + i
  SRNN_HD static uint64_t uid_of(const SrnnArgs& a, int64_t i) { return a.uid ? (uint64_t)a.uid[i] : (uint64_t)(a.lo + i); }
  SRNN_HD static ApplyCtx actx(const SrnnArgs& a, const SrnnCfg& c, uint64_t uid, uint32_t ctr, uint8_t* perm) {
    ApplyCtx x;
    x.rng = rng(a);
    x.uid = uid;
    x.ctr = ctr;
    x.aggregator = c.aggregator;
    x.shuffler = c.shuffler;
    x.perm = perm;
    return x;
  }

  // ---------------------------------------------------------------- init
  SRNN_HD static void init(const SrnnCfg&, const SrnnArgs& a, int64_t i, float4*, uint8_t*) {
    float w[P];
    Net::init(w, rng(a), uid_of(a, i));
    store(rowp(a.W, i), w);
  }

  // ---------------------------------------------------------------- apply (attack)
  SRNN_HD static void apply(const SrnnCfg& c, const SrnnArgs& a, int64_t i, float4*, uint8_t* perm) {
    int64_t fi = a.idx_f ? a.idx_f[i] : i;
    int64_t ti = a.idx_t ? a.idx_t[i] : i;
    int64_t oi = a.idx_o ? a.idx_o[i] : i;
    float f[P], t[P], o[P];
    load(rowp(a.W, fi), f);
    load(rowp(a.W, ti), t);
    uint64_t ouid = a.uid ? (uint64_t)a.uid[ti] : (uint64_t)ti;
    Net::apply(f, t, o, actx(a, c, ouid, a.ctr, perm));
    q(o);
    store(rowp(a.W2, oi), o);
  }

  // classification of the current weights (reference code/experiment.py:79-91)
  SRNN_HD static int8_t classify_w(const float* w, float eps, bool with_sec, const ApplyCtx& x) {
    if (is_diverged<P>(w)) return C_DIVERGENT;
    float f1[P];
    Net::apply(w, w, f1, x);
    q(f1);
    if (!is_diverged<P>(f1) && within_eps<P>(f1, w, eps)) return is_zero<P>(w, eps) ? C_FIX_ZERO : C_FIX_OTHER;
    if (with_sec) {
      float f2[P];
      Net::apply(w, f1, f2, x);
      q(f2);
      if (!is_diverged<P>(f2) && within_eps<P>(f2, w, eps)) return C_FIX_SEC;
    }
    return C_OTHER;
  }

  // ---------------------------------------------------------------- run_net
  // reference code/experiment.py:70-77: while i < limit and not diverged and not fixpoint: self_attack
  SRNN_HD static void run_fixpoint(const SrnnCfg& c, const SrnnArgs& a, int64_t i, float4*, uint8_t* perm) {
    float w[P], nw[P];
    load(rowp(a.W, i), w);
    uint64_t uid = uid_of(a, i);
    ApplyCtx x = actx(a, c, uid, a.ctr, perm);
    if (a.traj) store(rowp(a.traj, i), w);
    int s = 0;
    for (; s < a.steps; ++s) {
      if (a.early_exit) {
        if (is_diverged<P>(w)) break;
        Net::apply(w, w, nw, x);
        q(nw);
        if (!is_diverged<P>(nw) && within_eps<P>(nw, w, a.eps)) break;  // is_fixpoint()
      } else {
        Net::apply(w, w, nw, x);
        q(nw);
      }
      copy(w, nw);
      x.ctr += 1;
      if (a.traj) store(rowp(a.traj, (int64_t)(s + 1) * a.n + i), w);
    }
    store(rowp(a.W, i), w);
    if (a.nsteps) a.nsteps[i] = s;
    if (a.cls) a.cls[i] = classify_w(w, a.eps, (a.flags & 8) != 0, x);
  }

  // ---------------------------------------------------------------- known-fixpoint variation
  // reference code/setups/known-fixpoint-variation.py:66-83
  SRNN_HD static void vary_run(const SrnnCfg& c, const SrnnArgs& a, int64_t i, float4*, uint8_t* perm) {
    float w[P], nw[P];
    load(rowp(a.W, i), w);
    ApplyCtx x = actx(a, c, uid_of(a, i), a.ctr, perm);
    int tts = 0, taf = 0;
    bool still = true;
    for (int s = 0; s < a.steps; ++s) {
      Net::apply(w, w, nw, x);
      q(nw);
      copy(w, nw);
      if (is_zero<P>(w, a.eps) || is_diverged<P>(w)) break;
      Net::apply(w, w, nw, x);
      q(nw);
      bool fix = !is_diverged<P>(nw) && within_eps<P>(nw, w, a.eps);
      if (fix) {
        if (still) ++taf;
        else still = true;
      } else {
        still = false;
      }
      ++tts;
    }
    store(rowp(a.W, i), w);
    a.nsteps[i] = tts;
    a.loss[i] = (float)taf;
  }

  // ---------------------------------------------------------------- perturb (vary)
  SRNN_HD static void perturb(const SrnnCfg&, const SrnnArgs& a, int64_t i, float4*, uint8_t*) {
    float w[P];
    load(rowp(a.W, i), w);
    Rng r = rng(a);
    uint64_t uid = uid_of(a, i);
#pragma unroll
    for (int k = 0; k < P; ++k) {
      U4 u = r.draw(uid, a.ctr * 1024u + (uint32_t)k, P_PERTURB);
      double mag = (double)u01(u.y) * (double)a.eps;
      w[k] = u01(u.x) < 0.5f ? (float)((double)w[k] + mag) : (float)((double)w[k] - mag);
    }
    store(rowp(a.W, i), w);
  }

  // ---------------------------------------------------------------- train / learn_from
  SRNN_HD static void train(const SrnnCfg& c, const SrnnArgs& a, int64_t i, float4* samp, uint8_t* perm, bool learn) {
    float w[P], s[P];
    load(rowp(a.W, i), w);
    if (learn) load(rowp(a.W2, a.idx_t ? a.idx_t[i] : i), s);
    TrainCtx tc;
    tc.lr = a.lr;
    tc.rng = rng(a);
    tc.uid = uid_of(a, i);
    tc.ctr = a.ctr;
    tc.samp = samp;
    tc.perm = perm;
    tc.shuffle = (a.flags & 1) != 0;
    tc.stride = SAMP_STRIDE;
    tc.aggregator = c.aggregator;
    float loss = 0.f;
    if constexpr (Net::KIND == 0) {
      loss = learn ? Net::template train_epochs<false>(w, s, a.epochs, tc)
                   : Net::template train_epochs<true>(w, s, a.epochs, tc);
    } else {
      for (int e = 0; e < a.epochs; ++e) {
        if (!learn) copy(s, w);
        loss = Net::train_epoch(w, s, tc);
      }
    }
    store(rowp(a.W, i), w);
    if (a.loss) a.loss[i] = loss;
  }

  // ---------------------------------------------------------------- classify
  SRNN_HD static int8_t classify(const SrnnCfg& c, const SrnnArgs& a, int64_t i, uint8_t* perm) {
    float w[P];
    load(rowp(a.W, i), w);
    int8_t k = classify_w(w, a.eps, (a.flags & 8) != 0, actx(a, c, uid_of(a, i), a.ctr, perm));
    if (a.cls) a.cls[i] = k;
    return k;
  }

  // ---------------------------------------------------------------- soup
  // Decisions of global slot g in generation `gen` (reference code/soup.py:56-63): a pure
  // function of (seed, slot, generation), so any rank can recompute any slot's decision.
  SRNN_HD static void decision(const SrnnArgs& a, int64_t g, int32_t gen, int32_t& at, int32_t& te) {
    U4 d = rng(a).draw((uint64_t)g, (uint32_t)gen, P_SOUP);
    at = -1;
    te = -1;
    // partners are drawn inside the slot's sub-soup (segment) or the whole population
    const int64_t span = a.segment > 0 ? a.segment : a.n_total;
    const int64_t base = a.segment > 0 ? (g / a.segment) * a.segment : 0;
    if (u01(d.x) < a.attacking_rate) at = (int32_t)(base + (int64_t)(((uint64_t)d.y * (uint64_t)span) >> 32));
    if (u01(d.z) < a.learn_from_rate) te = (int32_t)(base + (int64_t)(((uint64_t)d.w * (uint64_t)span) >> 32));
  }
  SRNN_HD static int32_t gen_of(const SrnnArgs& a) { return a.gen_ptr ? a.gen_ptr[0] : a.gen; }
  // the next generation's counter: the other ring slot (gen_out) or in place
  SRNN_HD static void set_gen(const SrnnArgs& a, int32_t g) {
    if (a.gen_out) a.gen_out[0] = g;
    else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = g;
  }

  // Every global slot: link attacks on this rank's victims into per-victim lists
  // (head[victim] in i32e, pre-set to -1; next[attacker] in i32f).  Optional i32a/i32b
  // receive the decisions (diagnostics/tests).
  SRNN_HD static void soup_decide(const SrnnArgs& a, int64_t i) {
    int32_t at, te;
    decision(a, i, gen_of(a), at, te);
    if (a.i32a) a.i32a[i] = at;
    if (a.i32b) a.i32b[i] = te;
    link_decision(a, i, at, te, a.i32e, a.i32f);
  }
  // attacks on this rank's victims -> lists (head, next); rows other ranks will need ->
  // need masks (sharded)
  SRNN_HD static void link_decision(const SrnnArgs& a, int64_t i, int32_t at, int32_t te, int32_t* head,
                                    int32_t* next) {
    const bool i_local = i >= a.lo && i < a.lo + a.n;
    if (at >= a.lo && at < a.lo + a.n) {
#if defined(__HIP_DEVICE_COMPILE__)
      next[i] = atomicExch(head + (at - a.lo), (int32_t)i);
#else
      next[i] = __atomic_exchange_n(head + (at - a.lo), (int32_t)i, __ATOMIC_RELAXED);
#endif
    } else if (a.need && a.world > 1 && at >= 0 && i_local) {
      // my particle attacks a victim owned by another rank: ship my row there
      atomic_or_i32(a.need + (i - a.lo), 1 << shard_of(at, a.n_total, a.world));
    }
    if (a.need && a.world > 1 && te >= a.lo && te < a.lo + a.n && !i_local) {
      // a remote learner picked one of my particles as teacher
      atomic_or_i32(a.need + (te - a.lo), 1 << shard_of(i, a.n_total, a.world));
    }
  }

  // sharded soup: copy local row j to every rank that needs it this generation
  SRNN_HD static void soup_pack(const SrnnArgs& a, int64_t j) {
    int32_t m = a.need[j];
    if (!m) return;
    a.need[j] = 0;
    const int32_t gen = gen_of(a);
    const char* src = rowp(a.W2, j);
    while (m) {
      const int r = __builtin_ctz((unsigned)m);
      m &= m - 1;
      const int32_t pos = atomic_add_i32(a.sendcnt + r, 1);
      if (pos >= a.cap) {
        atomic_or_i32(a.ovf, 1);
        continue;
      }
      char* dst = reinterpret_cast<char*>(a.sendbuf) + ((int64_t)r * a.cap + pos) * XB;
      const uint2* s2 = reinterpret_cast<const uint2*>(src);
      uint2* d2 = reinterpret_cast<uint2*>(dst);
#pragma unroll
      for (int q = 0; q < RB / 8; ++q) d2[q] = s2[q];
      d2[RB / 8] = make_uint2((uint32_t)(a.lo + j), (uint32_t)gen);
      d2[RB / 8 + 1] = make_uint2(0u, 0u);
    }
  }
  // sharded soup: received row k -> rmap[slot]; rows of older generations are ignored
  SRNN_HD static void soup_unpack(const SrnnArgs& a, int64_t k) {
    if (k % a.cap < SR) return;  // stats rows
    const int32_t* tag = reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(a.recvbuf) + k * XB + RB);
    if (tag[1] == gen_of(a)) a.rmap[tag[0]] = (int32_t)k;
  }

  // Synchronous (Jacobi) generation for local row j: every read is from the
  // generation-start table W2 (global rows), the result goes to W (local rows).  The
  // particle's random streams (SGD shuffles, shuffle_random) are keyed by its global SLOT
  // and the generation -- not by its uid -- so a generation never waits for the uids of
  // the previous generation's newborns (their uid assignment overlaps the next generation).
  SRNN_HD static void soup_evolve(const SrnnCfg& c, const SrnnArgs& a, int64_t j, float4* samp, uint8_t* perm) {
    const int64_t g = a.lo + j;
    float w[P], f[P], o[P];
    load(rowp(a.W2, j), w);
    const uint64_t uid = (uint64_t)g;  // stream key of this slot
    const int32_t gen = gen_of(a);
    ApplyCtx x = actx(a, c, uid, (uint32_t)gen * 1024u, perm);
    // 1. attacks received, in ascending attacker slot order (the list is in arrival order)
    const int32_t head = a.i32e[j];
    a.i32e[j] = -1;  // list consumed: reset for the next generation's decide
    int32_t last = -1;
    while (head >= 0) {
      int32_t best = INT_MAX;
      for (int32_t r = head; r >= 0; r = a.i32f[r]) best = (r > last && r < best) ? r : best;
      if (best == INT_MAX) break;
      last = best;
      load(row_of(a, best), f);
      Net::apply(f, w, o, x);
      q(o);
      x.ctr += 1;
      copy(w, o);
    }
    int32_t my_at, te;
    decision(a, g, gen, my_at, te);
    int8_t act = A_NONE;
    int64_t cp = -1;
    if (my_at >= 0) {
      act = A_ATTACKING;
      cp = my_at;
    }
    TrainCtx tc;
    tc.lr = a.lr;
    tc.rng = rng(a);
    tc.uid = uid;
    tc.ctr = (uint32_t)gen * 1024u + 512u;
    tc.samp = samp;
    tc.perm = perm;
    tc.shuffle = (a.flags & 1) != 0;
    tc.stride = SAMP_STRIDE;
    tc.aggregator = c.aggregator;
    if ((a.flags & 131072) && a.perm_cur) {  // SGD permutations precomputed by helper waves
      tc.pre = reinterpret_cast<const unsigned long long*>(a.perm_cur) + j;
      tc.pre_stride = a.n;
      tc.pre_ctr0 = (uint32_t)gen * 1024u + 512u;
      tc.pre_n = a.perm_e;
    }
    float loss = 0.f;
    // 2. learn_from a teacher (its generation-start weights)
    if (te >= 0) {
      load(row_of(a, te), f);
      if constexpr (Net::KIND == 0) {
        if (a.severity > 0) loss = Net::template train_epochs<false>(w, f, a.severity, tc);
      } else {
        for (int e = 0; e < a.severity; ++e) loss = Net::train_epoch(w, f, tc);
      }
      act = A_LEARN_FROM;
      cp = te;
    }
    // 3. self-train
    if (a.epochs > 0) {
      if constexpr (Net::KIND == 0) {
        loss = Net::template train_epochs<true>(w, f, a.epochs, tc);
      } else {
        for (int e = 0; e < a.epochs; ++e) {
          copy(f, w);
          loss = Net::train_epoch(w, f, tc);
        }
      }
      act = A_TRAIN_SELF;
      cp = -1;
    }
    // 4. respawn flags (reference code/soup.py:77-86; zero test on the old particle)
    q(w);  // the stored state decides respawn
    int8_t rs = 0;
    if ((a.flags & 2) && is_diverged<P>(w)) rs = 1;
    else if ((a.flags & 4) && is_zero<P>(w, a.eps)) rs = 2;
    if (rs && (a.flags & 32)) Net::init(w, rng(a), respawn_key(gen, g));  // newborn, uid assigned later
    store(rowp(a.W, j), w);
    if (a.action) a.action[j] = act;
    if (a.counterpart) a.counterpart[j] = cp;
    if (a.loss) a.loss[j] = loss;
    a.respawn[j] = rs;
    if (a.i32c) {
#if defined(__HIP_DEVICE_COMPILE__)
      // one wave per block (TB == 64): per-block respawn count for k_respawn_seq
      (void)0;
#else
      a.i32c[j] = rs != 0 ? 1 : 0;
#endif
    }
  }

  // Sequential (Gauss-Seidel) generation step of particle j (reference Soup.evolve,
  // code/soup.py:51-87, semantics S11): the table W is updated IN PLACE in index order, so
  // particle j sees every earlier particle's changes of this generation.  Decisions as the
  // synchronous engine's (slot, generation) Philox stream; j attacks `at` (W[at] <- f_j(W[at]),
  // shuffle_random keyed by the attacker), learns from `te`'s CURRENT weights (severity
  // epochs), self-trains `epochs` epochs (SGD shuffles keyed by (slot, generation)), and is
  // re-initialised when divergent / zero (init key respawn_key(gen, j); the caller numbers
  // the newborns in index order).
  SRNN_HD static void soup_seq_one(const SrnnCfg& c, const SrnnArgs& a, int64_t j, int32_t gen, float4* samp,
                                   uint8_t* perm) {
    float w[P], f[P], o[P];
    int32_t at, te;
    decision(a, j, gen, at, te);
    int8_t act = A_NONE;
    int64_t cp = -1;
    if (at >= 0) {  // 1. attack: the victim's weights become f_j(victim)
      load(rowp(a.W, j), w);
      load(rowp(a.W, at), f);
      Net::apply(w, f, o, actx(a, c, (uint64_t)j, (uint32_t)gen * 1024u + 1u, perm));
      q(o);
      store(rowp(a.W, at), o);
      act = A_ATTACKING;
      cp = at;
    }
    load(rowp(a.W, j), w);  // (j may have attacked itself)
    TrainCtx tc;
    tc.lr = a.lr;
    tc.rng = rng(a);
    tc.uid = (uint64_t)j;
    tc.ctr = (uint32_t)gen * 1024u + 512u;
    tc.samp = samp;
    tc.perm = perm;
    tc.shuffle = (a.flags & 1) != 0;
    tc.stride = SAMP_STRIDE;
    tc.aggregator = c.aggregator;
    float loss = 0.f;
    if (te >= 0) {  // 2. learn_from the teacher's current weights
      load(rowp(a.W, te), f);
      if constexpr (Net::KIND == 0) {
        if (a.severity > 0) loss = Net::template train_epochs<false>(w, f, a.severity, tc);
      } else {
        for (int e = 0; e < a.severity; ++e) loss = Net::train_epoch(w, f, tc);
      }
      act = A_LEARN_FROM;
      cp = te;
    }
    if (a.epochs > 0) {  // 3. self-train
      if constexpr (Net::KIND == 0) {
        loss = Net::template train_epochs<true>(w, f, a.epochs, tc);
      } else {
        for (int e = 0; e < a.epochs; ++e) {
          copy(f, w);
          loss = Net::train_epoch(w, f, tc);
        }
      }
      act = A_TRAIN_SELF;
      cp = -1;
    }
    q(w);  // 4. respawn (the zero test on the old particle: at most one of the two)
    int8_t rs = 0;
    if ((a.flags & 2) && is_diverged<P>(w)) rs = 1;
    else if ((a.flags & 4) && is_zero<P>(w, a.eps)) rs = 2;
    if (a.W2) store(rowp(a.W2, j), w);  // recording: the particle's state before any respawn
    if (rs) Net::init(w, rng(a), respawn_key(gen, j));
    store(rowp(a.W, j), w);
    if (a.action) a.action[j] = act;
    // recording (W2 set): the counterpart's uid at the time of the action (a slot before j may
    // already hold a newborn this generation); otherwise its slot
    if (a.counterpart) a.counterpart[j] = (a.W2 && cp >= 0) ? a.uid_out[cp] : cp;
    if (a.loss) a.loss[j] = loss;
    if (a.respawn) a.respawn[j] = rs;
  }

  SRNN_HD static void respawn(const SrnnArgs& a, int64_t j) {
    if (a.respawn[j] == 0) return;
    float w[P];
    Net::init(w, rng(a), respawn_key(gen_of(a), a.lo + j));
    store(rowp(a.W, j), w);
  }

  // SGD permutations of local row j for generation `gen` (epoch counters gen*1024+512+k,
  // k < perm_e, keyed by the slot): exactly what train_epochs would draw, into
  // out[k * n + j] (k-major: the lanes of a wave write consecutive words)
  SRNN_HD static void perm_fill(const SrnnArgs& a, int64_t j, int32_t gen, uint64_t* out) {
    if constexpr (Net::KIND == 0 && P <= 16) {
      const uint64_t key = (uint64_t)(a.lo + j);
      const uint32_t c0 = (uint32_t)gen * 1024u + 512u;  // even: epochs (k, k+1) share a draw
      const Rng r = rng(a);
      for (int32_t k = 0; k < a.perm_e; k += 2) {
        const U4 d = perm_draw(r, key, c0 + (uint32_t)k, P_SHUFFLE);
        out[(int64_t)k * a.n + j] = perm_from_bits<P>(perm_bits(d, c0 + (uint32_t)k));
        if (k + 1 < a.perm_e) out[(int64_t)(k + 1) * a.n + j] = perm_from_bits<P>(perm_bits(d, c0 + (uint32_t)k + 1u));
      }
    }
  }
};

// ----------------------------------------------------------------------------------
// Helper waves of the fused generation (flag 131072).  At ~1.5 waves per SIMD the SIMDs
// carrying two generation waves are issue-saturated while the others run one wave at half
// issue rate.  The next generation's SGD permutations (the Philox + Fisher-Yates integer
// work, ~30 % of an epoch's instructions) are computed by extra workgroups that keep
// going only on SIMDs holding fewer than two generation waves, pulling 64-slot chunks from
// a work queue; generation waves drain whatever is left when they finish, so the queue
// always empties inside the launch.  Placement only affects speed, never the result.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ int simd_slot() {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
  const uint32_t simd = (hw >> 4) & 3u, cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
  return (int)((((((xcc & 7u) * 8u + se) * 2u + sh) * 16u + cu) * 4u) + simd);  // < 8192
}
constexpr int HELPER_CTL = 1 + 8192;  // queue head + per-SIMD generation-wave counts

template <class Net, class S>
__device__ void perm_drain(const SrnnArgs& a, int32_t gen_next) {
  using I = Item<Net, S>;
  const int64_t nch = (a.n + TB - 1) / TB;
  for (;;) {
    int32_t ch = 0;
    if (threadIdx.x == 0) ch = atomicAdd(a.helper_ctl, 1);
    ch = __shfl(ch, 0);
    if ((int64_t)ch >= nch) break;
    const int64_t j = (int64_t)ch * TB + threadIdx.x;
    if (j < a.n) I::perm_fill(a, j, gen_next, a.perm_next);
  }
}

// ==================================================================================
// Device kernels
// ==================================================================================
template <class Net, int OP, class S>
__global__ __launch_bounds__(TB) void k_op(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr bool NEED_SAMP = (OP == OP_TRAIN || OP == OP_LEARN || OP == OP_SOUP_EVOLVE) && Net::KIND == 0;
  constexpr int SAMP = NEED_SAMP ? P : 1;  // slot-major [P][TB]: lane fastest
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  float4* samp = s_samp + threadIdx.x;  // slot k of this lane at samp[k * TB]
  uint8_t* perm = s_perm + threadIdx.x * PERM;

  if constexpr (OP == OP_SOUP_DECIDE) {
    if (i < a.n_total) I::soup_decide(a, i);
    return;
  } else if constexpr (OP == OP_SOUP_UNPACK) {
    if (i == 0)  // packing of this generation is complete; data rows follow the stats rows
      for (int r = 0; r < a.world; ++r) a.sendcnt[r] = I::SR;
    if (i < (int64_t)a.world * a.cap) I::soup_unpack(a, i);
    return;
  } else if constexpr (OP == OP_SOUP_PACK) {
    if (i == 0) I::pack_stats(a);
    if (i < a.n) I::soup_pack(a, i);
    return;
  } else if constexpr (OP == OP_CLASSIFY) {
    if (i < a.n) I::classify(c, a, i, perm);  // histogram: k_classify_count
    return;
  } else {
    if (i >= a.n) return;
    if constexpr (OP == OP_INIT) I::init(c, a, i, samp, perm);
    else if constexpr (OP == OP_APPLY) I::apply(c, a, i, samp, perm);
    else if constexpr (OP == OP_RUN_FIXPOINT) I::run_fixpoint(c, a, i, samp, perm);
    else if constexpr (OP == OP_TRAIN) I::train(c, a, i, samp, perm, false);
    else if constexpr (OP == OP_LEARN) I::train(c, a, i, samp, perm, true);
    else if constexpr (OP == OP_PERTURB) I::perturb(c, a, i, samp, perm);
    else if constexpr (OP == OP_RESPAWN) I::respawn(a, i);
    else if constexpr (OP == OP_VARY_RUN) I::vary_run(c, a, i, samp, perm);
  }
}

// Fused soup generation body: one wave per block; after the per-particle work the wave
// publishes its 64-bit respawn ballot (i32c as u64[block]) for the single-rank respawn scan, or per-row
// flags (i32c[row]) when OP_SCAN follows (sharded path, a.i32d != null flags that mode).
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_soup_evolve(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr int SAMP = Net::KIND == 0 ? P : 1;
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  bool rs = false;
  if (i < a.n) {
    I::soup_evolve(c, a, i, s_samp + threadIdx.x, s_perm + threadIdx.x * PERM);
    rs = a.respawn[i] != 0;
  }
  if (a.i32c) {
    if (a.flags & 16) {
      if (i < a.n) a.i32c[i] = rs ? 1 : 0;
    } else {
      unsigned long long m = __ballot(rs);
      if (threadIdx.x == 0) reinterpret_cast<unsigned long long*>(a.i32c)[blockIdx.x] = m;
    }
  }
}

// ----------------------------------------------------------------------------------
// Post-exchange work of a sharded generation folded into its generation launch (flag
// 524288) instead of a separate launch between the all-to-all and the generation:
//   workgroup 0        -- uids of the previous generation's newborns (stats rows of the
//                         exchange: lower ranks' respawn counts; the previous generation's
//                         ballots in temp2) + the global census + send-counter reset;
//   workgroups 1..U    -- index the received rows (rmap[slot] = row, memory-side atomic
//                         stores), then bump xdone;
//   the rest           -- generation waves: the next generation's decisions first (they do
//                         not need the received rows), then wait for xdone == U (bounded
//                         spin, overflow flag 2 on timeout: never a hang), then evolve.
// The unpack workgroups have the lowest block ids, so they are dispatched before any
// generation wave can occupy the machine: the wait always ends.
// ----------------------------------------------------------------------------------
template <class Net, class S>
__device__ void post_uids(const SrnnArgs& a) {
  using I = Item<Net, S>;
  const int lane = threadIdx.x;
  if (lane < a.world) a.sendcnt[lane] = I::SR;  // the finish launch packs the next exchange
  int64_t pre = 0, tot = 0;
  if (lane == 0) {
    int64_t cen[5] = {0, 0, 0, 0, 0}, all = 0;
    for (int r = 0; r < a.world; ++r) {
      const int64_t k = I::stat(a, r, 5);
      if (r < a.rank) pre += k;
      tot += k;
      for (int q = 0; q < 5; ++q) cen[q] += I::stat(a, r, q);
    }
    for (int q = 0; q < 5; ++q) all += cen[q];
    if (a.census && all > 0)
      for (int q = 0; q < 5; ++q) a.census[q] = cen[q];
  }
  pre = __shfl(pre, 0);
  tot = __shfl(tot, 0);
  unsigned long long* masks = reinterpret_cast<unsigned long long*>(a.temp2);
  const int64_t nb = (a.n + TB - 1) / TB, ch = (nb + TB - 1) / TB;
  const int64_t b0 = (int64_t)lane * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t cnt = 0;
  for (int64_t b = b0; b < b1; ++b) cnt += __popcll(masks[b * 4]);
  int32_t incl = cnt;
#pragma unroll
  for (int off = 1; off < TB; off <<= 1) {
    const int32_t v = __shfl_up(incl, off);
    if (lane >= off) incl += v;
  }
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t u = base + pre + incl - cnt;
  for (int64_t b = b0; b < b1 && cnt; ++b) {
    unsigned long long m = masks[b * 4];
    masks[b * 4] = 0ull;
    while (m) {
      const int bit = __ffsll((long long)m) - 1;
      m &= m - 1;
      a.uid_out[b * TB + bit] = u++;
    }
  }
  if (lane == 0) ((int64_t*)a.uid_base)[0] = base + tot;
}
template <class Net, class S>
__device__ void post_unpack(const SrnnArgs& a, int64_t k) {
  using I = Item<Net, S>;
  if (k < (int64_t)a.world * a.cap && k % a.cap >= I::SR) {
    const int32_t* tag = reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(a.recvbuf) + k * I::XB + I::RB);
    if (tag[1] == I::gen_of(a)) __hip_atomic_store(a.rmap + tag[0], (int32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's index stores are at memory
  if (threadIdx.x == 0) __hip_atomic_fetch_add(a.xdone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void post_wait(const SrnnArgs& a, int32_t want) {
  int32_t ok = 1;
  if (threadIdx.x == 0) {
    uint32_t it = 0;
    while (__hip_atomic_load(a.xdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > (1u << 24)) {  // ~1 s: report instead of hanging the GPU
        ok = 0;
        break;
      }
    }
    if (!ok) atomic_or_i32(a.ovf, 2);
  }
}

// ----------------------------------------------------------------------------------
// Fused single-rank soup generation (OP_SOUP_GEN): ONE launch per generation instead of
// decide -> evolve -> respawn -> classify.  Per lane: the generation (attacks received,
// learn_from, self-train, respawn + inline re-init), then the NEXT generation's decision
// for its slot linked into the other list buffer (i32a = head, i32b = next; the decisions
// are a pure function of (seed, slot, generation)), then the census class of the stored
// row.  Each wave publishes its respawn ballot + class counts (temp: u64[4] per block)
// and bumps a done counter (i32d[0]) with an agent-scope atomic; the LAST wave to
// finish (no waiting anywhere: every wave exits) scans the ballots in slot order, assigns
// the globally sequential uids of the newborns, writes the census (counts[0..4]),
// advances next_uid and the generation counter and re-arms the done counter.
// flags: 1024 = census on (FIX_SEC bit 8 = with second-order fixpoints).
// ----------------------------------------------------------------------------------
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_soup_gen(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr int SAMP = Net::KIND == 0 ? P : 1;
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const bool post = (a.flags & 524288) != 0;
  int64_t xoff = 0;
  int32_t nunpack = 0;
  if (post) {
    nunpack = (int32_t)(((int64_t)a.world * a.cap + TB - 1) / TB);
    if (blockIdx.x == 0) {
      post_uids<Net, S>(a);
      return;
    }
    if ((int64_t)blockIdx.x <= nunpack) {
      post_unpack<Net, S>(a, (int64_t)(blockIdx.x - 1) * TB + threadIdx.x);
      return;
    }
    xoff = 1 + nunpack;
  }
  const int64_t gb = (int64_t)blockIdx.x - xoff;  // generation block: rows gb*64 ..
  const int64_t i = gb * TB + threadIdx.x;
  const int lane = threadIdx.x;
  uint8_t* perm = s_perm + lane * PERM;
  const int32_t gen = I::gen_of(a);
  const bool census = (a.flags & 1024) != 0;
  const bool pre = (a.flags & 131072) != 0;
  if (pre) {
    const int64_t nb_main = (a.n + TB - 1) / TB;
    if (gb >= nb_main) {
      // helper workgroup: work only where fewer than two generation waves share the SIMD
      int32_t cnt = 0;
      if (lane == 0) cnt = __hip_atomic_load(a.helper_ctl + 1 + simd_slot(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      cnt = __shfl(cnt, 0);
      if (cnt < 2) perm_drain<Net, S>(a, gen + 1);
      return;
    }
    if (lane == 0) atomicAdd(a.helper_ctl + 1 + simd_slot(), 1);
  }
  bool rs = false;
  int8_t k = -1;
  if (i < a.n && (a.flags & 4096)) {
    // sharded: the next generation's decisions of EVERY global slot (this lane takes
    // slots i, i + n, ...): attack lists of local victims + need masks for the pack.
    // First: they need nothing from the exchange, so they overlap the unpack workgroups
    for (int64_t g = i; g < a.n_total; g += a.n) {
      int32_t at, te;
      I::decision(a, g, gen + 1, at, te);
      I::link_decision(a, g, at, te, a.i32a, a.i32b);
    }
  }
  if (post) post_wait(a, nunpack);
  if (i < a.n) {
    I::soup_evolve(c, a, i, s_samp + lane, perm);
    rs = a.respawn[i] != 0;
    if (!(a.flags & 4096)) {
      int32_t at, te;
      I::decision(a, i, gen + 1, at, te);
      if (at >= 0) a.i32b[i] = atomicExch(a.i32a + at, (int32_t)i);
    }
    if (census) {
      float w[P];
      I::load(I::rowp(a.W, i), w);
      k = I::classify_w(w, a.eps, (a.flags & 8) != 0, I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
    }
  }
  if ((a.flags & 65536) && gb == 0 && threadIdx.x == 0) {
    // asynchronous finish: this launch advances the generation counter (the other ring
    // slot: no block of this launch reads it) so the next generation needs nothing from
    // the finish kernel, which runs beside it on a side stream
    I::set_gen(a, gen + 1);
  }
  const unsigned long long m = __ballot(rs);
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(k == q));
  // Hand-off to the last wave without an agent-scope release per wave (a release writes
  // back the XCD's whole L2: ~+30 us over 1563 waves).  The block stats are 8-byte
  // agent-scope atomic stores (memory-side, coherent across XCDs), drained with
  // s_waitcnt vmcnt(0) before the relaxed ticket add; the last wave acquires once and
  // reads them with agent-scope atomic loads (MI355X_MICROARCH "Valid forms").
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  if (a.flags & 2048) {  // two-phase: plain stores, k_gen_finish reads them after the kernel boundary
    if (lane == 0) {
      unsigned long long* mine = bs + gb * 4;
      mine[0] = m;
      mine[1] = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
      mine[2] = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
      mine[3] = (unsigned long long)cnt[4];
      // flag 1048576: the generation's newborn count after the block stats (batched finish)
      if ((a.flags & 1048576) && m) atomicAdd(bs + ((a.n + TB - 1) / TB) * 4, (unsigned long long)__popcll(m));
    }
    if (pre) perm_drain<Net, S>(a, gen + 1);  // whatever the helpers left
    return;
  }
  int32_t prev = 0;
  if (lane == 0) {
    unsigned long long* mine = bs + gb * 4;
    __hip_atomic_store(mine + 0, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 2, (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 3, (unsigned long long)cnt[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    prev = __hip_atomic_fetch_add(a.i32d, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  prev = __shfl(prev, 0);
  const int32_t nb = (int32_t)(gridDim.x - xoff);
  if (prev != nb - 1) return;
  // ---- last wave: census + sequential uids of the newborns (blocks in slot order)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int32_t ch = (nb + TB - 1) / TB;
  const int32_t b0 = lane * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t born = 0;
  uint64_t cs[5] = {0, 0, 0, 0, 0};
  for (int32_t b = b0; b < b1; ++b) {
    const unsigned long long* st = bs + (int64_t)b * 4;
    born += __popcll(__hip_atomic_load(st + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const unsigned long long c01 = __hip_atomic_load(st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long c23 = __hip_atomic_load(st + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long c4 = __hip_atomic_load(st + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cs[0] += (uint32_t)c01;
    cs[1] += (uint32_t)(c01 >> 32);
    cs[2] += (uint32_t)c23;
    cs[3] += (uint32_t)(c23 >> 32);
    cs[4] += (uint32_t)c4;
  }
  // wave inclusive scan of `born` (64 lanes)
  int32_t incl = born;
#pragma unroll
  for (int off = 1; off < TB; off <<= 1) {
    int32_t v = __shfl_up(incl, off);
    if (lane >= off) incl += v;
  }
  const int32_t total = __shfl(incl, TB - 1);
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int off = TB / 2; off > 0; off >>= 1) cs[q] += __shfl_xor(cs[q], off);
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t u = base + incl - born;
  for (int32_t b = b0; b < b1 && born; ++b) {
    unsigned long long mm = __hip_atomic_load(bs + (int64_t)b * 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (mm) {
      const int bit = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      a.uid_out[(int64_t)b * TB + bit] = u++;
    }
  }
  if (lane == 0) {
    ((int64_t*)a.uid_base)[0] = base + total;
    I::set_gen(a, gen + 1);
    if (a.counts) {
#pragma unroll
      for (int q = 0; q < 5; ++q) a.counts[q] = census ? cs[q] : 0ull;
      a.counts[5] = (uint64_t)total;
    }
    __hip_atomic_store(a.i32d, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
  }
}

// Inclusive scan over an NT-thread block: wave shuffles (no barrier) + one LDS pass over
// the NT/64 wave totals (one barrier) instead of a log2(NT)-round Hillis-Steele scan with
// two barriers per round.  *total receives the block sum.
template <int NT>
__device__ __forceinline__ int32_t block_incl_scan(int32_t v, int32_t* s_wave, int32_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wave[wv] = x;
  __syncthreads();
  int32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int32_t sw = s_wave[w];
    pre += (w < wv) ? sw : 0;
    tot += sw;
  }
  *total = tot;
  return x + pre;
}

// Second phase of the two-phase fused generation: one SRNN_FINISH_NT-thread workgroup reduces the
// per-wave census counts, scans the respawn ballots in slot order, assigns the newborns'
// uids and advances next_uid / the generation counter.  Sharded (flag 4096): only the
// counts (census + respawns, sent with the next exchange); uids wait for k_uid_assign.
#ifndef SRNN_FINISH_NT
#define SRNN_FINISH_NT 1024  // threads of the finish workgroup and its pack blocks (256: 7.27 us vs 6.68 us)
#endif
template <class Net, class S, int NT>
__global__ __launch_bounds__(NT) void k_gen_finish(SrnnArgs a, int32_t nb) {
  using I = Item<Net, S>;
  if (blockIdx.x > 0) {
    // flag 32768, blocks >= 1: pack the next generation's all-to-all (rows other ranks
    // need; generation-start rows of gen + 1 = this generation's output).  Block 0 only
    // writes the OTHER ring slot of the counter, so the gen read here is stable.
    SrnnArgs pa = a;
    pa.W2 = a.W;
    pa.gen_ptr = nullptr;
    pa.gen = I::gen_of(a) + 1;
    const int64_t j = (int64_t)(blockIdx.x - 1) * NT + threadIdx.x;
    if (j < a.n) I::soup_pack(pa, j);
    return;
  }
  __shared__ int32_t s_wave[NT / 64];
  __shared__ unsigned long long s_cs[5];
  const int t = threadIdx.x;
  if (t < 5) s_cs[t] = 0;
  if (t == 0 && a.xdone) *a.xdone = 0;  // re-armed for the next generation's unpack workgroups
  if ((a.flags & 131072) && a.helper_ctl)  // re-arm this parity's helper queue / SIMD counts
    for (int q = t; q < HELPER_CTL; q += NT) a.helper_ctl[q] = 0;
  const unsigned long long* bs = reinterpret_cast<const unsigned long long*>(a.temp);
  // the uid base and the generation counter are only written by thread 0 after the last
  // barrier: load them up front so their latency overlaps the per-block stats loads
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  const bool async = (a.flags & 65536) != 0;  // the generation kernel advanced the counter
  const int32_t gen = async ? 0 : I::gen_of(a);
  const int32_t ch = (nb + NT - 1) / NT;
  const int32_t b0 = t * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t born = 0;
  unsigned long long cs[5] = {0, 0, 0, 0, 0};
  for (int32_t b = b0; b < b1; ++b) {
    const unsigned long long* st = bs + (int64_t)b * 4;
    born += __popcll(st[0]);
    cs[0] += (uint32_t)st[1];
    cs[1] += (uint32_t)(st[1] >> 32);
    cs[2] += (uint32_t)st[2];
    cs[3] += (uint32_t)(st[2] >> 32);
    cs[4] += (uint32_t)st[3];
  }
  int32_t total_born;
  const int32_t incl = block_incl_scan<NT>(born, s_wave, &total_born);  // barrier inside
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    unsigned long long v = cs[q];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((t & 63) == 0 && v) atomicAdd(&s_cs[q], v);
  }
  const bool sharded = (a.flags & 4096) != 0;  // uids come after the exchange (k_uid_assign)
  int64_t u = base + incl - born;
  for (int32_t b = b0; b < b1 && born && !sharded; ++b) {
    unsigned long long mm = bs[(int64_t)b * 4];
    while (mm) {
      const int bit = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      a.uid_out[(int64_t)b * TB + bit] = u++;
    }
  }
  __syncthreads();
  if (t == 0) {
    const int32_t total = total_born;
    if (!sharded) ((int64_t*)a.uid_base)[0] = base + total;
    if (!async) I::set_gen(a, gen + 1);
    if (a.counts) {
      for (int q = 0; q < 5; ++q) a.counts[q] = (a.flags & 1024) ? s_cs[q] : 0ull;
      a.counts[5] = (uint64_t)total;
    }
    if (a.flags & 32768) I::pack_stats(a);  // this generation's stats ride on the next exchange
  }
}

// Batched finish of m single-rank fused generations (OP_GEN_FINISH with steps = m > 1):
// generation k left its block stats (respawn ballot + class counts per 64-row block) in
// temp + k * temp_bytes; one workgroup walks the generations in order -- census of each
// (counts[] keeps the last; a.census, when given, receives [m][6] history rows), newborn
// uids in slot order from the running next_uid -- then stores next_uid once.  One launch
// per graph chunk of generations instead of one per generation on the critical path.
template <class Net, class S, int NT>
__global__ __launch_bounds__(NT) void k_gen_finish_batch(SrnnArgs a, int32_t nb, int32_t m) {
  __shared__ int32_t s_wave[NT / 64];
  __shared__ unsigned long long s_cs[5];
  __shared__ int64_t s_base;
  const int t = threadIdx.x;
  if (t == 0) s_base = *(volatile const int64_t*)a.uid_base;
  const int32_t ch = (nb + NT - 1) / NT;
  const int32_t b0 = t * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  for (int32_t g = 0; g < m; ++g) {
    if (t < 5) s_cs[t] = 0;
    const unsigned long long* bs =
        reinterpret_cast<const unsigned long long*>(reinterpret_cast<const char*>(a.temp) + (int64_t)g * a.temp_bytes);
    int32_t born = 0;
    unsigned long long cs[5] = {0, 0, 0, 0, 0};
    for (int32_t b = b0; b < b1; ++b) {
      const unsigned long long* st = bs + (int64_t)b * 4;
      born += __popcll(st[0]);
      cs[0] += (uint32_t)st[1];
      cs[1] += (uint32_t)(st[1] >> 32);
      cs[2] += (uint32_t)st[2];
      cs[3] += (uint32_t)(st[2] >> 32);
      cs[4] += (uint32_t)st[3];
    }
    int32_t total_born;
    const int32_t incl = block_incl_scan<NT>(born, s_wave, &total_born);  // barrier inside (s_base, s_cs visible)
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      unsigned long long v = cs[q];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if ((t & 63) == 0 && v) atomicAdd(&s_cs[q], v);
    }
    const int64_t base = s_base;
    int64_t u = base + incl - born;
    for (int32_t b = b0; b < b1 && born; ++b) {
      unsigned long long mm = bs[(int64_t)b * 4];
      while (mm) {
        const int bit = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        a.uid_out[(int64_t)b * TB + bit] = u++;
      }
    }
    __syncthreads();
    if (t == 0) {
      s_base = base + total_born;
      const bool census = (a.flags & 1024) != 0;
      if (a.counts && g == m - 1) {
        for (int q = 0; q < 5; ++q) a.counts[q] = census ? s_cs[q] : 0ull;
        a.counts[5] = (uint64_t)total_born;
      }
      if (a.census) {
        for (int q = 0; q < 5; ++q) a.census[(int64_t)g * 6 + q] = census ? (int64_t)s_cs[q] : 0;
        a.census[(int64_t)g * 6 + 5] = total_born;
      }
    }
    // the next generation's scan reuses s_wave / s_cs: every thread past this iteration's reads
    __syncthreads();
  }
  if (t == 0) ((int64_t*)a.uid_base)[0] = s_base;
}

// Parallel form of k_gen_finish_batch (a.i32d given: a zeroed done counter): ONE workgroup
// per generation of the batch.  Workgroup g counts the newborns of generations < g (its uid
// base), reduces its own generation's census and numbers its newborns in slot order exactly
// as the sequential walk does, but writes a uid only where no later generation of the batch
// re-spawned the same slot (the later uid wins, as in the walk).  The last workgroup to finish
// (done counter) stores next_uid and re-arms the counter.  Same results as the one-workgroup
// walk; the m generations run side by side instead of one after another (27.8 us for a
// 16-generation batch, profiles/r2i_restore_check.md).
template <class Net, class S, int NT>
__global__ __launch_bounds__(NT) void k_gen_finish_par(SrnnArgs a, int32_t nb, int32_t m) {
  __shared__ int32_t s_wave[NT / 64], s_wave2[NT / 64], s_wave3[NT / 64];
  __shared__ unsigned long long s_cs[5];
  const int t = threadIdx.x;
  const int32_t g = (int32_t)blockIdx.x;
  if (t < 5) s_cs[t] = 0;
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  const int32_t ch = (nb + NT - 1) / NT;
  const int32_t b0 = t * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  auto ring = [&](int32_t k) {
    return reinterpret_cast<const unsigned long long*>(reinterpret_cast<const char*>(a.temp) + (int64_t)k * a.temp_bytes);
  };
  const bool totals = (a.flags & 1048576) != 0 && m <= NT;  // newborn count of generation k at ring(k)[4 nb]
  int32_t before = 0, all = 0;
  if (totals) {
    // thread k < m loads generation k's count: m loads in flight at once (a loop over k in
    // one thread paid one memory latency per generation, ~0.9 us each)
    if (t < m) {
      const int32_t c = (int32_t)ring(t)[(int64_t)nb * 4];
      all = c;
      before = t < g ? c : 0;
    }
  } else {
#pragma unroll 8  // independent loads in flight (the walk over generations is latency bound)
    for (int32_t k = 0; k < m; ++k) {
      const unsigned long long* bk = ring(k);
      int32_t c = 0;
      for (int32_t b = b0; b < b1; ++b) c += __popcll(bk[(int64_t)b * 4]);
      all += c;
      before += k < g ? c : 0;
    }
  }
  const unsigned long long* bs = ring(g);
  int32_t born = 0;
  unsigned long long cs[5] = {0, 0, 0, 0, 0};
  for (int32_t b = b0; b < b1; ++b) {
    const unsigned long long* st = bs + (int64_t)b * 4;
    born += __popcll(st[0]);
    cs[0] += (uint32_t)st[1];
    cs[1] += (uint32_t)(st[1] >> 32);
    cs[2] += (uint32_t)st[2];
    cs[3] += (uint32_t)(st[2] >> 32);
    cs[4] += (uint32_t)st[3];
  }
  int32_t total_born, total_before, total_all;
  const int32_t incl = block_incl_scan<NT>(born, s_wave, &total_born);
  (void)block_incl_scan<NT>(before, s_wave2, &total_before);
  (void)block_incl_scan<NT>(all, s_wave3, &total_all);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    unsigned long long v = cs[q];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((t & 63) == 0 && v) atomicAdd(&s_cs[q], v);
  }
  int64_t u = base + total_before + incl - born;
  for (int32_t b = b0; b < b1 && born; ++b) {
    unsigned long long later = 0;  // slots of this block re-spawned by a later generation
#pragma unroll 8
    for (int32_t k = g + 1; k < m; ++k) later |= ring(k)[(int64_t)b * 4];
    unsigned long long mm = bs[(int64_t)b * 4];
    while (mm) {
      const int bit = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      if (!((later >> bit) & 1ull)) a.uid_out[(int64_t)b * TB + bit] = u;
      ++u;
    }
  }
  __syncthreads();
  if (t == 0) {
    const bool census = (a.flags & 1024) != 0;
    if (a.counts && g == m - 1) {
      for (int q = 0; q < 5; ++q) a.counts[q] = census ? s_cs[q] : 0ull;
      a.counts[5] = (uint64_t)total_born;
    }
    if (a.census) {
      for (int q = 0; q < 5; ++q) a.census[(int64_t)g * 6 + q] = census ? (int64_t)s_cs[q] : 0;
      a.census[(int64_t)g * 6 + 5] = total_born;
    }
    // every workgroup read next_uid before its ticket: the last one may overwrite it
    __threadfence();
    const int32_t prev = atomicAdd(a.i32d, 1);
    if (prev == m - 1) {
      ((int64_t*)a.uid_base)[0] = base + total_all;
      if (totals)  // every workgroup has read the counts: re-armed for the next batch
        for (int32_t k = 0; k < m; ++k) const_cast<unsigned long long*>(ring(k))[(int64_t)nb * 4] = 0ull;
      __hip_atomic_store(a.i32d, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// SGD permutations of generation *gen_ptr for every local row into perm_next (OP_SOUP_PERMS:
// the first precomputed generation; later ones come from the helper waves)
template <class Net, class S>
__global__ __launch_bounds__(256) void k_soup_perms(SrnnArgs a) {
  using I = Item<Net, S>;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n) I::perm_fill(a, j, I::gen_of(a), a.perm_next);
}
template <class Net, class S>
int soup_perms(const SrnnCfg&, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (!(Net::KIND == 0 && Net::P <= 16)) return 0;  // no per-epoch permutations to precompute
  if (!a.perm_next || a.perm_e < 1) {
    set_error("soup_perms needs perm_next and perm_e >= 1");
    return -5;
  }
  if (!a.dev) {
    for (int64_t j = 0; j < a.n; ++j) I::perm_fill(a, j, I::gen_of(a), a.perm_next);
    return 0;
  }
  if (a.n <= 0) return 0;
  hipLaunchKernelGGL((k_soup_perms<Net, S>), dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, (hipStream_t)a.stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// Asynchronous finish of a single-rank fused generation (OP_GEN_FINISH, flag 65536): the
// census reduction + uids of the generation whose block stats are in a.temp, launched on a
// side stream after that generation and beside the next one (host: no-op, soup_gen did it).
template <class Net, class S>
int gen_finish(const SrnnCfg&, const SrnnArgs& a) {
  if (!a.dev) return 0;
  const int64_t blocks = (a.n + TB - 1) / TB;
  if (blocks <= 0) return 0;
  constexpr int FNT = SRNN_FINISH_NT;
  if (a.steps > 1 || (a.flags & 262144)) {  // batch of a.steps generations (ring in temp)
    if (a.steps < 1 || a.temp_bytes < blocks * 32) {
      set_error("batched finish needs steps >= 1 generations and temp_bytes >= 32 per block");
      return -5;
    }
    if (a.i32d)  // a zeroed done counter: one workgroup per generation
      hipLaunchKernelGGL((k_gen_finish_par<Net, S, FNT>), dim3((unsigned)a.steps), dim3(FNT), 0,
                         (hipStream_t)a.stream, a, (int32_t)blocks, a.steps);
    else
      hipLaunchKernelGGL((k_gen_finish_batch<Net, S, FNT>), dim3(1), dim3(FNT), 0, (hipStream_t)a.stream, a,
                         (int32_t)blocks, a.steps);
  } else {
    hipLaunchKernelGGL((k_gen_finish<Net, S, FNT>), dim3(1), dim3(FNT), 0, (hipStream_t)a.stream, a, (int32_t)blocks);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

template <class Net, class S>
int uid_assign(const SrnnCfg& c, const SrnnArgs& a);

// OP_SOUP_SEQ: `steps` sequential soup generations starting at generation *gen_ptr (or
// a.gen) on a host table, one particle after another (the reference order is serial by
// definition: a single CPU core runs it ~100x faster than per-particle device launches and
// faster than one GPU lane).  Newborns get uids from *uid_base in index order; uid_out
// receives them; the generation counter advances by `steps`.
// The same serial loop as ONE device lane (measured against the host loop: the dependent
// chain is slower on a GPU lane than on a CPU core, profiles/r2o_native_sequential_soups.md)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_soup_seq(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int SAMP = Net::KIND == 0 ? Net::P : 1;
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];  // lane 0's slots at s_samp[k * TB] (SAMP_STRIDE)
  __shared__ uint8_t s_perm[PERM];
  if (threadIdx.x != 0) return;
  const int32_t gen0 = I::gen_of(a);
  int64_t next = a.uid_base[0];
  for (int32_t s = 0; s < a.steps; ++s) {
    for (int64_t j = 0; j < a.n; ++j) {
      I::soup_seq_one(c, a, j, gen0 + s, s_samp, s_perm);
      if (a.respawn && a.respawn[j]) a.uid_out[j] = next++;
    }
  }
  ((int64_t*)a.uid_base)[0] = next;
  I::set_gen(a, gen0 + a.steps);
}

template <class Net, class S>
int soup_seq(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (a.world > 1 || a.lo != 0 || (a.n_total && a.n_total != a.n) || !a.uid_base || !a.uid_out) {
    set_error("sequential soup: one unsharded table, uid_base and uid_out needed");
    return -5;
  }
  if (a.dev) {
    hipLaunchKernelGGL((k_soup_seq<Net, S>), dim3(1), dim3(1), 0, (hipStream_t)a.stream, c, a);
    return 0;
  }
  float4 samp[Net::P + 1];
  uint8_t perm[Net::P + 4];
  const int32_t gen0 = I::gen_of(a);
  int64_t next = a.uid_base[0];
  for (int32_t s = 0; s < a.steps; ++s) {
    for (int64_t j = 0; j < a.n; ++j) {
      I::soup_seq_one(c, a, j, gen0 + s, samp, perm);
      if (a.respawn && a.respawn[j]) a.uid_out[j] = next++;
    }
  }
  ((int64_t*)a.uid_base)[0] = next;
  I::set_gen(a, gen0 + a.steps);
  return 0;
}

template <class Net, class S>
int soup_gen(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (!a.dev) {
    // host: the same steps in order (evolve all rows, link next decisions, census, uids)
    if (a.flags & 524288) {
      // post-exchange work first: previous generation's uids (ballots in temp2), received-row
      // index, send-counter reset -- the device's workgroup 0 and unpack workgroups
      SrnnArgs ua = a;
      ua.flags = (a.flags & ~524288) | 16384 | 8192;
      ua.temp = a.temp2;
      ua.counts = nullptr;
      uid_assign<Net, S>(c, ua);
    }
    const int32_t gen = I::gen_of(a);
    host_parallel(a.n, [&](int64_t i) {
      float4 samp[Net::P + 1];
      uint8_t perm[Net::P + 4];
      I::soup_evolve(c, a, i, samp, perm);
    });
    if (a.flags & 4096) {
      for (int64_t g = 0; g < a.n_total; ++g) {
        int32_t at, te;
        I::decision(a, g, gen + 1, at, te);
        I::link_decision(a, g, at, te, a.i32a, a.i32b);
      }
    } else {
      for (int64_t i = 0; i < a.n; ++i) {
        int32_t at, te;
        I::decision(a, i, gen + 1, at, te);
        if (at >= 0) {
          a.i32b[i] = a.i32a[at];
          a.i32a[at] = (int32_t)i;
        }
      }
    }
    uint64_t cs[5] = {0, 0, 0, 0, 0};
    if (a.flags & 1024) {
      std::vector<int8_t> ks((size_t)a.n);
      host_parallel(a.n, [&](int64_t i) {
        float w[Net::P];
        uint8_t perm[Net::P + 4];
        I::load(I::rowp(a.W, i), w);
        ks[(size_t)i] = I::classify_w(w, a.eps, (a.flags & 8) != 0, I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
      });
      for (int64_t i = 0; i < a.n; ++i) cs[ks[(size_t)i]]++;
    }
    int64_t u = a.uid_base[0], total = 0;
    if (a.flags & 4096) {
      // sharded: respawn ballots per 64-row block for k_uid_assign after the next exchange
      unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
      for (int64_t b = 0; b < (a.n + TB - 1) / TB; ++b) bs[b * 4] = 0ull;
      for (int64_t i = 0; i < a.n; ++i)
        if (a.respawn[i]) {
          bs[(i / TB) * 4] |= 1ull << (i % TB);
          ++total;
        }
    } else {
      for (int64_t i = 0; i < a.n; ++i)
        if (a.respawn[i]) {
          a.uid_out[i] = u++;
          ++total;
        }
      ((int64_t*)a.uid_base)[0] = u;
    }
    I::set_gen(a, gen + 1);
    if (a.counts) {
      for (int q = 0; q < 5; ++q) a.counts[q] = cs[q];
      a.counts[5] = (uint64_t)total;
    }
    if (a.flags & 32768) {
      I::pack_stats(a);
      SrnnArgs pa = a;
      pa.W2 = a.W;
      pa.gen_ptr = nullptr;
      pa.gen = gen + 1;
      for (int64_t j = 0; j < a.n; ++j) I::soup_pack(pa, j);
    }
    return 0;
  }
  const int64_t blocks = (a.n + TB - 1) / TB;
  if (blocks <= 0) return 0;
  if (blocks > 0x7fffffffLL) {
    set_error("grid too large");
    return -2;
  }
  const int64_t helpers = (a.flags & 131072) ? (a.helpers > 0 ? a.helpers : 0) : 0;
  int64_t xblocks = 0;
  if (a.flags & 524288) {
    if (!(a.flags & 4096) || !(a.flags & 2048) || !a.temp2 || !a.xdone || !a.rmap || !a.recvbuf || a.world > 64) {
      set_error("post-exchange generation needs a sharded two-phase generation, temp2, xdone, rmap, recvbuf");
      return -5;
    }
    xblocks = 1 + ((int64_t)a.world * a.cap + TB - 1) / TB;
  }
  if ((a.flags & 131072) && (!a.perm_cur || !a.perm_next || !a.helper_ctl || !(a.flags & 2048) || a.perm_e < 1)) {
    set_error("precomputed permutations need perm_cur / perm_next / helper_ctl, perm_e >= 1 and a two-phase generation");
    return -5;
  }
  hipLaunchKernelGGL((k_soup_gen<Net, S>), dim3((unsigned)(xblocks + blocks + helpers)), dim3(TB), 0,
                     (hipStream_t)a.stream, c, a);
  if ((a.flags & 2048) && !(a.flags & 65536)) {
    constexpr int FNT = SRNN_FINISH_NT;
    const int64_t pack_blocks = (a.flags & 32768) ? (a.n + FNT - 1) / FNT : 0;
    hipLaunchKernelGGL((k_gen_finish<Net, S, FNT>), dim3((unsigned)(1 + pack_blocks)), dim3(FNT), 0,
                       (hipStream_t)a.stream, a, (int32_t)blocks);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// Classification + 5-bin histogram: 256-thread blocks, per-wave ballots reduced in LDS,
// at most one atomic per (block, non-empty class) -- per-wave atomics on 5 addresses
// serialised at L2 (39 us for 100k particles in the first profile).
constexpr int TBC = 256;
template <class Net, class S>
__global__ __launch_bounds__(TBC) void k_classify_count(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ uint8_t s_perm[TBC * PERM];
  __shared__ uint32_t s_cnt[5];
  if (threadIdx.x < 5) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * TBC + threadIdx.x;
  int8_t k = -1;
  if (i < a.n) k = I::classify(c, a, i, s_perm + threadIdx.x * PERM);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    unsigned long long m = __ballot(k == q);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_cnt[q], (uint32_t)__popcll(m));
  }
  __syncthreads();
  if (threadIdx.x < 5 && s_cnt[threadIdx.x]) atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
  if (a.flags & 64) {  // respawns of this generation (sharded soup: uid prefix)
    unsigned long long m = __ballot(i < a.n && a.respawn[i] != 0);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(a.counts + 5, (uint64_t)__popcll(m));
  }
  // sharded soup: the census closes the generation (no later kernel of this generation
  // reads the counter)
  if ((a.flags & 512) && blockIdx.x == 0 && threadIdx.x == 0) I::set_gen(a, I::gen_of(a) + 1);
}

// ----------------------------------------------------------------------------------
// Weightwise self-application runs (OP_RUN_FIXPOINT) for SMALL populations: 16 lanes per
// particle.  Lane k owns point / weight k, every lane of the group holds the whole vector
// (the applying net), computes its own point, and the new vector is gathered with
// in-group shuffles; the predicates are group ballots.  A lane-per-particle launch of
// n <= ~65k particles leaves SIMDs idle and each wave latency-bound; this spreads the
// same work over 16x the lanes.  Same arithmetic per point as Item::run_fixpoint.
// ----------------------------------------------------------------------------------
// w[q] = v of lane q of this lane's 16-lane row, q < P (DPP row_newbcast, VALU only)
template <int Q>
__device__ __forceinline__ float row_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + Q, 0xF, 0xF, true));
}
template <int P, int Q = 0>
__device__ __forceinline__ void row_bcast_all(float v, float* w) {
  if constexpr (Q < P) {
    w[Q] = row_bcast<Q>(v);
    row_bcast_all<P, Q + 1>(v, w);
  }
}
constexpr int TBG = 256;
constexpr int64_t FIX_GROUP_MAX_N = 32768;  // measured crossover vs lane-per-particle (profiles/r1h)
template <class Net, class S>
__global__ __launch_bounds__(TBG) void k_fix_group(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  static_assert(P <= 16, "one 16-lane group per particle");
  const int lane = threadIdx.x & 63;
  const int k = lane & 15;
  const int gbase = lane & ~15;
  const int64_t i = ((int64_t)blockIdx.x * TBG + threadIdx.x) >> 4;
  if (i >= a.n) return;  // whole groups leave together
  const unsigned long long vmask = (((1ull << P) - 1ull) << gbase);
  float c0 = 0.f, c1 = 0.f, c2 = 0.f;
#pragma unroll
  for (int q = 0; q < P; ++q)
    if (k == q) {
      c0 = Net::coords.c[q][0];
      c1 = Net::coords.c[q][1];
      c2 = Net::coords.c[q][2];
    }
  float w[P];
  I::load(I::rowp(a.W, i), w);
  float wk = 0.f;
#pragma unroll
  for (int q = 0; q < P; ++q) wk = (k == q) ? w[q] : wk;
  if (a.traj && k == 0) I::store(I::rowp(a.traj, i), w);
  auto all_of = [&](bool pred) { return (__ballot(pred || k >= P) & vmask) == vmask; };
  int s = 0;
  for (; s < a.steps; ++s) {
    float x[4] = {wk, c0, c1, c2}, y[1];
    Net::Net::forward_only(w, x, y);
    const float nk = S::q(y[0]);
    if (a.early_exit) {
      if (!all_of(finitef(wk))) break;  // is_diverged(w)
      if (all_of(finitef(nk) && !(fabsf(nk - wk) >= a.eps))) break;  // is_fixpoint()
    }
    row_bcast_all<P>(nk, w);
    wk = nk;
    if (a.traj && k == 0) I::store(I::rowp(a.traj, (int64_t)(s + 1) * a.n + i), w);
  }
  if (k == 0) {
    I::store(I::rowp(a.W, i), w);
    if (a.nsteps) a.nsteps[i] = s;
  }
  if (a.cls) {  // classify_w with the group: f1 = f_w(w), f2 = f_w(f1) -- own points only
    int8_t cl;
    if (!all_of(finitef(wk))) {
      cl = C_DIVERGENT;
    } else {
      float x[4] = {wk, c0, c1, c2}, y[1];
      Net::Net::forward_only(w, x, y);
      const float f1 = S::q(y[0]);
      if (all_of(finitef(f1) && !(fabsf(f1 - wk) >= a.eps))) {
        cl = all_of((-a.eps <= wk) && (wk <= a.eps)) ? C_FIX_ZERO : C_FIX_OTHER;
      } else {
        cl = C_OTHER;
        if (a.flags & 8) {
          float x2[4] = {f1, c0, c1, c2};
          Net::Net::forward_only(w, x2, y);
          const float f2 = S::q(y[0]);
          if (all_of(finitef(f2) && !(fabsf(f2 - wk) >= a.eps))) cl = C_FIX_SEC;
        }
      }
    }
    if (k == 0) a.cls[i] = cl;
  }
}

template <class Net, int OP, class S>
int launch(const SrnnCfg& c, const SrnnArgs& a) {
  int64_t items = (OP == OP_SOUP_DECIDE) ? a.n_total : (OP == OP_SOUP_UNPACK) ? (int64_t)a.world * a.cap : a.n;
  if (OP == OP_SOUP_PACK && items < 1) items = 1;  // the stats rows are always written
  if (items <= 0) return 0;
  int64_t blocks = (items + TB - 1) / TB;
  if (blocks > 0x7fffffffLL) {
    set_error("grid too large");
    return -2;
  }
  hipStream_t st = (hipStream_t)a.stream;
  if constexpr (OP == OP_RUN_FIXPOINT && Net::KIND == 0 && Net::P <= 16) {
    // small populations: 16 lanes per particle (SRNN_FIX_GROUP=0/1 forces either form)
    const char* env = std::getenv("SRNN_FIX_GROUP");
    const bool group = env ? env[0] == '1' : a.n <= FIX_GROUP_MAX_N;
    if (group) {
      hipLaunchKernelGGL((k_fix_group<Net, S>), dim3((unsigned)((a.n * 16 + TBG - 1) / TBG)), dim3(TBG), 0, st, c,
                         a);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        set_error(hipGetErrorString(e));
        return -3;
      }
      return 0;
    }
  }
  if (OP == OP_SOUP_EVOLVE) {
    hipLaunchKernelGGL((k_soup_evolve<Net, S>), dim3((unsigned)blocks), dim3(TB), 0, st, c, a);
  } else if (OP == OP_CLASSIFY && a.counts) {
    hipLaunchKernelGGL((k_classify_count<Net, S>), dim3((unsigned)((items + TBC - 1) / TBC)), dim3(TBC), 0, st, c, a);
  } else {
    hipLaunchKernelGGL((k_op<Net, OP, S>), dim3((unsigned)blocks), dim3(TB), 0, st, c, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// ==================================================================================
// Host execution of the same per-item code (CPU tensors)
// ==================================================================================
template <class Net, int OP, class S>
int host_run(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  int64_t items = (OP == OP_SOUP_DECIDE) ? a.n_total : (OP == OP_SOUP_UNPACK) ? (int64_t)a.world * a.cap : a.n;
  if (OP == OP_SOUP_UNPACK)
    for (int r = 0; r < a.world; ++r) a.sendcnt[r] = I::SR;
  if (OP == OP_CLASSIFY && a.counts) {
    uint64_t local[5] = {0, 0, 0, 0, 0};
    std::vector<int8_t> ks((size_t)items);
    host_parallel(items, [&](int64_t i) {
      uint8_t perm[P + 4];
      ks[(size_t)i] = I::classify(c, a, i, perm);
    });
    for (int64_t i = 0; i < items; ++i) local[ks[(size_t)i]]++;
    for (int q = 0; q < 5; ++q) a.counts[q] += local[q];
    if (a.flags & 64)
      for (int64_t i = 0; i < items; ++i) a.counts[5] += a.respawn[i] != 0;
    if (a.flags & 512) I::set_gen(a, I::gen_of(a) + 1);
    return 0;
  }
  if (OP == OP_SOUP_PACK) {
    I::pack_stats(a);
    host_parallel(a.n, [&](int64_t i) { I::soup_pack(a, i); });
    return 0;
  }
  host_parallel(items, [&](int64_t i) {
    float4 samp[P + 1];
    uint8_t perm[P + 4];
    if constexpr (OP == OP_SOUP_DECIDE) I::soup_decide(a, i);
    else if constexpr (OP == OP_CLASSIFY) I::classify(c, a, i, perm);
    else if constexpr (OP == OP_INIT) I::init(c, a, i, samp, perm);
    else if constexpr (OP == OP_APPLY) I::apply(c, a, i, samp, perm);
    else if constexpr (OP == OP_RUN_FIXPOINT) I::run_fixpoint(c, a, i, samp, perm);
    else if constexpr (OP == OP_TRAIN) I::train(c, a, i, samp, perm, false);
    else if constexpr (OP == OP_LEARN) I::train(c, a, i, samp, perm, true);
    else if constexpr (OP == OP_PERTURB) I::perturb(c, a, i, samp, perm);
    else if constexpr (OP == OP_SOUP_EVOLVE) I::soup_evolve(c, a, i, samp, perm);
    else if constexpr (OP == OP_RESPAWN) I::respawn(a, i);
    else if constexpr (OP == OP_VARY_RUN) I::vary_run(c, a, i, samp, perm);
    else if constexpr (OP == OP_SOUP_PACK) I::soup_pack(a, i);
    else if constexpr (OP == OP_SOUP_UNPACK) I::soup_unpack(a, i);
  });
  return 0;
}

// Single-rank respawn: one 1024-thread workgroup scans the respawn flags in slot
// order, assigns the new uids (*uid_base is next_uid), re-initialises those rows, then
// advances next_uid and the generation counter -- replacing scan + torch bookkeeping
// kernels with one launch (the flags are sparse; each thread walks a contiguous chunk).
constexpr int TBR = 1024;
template <class Net, class S>
__global__ __launch_bounds__(TBR) void k_respawn_seq(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  __shared__ int32_t s_wave[TBR / 64];
  // i32c as u64[b] = respawn ballot of evolve block b (64 rows); thread t owns blocks
  // [t*ch, (t+1)*ch): no per-row memory traffic, bits give the rows in slot order.
  const unsigned long long* masks = reinterpret_cast<const unsigned long long*>(a.i32c);
  const int64_t nb = (a.n + TB - 1) / TB;
  const int64_t ch = (nb + TBR - 1) / TBR;
  const int64_t b0 = (int64_t)threadIdx.x * ch;
  const int64_t b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t cnt = 0;
  for (int64_t b = b0; b < b1; ++b) cnt += __popcll(masks[b]);
  int32_t total;
  const int32_t incl = block_incl_scan<TBR>(cnt, s_wave, &total);
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t k = base + incl - cnt;
  if (cnt) {
    for (int64_t b = b0; b < b1; ++b) {
      unsigned long long m = masks[b];
      while (m) {
        const int bit = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int64_t r = b * TB + bit;
        a.uid_out[r] = k;
        if (!(a.flags & 32)) {  // flag 32: re-initialised inline by the evolve kernel
          float w[Net::P];
          Net::init(w, I::rng(a), respawn_key(I::gen_of(a), a.lo + r));
          I::store(I::rowp(a.W, r), w);
        }
        ++k;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ((int64_t*)a.uid_base)[0] = base + total;
    I::set_gen(a, I::gen_of(a) + 1);
  }
  if (a.counts && threadIdx.x < 5) a.counts[threadIdx.x] = 0;  // fresh histogram for the census
}

template <class Net, class S>
int respawn_seq(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (a.dev) {
    hipLaunchKernelGGL((k_respawn_seq<Net, S>), dim3(1), dim3(TBR), 0, (hipStream_t)a.stream, c, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error(hipGetErrorString(e));
      return -3;
    }
    return 0;
  }
  int64_t k = a.uid_base[0];
  for (int64_t i = 0; i < a.n; ++i) {
    if (a.respawn[i] == 0) continue;
    a.uid_out[i] = k;
    if (!(a.flags & 32)) {
      float w[Net::P];
      Net::init(w, I::rng(a), respawn_key(I::gen_of(a), a.lo + i));
      I::store(I::rowp(a.W, i), w);
    }
    ++k;
  }
  ((int64_t*)a.uid_base)[0] = k;
  I::set_gen(a, I::gen_of(a) + 1);
  if (a.counts)
    for (int q = 0; q < 5; ++q) a.counts[q] = 0;
  return 0;
}

// Sharded soup: uids of the newborns of the previous generation.  The per-rank stats
// (the exchange's stats rows, flag 256, or the gathered [world][6] array) give the
// respawn counts of lower ranks (globally sequential uids, reference S13) and the global
// census; the 64-bit respawn ballots of the evolve waves give the local order.  Consumes
// the ballots (zeroed), advances next_uid (*uid_base) and zeroes counts[0..5]; with no
// stats pending (all zero) it is a no-op apart from that.
template <class Net, class S>
__global__ __launch_bounds__(TBR) void k_uid_assign(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  __shared__ int32_t s_wave[TBR / 64];
  __shared__ int64_t s_prefix, s_total;
  if (blockIdx.x > 0) {
    // flag 16384, blocks >= 1: index the received rows (OP_SOUP_UNPACK); block 0 resets
    // the send counters (the pack that used them ran in an earlier launch)
    const int64_t k = (int64_t)(blockIdx.x - 1) * TBR + threadIdx.x;
    if (k < (int64_t)a.world * a.cap) I::soup_unpack(a, k);
    return;
  }
  if ((a.flags & 16384) && threadIdx.x < a.world) a.sendcnt[threadIdx.x] = I::SR;
  if (threadIdx.x == 0) {
    int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
    for (int r = 0; r < a.world; ++r) {
      const int64_t k = I::stat(a, r, 5);
      if (r < a.rank) pre += k;
      tot += k;
      for (int q = 0; q < 5; ++q) cen[q] += I::stat(a, r, q);
    }
    for (int q = 0; q < 5; ++q) all += cen[q];
    s_prefix = pre;
    s_total = tot;
    if (a.census && all > 0)
      for (int q = 0; q < 5; ++q) a.census[q] = cen[q];
  }
  // 64-bit respawn ballot of evolve wave b: i32c as u64[b], or the fused generation's
  // block stats (flag 8192: u64[4] per block, ballot first)
  unsigned long long* masks = reinterpret_cast<unsigned long long*>((a.flags & 8192) ? a.temp : (void*)a.i32c);
  const int mstride = (a.flags & 8192) ? 4 : 1;
  const int64_t nb = (a.n + TB - 1) / TB;
  const int64_t ch = (nb + TBR - 1) / TBR;
  const int64_t b0 = (int64_t)threadIdx.x * ch;
  const int64_t b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t cnt = 0;
  for (int64_t b = b0; b < b1; ++b) cnt += __popcll(masks[b * mstride]);
  int32_t total_local;
  const int32_t incl = block_incl_scan<TBR>(cnt, s_wave, &total_local);  // barrier inside
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t k = base + s_prefix + incl - cnt;
  for (int64_t b = b0; b < b1 && cnt; ++b) {
    unsigned long long m = masks[b * mstride];
    masks[b * mstride] = 0ull;
    while (m) {
      const int bit = __ffsll((long long)m) - 1;
      m &= m - 1;
      a.uid_out[b * TB + bit] = k++;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) ((int64_t*)a.uid_base)[0] = base + s_total;
  if (a.counts && threadIdx.x < 6) a.counts[threadIdx.x] = 0;
}

template <class Net, class S>
int uid_assign(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (a.dev) {
    const int64_t unpack_blocks = (a.flags & 16384) ? ((int64_t)a.world * a.cap + TBR - 1) / TBR : 0;
    hipLaunchKernelGGL((k_uid_assign<Net, S>), dim3((unsigned)(1 + unpack_blocks)), dim3(TBR), 0,
                       (hipStream_t)a.stream, c, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error(hipGetErrorString(e));
      return -3;
    }
    return 0;
  }
  if (a.flags & 16384) {  // post-exchange: index the received rows too
    for (int64_t k = 0; k < (int64_t)a.world * a.cap; ++k) I::soup_unpack(a, k);
    for (int r = 0; r < a.world; ++r) a.sendcnt[r] = I::SR;
  }
  int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
  for (int r = 0; r < a.world; ++r) {
    const int64_t k = I::stat(a, r, 5);
    if (r < a.rank) pre += k;
    tot += k;
    for (int q = 0; q < 5; ++q) cen[q] += I::stat(a, r, q);
  }
  for (int q = 0; q < 5; ++q) all += cen[q];
  if (a.census && all > 0)
    for (int q = 0; q < 5; ++q) a.census[q] = cen[q];
  // host path: per-row respawn flags in i32c (evolve with flag 16) or the fused
  // generation's block ballots (flag 8192), consumed here
  int64_t k = a.uid_base[0] + pre;
  if (a.flags & 8192) {
    unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
    for (int64_t b = 0; b < (a.n + TB - 1) / TB; ++b) {
      unsigned long long m = bs[b * 4];
      bs[b * 4] = 0ull;
      while (m) {
        const int bit = __builtin_ctzll(m);
        m &= m - 1;
        a.uid_out[b * TB + bit] = k++;
      }
    }
  } else {
    for (int64_t i = 0; i < a.n; ++i)
      if (a.i32c[i]) {
        a.uid_out[i] = k++;
        a.i32c[i] = 0;
      }
  }
  ((int64_t*)a.uid_base)[0] += tot;
  if (a.counts)
    for (int q = 0; q < 6; ++q) a.counts[q] = 0;
  return 0;
}

template <class Net, int OP, class S>
int run_one(const SrnnCfg& c, const SrnnArgs& a) {
  return a.dev ? launch<Net, OP, S>(c, a) : host_run<Net, OP, S>(c, a);
}

template <class Net, class S = StF32>
int run_net_op(int op, const SrnnCfg& c, const SrnnArgs& a) {
  switch (op) {
    case OP_INIT: return run_one<Net, OP_INIT, S>(c, a);
    case OP_APPLY: return run_one<Net, OP_APPLY, S>(c, a);
    case OP_RUN_FIXPOINT: return run_one<Net, OP_RUN_FIXPOINT, S>(c, a);
    case OP_TRAIN: return run_one<Net, OP_TRAIN, S>(c, a);
    case OP_LEARN: return run_one<Net, OP_LEARN, S>(c, a);
    case OP_CLASSIFY: return run_one<Net, OP_CLASSIFY, S>(c, a);
    case OP_PERTURB: return run_one<Net, OP_PERTURB, S>(c, a);
    case OP_SOUP_DECIDE: return run_one<Net, OP_SOUP_DECIDE, S>(c, a);
    case OP_RESPAWN_SEQ: return respawn_seq<Net, S>(c, a);
    case OP_SOUP_PACK: return run_one<Net, OP_SOUP_PACK, S>(c, a);
    case OP_SOUP_UNPACK: return run_one<Net, OP_SOUP_UNPACK, S>(c, a);
    case OP_UID_ASSIGN: return uid_assign<Net, S>(c, a);
    case OP_SOUP_EVOLVE: return run_one<Net, OP_SOUP_EVOLVE, S>(c, a);
    case OP_RESPAWN: return run_one<Net, OP_RESPAWN, S>(c, a);
    case OP_VARY_RUN: return run_one<Net, OP_VARY_RUN, S>(c, a);
    case OP_SOUP_GEN: return soup_gen<Net, S>(c, a);
    case OP_GEN_FINISH: return gen_finish<Net, S>(c, a);
    case OP_SOUP_PERMS: return soup_perms<Net, S>(c, a);
    case OP_SOUP_SEQ: return soup_seq<Net, S>(c, a);
    default: set_error("unknown op"); return -1;
  }
}

}  // namespace srnn

// Registration: each srnn_<kind>.hip lists its instantiated shapes with this macro and
// exports `int srnn_dispatch_<kind>(int op, const SrnnCfg*, const SrnnArgs*)`
// returning 1 on "shape not instantiated".
#define SRNN_TRY(NETTYPE, W_, D_, A_)                                                  \
  if (c->width == (W_) && c->depth == (D_) && c->aggregates == (A_)) {                 \
    if (c->p != NETTYPE::P || c->pp != NETTYPE::PP) {                                  \
      srnn::set_error("layout mismatch (p/pp) for instantiated shape");                \
      return -4;                                                                       \
    }                                                                                  \
    if (c->dtype != 0) return 1; /* 16-bit tables: srnn_lowp.hip */                    \
    if (op < 0) return 0;                                                              \
    return srnn::run_net_op<NETTYPE>(op, *c, *a);                                      \
  }

// 16-bit weight tables (bf16 / fp16 storage, fp32 arithmetic) for a shape
#define SRNN_TRY_LOWP(NETTYPE, W_, D_, A_)                                             \
  if (c->width == (W_) && c->depth == (D_) && c->aggregates == (A_)) {                 \
    if (c->p != NETTYPE::P || c->pp != NETTYPE::PP) {                                  \
      srnn::set_error("layout mismatch (p/pp) for instantiated shape");                \
      return -4;                                                                       \
    }                                                                                  \
    if (c->dtype != 1 && c->dtype != 2) return 1;                                      \
    if (op < 0) return 0;                                                              \
    if (c->dtype == 1) return srnn::run_net_op<NETTYPE, srnn::StBF16>(op, *c, *a);     \
    return srnn::run_net_op<NETTYPE, srnn::StF16>(op, *c, *a);                         \
  }
