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
#include <type_traits>
#include <vector>
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>

extern "C" int srnn_x2_run(int op, const SrnnCfg* c, const SrnnArgs* a);  // srnn_shard.hip

namespace srnn {

void set_error(const char* msg);
int knob(int id, int dflt);  // srnn_common.hip: execution knob in force (SrnnKnob)

constexpr int TB = 64;  // threads per block: one wave; lane-private LDS scratch per thread
// waves of the X2 remote evolve (grid-stride over the remote-dependent list, whose length is
// only known on the device): 4 per SIMD of a 256-CU MI355X
constexpr int64_t X2_REMOTE_WAVES = 4096;

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

// float4 sample slots per lane of a net's training scratch (Weightwise::SAMP_F4; the other
// kinds keep their samples in registers) and the lane's base pointer: float4 slots, or for
// value-only samples (Weightwise P > 16) float slots, both slot-major with the lane fastest
template <class Net>
constexpr int samp_slots() {
  if constexpr (Net::KIND == 0) return Net::SAMP_F4;
  else return 1;
}
template <class Net>
SRNN_HD float4* samp_lane(float4* base, int lane) {
  if constexpr (Net::KIND == 0 && Net::P > 16) return reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + lane);
  else return base + lane;
}

SRNN_HD int32_t atomic_or_i32(int32_t* p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicOr(p, v);
#else
  return __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}

// rank owning global slot g under the contiguous sharding lo_r = floor(r * N / R)
SRNN_HD int32_t shard_of(int64_t g, int64_t n_total, int32_t world) {
  // g * world < 2^63 for any population that fits a node (< 2^58 slots)
  int32_t r = (int32_t)((g * world) / n_total);
  while (r + 1 < world && ((int64_t)(r + 1) * n_total) / world <= g) ++r;
  while (r > 0 && ((int64_t)r * n_total) / world > g) --r;
  return r;
}
SRNN_HD int64_t shard_lo(int32_t r, int64_t n_total, int32_t world) { return ((int64_t)r * n_total) / world; }

// init key of the particle born in slot g at generation `gen` (rank-count invariant).
// Slots below 2^32: bit 62 | gen << 32 | slot; larger slots (HBM-filling sharded soups):
// bit 63 | (gen mod 2^23) << 40 | slot.  Initial particles are keyed by their uid (< 2^62).
SRNN_HD uint64_t respawn_key(int32_t gen, int64_t g) {
  if ((uint64_t)g < (1ull << 32)) return (1ull << 62) | ((uint64_t)(uint32_t)gen << 32) | (uint64_t)g;
  return (1ull << 63) | ((uint64_t)((uint32_t)gen & 0x7FFFFFu) << 40) | ((uint64_t)g & ((1ull << 40) - 1));
}

// ----------------------------------------------------------------------------------
// Soup row sources and attack lists, shape independent (rb = bytes of a table row).
// A victim's list holds its attackers' entries (SRNN_NIL-terminated, see srnn_abi.h):
//   single rank       entry = the attacker's row (= slot, lo = 0), row in W2
//   SRNN_F_FULL_TABLE entry = global slot, row in W2 (own shard) or the gathered table
//   SRNN_F_X2         entry < n: local row in W2; entry >= n: received row e - n of the
//                     all-to-all (block q = k / x_cr, position k % x_cr), slot in x_rslot
// ----------------------------------------------------------------------------------
constexpr int64_t X2_HB = (int64_t)SRNN_X2_HDR * 8;  // header bytes of an exchange block
SRNN_HD int64_t x2_xb(int64_t rb) { return rb + 16; }  // exchange row: weights + (int64 slot, int64 gen)
SRNN_HD const char* x2_row(const SrnnArgs& a, int64_t k, int64_t rb) {
  const int64_t q = k / a.x_cr, pos = k - q * a.x_cr;
  return a.recvbuf + q * a.x_blk + X2_HB + pos * x2_xb(rb);
}
SRNN_HD uint64_t ent_slot(const SrnnArgs& a, uint32_t e) {
  if (a.flags & SRNN_F_FULL_TABLE) return e;
  if ((int64_t)e < a.n) return (uint64_t)(a.lo + (int64_t)e);
  return (uint64_t)a.x_rslot[(int64_t)e - a.n];
}
SRNN_HD const char* ent_row(const SrnnArgs& a, uint32_t e, int64_t rb) {
  if (a.flags & SRNN_F_FULL_TABLE) {
    const int64_t g = (int64_t)e;
    if (g >= a.lo && g < a.lo + a.n) return reinterpret_cast<const char*>(a.W2) + (g - a.lo) * rb;
    return a.recvbuf + g * rb;
  }
  if ((int64_t)e < a.n) return reinterpret_cast<const char*>(a.W2) + (int64_t)e * rb;
  return x2_row(a, (int64_t)e - a.n, rb);
}
// generation-start row of teacher slot te (tk: its received row under SRNN_F_X2)
SRNN_HD const char* teacher_row(const SrnnArgs& a, int64_t te, uint32_t tk, int64_t rb) {
  if (te >= a.lo && te < a.lo + a.n) return reinterpret_cast<const char*>(a.W2) + (te - a.lo) * rb;
  if (a.flags & SRNN_F_FULL_TABLE) return a.recvbuf + te * rb;
  return x2_row(a, (int64_t)tk, rb);
}
SRNN_HD void err_or(int32_t* p, int32_t v) {
  if (!p) return;
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}
// a received row must carry the slot and generation the receiver expects (protocol check)
SRNN_HD void x2_check(const SrnnArgs& a, const char* row, int64_t rb, int64_t slot, int32_t gen) {
  const int64_t* t = reinterpret_cast<const int64_t*>(row + rb);
  if (t[0] != slot || t[1] != (int64_t)gen) err_or(a.err, 4);
}
// Visit the attackers of local victim j in ascending attacker-slot order (the list is in
// arrival order; lists are short: Poisson(attacking_rate)).  Consumes the list head.
// SINGLE: single-rank lists (entry = slot = row): no flag tests on the hot path.
// Sharded lists (!SINGLE) are bounded: a list that does not end within 2^16 steps (a
// protocol bug) sets error bit 4 and ends the walk instead of hanging the GPU.
template <bool SINGLE, class F>
SRNN_HD void for_each_attacker(const SrnnArgs& a, int64_t j, F&& f) {
  const uint32_t head = a.heads[j];
  if (head == SRNN_NIL) return;
  a.heads[j] = SRNN_NIL;  // consumed: NIL for the generation after next
  uint64_t last = 0;
  bool first = true;
  uint32_t steps = 0;
  for (;;) {
    uint64_t best = ~0ull;
    uint32_t be = SRNN_NIL;
    for (uint32_t e = head; e != SRNN_NIL; e = a.nexts[e]) {
      if (!SINGLE && ++steps > (1u << 16)) {
        err_or(a.err, 4);
        return;
      }
      const uint64_t sl = SINGLE ? (uint64_t)e : ent_slot(a, e);
      if ((first || sl > last) && sl < best) best = sl, be = e;
    }
    if (be == SRNN_NIL) break;
    first = false;
    last = best;
    f(be, (int64_t)best);
  }
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
  SRNN_HD static char* rowp(float* base, int64_t i) { return reinterpret_cast<char*>(base) + i * RB; }
  SRNN_HD static const char* rowp(const float* base, int64_t i) { return reinterpret_cast<const char*>(base) + i * RB; }

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
    if (a.cls) a.cls[i] = classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, x);
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
    tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
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
    int8_t k = classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, actx(a, c, uid_of(a, i), a.ctr, perm));
    if (a.cls) a.cls[i] = k;
    return k;
  }

  // ---------------------------------------------------------------- soup
  // Decisions of global slot g in generation `gen` (reference code/soup.py:56-63): a pure
  // function of (seed, slot, generation), so any rank can recompute any slot's decision.
  // Partners are uniform over the slot's sub-soup (segment) or the whole population; spans
  // above 2^32 slots take 64-bit partner draws from a second stream.
  SRNN_HD static void decision(const SrnnArgs& a, int64_t g, int32_t gen, int64_t& at, int64_t& te) {
    const Rng r = rng(a);
    const U4 d = r.draw((uint64_t)g, (uint32_t)gen, P_SOUP);
    at = -1;
    te = -1;
    const int64_t span = a.segment > 0 ? a.segment : a.n_total;
    const int64_t base = a.segment > 0 ? (g / a.segment) * a.segment : 0;
    const bool atk = u01(d.x) < a.attacking_rate, lrn = u01(d.z) < a.learn_from_rate;
    if (!atk && !lrn) return;
    if ((uint64_t)span <= 0xFFFFFFFFull) {
      if (atk) at = base + (int64_t)(((uint64_t)d.y * (uint64_t)span) >> 32);
      if (lrn) te = base + (int64_t)(((uint64_t)d.w * (uint64_t)span) >> 32);
    } else {
      const U4 e = r.draw((uint64_t)g, (uint32_t)gen, P_SOUP_WIDE);
      if (atk) at = base + (int64_t)mulhi64((((uint64_t)e.x) << 32) | e.y, (uint64_t)span);
      if (lrn) te = base + (int64_t)mulhi64((((uint64_t)e.z) << 32) | e.w, (uint64_t)span);
    }
  }
  SRNN_HD static uint64_t mulhi64(uint64_t x, uint64_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(x, y);
#else
    return (uint64_t)(((unsigned __int128)x * y) >> 64);
#endif
  }
  SRNN_HD static int32_t gen_of(const SrnnArgs& a) { return a.gen_ptr ? a.gen_ptr[0] : a.gen; }
  // the next generation's counter: the other ring slot (gen_out) or in place
  SRNN_HD static void set_gen(const SrnnArgs& a, int32_t g) {
    if (a.gen_out) a.gen_out[0] = g;
    else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = g;
  }

  // Every global slot (single rank or all-gather exchange): link attacks on this rank's
  // victims into per-victim lists (heads pre-set to NIL).  Entries are global slots (single
  // rank: lo = 0, slot = row).  Optional dec_at / dec_te receive the decisions.
  SRNN_HD static void soup_decide(const SrnnArgs& a, int64_t i) {
    int64_t at, te;
    decision(a, i, gen_of(a), at, te);
    if (a.dec_at) a.dec_at[i] = at;
    if (a.dec_te) a.dec_te[i] = te;
    if (at >= a.lo && at < a.lo + a.n) link(a.heads, a.nexts, at - a.lo, (uint32_t)i);
  }
  // entry e joins the list of local victim v
  SRNN_HD static void link(uint32_t* heads, uint32_t* nexts, int64_t v, uint32_t e) {
#if defined(__HIP_DEVICE_COMPILE__)
    nexts[e] = atomicExch(heads + v, e);
#else
    nexts[e] = __atomic_exchange_n(heads + v, e, __ATOMIC_RELAXED);
#endif
  }

  // Synchronous (Jacobi) generation for local row j: every read is from the
  // generation-start table W2 (own rows) or received / gathered rows of other ranks, the
  // result goes to W (local rows).  The particle's random streams (SGD shuffles,
  // shuffle_random) are keyed by its global SLOT and the generation -- not by its uid -- so
  // a generation never waits for the uids of the previous generation's newborns.
  // SINGLE: single-rank source rows (no exchange); tk: the received row of a remote teacher
  // (SRNN_F_X2).  Returns the respawn code (also in respawn[j]).
  // TAB = false compiles the permutation-table path out (the launches that never get one)
  template <bool SINGLE = false, bool TAB = true>
  SRNN_HD static int8_t soup_evolve(const SrnnCfg& c, const SrnnArgs& a, int64_t j, float4* samp, uint8_t* perm,
                                    uint32_t tk = SRNN_NIL, float* wout = nullptr) {
    const int64_t g = a.lo + j;
    float w[P], f[P], o[P];
    load(rowp(a.W2, j), w);
    const uint64_t uid = (uint64_t)g;  // stream key of this slot
    const int32_t gen = gen_of(a);
    ApplyCtx x = actx(a, c, uid, (uint32_t)gen * 1024u, perm);
    const bool x2 = !SINGLE && (a.flags & SRNN_F_X2);
    // this slot's decisions and its teacher's row first: the teacher's load is in flight
    // while the attacks are applied (generation-start rows: nothing of this generation
    // writes them)
    int64_t my_at, te;
    decision(a, g, gen, my_at, te);
    float tw[P];
    const char* tr = nullptr;
    if (te >= 0) {
      tr = SINGLE ? rowp(a.W2, te) : teacher_row(a, te, tk, RB);
      load(tr, tw);
    }
    // 1. attacks received, in ascending attacker slot order (generation-start attacker rows)
    for_each_attacker<SINGLE>(a, j, [&](uint32_t e, int64_t slot) {
      const char* r = SINGLE ? rowp(a.W2, (int64_t)e) : ent_row(a, e, RB);
      if (x2 && (int64_t)e >= a.n) x2_check(a, r, RB, slot, gen);
      load(r, f);
      Net::apply(f, w, o, x);
      q(o);
      x.ctr += 1;
      copy(w, o);
    });
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
    tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
    tc.stride = SAMP_STRIDE;
    tc.aggregator = c.aggregator;
    if (TAB && a.ptab && a.dev) {  // this generation's permutations, precomputed (k_perm_table)
      tc.ptab = a.ptab + j;
      tc.pstride = a.n;
      tc.pbase = tc.ctr;
    }
    float loss = 0.f;
    // 2. learn_from a teacher (its generation-start weights)
    if (te >= 0) {
      if (x2 && tk != SRNN_NIL) x2_check(a, tr, RB, te, gen);
      copy(f, tw);
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
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && is_diverged<P>(w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && is_zero<P>(w, a.eps)) rs = 2;
    if (rs && (a.flags & SRNN_F_RESPAWN_INLINE)) Net::init(w, rng(a), respawn_key(gen, g));  // newborn
    store(rowp(a.W, j), w);
    if (wout) {  // the stored row as a reload would see it (the census classifies it from registers)
      copy(wout, w);
      q(wout);
    }
    if (a.action) a.action[j] = act;
    if (a.counterpart) a.counterpart[j] = cp;
    if (a.loss) a.loss[j] = loss;
    if (a.respawn) a.respawn[j] = rs;
    return rs;
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
    int64_t at, te;
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
    tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
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
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && is_diverged<P>(w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && is_zero<P>(w, a.eps)) rs = 2;
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
};

// ==================================================================================
// Device kernels
// ==================================================================================
template <class Net, int OP, class S>
__global__ __launch_bounds__(TB) void k_op(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr bool NEED_SAMP = (OP == OP_TRAIN || OP == OP_LEARN) && Net::KIND == 0;
  constexpr int SAMP = NEED_SAMP ? samp_slots<Net>() : 1;  // slot-major [P][TB]: lane fastest
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  float4* samp = samp_lane<Net>(s_samp, threadIdx.x);  // slot k of this lane at samp[k * TB]
  uint8_t* perm = s_perm + threadIdx.x * PERM;

  if constexpr (OP == OP_SOUP_DECIDE) {
    if (i < a.n_total) I::soup_decide(a, i);
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

// Epoch permutations of a soup generation ahead of it (SrnnArgs::ptab): thread (row, pair)
// draws the Philox block of epochs 2p, 2p + 1 (counters gen*1024 + 512 + e, keyed by the
// row's global slot) and stores both nibble permutations -- exactly what train_epochs would
// compute inline, moved off the latency-bound SGD chains into one fully parallel launch.
constexpr int TBP = 256;
template <class Net>
__global__ __launch_bounds__(TBP) void k_perm_table(SrnnArgs a, int32_t E) {
  constexpr int P = Net::P;
  // grid (rows, epoch pairs): no 64-bit division on the index
  const int64_t row = (int64_t)blockIdx.x * TBP + threadIdx.x, p = blockIdx.y;
  if (row >= a.n) return;
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const uint32_t c0 = (uint32_t)gen * 1024u + 512u + 2u * (uint32_t)p;  // even: one draw, two epochs
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const U4 r = perm_draw(rng, (uint64_t)(a.lo + row), c0, P_SHUFFLE);
  a.ptab[2 * p * a.n + row] = perm_from_bits<P>(perm_bits(r, c0));
  if (2 * p + 1 < E) a.ptab[(2 * p + 1) * a.n + row] = perm_from_bits<P>(perm_bits(r, c0 + 1u));
}
// the same entries from a shape-independent kernel (the sharded exchange's pack builds the
// table of the generation it prepares; runtime P, identical permutations)
__device__ __forceinline__ void perm_table_entry(const SrnnArgs& a, int P, int64_t row, int32_t p, int32_t gen,
                                                 int32_t E) {
  const uint32_t c0 = (uint32_t)gen * 1024u + 512u + 2u * (uint32_t)p;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const U4 r = perm_draw(rng, (uint64_t)(a.lo + row), c0, P_SHUFFLE);
  a.ptab[2 * p * a.n + row] = perm_from_bits_n(P, perm_bits(r, c0));
  if (2 * p + 1 < E) a.ptab[(2 * p + 1) * a.n + row] = perm_from_bits_n(P, perm_bits(r, c0 + 1u));
}
// workgroups of NT threads that build a generation's table inside another launch (0: none --
// no table given, host, not a nibble Weightwise net, no shuffle, no epochs)
inline int64_t pack_ptab_blocks(const SrnnCfg& c, const SrnnArgs& a, int NT) {
  const int32_t E = (a.severity > 0 ? a.severity : 0) + (a.epochs > 0 ? a.epochs : 0);
  if (!a.ptab || !a.dev || !(a.flags & SRNN_F_SHUFFLE) || c.kind != 0 || c.p > 16 || E <= 0 || a.n <= 0) return 0;
  return ((a.n + NT - 1) / NT) * ((E + 1) / 2);
}
// launch the permutation table of this generation when the caller gave one (nibble nets);
// SRNN_F_PTAB_READY: an earlier launch of the generation (the sharded pack) built it already
template <class Net>
int perm_table(const SrnnArgs& a) {
  if constexpr (Net::KIND != 0 || Net::P > 16) {
    return 0;
  } else {
    const int32_t E = (a.severity > 0 ? a.severity : 0) + (a.epochs > 0 ? a.epochs : 0);
    if (!a.ptab || !a.dev || !(a.flags & SRNN_F_SHUFFLE) || E <= 0 || a.n <= 0 || (a.flags & SRNN_F_PTAB_READY)) return 0;
    hipLaunchKernelGGL((k_perm_table<Net>), dim3((unsigned)((a.n + TBP - 1) / TBP), (unsigned)((E + 1) / 2)),
                       dim3(TBP), 0, (hipStream_t)a.stream, a, E);
    return 0;
  }
}

// Inclusive scan over an NT-thread block: wave shuffles (no barrier) + one LDS pass over
// the NT/64 wave totals (one barrier) instead of a log2(NT)-round Hillis-Steele scan with
// two barriers per round.  *total receives the block sum.
template <int NT, class T = int32_t>
__device__ __forceinline__ T block_incl_scan(T v, T* s_wave, T* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wave[wv] = x;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const T sw = s_wave[w];
    pre += (w < wv) ? sw : 0;
    tot += sw;
  }
  *total = tot;
  return x + pre;
}

// the sharded exchange protocol's steps (pack / post roles), used by the single-launch X2 evolve
#include "srnn_shard.h"

// ----------------------------------------------------------------------------------
// X2 block stats (u64[4] per 64-row block of a generation: respawn ballot; class counts
// c0 | c1 << 32, c2 | c3 << 32, c4) are accumulated with atomics: the local and the remote
// evolve of a sharded generation run at the same time and share blocks.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ void bs_publish_wave(unsigned long long* bs, int64_t b, bool rs, int8_t k) {
  const unsigned long long m = __ballot(rs);
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(k == q));
  if (threadIdx.x % TB == 0) {
    unsigned long long* st = bs + b * 4;
    if (m) atomicOr(st, m);
    const unsigned long long c01 = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
    const unsigned long long c23 = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
    if (c01) atomicAdd(st + 1, c01);
    if (c23) atomicAdd(st + 2, c23);
    if (cnt[4]) atomicAdd(st + 3, (unsigned long long)cnt[4]);
  }
}
__device__ __forceinline__ void bs_publish_lane(unsigned long long* bs, int64_t row, bool rs, int8_t k) {
  unsigned long long* st = bs + (row >> 6) * 4;
  if (rs) atomicOr(st, 1ull << (row & 63));
  if (k >= 0) atomicAdd(st + 1 + (k >> 1), 1ull << (32 * (k & 1)));
}
// host form of the same accumulation (the X2 evolve on CPU tensors)
inline void bs_publish_host(unsigned long long* bs, int64_t row, bool rs, int8_t k) {
  unsigned long long* st = bs + (row >> 6) * 4;
  if (rs) __atomic_fetch_or(st, 1ull << (row & 63), __ATOMIC_RELAXED);
  if (k >= 0) __atomic_fetch_add(st + 1 + (k >> 1), 1ull << (32 * (k & 1)), __ATOMIC_RELAXED);
}
// X2 local evolve: is row i remote-dependent this generation?
SRNN_HD bool x2_dep(const SrnnArgs& a, int64_t i) { return (a.x_dep[i >> 5] >> (i & 31)) & 1u; }
// most entries the remote list of a generation can hold (a slot joins it through a received
// notice or one of its requests): the remote evolve's grid is sized by this bound, not by n
// (every wave of that launch takes one ticket on the re-arm counter)
SRNN_HD int64_t x2_remote_bound(const SrnnArgs& a) {
  if (a.x_emul && a.world == 1) return a.n > 1 ? a.n : 1;  // timing model: any local slot
  const int64_t b = (int64_t)a.world * (a.x_cn + a.x_cq);
  return b < a.n ? (b > 1 ? b : 1) : (a.n > 1 ? a.n : 1);
}
// workgroups of the remote-list walk (grid-stride over the bound, at most X2_REMOTE_WAVES)
SRNN_HD int64_t x2_remote_blocks(const SrnnArgs& a) {
  const int64_t rb = (x2_remote_bound(a) + TB - 1) / TB;
  return rb < X2_REMOTE_WAVES ? rb : X2_REMOTE_WAVES;
}

// Soup evolve (OP_SOUP_EVOLVE), one wave per block, lane per slot:
//  * single rank / all-gather exchange: rows blockIdx * 64 + lane; each wave publishes its
//    64-bit respawn ballot (ballots[block]) or per-row flags (rowflags, SRNN_F_ROW_FLAGS)
//  * SRNN_F_X2, local: the same rows minus the remote-dependent ones (x_dep bits, reset
//    here for the generation after next)
//  * SRNN_F_X2 | SRNN_F_X2_REMOTE: the (row, teacher row) entries of x_rlist, grid-stride
//    over a bounded grid; the last wave re-arms the list counter
//  X2 evolves accumulate the generation's block stats (temp), with SRNN_F_FUSED_CENSUS the
//  census class of each stored row too.
template <class Net, class S, bool TAB = false>
__global__ __launch_bounds__(TB) void k_soup_evolve(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int lane = threadIdx.x;
  float4* samp = samp_lane<Net>(s_samp, lane);
  uint8_t* perm = s_perm + lane * PERM;
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  auto classify_w_ = [&](const float* w, int64_t i) -> int8_t {  // census class of stored row i
    return I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0,
                         I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
  };
  auto classify_stored = [&](int64_t i) -> int8_t {
    float w[P];
    I::load(I::rowp(a.W, i), w);
    return classify_w_(w, i);
  };
  if (!(a.flags & SRNN_F_X2)) {
    const int64_t i = (int64_t)blockIdx.x * TB + lane;
    bool rs = false;
    if (i < a.n) rs = I::template soup_evolve<false, TAB>(c, a, i, samp, perm) != 0;
    if (a.flags & SRNN_F_ROW_FLAGS) {
      if (i < a.n && a.rowflags) a.rowflags[i] = rs ? 1 : 0;
    } else if (a.ballots) {
      const unsigned long long m = __ballot(rs);
      if (lane == 0) a.ballots[blockIdx.x] = m;
    }
    return;
  }
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  if (a.flags & SRNN_F_X2_BOTH) {
    // SRNN_F_X2_POST_FUSED: the first workgroups are the post of this generation's exchange
    // (uids of the last generation's newborns, census, the next generation's notices and
    // requests); nothing the evolve reads is written by it
    const int64_t npb = (a.flags & SRNN_F_X2_POST_FUSED) ? x2::post_blocks<TB>(a) : 0;
    if ((int64_t)blockIdx.x < npb) {
      if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
      x2::post_block<TB>(x2::geom(c), a, reinterpret_cast<unsigned long long*>(a.temp2), blockIdx.x);
      return;
    }
    const int64_t eb = (int64_t)blockIdx.x - npb;  // this wave's 64-row block
    // one launch for the whole generation, n/64 waves: a lane whose own slot is
    // remote-dependent (x_dep) takes an entry of the remote list instead -- there are exactly as
    // many such lanes as entries (a slot joins the list when its bit is first set), so every
    // lane evolves one slot and no wave is added for the remote ones
    const int64_t i = eb * TB + lane;
    const bool valid = i < a.n;
    const bool dep = valid && x2_dep(a, i);
    const int64_t cnt = *(volatile const int32_t*)a.x_rcount;
    const unsigned long long hm = __ballot(dep);
    // this wave's first list entry: holes before its block (prefix from pack, x_hpre / x_hgrp)
    const int64_t nbk = (a.n + TB - 1) / TB, per = (nbk + a.x_groups - 1) / a.x_groups;
    const int64_t base = hm ? (int64_t)a.x_hpre[eb] + a.x_hgrp[eb / per] : 0;
    const int64_t pos = base + (int64_t)__popcll(hm & ((1ull << lane) - 1ull));
    int64_t j = i;
    uint32_t tk = SRNN_NIL;
    bool on = valid && !dep;
    if (dep && pos < cnt) {
      j = a.x_rlist[2 * pos];
      tk = a.x_rlist[2 * pos + 1];
      on = true;
    }
    bool rs = false;
    int8_t k = -1;
    if (on) {
      float w[P];
      rs = I::template soup_evolve<false, TAB>(c, a, j, samp, perm, tk, w) != 0;
      if (census) k = classify_w_(w, j);
    }
    const int64_t wd = eb * 2 + lane;
    if (lane < 2 && wd * 32 < a.n) a.x_dep[wd] = 0u;
    // own slots in the wave's block stats, taken list entries lane by lane
    bs_publish_wave(bs, eb, on && !dep && rs, dep ? (int8_t)-1 : k);
    if (dep && on) bs_publish_lane(bs, j, rs, k);
    int32_t prev = 0;
    if (lane == 0) prev = atomicAdd(a.x_ctl + 3, 1);
    prev = __shfl(prev, 0);
    if (prev == (int32_t)((int64_t)gridDim.x - npb) - 1 && lane == 0) {  // last wave: the list is re-armed
      *a.x_rcount = 0;
      a.x_ctl[3] = 0;
    }
    return;
  }
  if (!(a.flags & SRNN_F_X2_REMOTE)) {
    const int64_t i = (int64_t)blockIdx.x * TB + lane;
    const bool on = i < a.n && !x2_dep(a, i);
    bool rs = false;
    int8_t k = -1;
    if (on) {
      float w[P];
      rs = I::template soup_evolve<false, TAB>(c, a, i, samp, perm, SRNN_NIL, w) != 0;
      if (census) k = classify_w_(w, i);
    }
    // this wave's two dependency words are consumed (every lane read its bit above)
    const int64_t wd = (int64_t)blockIdx.x * 2 + lane;
    if (lane < 2 && wd * 32 < a.n) a.x_dep[wd] = 0u;
    bs_publish_wave(bs, blockIdx.x, rs, k);
    return;
  }
  if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);  // the exchange chain's tail
  const int64_t cnt = *(volatile const int32_t*)a.x_rcount;
  for (int64_t base = (int64_t)blockIdx.x * TB; base < cnt; base += (int64_t)gridDim.x * TB) {
    const int64_t q = base + lane;
    if (q < cnt) {
      const int64_t j = a.x_rlist[2 * q];
      const uint32_t tk = a.x_rlist[2 * q + 1];
      const bool rs = I::template soup_evolve<false, TAB>(c, a, j, samp, perm, tk) != 0;
      const int8_t k = census ? classify_stored(j) : (int8_t)-1;
      bs_publish_lane(bs, j, rs, k);
    }
  }
  // last wave: the counter is free again (the list of the generation after next appends to it;
  // no data is handed over, every wave read the counter before its ticket)
  int32_t prev = 0;
  if (lane == 0) prev = atomicAdd(a.x_ctl + 3, 1);
  prev = __shfl(prev, 0);
  if (prev == (int32_t)gridDim.x - 1 && lane == 0) {
    *a.x_rcount = 0;
    a.x_ctl[3] = 0;
  }
}

// ----------------------------------------------------------------------------------
// Fused single-rank soup generation (OP_SOUP_GEN): ONE launch per generation instead of
// decide -> evolve -> respawn -> classify.  Per lane: the generation (attacks received,
// learn_from, self-train, respawn + inline re-init), then the NEXT generation's decision
// for its slot linked into the other list buffer (heads_next / nexts_next; the decisions
// are a pure function of (seed, slot, generation)), then the census class of the stored
// row.  Each wave publishes its respawn ballot + class counts (temp: u64[4] per block).
//  * SRNN_F_TWO_PHASE: plain stores; a finish launch (k_gen_finish / the batched finish)
//    numbers the newborns and reduces the census after the kernel boundary
//    (SRNN_F_GEN_COUNTS: this launch advances the generation counter itself;
//    SRNN_F_BORN_TOTAL: it also adds its newborn count after the block stats)
//  * otherwise the LAST wave to finish (done ticket, no waiting anywhere) scans the
//    ballots in slot order, assigns the newborns' uids, writes the census (counts[0..4]),
//    advances next_uid and the generation counter and re-arms the ticket.
// ----------------------------------------------------------------------------------
template <class Net, class S, bool TAB = false>
__global__ __launch_bounds__(TB) void k_soup_gen(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t gb = blockIdx.x;  // rows gb*64 ..
  const int64_t i = gb * TB + threadIdx.x;
  const int lane = threadIdx.x;
  uint8_t* perm = s_perm + lane * PERM;
  const int32_t gen = I::gen_of(a);
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  bool rs = false;
  int8_t k = -1;
  if (i < a.n) {
    // the next generation's attack first (its own lists: the atomic's round trip overlaps
    // this generation's loads instead of ending the wave; list order is irrelevant, attacks
    // are applied in ascending attacker order)
    int64_t at, te;
    I::decision(a, i, gen + 1, at, te);
    if (at >= 0) I::link(a.heads_next, a.nexts_next, at, (uint32_t)i);
    float w[P];  // the stored row (no reload of what this lane just wrote)
    rs = I::template soup_evolve<true, TAB>(c, a, i, samp_lane<Net>(s_samp, lane), perm, SRNN_NIL, w) != 0;
    if (census)
      k = I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0,
                        I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
  }
  if ((a.flags & SRNN_F_GEN_COUNTS) && gb == 0 && threadIdx.x == 0) {
    // this launch advances the generation counter (the other ring slot: no block of this
    // launch reads it), so the next generation needs nothing from the finish launch
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
  if (a.flags & SRNN_F_TWO_PHASE) {  // plain stores, the finish reads them after the kernel boundary
    if (lane == 0) {
      unsigned long long* mine = bs + gb * 4;
      mine[0] = m;
      mine[1] = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
      mine[2] = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
      mine[3] = (unsigned long long)cnt[4];
      // the generation's newborn count after the block stats (batched finish)
      if ((a.flags & SRNN_F_BORN_TOTAL) && m) atomicAdd(bs + ((a.n + TB - 1) / TB) * 4, (unsigned long long)__popcll(m));
    }
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
    prev = __hip_atomic_fetch_add(a.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  prev = __shfl(prev, 0);
  const int32_t nb = (int32_t)gridDim.x;
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
    a.uid_base[0] = base + total;
    I::set_gen(a, gen + 1);
    if (a.counts) {
#pragma unroll
      for (int q = 0; q < 5; ++q) a.counts[q] = census ? cs[q] : 0ull;
      a.counts[5] = (uint64_t)total;
    }
    __hip_atomic_store(a.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
  }
}


// Second phase of the two-phase fused single-rank generation: one SRNN_FINISH_NT-thread
// workgroup reduces the per-wave census counts, scans the respawn ballots in slot order,
// assigns the newborns' uids and advances next_uid / the generation counter.
#ifndef SRNN_FINISH_NT
#define SRNN_FINISH_NT 1024  // threads of the finish workgroup (256: 7.27 us vs 6.68 us)
#endif
template <class Net, class S, int NT>
__global__ __launch_bounds__(NT) void k_gen_finish(SrnnArgs a, int32_t nb) {
  using I = Item<Net, S>;
  __shared__ int32_t s_wave[NT / 64];
  __shared__ unsigned long long s_cs[5];
  const int t = threadIdx.x;
  if (t < 5) s_cs[t] = 0;
  const unsigned long long* bs = reinterpret_cast<const unsigned long long*>(a.temp);
  // the uid base and the generation counter are only written by thread 0 after the last
  // barrier: load them up front so their latency overlaps the per-block stats loads
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  const bool advanced = (a.flags & SRNN_F_GEN_COUNTS) != 0;  // the generation kernel advanced the counter
  const int32_t gen = advanced ? 0 : I::gen_of(a);
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
    a.uid_base[0] = base + total_born;
    if (!advanced) I::set_gen(a, gen + 1);
    if (a.counts) {
      for (int q = 0; q < 5; ++q) a.counts[q] = (a.flags & SRNN_F_FUSED_CENSUS) ? s_cs[q] : 0ull;
      a.counts[5] = (uint64_t)total_born;
    }
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
      const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
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
  if (t == 0) a.uid_base[0] = s_base;
}

// Parallel form of k_gen_finish_batch (a.done given: a zeroed done counter): ONE workgroup
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
  const bool totals = (a.flags & SRNN_F_BORN_TOTAL) != 0 && m <= NT;  // newborns of generation k at ring(k)[4 nb]
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
    const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
    if (a.counts && g == m - 1) {
      for (int q = 0; q < 5; ++q) a.counts[q] = census ? s_cs[q] : 0ull;
      a.counts[5] = (uint64_t)total_born;
    }
    if (a.census) {
      for (int q = 0; q < 5; ++q) a.census[(int64_t)g * 6 + q] = census ? (int64_t)s_cs[q] : 0;
      a.census[(int64_t)g * 6 + 5] = total_born;
    }
    // every workgroup read next_uid (and the newborn totals) before its ticket -- the loads
    // completed, their values are in use -- so the last one may overwrite them; the other
    // workgroups' uid / census stores need no release: only later launches read them
    const int32_t prev = atomicAdd(a.done, 1);
    if (prev == m - 1) {
      a.uid_base[0] = base + total_all;
      if (totals)  // every workgroup has read the counts: re-armed for the next batch
        for (int32_t k = 0; k < m; ++k) const_cast<unsigned long long*>(ring(k))[(int64_t)nb * 4] = 0ull;
      __hip_atomic_store(a.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Finish of single-rank fused generations (OP_GEN_FINISH): census + newborn uids of the
// generation(s) whose block stats are in a.temp (host: no-op, soup_gen did it).
template <class Net, class S>
int gen_finish(const SrnnCfg&, const SrnnArgs& a) {
  if (!a.dev) return 0;
  const int64_t blocks = (a.n + TB - 1) / TB;
  if (blocks <= 0) return 0;
  constexpr int FNT = SRNN_FINISH_NT;
  if (a.steps > 1 || (a.flags & SRNN_F_FINISH_BATCH)) {  // batch of a.steps generations (ring in temp)
    if (a.steps < 1 || a.temp_bytes < blocks * 32) {
      set_error("batched finish needs steps >= 1 generations and temp_bytes >= 32 per block");
      return -5;
    }
    if (a.done)  // a zeroed done counter: one workgroup per generation
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

// reference-order generations scheduled by dependency level (OP_SOUP_ORDERED), and the
// two-lanes-per-particle WW(2,2) generations (srnn_pair.h, included from srnn_ordered.h)
#include "srnn_ordered.h"

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
  constexpr int SAMP = samp_slots<Net>();
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
  a.uid_base[0] = next;
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
  a.uid_base[0] = next;
  I::set_gen(a, gen0 + a.steps);
  return 0;
}

template <class Net, class S>
int soup_gen(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  if (a.world > 1 || a.lo != 0 || a.n_total != a.n || a.n >= (int64_t)SRNN_NIL) {
    set_error("fused soup generation: one unsharded table of < 2^32 rows");
    return -5;
  }
  if (!a.dev) {
    // host: the same steps in order (evolve all rows, link next decisions, census, uids)
    const int32_t gen = I::gen_of(a);
    host_parallel(a.n, [&](int64_t i) {
      float4 samp[Net::P + 1];
      uint8_t perm[Net::P + 4];
      I::template soup_evolve<true>(c, a, i, samp, perm);
    });
    for (int64_t i = 0; i < a.n; ++i) {
      int64_t at, te;
      I::decision(a, i, gen + 1, at, te);
      if (at >= 0) {
        a.nexts_next[i] = a.heads_next[at];
        a.heads_next[at] = (uint32_t)i;
      }
    }
    uint64_t cs[5] = {0, 0, 0, 0, 0};
    if (a.flags & SRNN_F_FUSED_CENSUS) {
      std::vector<int8_t> ks((size_t)a.n);
      host_parallel(a.n, [&](int64_t i) {
        float w[Net::P];
        uint8_t perm[Net::P + 4];
        I::load(I::rowp(a.W, i), w);
        ks[(size_t)i] = I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0,
                                      I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
      });
      for (int64_t i = 0; i < a.n; ++i) cs[ks[(size_t)i]]++;
    }
    int64_t u = a.uid_base[0], total = 0;
    for (int64_t i = 0; i < a.n; ++i)
      if (a.respawn[i]) {
        a.uid_out[i] = u++;
        ++total;
      }
    a.uid_base[0] = u;
    I::set_gen(a, gen + 1);
    if (a.counts) {
      for (int q = 0; q < 5; ++q) a.counts[q] = cs[q];
      a.counts[5] = (uint64_t)total;
    }
    return 0;
  }
  const int64_t blocks = (a.n + TB - 1) / TB;
  if (blocks <= 0) return 0;
  if (blocks > 0x7fffffffLL) {
    set_error("grid too large");
    return -2;
  }
  if (!a.temp || !a.heads_next || !a.nexts_next || (!(a.flags & SRNN_F_TWO_PHASE) && !a.done)) {
    set_error("fused soup generation needs block stats (temp), the next lists and a done counter");
    return -5;
  }
  perm_table<Net>(a);
  bool pairs = false;
  if constexpr (std::is_same_v<Net, Weightwise<2, 2>>) pairs = (a.flags & SRNN_F_TWO_PHASE) && use_pairs(a.n);
  if (pairs) {  // below ~0.6 waves per SIMD: two lanes per particle (srnn_pair.h)
    if constexpr (std::is_same_v<Net, Weightwise<2, 2>>)
      hipLaunchKernelGGL((k_soup_gen2<S>), dim3((unsigned)blocks), dim3(pair::TBW), 0, (hipStream_t)a.stream, c, a);
  } else {
    bool tab = false;
    if constexpr (Net::KIND == 0 && Net::P <= 16) tab = a.ptab != nullptr;
    if (tab) {
      if constexpr (Net::KIND == 0 && Net::P <= 16)
        hipLaunchKernelGGL((k_soup_gen<Net, S, true>), dim3((unsigned)blocks), dim3(TB), 0, (hipStream_t)a.stream, c, a);
    } else {
      hipLaunchKernelGGL((k_soup_gen<Net, S, false>), dim3((unsigned)blocks), dim3(TB), 0, (hipStream_t)a.stream, c, a);
    }
  }
  if ((a.flags & SRNN_F_TWO_PHASE) && !(a.flags & SRNN_F_GEN_COUNTS)) {
    constexpr int FNT = SRNN_FINISH_NT;
    hipLaunchKernelGGL((k_gen_finish<Net, S, FNT>), dim3(1), dim3(FNT), 0, (hipStream_t)a.stream, a, (int32_t)blocks);
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
  if (a.flags & SRNN_F_COUNT_RESPAWNS) {  // respawns of this generation (sharded soup: uid prefix)
    unsigned long long m = __ballot(i < a.n && a.respawn[i] != 0);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(a.counts + 5, (uint64_t)__popcll(m));
  }
  // sharded soup: the census closes the generation (no later kernel of this generation
  // reads the counter)
  if ((a.flags & SRNN_F_GEN_ADVANCE) && blockIdx.x == 0 && threadIdx.x == 0) I::set_gen(a, I::gen_of(a) + 1);
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
        if (a.flags & SRNN_F_FIX_SEC) {
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
  const int64_t items = (OP == OP_SOUP_DECIDE) ? a.n_total : a.n;
  if (items <= 0) return 0;
  int64_t blocks = (items + TB - 1) / TB;
  if (blocks > 0x7fffffffLL) {
    set_error("grid too large");
    return -2;
  }
  hipStream_t st = (hipStream_t)a.stream;
  if constexpr (OP == OP_RUN_FIXPOINT && Net::KIND == 0 && Net::P <= 16) {
    // small populations: 16 lanes per particle (knob SRNN_KNOB_FIX_GROUP 0/1 forces either form)
    const int kg = knob(SRNN_KNOB_FIX_GROUP, -1);
    const bool group = kg >= 0 ? kg == 1 : a.n <= FIX_GROUP_MAX_N;
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
    if ((a.flags & SRNN_F_X2) && (a.flags & SRNN_F_X2_REMOTE)) {
      // bounded grid over the remote-dependent list (its length is on the device), after the
      // local blocks with SRNN_F_X2_BOTH
      if (!(a.flags & SRNN_F_X2_BOTH)) blocks = x2_remote_blocks(a);  // (BOTH: n/64 waves)
      else if (a.flags & SRNN_F_X2_POST_FUSED) blocks += x2::post_blocks<TB>(a);  // + post's workgroups
    }
    if ((a.flags & SRNN_F_X2_POST_FUSED) && (!(a.flags & SRNN_F_X2_BOTH) || !a.temp2 || !a.recvbuf)) {
      set_error("X2 evolve with the fused post needs X2_BOTH, temp2 (the last generation's block stats), recvbuf");
      return -5;
    }
    if ((a.flags & SRNN_F_X2_BOTH) && (!a.x_hpre || !a.x_hgrp || a.x_groups < 1)) {
      set_error("single-launch X2 evolve needs the hole prefixes of pack (x_hpre, x_hgrp)");
      return -5;
    }
    if ((a.flags & SRNN_F_X2) && (!a.temp || !a.x_dep || !a.x_rlist || !a.x_rcount || !a.x_ctl)) {
      set_error("X2 evolve needs block stats (temp), x_dep, x_rlist, x_rcount and x_ctl");
      return -5;
    }
    // the generation's permutation table: computed right before a launch that evolves every slot
    // of the generation (single rank / all-gather, or the single-launch X2 evolve); a launch that
    // evolves only part of them (the overlap schedule's local / remote halves) computes inline
    const bool whole = !(a.flags & SRNN_F_X2) || ((a.flags & SRNN_F_X2_REMOTE) && (a.flags & SRNN_F_X2_BOTH));
    if (a.ptab && !whole) {
      SrnnArgs b = a;
      b.ptab = nullptr;
      hipLaunchKernelGGL((k_soup_evolve<Net, S, false>), dim3((unsigned)blocks), dim3(TB), 0, st, c, b);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        set_error(hipGetErrorString(e));
        return -3;
      }
      return 0;
    }
    perm_table<Net>(a);
    if constexpr (std::is_same_v<Net, Weightwise<2, 2>>) {
      const uint32_t both = SRNN_F_X2 | SRNN_F_X2_REMOTE | SRNN_F_X2_BOTH;
      if ((a.flags & both) == both && use_pairs(a.n)) {  // the sharded generation on lane pairs
        const int64_t pb = (a.flags & SRNN_F_X2_POST_FUSED) ? x2::post_blocks<pair::TBW>(a) : 0;
        hipLaunchKernelGGL((k_soup_evolve2<S>), dim3((unsigned)(pb + (a.n + 63) / 64)), dim3(pair::TBW), 0, st, c, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
          set_error(hipGetErrorString(e));
          return -3;
        }
        return 0;
      }
    }
    bool tab = false;
    if constexpr (Net::KIND == 0 && Net::P <= 16) tab = a.ptab != nullptr;
    if (tab) {
      if constexpr (Net::KIND == 0 && Net::P <= 16)
        hipLaunchKernelGGL((k_soup_evolve<Net, S, true>), dim3((unsigned)blocks), dim3(TB), 0, st, c, a);
    } else {
      hipLaunchKernelGGL((k_soup_evolve<Net, S, false>), dim3((unsigned)blocks), dim3(TB), 0, st, c, a);
    }
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
// X2 evolve on the host: the local rows minus the remote-dependent ones, or the remote list;
// same block-stats accumulation as the device kernels (census with SRNN_F_FUSED_CENSUS)
template <class Net, class S, class EvolveFn, class ClassifyFn>
void host_x2_evolve(const SrnnArgs& a, EvolveFn&& evolve, ClassifyFn&& classify) {
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  if (!(a.flags & SRNN_F_X2_REMOTE) || (a.flags & SRNN_F_X2_BOTH)) {
    host_parallel(a.n, [&](int64_t i) {
      if (x2_dep(a, i)) return;
      const bool rs = evolve(i, SRNN_NIL) != 0;
      bs_publish_host(bs, i, rs, census ? classify(i) : (int8_t)-1);
    });
    for (int64_t w = 0; w < (a.n + 31) / 32; ++w) a.x_dep[w] = 0u;
    if (!(a.flags & SRNN_F_X2_BOTH)) return;
  }
  const int64_t cnt = *a.x_rcount;
  host_parallel(cnt, [&](int64_t q) {
    const int64_t j = a.x_rlist[2 * q];
    const bool rs = evolve(j, a.x_rlist[2 * q + 1]) != 0;
    bs_publish_host(bs, j, rs, census ? classify(j) : (int8_t)-1);
  });
  *a.x_rcount = 0;
}

template <class Net, int OP, class S>
int host_run(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  constexpr int P = Net::P;
  const int64_t items = (OP == OP_SOUP_DECIDE) ? a.n_total : a.n;
  if (OP == OP_CLASSIFY && a.counts) {
    uint64_t local[5] = {0, 0, 0, 0, 0};
    std::vector<int8_t> ks((size_t)items);
    host_parallel(items, [&](int64_t i) {
      uint8_t perm[P + 4];
      ks[(size_t)i] = I::classify(c, a, i, perm);
    });
    for (int64_t i = 0; i < items; ++i) local[ks[(size_t)i]]++;
    for (int q = 0; q < 5; ++q) a.counts[q] += local[q];
    if (a.flags & SRNN_F_COUNT_RESPAWNS)
      for (int64_t i = 0; i < items; ++i) a.counts[5] += a.respawn[i] != 0;
    if (a.flags & SRNN_F_GEN_ADVANCE) I::set_gen(a, I::gen_of(a) + 1);
    return 0;
  }
  if (OP == OP_SOUP_EVOLVE) {
    auto evolve = [&](int64_t i, uint32_t tk) -> int8_t {
      float4 samp[P + 1];
      uint8_t perm[P + 4];
      return I::soup_evolve(c, a, i, samp, perm, tk);
    };
    if (a.flags & SRNN_F_X2) {
      auto classify = [&](int64_t i) -> int8_t {
        float w[P];
        uint8_t perm[P + 4];
        I::load(I::rowp(a.W, i), w);
        return I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0,
                             I::actx(a, c, (uint64_t)(a.lo + i), 0x7FFFFFF0u, perm));
      };
      if (a.flags & SRNN_F_X2_POST_FUSED) {  // the post of this exchange first (host order)
        SrnnArgs pa = a;
        pa.temp = a.temp2;
        pa.flags &= ~(uint32_t)(SRNN_F_X2_POST_FUSED | SRNN_F_X2_BOTH | SRNN_F_X2_REMOTE);
        const int r = srnn_x2_run(OP_X2_POST, &c, &pa);
        if (r) return r;
      }
      host_x2_evolve<Net, S>(a, evolve, classify);
      return 0;
    }
    host_parallel(a.n, [&](int64_t i) { evolve(i, SRNN_NIL); });
    if (a.flags & SRNN_F_ROW_FLAGS) {
      if (a.rowflags)
        for (int64_t i = 0; i < a.n; ++i) a.rowflags[i] = a.respawn[i] != 0 ? 1 : 0;
    } else if (a.ballots) {
      for (int64_t b = 0; b < (a.n + TB - 1) / TB; ++b) {
        unsigned long long m = 0;
        for (int64_t i = b * TB; i < a.n && i < (b + 1) * TB; ++i)
          if (a.respawn[i]) m |= 1ull << (i - b * TB);
        a.ballots[b] = m;
      }
    }
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
    else if constexpr (OP == OP_RESPAWN) I::respawn(a, i);
    else if constexpr (OP == OP_VARY_RUN) I::vary_run(c, a, i, samp, perm);
  });
  return 0;
}

// Single-rank respawn: one 1024-thread workgroup scans the respawn ballots in slot
// order, assigns the new uids (*uid_base is next_uid), re-initialises those rows, then
// advances next_uid and the generation counter -- replacing scan + torch bookkeeping
// kernels with one launch (the flags are sparse; each thread walks a contiguous chunk).
constexpr int TBR = 1024;
template <class Net, class S>
__global__ __launch_bounds__(TBR) void k_respawn_seq(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  __shared__ int32_t s_wave[TBR / 64];
  // ballots[b] = respawn ballot of evolve block b (64 rows); thread t owns blocks
  // [t*ch, (t+1)*ch): no per-row memory traffic, bits give the rows in slot order.
  const unsigned long long* masks = a.ballots;
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
        if (!(a.flags & SRNN_F_RESPAWN_INLINE)) {
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
    a.uid_base[0] = base + total;
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
    if (!(a.flags & SRNN_F_RESPAWN_INLINE)) {
      float w[Net::P];
      Net::init(w, I::rng(a), respawn_key(I::gen_of(a), a.lo + i));
      I::store(I::rowp(a.W, i), w);
    }
    ++k;
  }
  a.uid_base[0] = k;
  I::set_gen(a, I::gen_of(a) + 1);
  if (a.counts)
    for (int q = 0; q < 5; ++q) a.counts[q] = 0;
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
    case OP_SOUP_EVOLVE: return run_one<Net, OP_SOUP_EVOLVE, S>(c, a);
    case OP_RESPAWN: return run_one<Net, OP_RESPAWN, S>(c, a);
    case OP_VARY_RUN: return run_one<Net, OP_VARY_RUN, S>(c, a);
    case OP_SOUP_GEN: return soup_gen<Net, S>(c, a);
    case OP_GEN_FINISH: return gen_finish<Net, S>(c, a);
    case OP_SOUP_SEQ: return soup_seq<Net, S>(c, a);
    case OP_SOUP_ORDERED: return soup_ordered<Net, S>(c, a);
    case OP_SOUP_ORDERED_SH: return soup_ordered_sh<Net, S>(c, a);
    case OP_ORD_PLAN: return soup_ord_plan<Net, S>(c, a);
    case OP_ORD_CENSUS: return soup_ord_census<Net, S>(c, a);
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
