// srnn_pair.h — soup generations of the headline net, Weightwise(2, 2), on TWO lanes per
// particle (lane u of a pair computes hidden unit u).  Included by srnn_kernels.h inside
// namespace srnn, after srnn_ordered.h.
//
// Below one wave per SIMD (a 100k soup strong-scaled over 2-8 GPUs) the lane-per-particle
// kernels are latency-bound: every SIMD that
// has a wave at all runs ONE particle's 280-step SGD chain per lane at ~5 cycles per dependent
// instruction, and most SIMDs are idle.  Splitting a particle over a lane pair cuts the
// instructions each lane issues per SGD step from 37 to 25 (the dot products of a unit stay on
// one lane in the lane path's order; the other unit's hidden values come by DPP quad
// broadcasts), halves the work of every attack and census self-application (7 of the 14 points
// per lane, gathered back by DPP) and doubles the waves.  Lane u holds column u of the first
// kernel (4 weights), column u AND row u of the 2x2 kernel (its diagonal entry twice, updated
// by the same fma) and the 2-weight output kernel.  Every fma is the lane path's
// (MLP::forward / backward_update in folded form, Net::apply per point), so results are
// bitwise equal to k_soup_gen / k_soup_evolve (tests/test_pair_soup_gpu.py).
#pragma once

namespace pair {

using WW22 = Weightwise<2, 2>;
constexpr int P = WW22::P;  // 14
constexpr int TBW = 128;    // threads per workgroup: 64 particles = one 64-row block
constexpr int64_t PAIR_MAX_N = 20480;  // auto: pairs for populations (levels) up to this size

// DPP quad permutations (quad_perm encodings): the value of pair lane 0 / 1, the partner's
__device__ __forceinline__ float pb0(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xA0, 0xF, 0xF, true));  // [0,0,2,2]
}
__device__ __forceinline__ float pb1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xF5, 0xF, 0xF, true));  // [1,1,3,3]
}
__device__ __forceinline__ int pswap_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // [1,0,3,2]
}

// normalised (layer, row, col) of point 2m + u (flat Keras order: K0 (4,2) at 2i+j, K1 (2,2) at
// 8+2i+j, K2 (2,1) at 12+i; normalize_id v/m for m > 1 else v): the lane path's coordinate table
__device__ __forceinline__ void point_coords(int m, int u, float& cl, float& cr, float& cc) {
  const float fu = (float)u;
  if (m < 6) {
    cl = WW22::coords.c[2 * m][0];
    cr = WW22::coords.c[2 * m][1];
    cc = fu;
  } else {
    cl = WW22::coords.c[12][0];
    cr = fu;
    cc = 0.f;
  }
}

// o = f_a(t) on the pair: lane u evaluates the points 2m + u, both halves are gathered back
// (every lane ends with all 14 outputs, each computed exactly as Net::apply computes it)
__device__ __forceinline__ void apply(const float* __restrict__ a, const float* __restrict__ t, float* __restrict__ o,
                                      int u) {
  float own[7];
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    float cl, cr, cc;
    point_coords(m, u, cl, cr, cc);
    float x[4] = {u ? t[2 * m + 1] : t[2 * m], cl, cr, cc}, y[1];
    WW22::Net::forward_only(a, x, y);
    own[m] = y[0];
  }
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    o[2 * m] = pb0(own[m]);
    o[2 * m + 1] = pb1(own[m]);
  }
}

// Item::classify_w on the pair (both lanes return the class)
template <class S>
__device__ __forceinline__ int8_t classify(const float* w, float eps, bool with_sec, int u) {
  using I = Item<WW22, S>;
  if (is_diverged<P>(w)) return C_DIVERGENT;
  float f1[P];
  apply(w, w, f1, u);
  I::q(f1);
  if (!is_diverged<P>(f1) && within_eps<P>(f1, w, eps)) return is_zero<P>(w, eps) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    float f2[P];
    apply(w, f1, f2, u);
    I::q(f2);
    if (!is_diverged<P>(f2) && within_eps<P>(f2, w, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}

// the split weights of pair lane u
struct Regs {
  float k0[4];     // K0[i][u]
  float cl0, cl1;  // K1[0][u], K1[1][u]  (column u)
  float rw0, rw1;  // K1[u][0], K1[u][1]  (row u; K1[u][u] is also cl_u)
  float k2[2];     // K2[0], K2[1]
};
__device__ __forceinline__ void split(const float* w, Regs& r, int u) {
#pragma unroll
  for (int i = 0; i < 4; ++i) r.k0[i] = u ? w[2 * i + 1] : w[2 * i];
  r.cl0 = u ? w[9] : w[8];
  r.cl1 = u ? w[11] : w[10];
  r.rw0 = u ? w[10] : w[8];
  r.rw1 = u ? w[11] : w[9];
  r.k2[0] = w[12];
  r.k2[1] = w[13];
}
__device__ __forceinline__ void join(const Regs& r, float* w) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = pb0(r.k0[i]);
    w[2 * i + 1] = pb1(r.k0[i]);
  }
  w[8] = pb0(r.cl0);
  w[9] = pb1(r.cl0);
  w[10] = pb0(r.cl1);
  w[11] = pb1(r.cl1);
  w[12] = r.k2[0];
  w[13] = r.k2[1];
}
// the weight of point 2m + u
__device__ __forceinline__ float own_val(const Regs& r, int m, int u) {
  if (m < 4) return r.k0[m];
  if (m == 4) return r.cl0;
  if (m == 5) return r.cl1;
  return u ? r.k2[1] : r.k2[0];
}

// one SGD step of MLP<4,2,2,1> (forward, then backward_update in folded form) on the pair
template <bool LOSS>
__device__ __forceinline__ void sgd_step(Regs& r, const float4 s, float lr2, float& acc, int u) {
  float h1u = s.x * r.k0[0];
  h1u = fmaf(s.y, r.k0[1], h1u);
  h1u = fmaf(s.z, r.k0[2], h1u);
  h1u = fmaf(s.w, r.k0[3], h1u);
  const float h1_0 = pb0(h1u), h1_1 = pb1(h1u);
  float h2u = h1_0 * r.cl0;
  h2u = fmaf(h1_1, r.cl1, h2u);
  const float h2_0 = pb0(h2u), h2_1 = pb1(h2u);
  float y = h2_0 * r.k2[0];
  y = fmaf(h2_1, r.k2[1], y);
  const float err = y - s.x;
  if constexpr (LOSS) acc += err * err;
  const float so = -lr2 * err;
  const float si2_0 = r.k2[0] * so, si2_1 = r.k2[1] * so;  // pre-update K2
  r.k2[0] = fmaf(h2_0, so, r.k2[0]);
  r.k2[1] = fmaf(h2_1, so, r.k2[1]);
  float si1u = r.rw0 * si2_0;  // pre-update row u of K1
  si1u = fmaf(r.rw1, si2_1, si1u);
  const float si2u = u ? si2_1 : si2_0;
  r.cl0 = fmaf(h1_0, si2u, r.cl0);
  r.cl1 = fmaf(h1_1, si2u, r.cl1);
  r.rw0 = fmaf(h1u, si2_0, r.rw0);
  r.rw1 = fmaf(h1u, si2_1, r.rw1);
  r.k0[0] = fmaf(s.x, si1u, r.k0[0]);
  r.k0[1] = fmaf(s.y, si1u, r.k0[1]);
  r.k0[2] = fmaf(s.z, si1u, r.k0[2]);
  r.k0[3] = fmaf(s.w, si1u, r.k0[3]);
}

// E epochs of Weightwise::train_epochs (SELF: samples = the weights at each epoch start, else
// the fixed teacher row t) on the pair; sp = the particle's sample slot 0 (stride c.stride).
// Permutations from the precomputed table when given (train_epochs_tab), else drawn inline
// exactly as train_epochs draws them.  Returns the last epoch's loss.
template <bool SELF>
__device__ __forceinline__ float train(Regs& r, const float* __restrict__ t, int E, TrainCtx& c, int u, float4* sp) {
  if (E <= 0) return 0.f;
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    float cl, cr, cc;
    point_coords(m, u, cl, cr, cc);
    const float v = SELF ? own_val(r, m, u) : (u ? t[2 * m + 1] : t[2 * m]);
    sp[(2 * m + u) * c.stride] = make_float4(v, cl, cr, cc);
  }
  uint64_t ident = 0;
#pragma unroll
  for (int k = 0; k < P; ++k) ident |= (uint64_t)k << (4 * k);
  const bool tab = c.ptab != nullptr && c.shuffle;
  const uint64_t* pt = tab ? c.ptab + (int64_t)(c.ctr - c.pbase) * c.pstride : nullptr;
  U4 rr{0, 0, 0, 0};
  uint32_t pr = c.ctr >> 1;
  uint64_t pn = ident;
  if (tab) {
    pn = pt[0];
    perm_prologue_wait();
  } else if (c.shuffle) {
    rr = perm_draw(c.rng, c.uid, c.ctr, P_SHUFFLE);
    pn = perm_from_bits<P>(perm_bits(rr, c.ctr));
  }
  const float lr2 = 2.0f * c.lr;
  float loss = 0.f;
  for (int e = 0; e < E; ++e) {
    if (SELF && e > 0)
#pragma unroll
      for (int m = 0; m < 7; ++m) reinterpret_cast<float*>(&sp[(2 * m + u) * c.stride])[0] = own_val(r, m, u);
    __builtin_amdgcn_wave_barrier();  // the partner lane's sample writes precede these reads
    const bool last = e + 1 == E;
    uint64_t pn_next = ident;
    if (tab) {
      pn_next = last ? 0ull : pt[(int64_t)(e + 1) * c.pstride];
    } else if (c.shuffle) {
      const uint32_t nx = c.ctr + 1u;
      if ((nx >> 1) != pr) {
        pr = nx >> 1;
        rr = perm_draw(c.rng, c.uid, nx, P_SHUFFLE);
      }
      pn_next = perm_from_bits<P>(perm_bits(rr, nx));
    }
    float4 smp[P];
#pragma unroll
    for (int q = 0; q < P; ++q) smp[q] = sp[(int)((pn >> (4 * q)) & 15u) * c.stride];
    __builtin_amdgcn_wave_barrier();  // ... and the next epoch's sample writes follow them
    float acc = 0.f;
    if (!last) {
#pragma unroll
      for (int q = 0; q < P; ++q) sgd_step<false>(r, smp[q], lr2, acc, u);
    } else {
#pragma unroll
      for (int q = 0; q < P; ++q) sgd_step<true>(r, smp[q], lr2, acc, u);
      loss = acc / (float)P;
    }
    c.ctr += 1;
    pn = pn_next;
  }
  return loss;
}

// learn_from (severity epochs on the teacher row f) then self-train (epochs) of the full row w
// in place, as Item::soup_evolve / Ord::turn run them; returns the last loss
template <class S>
__device__ __forceinline__ float learn_and_train(const SrnnArgs& a, float* w, const float* f, bool learn, TrainCtx& tc,
                                                 int u, float4* sp) {
  if (!(learn && a.severity > 0) && a.epochs <= 0) return 0.f;
  Regs r;
  split(w, r, u);
  float loss = 0.f;
  if (learn && a.severity > 0) loss = train<false>(r, f, a.severity, tc, u, sp);
  if (a.epochs > 0) loss = train<true>(r, nullptr, a.epochs, tc, u, sp);
  join(r, w);
  return loss;
}

// (row >= 0 with a table: the particle's permutations are column `row` of a.ptab, stride
// pstride (default n); row < 0: drawn inline)
__device__ __forceinline__ void train_ctx(const SrnnArgs& a, TrainCtx& tc, uint64_t uid, int32_t gen, int64_t row,
                                          int64_t pstride = -1) {
  tc.lr = a.lr;
  tc.rng = Rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  tc.uid = uid;
  tc.ctr = (uint32_t)gen * 1024u + 512u;
  tc.samp = nullptr;
  tc.perm = nullptr;
  tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
  tc.stride = 64;  // particles per workgroup: sample slot k of particle pi at sp[k * 64]
  tc.aggregator = 0;
  if (a.ptab && row >= 0) {
    tc.ptab = a.ptab + row;
    tc.pstride = pstride >= 0 ? pstride : a.n;
    tc.pbase = tc.ctr;
  }
}

// single-rank synchronous generation of row i (Item::soup_evolve<SINGLE = true>) on the pair;
// w receives the stored row
template <class S>
__device__ __forceinline__ int8_t evolve(const SrnnArgs& a, int64_t i, int32_t gen, int u, float4* sp, float* w) {
  using I = Item<WW22, S>;
  float f[P], o[P], tw[P];
  I::load(I::rowp(a.W2, i), w);
  // the decisions and the teacher's generation-start row first (its load overlaps the attacks)
  int64_t my_at, te;
  I::decision(a, i, gen, my_at, te);
  if (te >= 0) I::load(I::rowp(a.W2, te), tw);
  // 1. attacks received, ascending attacker slot, generation-start attacker rows (the list is
  // consumed by both lanes of the pair: same wave, the loads precede the NIL store)
  for_each_attacker<true>(a, i, [&](uint32_t e, int64_t) {
    I::load(I::rowp(a.W2, (int64_t)e), f);
    apply(f, w, o, u);
    I::q(o);
    I::copy(w, o);
  });
  int8_t act = my_at >= 0 ? A_ATTACKING : A_NONE;
  int64_t cp = my_at >= 0 ? my_at : -1;
  TrainCtx tc;
  train_ctx(a, tc, (uint64_t)i, gen, i);
  const float loss = learn_and_train<S>(a, w, tw, te >= 0, tc, u, sp);  // 2. learn_from, 3. self-train
  if (te >= 0) {
    act = A_LEARN_FROM;
    cp = te;
  }
  if (a.epochs > 0) {  // 3. self-train
    act = A_TRAIN_SELF;
    cp = -1;
  }
  I::q(w);  // 4. respawn
  int8_t rs = 0;
  if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && is_diverged<P>(w)) rs = 1;
  else if ((a.flags & SRNN_F_REMOVE_ZERO) && is_zero<P>(w, a.eps)) rs = 2;
  if (rs && (a.flags & SRNN_F_RESPAWN_INLINE)) WW22::init(w, I::rng(a), respawn_key(gen, i));
  I::store(I::rowp(a.W, i), w);
  I::q(w);
  if (u == 0) {
    if (a.action) a.action[i] = act;
    if (a.counterpart) a.counterpart[i] = cp;
    if (a.loss) a.loss[i] = loss;
    if (a.respawn) a.respawn[i] = rs;
  }
  return rs;
}

// even-lane bits of a 64-lane ballot -> 32 bits (pair p at bit p)
__device__ __forceinline__ uint32_t even_bits(unsigned long long x) {
  x &= 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  return (uint32_t)x;
}

}  // namespace pair

// OP_SOUP_GEN on pairs (two-phase form): workgroup = 64 particles = one 64-row block, so the
// block stats are the lane kernel's (k_gen_finish / the batched finish read them unchanged)
template <class S>
__global__ __launch_bounds__(pair::TBW) void k_soup_gen2(SrnnCfg c, SrnnArgs a) {
  using I = Item<pair::WW22, S>;
  __shared__ float4 s_samp[pair::P * 64];
  __shared__ unsigned long long s_bs[2][4];
  const int tid = threadIdx.x, u = tid & 1, pi = tid >> 1, wv = tid >> 6, lane = tid & 63;
  const int64_t gb = blockIdx.x;
  const int64_t i = gb * 64 + pi;
  const int32_t gen = I::gen_of(a);
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  bool rs = false;
  int8_t k = -1;
  if (i < a.n) {
    if (u == 0) {  // the next generation's attack first (the atomic overlaps this generation)
      int64_t at, te;
      I::decision(a, i, gen + 1, at, te);
      if (at >= 0) I::link(a.heads_next, a.nexts_next, at, (uint32_t)i);
    }
    float w[pair::P];
    rs = pair::evolve<S>(a, i, gen, u, s_samp + pi, w) != 0;
    if (census) k = pair::classify<S>(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, u);
  }
  if ((a.flags & SRNN_F_GEN_COUNTS) && gb == 0 && tid == 0) I::set_gen(a, gen + 1);
  const bool lead = u == 0;
  const uint32_t m = pair::even_bits(__ballot(rs && lead));
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(lead && k == q));
  if (lane == 0) {
    s_bs[wv][0] = m;
    s_bs[wv][1] = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
    s_bs[wv][2] = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
    s_bs[wv][3] = (unsigned long long)cnt[4];
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
    unsigned long long* mine = bs + gb * 4;
    const unsigned long long mm = s_bs[0][0] | (s_bs[1][0] << 32);
    mine[0] = mm;
    mine[1] = s_bs[0][1] + s_bs[1][1];  // per-half counts < 2^32: no carry across the halves
    mine[2] = s_bs[0][2] + s_bs[1][2];
    mine[3] = s_bs[0][3] + s_bs[1][3];
    if ((a.flags & SRNN_F_BORN_TOTAL) && mm) atomicAdd(bs + ((a.n + TB - 1) / TB) * 4, (unsigned long long)__popcll(mm));
  }
}

// lanes per particle of a WW(2,2) launch over `count` particles: knob SRNN_KNOB_SOUP_LANES
// (1 lane, 2 pair; 0 / unset: pairs up to PAIR_MAX_N particles)
inline bool use_pairs(int64_t count) {
  const int k = knob(SRNN_KNOB_SOUP_LANES, 0);
  if (k == 1) return false;
  if (k == 2) return true;
  return count <= pair::PAIR_MAX_N;
}

namespace pair {
// sharded (X2) generation of local row j on the pair (Item::soup_evolve<false>): attackers and
// teachers may be received rows (list entries >= n, tk); w receives the stored row
template <class S>
__device__ __forceinline__ int8_t evolve_x2(const SrnnArgs& a, int64_t j, uint32_t tk, int u, float4* sp, float* w) {
  using I = Item<WW22, S>;
  constexpr int64_t RB = I::RB;
  const int64_t g = a.lo + j;
  const int32_t gen = I::gen_of(a);
  float f[P], o[P], tw[P];
  I::load(I::rowp(a.W2, j), w);
  int64_t my_at, te;  // (the teacher's row load overlaps the attacks)
  I::decision(a, g, gen, my_at, te);
  const char* tr = nullptr;
  if (te >= 0) {
    tr = teacher_row(a, te, tk, RB);
    I::load(tr, tw);
  }
  for_each_attacker<false>(a, j, [&](uint32_t e, int64_t slot) {
    const char* r = ent_row(a, e, RB);
    if ((int64_t)e >= a.n) x2_check(a, r, RB, slot, gen);
    I::load(r, f);
    apply(f, w, o, u);
    I::q(o);
    I::copy(w, o);
  });
  int8_t act = my_at >= 0 ? A_ATTACKING : A_NONE;
  int64_t cp = my_at >= 0 ? my_at : -1;
  TrainCtx tc;
  train_ctx(a, tc, (uint64_t)g, gen, j);
  if (te >= 0 && tk != SRNN_NIL) x2_check(a, tr, RB, te, gen);
  const float loss = learn_and_train<S>(a, w, tw, te >= 0, tc, u, sp);
  if (te >= 0) {
    act = A_LEARN_FROM;
    cp = te;
  }
  if (a.epochs > 0) {
    act = A_TRAIN_SELF;
    cp = -1;
  }
  I::q(w);
  int8_t rs = 0;
  if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && is_diverged<P>(w)) rs = 1;
  else if ((a.flags & SRNN_F_REMOVE_ZERO) && is_zero<P>(w, a.eps)) rs = 2;
  if (rs && (a.flags & SRNN_F_RESPAWN_INLINE)) WW22::init(w, I::rng(a), respawn_key(gen, g));
  I::store(I::rowp(a.W, j), w);
  I::q(w);
  if (u == 0) {
    if (a.action) a.action[j] = act;
    if (a.counterpart) a.counterpart[j] = cp;
    if (a.loss) a.loss[j] = loss;
    if (a.respawn) a.respawn[j] = rs;
  }
  return rs;
}
}  // namespace pair

// The single-launch sharded generation (k_soup_evolve with SRNN_F_X2 | X2_REMOTE | X2_BOTH,
// optionally POST_FUSED) on pairs: workgroup = one 64-row block; a pair whose own slot is
// remote-dependent takes an entry of the remote list (the block's 64 dependency bits are two
// x_dep words, its first entry x_hpre + x_hgrp as in the lane kernel); block stats by atomics
// (local and remote slots share blocks).
template <class S>
__global__ __launch_bounds__(pair::TBW) void k_soup_evolve2(SrnnCfg c, SrnnArgs a) {
  __shared__ float4 s_samp[pair::P * 64];
  const int64_t npb = (a.flags & SRNN_F_X2_POST_FUSED) ? x2::post_blocks<pair::TBW>(a) : 0;
  if ((int64_t)blockIdx.x < npb) {
    if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
    x2::post_block<pair::TBW>(x2::geom(c), a, reinterpret_cast<unsigned long long*>(a.temp2), blockIdx.x);
    return;
  }
  const int tid = threadIdx.x, u = tid & 1, pi = tid >> 1, wv = tid >> 6, lane = tid & 63;
  const int64_t eb = (int64_t)blockIdx.x - npb;
  const int64_t i = eb * 64 + pi;
  const bool valid = i < a.n;
  const int64_t nw = (a.n + 31) / 32;
  const uint64_t hm = (uint64_t)a.x_dep[2 * eb] | (2 * eb + 1 < nw ? (uint64_t)a.x_dep[2 * eb + 1] << 32 : 0ull);
  const bool dep = valid && ((hm >> pi) & 1ull);
  const int64_t cnt = *(volatile const int32_t*)a.x_rcount;
  const int64_t nbk = (a.n + 63) / 64, per = (nbk + a.x_groups - 1) / a.x_groups;
  const int64_t base = hm ? (int64_t)a.x_hpre[eb] + a.x_hgrp[eb / per] : 0;
  const int64_t pos = base + (int64_t)__popcll(hm & ((1ull << pi) - 1ull));
  int64_t j = i;
  uint32_t tk = SRNN_NIL;
  bool on = valid && !dep;
  if (dep && pos < cnt) {
    j = a.x_rlist[2 * pos];
    tk = a.x_rlist[2 * pos + 1];
    on = true;
  }
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  bool rs = false;
  int8_t k = -1;
  if (on) {
    float w[pair::P];
    rs = pair::evolve_x2<S>(a, j, tk, u, s_samp + pi, w) != 0;
    if (census) k = pair::classify<S>(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, u);
  }
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  // own slots in the block's stats (bit pi of block eb), taken list entries slot by slot
  const bool lead = u == 0;
  const unsigned long long m = (unsigned long long)pair::even_bits(__ballot(lead && on && !dep && rs)) << (32 * wv);
  uint32_t cn[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cn[q] = (uint32_t)__popcll(__ballot(lead && on && !dep && k == q));
  if (lane == 0) {
    unsigned long long* st = bs + eb * 4;
    if (m) atomicOr(st, m);
    const unsigned long long c01 = (unsigned long long)cn[0] | ((unsigned long long)cn[1] << 32);
    const unsigned long long c23 = (unsigned long long)cn[2] | ((unsigned long long)cn[3] << 32);
    if (c01) atomicAdd(st + 1, c01);
    if (c23) atomicAdd(st + 2, c23);
    if (cn[4]) atomicAdd(st + 3, (unsigned long long)cn[4]);
  }
  if (lead && dep && on) bs_publish_lane(bs, j, rs, k);
  __syncthreads();  // every pair read its dependency bits and the list counter
  if (tid < 2 && (2 * eb + tid) * 32 < a.n) a.x_dep[2 * eb + tid] = 0u;
  if (tid == 0) {
    const int32_t prev = atomicAdd(a.x_ctl + 3, 1);
    if (prev == (int32_t)((int64_t)gridDim.x - npb) - 1) {  // last workgroup: the list is re-armed
      *a.x_rcount = 0;
      a.x_ctl[3] = 0;
    }
  }
}
