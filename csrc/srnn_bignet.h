// srnn_bignet.h — kernels of the big aggregating nets (one shape per srnn_bignet_*.hip
// translation unit, compiled in parallel; dispatch in srnn_bignet.hip).  Wave-per-particle kernels for Aggregating nets too large for the
// lane-per-particle register kernels (north-star config: Aggregating(4, 10, 3), P = 280,
// 1M particles; reference code/network.py:292-439).
//
// One 64-lane wave owns one particle: the row is streamed HBM -> LDS with float4 loads
// (coalesced, 1120 B per particle), chunk means are wave reductions (fp64, like the
// reference's python-float sums), every dense layer is computed by lanes j < out reading
// column j of the kernel from LDS, and the output row is written back coalesced.
//
// Self-application to convergence runs on a 4-number state: after one application an
// aggregating net's weights are constant over each aggregation chunk (no shuffle), the
// chunk means of such a vector are exactly those constants (double sums of identical
// floats), so every further application is a function of the A chunk values only --
// bit-identical to re-evaluating the expanded weights, with no memory traffic until the
// final write.  MFMA does not apply: each particle is a GEMV chain with its own weights
// (M = 1), see docs/kernels.md.
#pragma once
#include "srnn_kernels.h"
#include <cstdlib>
#include <utility>

namespace srnn {

constexpr int BW = 4;            // waves (particles) per block
constexpr int TBB = 64 * BW;

template <int A_, int W_, int D_>
struct AggBig {
  static constexpr int A = A_, W = W_, D = D_;
  using Net = MLP<A, W, D, A>;
  static constexpr int P = Net::P;
  static constexpr int PP = (P + 3) & ~3;
  static constexpr int NL = D + 1;
  static constexpr int CS = P / A;
  static_assert(P / CS == A, "invalid aggregation (SURVEY S4)");
  static constexpr int MAXW = (A > W ? A : W);
  static constexpr int rows(int l) { return l == 0 ? A : W; }
  static constexpr int cols(int l) { return l == D ? A : W; }
  static constexpr int off(int l) { return Net::off(l); }
  __device__ static int chunk(int k) { int c = k / CS; return c < A ? c : A - 1; }
  static constexpr int chunk_c(int k) { return k / CS < A ? k / CS : A - 1; }
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    float u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}
__device__ __forceinline__ bool wave_all(bool b) { return __ballot(!b) == 0ull; }

// per-wave LDS scratch: weights [PP] + vectors for backprop
template <class T>
struct WaveLds {
  float w[T::PP];
  float t[T::PP];             // second row (attack target)
  float act[T::NL][T::MAXW];  // input of every layer
  float st[T::MAXW];          // propagated step
  float st2[T::MAXW];
};

template <class T>
__device__ void load_row(float* __restrict__ sw, const float* __restrict__ row, int lane) {
  const float4* r4 = reinterpret_cast<const float4*>(row);
  float4* s4 = reinterpret_cast<float4*>(sw);
  for (int q = lane; q < T::PP / 4; q += 64) s4[q] = r4[q];
}
template <class T>
__device__ void store_state(float* __restrict__ row, const float* s, int lane) {
  // expand the chunk state into the full row
  float4* r4 = reinterpret_cast<float4*>(row);
  for (int q = lane; q < T::PP / 4; q += 64) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * q + e;
      float x = 0.f;
#pragma unroll
      for (int c = 0; c < T::A; ++c) x = (k < T::P && T::chunk(k) == c) ? s[c] : x;
      v[e] = x;
    }
    r4[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
}
template <class T>
__device__ void store_lds(float* __restrict__ row, const float* __restrict__ sw, int lane) {
  float4* r4 = reinterpret_cast<float4*>(row);
  const float4* s4 = reinterpret_cast<const float4*>(sw);
  for (int q = lane; q < T::PP / 4; q += 64) r4[q] = s4[q];
}

// chunk aggregation of an LDS row (aggregator: 0 mean, 1 max, 2 max with the reference quirk)
template <class T>
__device__ void aggregate_lds(const float* __restrict__ sw, float* g, int lane, int aggregator) {
#pragma unroll
  for (int c = 0; c < T::A; ++c) {
    const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
    if (aggregator == 0) {
      double acc = 0.0;
      for (int k = b + lane; k < e; k += 64) acc += (double)sw[k];
      g[c] = (float)(wave_sum(acc) / (double)(e - b));
    } else {
      // sequential semantics of the reference loop (first element seeds the max)
      float m = sw[b];
      if (lane == 0)
        for (int k = b; k < e; ++k) {
          const float v = sw[k];
          m = (aggregator == 1) ? (v > m ? v : m) : ((v > m && v != 0.0f) ? v : m);
        }
      g[c] = __shfl(m, 0, 64);
    }
  }
}

// y = x . K for the layer at LDS offset `o` (rows I, cols O); x replicated in all lanes,
// y returned replicated.  Lane j < O accumulates column j in the kernels' order.
template <int I, int O>
__device__ void dense_lds(const float* __restrict__ k, const float* x, float* y, int lane) {
  float acc = 0.f;
  if (lane < O) {
    acc = x[0] * k[lane];
#pragma unroll
    for (int i = 1; i < I; ++i) acc = fmaf(x[i], k[i * O + lane], acc);
  }
#pragma unroll
  for (int j = 0; j < O; ++j) y[j] = __shfl(acc, j, 64);
}

// same with piecewise-constant weights: K[i][j] = s[chunk(o + i*O + j)]
template <class T, int I, int O>
__device__ void dense_state(int o, const float* s, const float* x, float* y, int lane) {
  float acc = 0.f;
  if (lane < O) {
    float kv = 0.f;
    int f = o + lane;
    int c = T::chunk(f);
#pragma unroll
    for (int q = 0; q < T::A; ++q) kv = (c == q) ? s[q] : kv;
    acc = x[0] * kv;
#pragma unroll
    for (int i = 1; i < I; ++i) {
      f = o + i * O + lane;
      c = T::chunk(f);
#pragma unroll
      for (int q = 0; q < T::A; ++q) kv = (c == q) ? s[q] : kv;
      acc = fmaf(x[i], kv, acc);
    }
  }
#pragma unroll
  for (int j = 0; j < O; ++j) y[j] = __shfl(acc, j, 64);
}

template <class T>
__device__ void mlp_lds(const float* __restrict__ sw, const float* g, float* h, int lane) {
  float x[T::MAXW], y[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
  dense_lds<T::A, T::W>(sw + T::off(0), x, y, lane);
#pragma unroll
  for (int l = 1; l < T::D; ++l) {
#pragma unroll
    for (int i = 0; i < T::W; ++i) x[i] = y[i];
    dense_lds<T::W, T::W>(sw + T::off(l), x, y, lane);
  }
#pragma unroll
  for (int i = 0; i < T::W; ++i) x[i] = y[i];
  dense_lds<T::W, T::A>(sw + T::off(T::D), x, h, lane);
}

template <class T>
__device__ void mlp_state(const float* s, const float* g, float* h, int lane) {
  float x[T::MAXW], y[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
  dense_state<T, T::A, T::W>(T::off(0), s, x, y, lane);
#pragma unroll
  for (int l = 1; l < T::D; ++l) {
#pragma unroll
    for (int i = 0; i < T::W; ++i) x[i] = y[i];
    dense_state<T, T::W, T::W>(T::off(l), s, x, y, lane);
  }
#pragma unroll
  for (int i = 0; i < T::W; ++i) x[i] = y[i];
  dense_state<T, T::W, T::A>(T::off(T::D), s, x, h, lane);
}

template <class T>
__device__ bool finite_all(const float* v) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < T::A; ++i) ok &= finitef(v[i]);
  return ok;
}
template <class T>
__device__ bool close_all(const float* a, const float* b, float eps) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < T::A; ++i) ok &= !(fabsf(a[i] - b[i]) >= eps);
  return ok;
}
template <class T>
__device__ bool lds_finite(const float* sw, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) ok &= finitef(sw[k]);
  return wave_all(ok);
}
// |state-expanded(s) - lds weights| < eps for every weight
template <class T>
__device__ bool lds_close_state(const float* sw, const float* s, float eps, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) {
    const int c = T::chunk(k);
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < T::A; ++q) v = (c == q) ? s[q] : v;
    ok &= !(fabsf(v - sw[k]) >= eps);
  }
  return wave_all(ok);
}
template <class T>
__device__ bool lds_zero(const float* sw, float eps, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) ok &= (-eps <= sw[k]) && (sw[k] <= eps);
  return wave_all(ok);
}

// classification of general (LDS) weights: f = f_W(W) = expand(h1), f2 = expand(h2)
template <class T>
__device__ int8_t classify_lds(const float* sw, float eps, bool with_sec, int aggregator, int lane) {
  if (!lds_finite<T>(sw, lane)) return C_DIVERGENT;
  float g[T::A], h1[T::A], h2[T::A];
  aggregate_lds<T>(sw, g, lane, aggregator);
  mlp_lds<T>(sw, g, h1, lane);
  if (finite_all<T>(h1) && lds_close_state<T>(sw, h1, eps, lane))
    return lds_zero<T>(sw, eps, lane) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    mlp_lds<T>(sw, h1, h2, lane);  // aggregate(expand(h1)) == h1 exactly
    if (finite_all<T>(h2) && lds_close_state<T>(sw, h2, eps, lane)) return C_FIX_SEC;
  }
  return C_OTHER;
}
// classification of chunk-constant weights expand(s)
template <class T>
__device__ int8_t classify_state(const float* s, float eps, bool with_sec, int lane) {
  if (!finite_all<T>(s)) return C_DIVERGENT;
  float h1[T::A], h2[T::A];
  mlp_state<T>(s, s, h1, lane);
  if (finite_all<T>(h1) && close_all<T>(h1, s, eps)) {
    bool zero = true;
#pragma unroll
    for (int i = 0; i < T::A; ++i) zero &= (-eps <= s[i]) && (s[i] <= eps);
    return zero ? C_FIX_ZERO : C_FIX_OTHER;
  }
  if (with_sec) {
    mlp_state<T>(s, h1, h2, lane);
    if (finite_all<T>(h2) && close_all<T>(h2, s, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}

// one SGD step on x = y = aggregate(own or teacher weights); weights in LDS (updated)
template <class T>
__device__ float train_step_lds(float* sw, WaveLds<T>& L, const float* g, float lr, int lane) {
  // forward keeping every layer input
  float x[T::MAXW], y[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
#pragma unroll
  for (int l = 0; l <= T::D; ++l) {
    if (lane < T::rows(l)) {
      float v = x[0];
#pragma unroll
      for (int i = 1; i < T::MAXW; ++i) v = (lane == i) ? x[i] : v;
      L.act[l][lane] = v;
    }
    if (l == 0) dense_lds<T::A, T::W>(sw + T::off(0), x, y, lane);
    else if (l < T::D) dense_lds<T::W, T::W>(sw + T::off(l), x, y, lane);
    else dense_lds<T::W, T::A>(sw + T::off(T::D), x, y, lane);
#pragma unroll
    for (int i = 0; i < T::MAXW; ++i) x[i] = y[i];
  }
  // loss mean over A, step = -lr * dL/dh
  float loss = 0.f;
  float st = 0.f;
#pragma unroll
  for (int k = 0; k < T::A; ++k) {
    const float e = x[k] - g[k];
    loss += e * e;
    if (lane == k) st = -lr * (2.0f * e / (float)T::A);
  }
  if (lane < T::A) L.st[lane] = st;
  __builtin_amdgcn_wave_barrier();
  // backward: st_in = K . st_out (pre-update K), K += act (x) st_out
#pragma unroll
  for (int l = T::D; l >= 0; --l) {
    const int R = T::rows(l), Cc = T::cols(l);
    float* k = sw + T::off(l);
    if (l > 0 && lane < R) {
      float acc = k[lane * Cc] * L.st[0];
      for (int j = 1; j < Cc; ++j) acc = fmaf(k[lane * Cc + j], L.st[j], acc);
      L.st2[lane] = acc;
    }
    __builtin_amdgcn_wave_barrier();
    for (int f = lane; f < R * Cc; f += 64) {
      const int i = f / Cc, j = f - i * Cc;
      k[f] = fmaf(L.act[l][i], L.st[j], k[f]);
    }
    __builtin_amdgcn_wave_barrier();
    if (l > 0 && lane < R) L.st[lane] = L.st2[lane];
    __builtin_amdgcn_wave_barrier();
  }
  return loss / (float)T::A;
}

// ------------------------------------------------------------------------------ kernel
template <class T, int OP>
__global__ __launch_bounds__(TBB) void k_big(SrnnCfg c, SrnnArgs a) {
  __shared__ WaveLds<T> lds[BW];
  __shared__ uint32_t s_cnt[5];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * BW + wv;  // particle (wave-uniform)
  WaveLds<T>& L = lds[wv];
  if (OP == OP_CLASSIFY && threadIdx.x < 5) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  int8_t cls = -1;
  if (p < a.n) {
    if constexpr (OP == OP_APPLY) {
      const int64_t fi = a.idx_f ? a.idx_f[p] : p, ti = a.idx_t ? a.idx_t[p] : p, oi = a.idx_o ? a.idx_o[p] : p;
      // both rows in flight at once, then aggregate the target and run the attacker's net
      {
        const float4* f4 = reinterpret_cast<const float4*>(a.W + fi * T::PP);
        const float4* t4 = reinterpret_cast<const float4*>(a.W + ti * T::PP);
        float4* sw4 = reinterpret_cast<float4*>(L.w);
        float4* st4 = reinterpret_cast<float4*>(L.t);
        for (int q = lane; q < T::PP / 4; q += 64) {
          const float4 x = f4[q], y = t4[q];
          sw4[q] = x;
          st4[q] = y;
        }
      }
      __builtin_amdgcn_wave_barrier();
      float g[T::A], h[T::A];
      aggregate_lds<T>(L.t, g, lane, c.aggregator);
      mlp_lds<T>(L.w, g, h, lane);
      store_state<T>(a.W2 + oi * T::PP, h, lane);
    } else if constexpr (OP == OP_RUN_FIXPOINT || OP == OP_CLASSIFY) {
      load_row<T>(L.w, a.W + p * T::PP, lane);
      __builtin_amdgcn_wave_barrier();
      const bool with_sec = (a.flags & SRNN_F_FIX_SEC) != 0;
      int s = 0;
      float st[T::A];
      bool compressed = false;
      if constexpr (OP == OP_RUN_FIXPOINT) {
        float g[T::A], h[T::A];
        for (; s < a.steps; ++s) {
          if (!compressed) {
            if (a.early_exit && !lds_finite<T>(L.w, lane)) break;
            aggregate_lds<T>(L.w, g, lane, c.aggregator);
            mlp_lds<T>(L.w, g, h, lane);
            if (a.early_exit && finite_all<T>(h) && lds_close_state<T>(L.w, h, a.eps, lane)) break;
          } else {
            if (a.early_exit && !finite_all<T>(st)) break;
            mlp_state<T>(st, st, h, lane);
            if (a.early_exit && finite_all<T>(h) && close_all<T>(h, st, a.eps)) break;
          }
#pragma unroll
          for (int i = 0; i < T::A; ++i) st[i] = h[i];
          compressed = true;
        }
        if (compressed) store_state<T>(a.W + p * T::PP, st, lane);
        if (a.nsteps && lane == 0) a.nsteps[p] = s;
      }
      cls = compressed ? classify_state<T>(st, a.eps, with_sec, lane)
                       : classify_lds<T>(L.w, a.eps, with_sec, c.aggregator, lane);
      if (a.cls && lane == 0) a.cls[p] = cls;
    } else if constexpr (OP == OP_TRAIN || OP == OP_LEARN) {
      load_row<T>(L.w, a.W + p * T::PP, lane);
      float g[T::A];
      if constexpr (OP == OP_LEARN) {
        // teacher samples are fixed: aggregate the teacher row once (through L.act as scratch)
        const float* tr = a.W2 + (a.idx_t ? a.idx_t[p] : p) * T::PP;
        if (c.aggregator != 0) {  // max aggregators: stage the teacher row, sequential semantics
          load_row<T>(L.t, tr, lane);
          __builtin_amdgcn_wave_barrier();
          aggregate_lds<T>(L.t, g, lane, c.aggregator);
        }
        double acc[T::A];
#pragma unroll
        for (int q = 0; q < T::A; ++q) acc[q] = 0.0;
        for (int k = lane; k < T::P; k += 64) {
          const int ch = T::chunk(k);
#pragma unroll
          for (int q = 0; q < T::A; ++q) acc[q] += (ch == q) ? (double)tr[k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < T::A; ++q) {
          const int b = q * T::CS, e = (q == T::A - 1) ? T::P : b + T::CS;
          const float mean = (float)(wave_sum(acc[q]) / (double)(e - b));
          if (c.aggregator == 0) g[q] = mean;
        }
      }
      __builtin_amdgcn_wave_barrier();
      float loss = 0.f;
      for (int e = 0; e < a.epochs; ++e) {
        if constexpr (OP == OP_TRAIN) aggregate_lds<T>(L.w, g, lane, c.aggregator);
        loss = train_step_lds<T>(L.w, L, g, a.lr, lane);
      }
      __builtin_amdgcn_wave_barrier();
      store_lds<T>(a.W + p * T::PP, L.w, lane);
      if (a.loss && lane == 0) a.loss[p] = loss;
    }
  }
  if constexpr (OP == OP_CLASSIFY) {
    if (a.counts && lane == 0 && cls >= 0) atomicAdd(&s_cnt[cls], 1u);
    __syncthreads();
    if (a.counts && threadIdx.x < 5 && s_cnt[threadIdx.x]) atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
  }
}

// ------------------------------------------------------------------ run_fixpoint, 3 phases
// phase 1 (wave per particle): step-0 checks and the first application on the full row;
// phase 2 (lane per particle): every further step on the A-float chunk state, with the
//   chunk index of every weight a compile-time constant (fully unrolled MLP);
// phase 3 (wave per particle): expand the final state into the row, coalesced.
// temp = state float[n][A] followed by flags int8[n] (1 = continues in phase 2).

template <class T, int L>
__device__ __forceinline__ void dense_state_lane(const float* s, const float* x, float* y) {
  constexpr int I = T::rows(L), O = T::cols(L), OFF = T::off(L);
#pragma unroll
  for (int j = 0; j < O; ++j) {
    float acc = x[0] * s[T::chunk_c(OFF + j)];
#pragma unroll
    for (int i = 1; i < I; ++i) acc = fmaf(x[i], s[T::chunk_c(OFF + i * O + j)], acc);
    y[j] = acc;
  }
}
template <class T, int L>
__device__ __forceinline__ void mlp_state_lane_rec(const float* s, float* x) {
  float y[T::MAXW];
  dense_state_lane<T, L>(s, x, y);
#pragma unroll
  for (int j = 0; j < T::cols(L); ++j) x[j] = y[j];
  if constexpr (L < T::D) mlp_state_lane_rec<T, L + 1>(s, x);
}
template <class T>
__device__ __forceinline__ void mlp_state_lane(const float* s, const float* g, float* h) {
  float x[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
  mlp_state_lane_rec<T, 0>(s, x);
#pragma unroll
  for (int i = 0; i < T::A; ++i) h[i] = x[i];
}

template <class T>
__global__ __launch_bounds__(TBB) void k_big_fix1(SrnnCfg c, SrnnArgs a) {
  __shared__ WaveLds<T> lds[BW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * BW + wv;
  if (p >= a.n) return;
  WaveLds<T>& L = lds[wv];
  float* state = reinterpret_cast<float*>(a.temp);
  int8_t* flag = reinterpret_cast<int8_t*>(state + a.n * T::A);
  load_row<T>(L.w, a.W + p * T::PP, lane);
  __builtin_amdgcn_wave_barrier();
  const bool with_sec = (a.flags & SRNN_F_FIX_SEC) != 0;
  bool stop = a.steps <= 0;
  float g[T::A], h[T::A];
  if (!stop && a.early_exit && !lds_finite<T>(L.w, lane)) stop = true;
  if (!stop) {
    aggregate_lds<T>(L.w, g, lane, c.aggregator);
    mlp_lds<T>(L.w, g, h, lane);
    if (a.early_exit && finite_all<T>(h) && lds_close_state<T>(L.w, h, a.eps, lane)) stop = true;
  }
  if (stop) {  // no step taken: the row is unchanged, classify the general weights
    const int8_t k = classify_lds<T>(L.w, a.eps, with_sec, c.aggregator, lane);
    if (lane == 0) {
      flag[p] = 0;
      if (a.nsteps) a.nsteps[p] = 0;
      if (a.cls) a.cls[p] = k;
    }
  } else if (lane < T::A) {
    float v = h[0];
#pragma unroll
    for (int q = 1; q < T::A; ++q) v = (lane == q) ? h[q] : v;
    state[p * T::A + lane] = v;
    if (lane == 0) flag[p] = 1;
  }
}

template <class T>
__global__ __launch_bounds__(256) void k_big_fix2(SrnnCfg c, SrnnArgs a) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= a.n) return;
  float* state = reinterpret_cast<float*>(a.temp);
  const int8_t* flag = reinterpret_cast<const int8_t*>(state + a.n * T::A);
  if (!flag[p]) return;
  float st[T::A], h[T::A];
#pragma unroll
  for (int i = 0; i < T::A; ++i) st[i] = state[p * T::A + i];
  int taken = 1;
  for (int k = 1; k < a.steps; ++k) {
    if (a.early_exit && !finite_all<T>(st)) break;
    mlp_state_lane<T>(st, st, h);
    if (a.early_exit && finite_all<T>(h) && close_all<T>(h, st, a.eps)) break;
#pragma unroll
    for (int i = 0; i < T::A; ++i) st[i] = h[i];
    ++taken;
  }
#pragma unroll
  for (int i = 0; i < T::A; ++i) state[p * T::A + i] = st[i];
  if (a.nsteps) a.nsteps[p] = taken;
  if (a.cls) {
    // classify the chunk-constant weights expand(st)
    int8_t k;
    if (!finite_all<T>(st)) k = C_DIVERGENT;
    else {
      float h1[T::A], h2[T::A];
      mlp_state_lane<T>(st, st, h1);
      if (finite_all<T>(h1) && close_all<T>(h1, st, a.eps)) {
        bool zero = true;
#pragma unroll
        for (int i = 0; i < T::A; ++i) zero &= (-a.eps <= st[i]) && (st[i] <= a.eps);
        k = zero ? C_FIX_ZERO : C_FIX_OTHER;
      } else {
        k = C_OTHER;
        if (a.flags & SRNN_F_FIX_SEC) {
          mlp_state_lane<T>(st, h1, h2);
          if (finite_all<T>(h2) && close_all<T>(h2, st, a.eps)) k = C_FIX_SEC;
        }
      }
    }
    a.cls[p] = k;
  }
}

template <class T>
__global__ __launch_bounds__(TBB) void k_big_fix3(SrnnCfg c, SrnnArgs a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * BW + wv;
  if (p >= a.n) return;
  const float* state = reinterpret_cast<const float*>(a.temp);
  const int8_t* flag = reinterpret_cast<const int8_t*>(state + a.n * T::A);
  if (!flag[p]) return;
  float st[T::A];
#pragma unroll
  for (int i = 0; i < T::A; ++i) st[i] = state[p * T::A + i];
  store_state<T>(a.W + p * T::PP, st, lane);
}

// lane-per-particle ops writing straight to global memory (init, perturb)
template <class T, int OP>
__global__ __launch_bounds__(256) void k_big_lane(SrnnCfg c, SrnnArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  float* row = a.W + i * T::PP;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const uint64_t uid = a.uid ? (uint64_t)a.uid[i] : (uint64_t)i;
  if constexpr (OP == OP_INIT) {
    glorot_fill(row, 0, T::A, T::W, rng, uid);
    for (int l = 1; l < T::D; ++l) glorot_fill(row, T::off(l), T::W, T::W, rng, uid);
    glorot_fill(row, T::off(T::D), T::W, T::A, rng, uid);
    for (int k = T::P; k < T::PP; ++k) row[k] = 0.f;
  } else {
    for (int k = 0; k < T::P; ++k) {
      U4 u = rng.draw(uid, a.ctr * 1024u + (uint32_t)k, P_PERTURB);
      double mag = (double)u01(u.y) * (double)a.eps;
      row[k] = u01(u.x) < 0.5f ? (float)((double)row[k] + mag) : (float)((double)row[k] - mag);
    }
  }
}

// ------------------------------------------------------------------ lane per particle
// classify / attack / train with the particle's whole row in VGPRs (P = 280 floats:
// ~360 VGPRs, one wave per SIMD): every lane does useful work instead of the 10 of 64
// lanes of the wave-per-particle layers, and the kernels become HBM-bound (1.1 KB row per
// particle).  Arithmetic in the same order as the wave kernels (dense: x[0]*k then fma
// over the inputs; chunk means as double sums, here in index order).
template <class T>
__device__ __forceinline__ void lrow_load(const float* __restrict__ row, float (&w)[T::P]) {
  const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll
  for (int q = 0; q < T::PP / 4; ++q) {
    const float4 v = r4[q];
    if (4 * q + 0 < T::P) w[4 * q + 0] = v.x;
    if (4 * q + 1 < T::P) w[4 * q + 1] = v.y;
    if (4 * q + 2 < T::P) w[4 * q + 2] = v.z;
    if (4 * q + 3 < T::P) w[4 * q + 3] = v.w;
  }
}
template <class T>
__device__ __forceinline__ void lrow_store(float* __restrict__ row, const float (&w)[T::P]) {
  float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
  for (int q = 0; q < T::PP / 4; ++q) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (4 * q + e < T::P) ? w[4 * q + e] : 0.f;
    r4[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
}
template <class T>
__device__ __forceinline__ void lrow_store_state(float* __restrict__ row, const float* h) {
  float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
  for (int q = 0; q < T::PP / 4; ++q) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (4 * q + e < T::P) ? h[T::chunk_c(4 * q + e)] : 0.f;
    r4[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
}
// chunk aggregation of a register row (reference: python-float sums / sequential max)
template <class T>
__device__ __forceinline__ void lrow_aggregate(const float (&w)[T::P], float* g, int aggregator) {
#pragma unroll
  for (int c = 0; c < T::A; ++c) {
    constexpr int dummy = 0;
    (void)dummy;
    const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
    if (aggregator == 0) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < T::P; ++k)
        if (k >= b && k < e) acc += (double)w[k];
      g[c] = (float)(acc / (double)(e - b));
    } else {
      float m = w[b];
#pragma unroll
      for (int k = 0; k < T::P; ++k)
        if (k >= b && k < e) m = (aggregator == 1) ? (w[k] > m ? w[k] : m) : ((w[k] > m && w[k] != 0.0f) ? w[k] : m);
      g[c] = m;
    }
  }
}
// aggregation of a streamed row (attack target / teacher): float4 by float4 into the
// chunk accumulators (same per-chunk order as lrow_aggregate), the row is never held
template <class T>
__device__ __forceinline__ void lstream_aggregate(const float* __restrict__ row, float* g, int aggregator) {
  const float4* r4 = reinterpret_cast<const float4*>(row);
  double acc[T::A];
  float m[T::A];
#pragma unroll
  for (int c = 0; c < T::A; ++c) acc[c] = 0.0;
#pragma unroll
  for (int q = 0; q < T::PP / 4; ++q) {
    const float4 v4 = r4[q];
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * q + e;
      if (k >= T::P) continue;
      const int c = T::chunk_c(k);
      if (aggregator == 0) {
        acc[c] += (double)v[e];
      } else if (k == c * T::CS) {
        m[c] = v[e];
      } else {
        m[c] = (aggregator == 1) ? (v[e] > m[c] ? v[e] : m[c]) : ((v[e] > m[c] && v[e] != 0.0f) ? v[e] : m[c]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < T::A; ++c) {
    const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
    g[c] = aggregator == 0 ? (float)(acc[c] / (double)(e - b)) : m[c];
  }
}
template <class T, int L>
__device__ __forceinline__ void lmlp_rec(const float (&w)[T::P], float* x) {
  constexpr int I = T::rows(L), O = T::cols(L), OFF = T::off(L);
  float y[T::MAXW];
#pragma unroll
  for (int j = 0; j < O; ++j) {
    float acc = x[0] * w[OFF + j];
#pragma unroll
    for (int i = 1; i < I; ++i) acc = fmaf(x[i], w[OFF + i * O + j], acc);
    y[j] = acc;
  }
#pragma unroll
  for (int j = 0; j < O; ++j) x[j] = y[j];
  if constexpr (L < T::D) lmlp_rec<T, L + 1>(w, x);
}
template <class T>
__device__ __forceinline__ void lmlp(const float (&w)[T::P], const float* g, float* h) {
  float x[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
  lmlp_rec<T, 0>(w, x);
#pragma unroll
  for (int i = 0; i < T::A; ++i) h[i] = x[i];
}
template <class T>
__device__ __forceinline__ bool lrow_close_state(const float (&w)[T::P], const float* h, float eps) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < T::P; ++k) ok &= !(fabsf(h[T::chunk_c(k)] - w[k]) >= eps);
  return ok;
}
// One pass over a register row for the census: chunk sums (double, index order = the mean
// aggregator's sums), per-chunk min / max.  Every census predicate is a function of these:
//   all weights finite   <=> every chunk sum finite (a NaN or an infinity in a chunk makes its
//                            double sum non-finite; finite floats cannot overflow a double sum)
//   all |w| <= eps       <=> min >= -eps and max <= eps
//   all |h[c(k)] - w[k]| < eps  <=>  h[c] - min_c < eps and max_c - h[c] < eps for every chunk:
//     fl(h - w) is monotone in w and fl(w - h) = -fl(h - w), so the largest rounded distance of
//     a chunk is attained at its min or max -- the same decisions as the per-weight test with
//     ~16 instead of ~1100 instructions (the per-weight compares made the census issue-bound)
template <class T>
struct RowSummary {
  double sum[T::A];
  float mn[T::A], mx[T::A];
  __device__ __forceinline__ explicit RowSummary(const float (&w)[T::P]) {
#pragma unroll
    for (int c = 0; c < T::A; ++c) {
      const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
      double acc = 0.0;  // index order (the reference's sums)
      float lo[4] = {w[b], w[b], w[b], w[b]}, hi[4] = {w[b], w[b], w[b], w[b]};  // order-free: 4 chains
#pragma unroll
      for (int k = 0; k < T::P; ++k)
        if (k >= b && k < e) {
          acc += (double)w[k];
          lo[k & 3] = fminf(lo[k & 3], w[k]);
          hi[k & 3] = fmaxf(hi[k & 3], w[k]);
        }
      sum[c] = acc;
      mn[c] = fminf(fminf(lo[0], lo[1]), fminf(lo[2], lo[3]));
      mx[c] = fmaxf(fmaxf(hi[0], hi[1]), fmaxf(hi[2], hi[3]));
    }
  }
  __device__ __forceinline__ bool finite() const {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < T::A; ++c) ok &= __builtin_isfinite(sum[c]) != 0;
    return ok;
  }
  __device__ __forceinline__ bool zero(float eps) const {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < T::A; ++c) ok &= (-eps <= mn[c]) && (mx[c] <= eps);
    return ok;
  }
  // every |expand(h)[k] - w[k]| < eps (h finite, w finite)
  __device__ __forceinline__ bool close(const float* h, float eps) const {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < T::A; ++c) ok &= !(h[c] - mn[c] >= eps) && !(mx[c] - h[c] >= eps);
    return ok;
  }
  // chunk means (aggregator 0) exactly as lrow_aggregate; the max aggregators walk the row
  __device__ __forceinline__ void aggregate(const float (&w)[T::P], float* g, int aggregator) const {
    if (aggregator == 0) {
#pragma unroll
      for (int c = 0; c < T::A; ++c) {
        const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
        g[c] = (float)(sum[c] / (double)(e - b));
      }
    } else {
      lrow_aggregate<T>(w, g, aggregator);
    }
  }
};

template <class T>
__device__ __forceinline__ int8_t lclassify(const float (&w)[T::P], float eps, bool with_sec, int aggregator) {
  bool fin = true;
#pragma unroll
  for (int k = 0; k < T::P; ++k) fin &= finitef(w[k]);
  if (!fin) return C_DIVERGENT;
  float g[T::A], h1[T::A], h2[T::A];
  lrow_aggregate<T>(w, g, aggregator);
  lmlp<T>(w, g, h1);
  if (finite_all<T>(h1) && lrow_close_state<T>(w, h1, eps)) {
    bool zero = true;
#pragma unroll
    for (int k = 0; k < T::P; ++k) zero &= (-eps <= w[k]) && (w[k] <= eps);
    return zero ? C_FIX_ZERO : C_FIX_OTHER;
  }
  if (with_sec) {
    lmlp<T>(w, h1, h2);  // aggregate(expand(h1)) == h1 exactly
    if (finite_all<T>(h2) && lrow_close_state<T>(w, h2, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}
// one SGD step on x = y = g (same order as train_step_lds)
template <class T>
__device__ __forceinline__ float ltrain_step(float (&w)[T::P], const float* g, float lr) {
  float act[T::NL][T::MAXW];
  float x[T::MAXW];
#pragma unroll
  for (int i = 0; i < T::A; ++i) x[i] = g[i];
#pragma unroll
  for (int l = 0; l <= T::D; ++l) {
#pragma unroll
    for (int i = 0; i < T::MAXW; ++i) act[l][i] = x[i];
    const int I = T::rows(l), O = T::cols(l), OFF = T::off(l);
    float y[T::MAXW];
#pragma unroll
    for (int j = 0; j < T::MAXW; ++j) {
      if (j < O) {
        float acc = x[0] * w[OFF + j];
#pragma unroll
        for (int i = 1; i < T::MAXW; ++i)
          if (i < I) acc = fmaf(x[i], w[OFF + i * O + j], acc);
        y[j] = acc;
      } else {
        y[j] = 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < T::MAXW; ++j) x[j] = y[j];
  }
  float loss = 0.f, st[T::MAXW], st2[T::MAXW];
#pragma unroll
  for (int k = 0; k < T::MAXW; ++k) st[k] = 0.f;
#pragma unroll
  for (int k = 0; k < T::A; ++k) {
    const float e = x[k] - g[k];
    loss += e * e;
    st[k] = -lr * (2.0f * e / (float)T::A);
  }
#pragma unroll
  for (int l = T::D; l >= 0; --l) {
    const int R = T::rows(l), Cc = T::cols(l), OFF = T::off(l);
    if (l > 0) {
#pragma unroll
      for (int i = 0; i < T::MAXW; ++i) {
        if (i < R) {
          float acc = w[OFF + i * Cc] * st[0];
#pragma unroll
          for (int j = 1; j < T::MAXW; ++j)
            if (j < Cc) acc = fmaf(w[OFF + i * Cc + j], st[j], acc);
          st2[i] = acc;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < T::MAXW; ++i)
#pragma unroll
      for (int j = 0; j < T::MAXW; ++j)
        if (i < R && j < Cc) w[OFF + i * Cc + j] = fmaf(act[l][i], st[j], w[OFF + i * Cc + j]);
    if (l > 0) {
#pragma unroll
      for (int i = 0; i < T::MAXW; ++i) st[i] = (i < R) ? st2[i] : 0.f;
    }
  }
  return loss / (float)T::A;
}

constexpr int TBROW = 256;  // 4 waves: one per SIMD at ~360 VGPRs

// ---- coalesced row staging through LDS --------------------------------------------------
// A lane-per-row load has every wave instruction fetch 16-byte pieces of 64 rows 1120 B
// apart (64 cache lines per instruction): 3.9 TB/s measured on 1M rows.  Staged, the wave
// moves its 64 rows in passes of Q 16-byte pieces per row: piece slot k of lane L is piece
// (64 k + L) % Q of row (64 k + L) / Q, so one wave instruction covers ~64/Q consecutive row
// segments (5.6-5.8 TB/s, the streaming-read ceiling 5.85; bench/micro/row_load.hip), goes
// through this wave's LDS area (row pitch Q|1 pieces: an odd multiple of 4 dwords, so the
// 16 lanes of a ds_read_b128 quarter-wave hit distinct bank groups) and each lane then reads
// its own row segment.  Rows are addressed by a 32-bit index into one table (idx < 0: no
// row); every lane of the wave must execute the call (wave-uniform control flow).
#ifndef SRNN_STAGE_Q
#define SRNN_STAGE_Q 18
#endif
template <int NQ>  // 16-byte pieces per row
struct Stage {
  static constexpr int Q = SRNN_STAGE_Q < NQ ? SRNN_STAGE_Q : NQ;
  static constexpr int PI = Q | 1;
  static constexpr int NPASS = (NQ + Q - 1) / Q;
  static constexpr int WAVE_U4 = 64 * PI;  // LDS uint4 per wave
  static constexpr int len(int s) { return NQ - Q * s < Q ? NQ - Q * s : Q; }
};
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// per piece slot k: the row index of its owner lane and the piece within the pass (every
// loop over slots / pieces is a compile-time fold: a runtime index into these arrays or into
// the row registers would put them in scratch memory)
template <int NQ>
struct StageMap {
  static constexpr int Q = Stage<NQ>::Q, PI = Stage<NQ>::PI;
  int32_t rk[Q];
  int32_t fk[Q];
  template <int K>
  __device__ __forceinline__ void set(int32_t idx, int L) {
    const int t = 64 * K + L, r = t / Q;
    fk[K] = t - r * Q;
    rk[K] = __shfl(idx, r);
  }
  template <int... K>
  __device__ __forceinline__ void init(int32_t idx, int L, std::integer_sequence<int, K...>) {
    (set<K>(idx, L), ...);
  }
  __device__ __forceinline__ StageMap(int32_t idx, int L) { init(idx, L, std::make_integer_sequence<int, Q>{}); }
  // LDS slot (uint4) of piece slot k: row r at r * PI + f
  __device__ __forceinline__ static int lds_slot(int k, int L) {
    const int t = 64 * k + L, r = t / Q;
    return r * PI + (t - r * Q);
  }
};
template <int NQ, int S, int K>
__device__ __forceinline__ uint4 stage_fetch(const char* __restrict__ base, const StageMap<NQ>& m) {
  constexpr int Q = Stage<NQ>::Q, LEN = Stage<NQ>::len(S);
  constexpr int64_t RB = (int64_t)NQ * 16;
  const bool ok = m.rk[K] >= 0 && m.fk[K] < LEN;  // else a harmless load of piece 0 of row 0
  const int64_t off = ok ? (int64_t)m.rk[K] * RB + (int64_t)(Q * S + m.fk[K]) * 16 : 0;
  return *reinterpret_cast<const uint4*>(base + off);
}
template <int NQ, int S, int K>
__device__ __forceinline__ void stage_put(char* __restrict__ base, const StageMap<NQ>& m, const uint4* st, int L) {
  constexpr int Q = Stage<NQ>::Q, LEN = Stage<NQ>::len(S);
  constexpr int64_t RB = (int64_t)NQ * 16;
  const uint4 v = st[StageMap<NQ>::lds_slot(K, L)];
  if (m.rk[K] >= 0 && m.fk[K] < LEN)
    *reinterpret_cast<uint4*>(base + (int64_t)m.rk[K] * RB + (int64_t)(Q * S + m.fk[K]) * 16) = v;
}
// pass S of a staged load in two halves: fetch (the wave's global loads, into registers)
// and commit (after every lane's reads of the previous pass: pieces to LDS, wave barrier).
// The loads of pass S + 1 are issued before pass S is committed, so a wave keeps one pass of
// loads in flight while it stages and decodes the previous one.
template <int NQ>
struct StageBuf {
  uint4 v[Stage<NQ>::Q];
};
template <int NQ, int S, int... K>
__device__ __forceinline__ StageBuf<NQ> stage_fetch_(const char* __restrict__ base, const StageMap<NQ>& m,
                                                     std::integer_sequence<int, K...>) {
  return StageBuf<NQ>{{stage_fetch<NQ, S, K>(base, m)...}};
}
template <int NQ, int S>
__device__ __forceinline__ StageBuf<NQ> stage_fetch_pass(const char* __restrict__ base, const StageMap<NQ>& m) {
  return stage_fetch_<NQ, S>(base, m, std::make_integer_sequence<int, Stage<NQ>::Q>{});
}
template <int NQ, int... K>
__device__ __forceinline__ void stage_commit_(const StageBuf<NQ>& b, uint4* st, int L, std::integer_sequence<int, K...>) {
  wave_lds_sync();  // every lane is done reading the previous pass's segment
  ((st[StageMap<NQ>::lds_slot(K, L)] = b.v[K]), ...);
  wave_lds_sync();
}
template <int NQ>
__device__ __forceinline__ void stage_commit(const StageBuf<NQ>& b, uint4* st, int L) {
  stage_commit_<NQ>(b, st, L, std::make_integer_sequence<int, Stage<NQ>::Q>{});
}
template <int NQ, int S, int... K>
__device__ __forceinline__ void stage_pass_out_(char* __restrict__ base, const StageMap<NQ>& m, const uint4* st, int L,
                                                std::integer_sequence<int, K...>) {
  wave_lds_sync();
  (stage_put<NQ, S, K>(base, m, st, L), ...);
  wave_lds_sync();
}
template <int NQ, int S>
__device__ __forceinline__ void stage_pass_out(char* __restrict__ base, const StageMap<NQ>& m, const uint4* st, int L) {
  stage_pass_out_<NQ, S>(base, m, st, L, std::make_integer_sequence<int, Stage<NQ>::Q>{});
}

template <class T, class S> struct BRow;
// census class of a register row from its summary (no shuffler): f1 = apply(w, w), f2 =
// apply(w, f1) with aggregate(expand(f1)) == f1, both rounded to the storage format
template <class T, class S>
__device__ __forceinline__ int8_t sclassify(const float (&w)[T::P], const RowSummary<T>& sm, float eps, bool with_sec,
                                            int aggregator) {
  if (!sm.finite()) return C_DIVERGENT;
  float g[T::A], h1[T::A], h2[T::A];
  sm.aggregate(w, g, aggregator);
  lmlp<T>(w, g, h1);
  BRow<T, S>::quant_a(h1);
  if (finite_all<T>(h1) && sm.close(h1, eps)) return sm.zero(eps) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    lmlp<T>(w, h1, h2);
    BRow<T, S>::quant_a(h2);
    if (finite_all<T>(h2) && sm.close(h2, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}
template <class T>
__global__ __launch_bounds__(TBROW) void k_big_fix1_row(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, StF32>;
  __shared__ uint4 s_stg[(TBROW / 64) * R::G::WAVE_U4];
  const int64_t p = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  if (blockIdx.x * (int64_t)TBROW + (threadIdx.x & ~63) >= a.n) return;  // whole wave past n
  float* state = reinterpret_cast<float*>(a.temp);
  int8_t* flag = reinterpret_cast<int8_t*>(state + a.n * T::A);
  float w[T::P];
  R::load_staged(a.W, p < a.n ? (int32_t)p : -1, w, s_stg + (threadIdx.x >> 6) * R::G::WAVE_U4);
  if (p >= a.n) return;
  const RowSummary<T> sm(w);
  bool stop = a.steps <= 0;
  if (!stop && a.early_exit) stop = !sm.finite();
  float g[T::A], h[T::A];
  if (!stop) {
    sm.aggregate(w, g, c.aggregator);
    lmlp<T>(w, g, h);
    // (a non-finite row never gets here with early_exit; without it the close test is off)
    if (a.early_exit && finite_all<T>(h) && sm.close(h, a.eps)) stop = true;
  }
  if (stop) {  // no step taken: the row is unchanged, classify the general weights
    flag[p] = 0;
    if (a.nsteps) a.nsteps[p] = 0;
    if (a.cls) a.cls[p] = sclassify<T, StF32>(w, sm, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, c.aggregator);
  } else {
#pragma unroll
    for (int i = 0; i < T::A; ++i) state[p * T::A + i] = h[i];
    flag[p] = 1;
  }
}
template <class T, int OP>
__global__ __launch_bounds__(TBROW) void k_big_row(SrnnCfg c, SrnnArgs a) {
  const int64_t p = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  float w[T::P];
  if constexpr (OP == OP_CLASSIFY) {
    __shared__ uint32_t s_cnt[5];
    if (threadIdx.x < 5) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    int8_t k = -1;
    if (p < a.n) {
      lrow_load<T>(a.W + p * T::PP, w);
      k = lclassify<T>(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, c.aggregator);
      if (a.cls) a.cls[p] = k;
    }
    if (a.counts) {  // histogram: wave ballots -> LDS -> one atomic per (block, class)
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const unsigned long long m = __ballot(k == q);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_cnt[q], (uint32_t)__popcll(m));
      }
      __syncthreads();
      if (threadIdx.x < 5 && s_cnt[threadIdx.x]) atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
    }
    return;
  }
  if (p >= a.n) return;
  if constexpr (OP == OP_APPLY) {
    const int64_t fi = a.idx_f ? a.idx_f[p] : p, ti = a.idx_t ? a.idx_t[p] : p, oi = a.idx_o ? a.idx_o[p] : p;
    float g[T::A], h[T::A];
    {  // target row into registers (all 70 loads in flight), aggregated, then dropped
      float t[T::P];
      lrow_load<T>(a.W + ti * T::PP, t);
      lrow_aggregate<T>(t, g, c.aggregator);
    }
    lrow_load<T>(a.W + fi * T::PP, w);
    lmlp<T>(w, g, h);
    lrow_store_state<T>(a.W2 + oi * T::PP, h);
  } else {  // OP_TRAIN / OP_LEARN
    float g[T::A];
    // teacher samples first (its row dies after the aggregation: one row live at a time)
    if constexpr (OP == OP_LEARN) lstream_aggregate<T>(a.W2 + (a.idx_t ? a.idx_t[p] : p) * T::PP, g, c.aggregator);
    lrow_load<T>(a.W + p * T::PP, w);
    float loss = 0.f;
    for (int e = 0; e < a.epochs; ++e) {
      if constexpr (OP == OP_TRAIN) lrow_aggregate<T>(w, g, c.aggregator);
      loss = ltrain_step<T>(w, g, a.lr);
    }
    lrow_store<T>(a.W + p * T::PP, w);
    if (a.loss) a.loss[p] = loss;
  }
}

// ==================================================================================
// Storage formats, shuffle_random and soups of the big nets (lane per particle).
//
// Rows are fp32, bf16 or fp16 (S = StF32 / StBF16 / StF16 of srnn_kernels.h): decoded to
// fp32 registers on load, rounded on every store and after every application, exactly
// where the runtime-shape engine rounds (g_quant / g_store of srnn_generic.hip), so a big
// net gives the same bits here as on the runtime-shape engine on the same device.
//
// shuffle_random (reference code/network.py:319-322, applied to the output of
// apply_to_weights): the output of an aggregating net is chunk-constant, out = expand(h),
// so the shuffled output out[k] = expand(h)[perm[k]] = h[chunk(perm[k])].  Fisher-Yates is
// therefore run directly on the CHUNK IDS (4 bits per weight, 35 words per lane in LDS)
// with the draws of fisher_yates(P_AGGSHUF): swapping entries of perm swaps the entries of
// chunk o perm, so no 280-entry index permutation is ever materialised.
// ==================================================================================
template <class T, class S>
struct BRow {
  static constexpr int RB = T::PP * S::BYTES;  // bytes per table row
  static constexpr int XB = RB + 16;           // exchange row: weights + (slot, gen) tags
  __device__ static const char* at(const float* base, int64_t i) {
    return reinterpret_cast<const char*>(base) + i * RB;
  }
  __device__ static char* at(float* base, int64_t i) { return reinterpret_cast<char*>(base) + i * RB; }
  __device__ static void load(const char* row, float (&w)[T::P]) {
    if constexpr (S::ID == 0) {
      // integer-typed loads (as for the 16-bit formats): with float loads the compiler
      // reorders/duplicates row loads across the soup kernel's control flow and spills
      const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
      for (int q = 0; q < T::PP / 4; ++q) {
        const uint4 v = r4[q];
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * q + e < T::P) w[4 * q + e] = __uint_as_float(u[e]);
      }
    } else {
      const uint2* r2 = reinterpret_cast<const uint2*>(row);
#pragma unroll
      for (int q = 0; q < T::PP / 4; ++q) {
        const uint2 v = r2[q];
        const uint16_t h[4] = {(uint16_t)(v.x & 0xffffu), (uint16_t)(v.x >> 16), (uint16_t)(v.y & 0xffffu),
                               (uint16_t)(v.y >> 16)};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * q + e < T::P) w[4 * q + e] = S::dec(h[e]);
      }
    }
  }
  __device__ static void store(char* row, const float (&w)[T::P]) {
    if constexpr (S::ID == 0) {
      uint4* r4 = reinterpret_cast<uint4*>(row);
#pragma unroll
      for (int q = 0; q < T::PP / 4; ++q) {
        uint32_t u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = (4 * q + e < T::P) ? __float_as_uint(w[4 * q + e]) : 0u;
        r4[q] = make_uint4(u[0], u[1], u[2], u[3]);
      }
    } else {
      uint2* r2 = reinterpret_cast<uint2*>(row);
#pragma unroll
      for (int q = 0; q < T::PP / 4; ++q) {
        uint32_t h[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = (4 * q + e < T::P) ? (uint32_t)S::enc(w[4 * q + e]) : 0u;
        r2[q] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
      }
    }
  }
  __device__ static void quant(float (&w)[T::P]) {
    if constexpr (S::ID != 0) {
#pragma unroll
      for (int k = 0; k < T::P; ++k) w[k] = S::q(w[k]);
    }
  }
  __device__ static void quant_a(float* h) {
    if constexpr (S::ID != 0) {
#pragma unroll
      for (int k = 0; k < T::A; ++k) h[k] = S::q(h[k]);
    }
  }
  // chunk aggregation of a streamed row (teacher / attack target): the row is never held
  __device__ static void stream_aggregate(const char* row, float* g, int aggregator) {
    {
      double acc[T::A];
      float m[T::A];
#pragma unroll
      for (int c = 0; c < T::A; ++c) acc[c] = 0.0, m[c] = 0.f;
#pragma unroll
      for (int q = 0; q < T::PP / 4; ++q) {
        float v[4];
        if constexpr (S::ID == 0) {
          const uint4 u = reinterpret_cast<const uint4*>(row)[q];
          v[0] = __uint_as_float(u.x), v[1] = __uint_as_float(u.y), v[2] = __uint_as_float(u.z),
          v[3] = __uint_as_float(u.w);
        } else {
          const uint2 u = reinterpret_cast<const uint2*>(row)[q];
          v[0] = S::dec((uint16_t)(u.x & 0xffffu)), v[1] = S::dec((uint16_t)(u.x >> 16)),
          v[2] = S::dec((uint16_t)(u.y & 0xffffu)), v[3] = S::dec((uint16_t)(u.y >> 16));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * q + e;
          if (k >= T::P) continue;
          const int c = T::chunk_c(k);
          if (aggregator == 0) acc[c] += (double)v[e];
          else if (k == c * T::CS) m[c] = v[e];
          else m[c] = (aggregator == 1) ? (v[e] > m[c] ? v[e] : m[c]) : ((v[e] > m[c] && v[e] != 0.0f) ? v[e] : m[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < T::A; ++c) {
        const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
        g[c] = aggregator == 0 ? (float)(acc[c] / (double)(e - b)) : m[c];
      }
    }
  }
  // glorot init of a particle straight into its (global) row: the draws and values of
  // glorot_fill / g_glorot, encoded to the storage format
  __device__ static void init_row(char* row, const Rng& rng, uint64_t uid) {
    for (int l = 0; l <= T::D; ++l) {
      const int r = T::rows(l), cc = T::cols(l), off = T::off(l), n = r * cc;
      const float lim = sqrtf(6.0f / (float)(r + cc));
      for (int b = 0; b < (n + 3) / 4; ++b) {
        const U4 u = rng.draw(uid, (uint32_t)off * 1024u + (uint32_t)b, P_INIT);
        const uint32_t xs[4] = {u.x, u.y, u.z, u.w};
        for (int q = 0; q < 4; ++q) {
          const int k = b * 4 + q;
          if (k < n) put(row, off + k, -lim + 2.0f * lim * u01(xs[q]));
        }
      }
    }
    for (int k = T::P; k < T::PP; ++k) put(row, k, 0.f);
  }
  __device__ static void put(char* row, int k, float v) {
    if constexpr (S::ID == 0) reinterpret_cast<float*>(row)[k] = v;
    else reinterpret_cast<uint16_t*>(row)[k] = S::enc(v);
  }
  // ---- staged (coalesced) row transfers: row idx of the table at base <-> w (see Stage)
  static constexpr int NQ = RB / 16;
  static_assert(RB % 16 == 0, "staged rows move 16-byte pieces");
  using G = Stage<NQ>;
  __device__ __forceinline__ static void dec_piece(int j, const uint4& u, float (&w)[T::P]) {
    if constexpr (S::ID == 0) {
      const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * j + e < T::P) w[4 * j + e] = __uint_as_float(x[e]);
    } else {
      const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * j + e < T::P) w[8 * j + e] = S::dec((uint16_t)((x[e >> 1] >> (16 * (e & 1))) & 0xffffu));
    }
  }
  __device__ __forceinline__ static uint4 enc_piece(int j, const float (&w)[T::P]) {
    uint32_t x[4];
    if constexpr (S::ID == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = (4 * j + e < T::P) ? __float_as_uint(w[4 * j + e]) : 0u;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t lo = (8 * j + 2 * e < T::P) ? (uint32_t)S::enc(w[8 * j + 2 * e]) : 0u;
        const uint32_t hi = (8 * j + 2 * e + 1 < T::P) ? (uint32_t)S::enc(w[8 * j + 2 * e + 1]) : 0u;
        x[e] = lo | (hi << 16);
      }
    }
    return make_uint4(x[0], x[1], x[2], x[3]);
  }
  template <int PS, int... Qi>
  __device__ __forceinline__ static void dec_pass(const uint4* st, int L, float (&w)[T::P], std::integer_sequence<int, Qi...>) {
    (dec_piece(G::Q * PS + Qi, st[L * G::PI + Qi], w), ...);
  }
  template <int PS>
  __device__ __forceinline__ static void load_passes(const char* base, const StageMap<NQ>& m, const StageBuf<NQ>& cur,
                                                     float (&w)[T::P], uint4* st, int L) {
    if constexpr (PS < G::NPASS) {
      if constexpr (PS + 1 < G::NPASS) {
        const StageBuf<NQ> nxt = stage_fetch_pass<NQ, PS + 1>(base, m);  // in flight during this pass
        stage_commit<NQ>(cur, st, L);
        dec_pass<PS>(st, L, w, std::make_integer_sequence<int, G::len(PS)>{});
        load_passes<PS + 1>(base, m, nxt, w, st, L);
      } else {
        stage_commit<NQ>(cur, st, L);
        dec_pass<PS>(st, L, w, std::make_integer_sequence<int, G::len(PS)>{});
      }
    }
  }
  // sources of a staged store: a register row, or the chunk state of a chunk-constant row
  struct RowSrc {
    const float (&w)[T::P];
    template <int J>
    __device__ __forceinline__ uint4 piece() const { return enc_piece(J, w); }
  };
  struct StateSrc {
    const float* s;  // T::A chunk values
    template <int J>
    __device__ __forceinline__ uint4 piece() const {
      constexpr int j = J;
      float v[8];
      constexpr int E = S::ID == 0 ? 4 : 8;
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = (E * j + e < T::P) ? s[T::chunk_c(E * j + e)] : 0.f;
      uint32_t x[4];
      if constexpr (S::ID == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = __float_as_uint(v[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (uint32_t)S::enc(v[2 * e]) | ((uint32_t)S::enc(v[2 * e + 1]) << 16);
      }
      return make_uint4(x[0], x[1], x[2], x[3]);
    }
  };
  template <int PS, class Src, int... Qi>
  __device__ __forceinline__ static void enc_pass(uint4* st, int L, const Src& src, std::integer_sequence<int, Qi...>) {
    ((st[L * G::PI + Qi] = src.template piece<G::Q * PS + Qi>()), ...);
  }
  template <int PS, class Src>
  __device__ __forceinline__ static void store_passes(char* base, const StageMap<NQ>& m, const Src& src, uint4* st, int L) {
    if constexpr (PS < G::NPASS) {
      enc_pass<PS>(st, L, src, std::make_integer_sequence<int, G::len(PS)>{});
      stage_pass_out<NQ, PS>(base, m, st, L);
      store_passes<PS + 1>(base, m, src, st, L);
    }
  }
  // w <- row idx of the table (idx < 0: w unchanged); st: this wave's G::WAVE_U4 LDS area
  __device__ __forceinline__ static void load_staged(const float* table, int32_t idx, float (&w)[T::P], uint4* st) {
    const int L = threadIdx.x & 63;
    const StageMap<NQ> m(idx, L);
    const char* base = reinterpret_cast<const char*>(table);
    load_passes<0>(base, m, stage_fetch_pass<NQ, 0>(base, m), w, st, L);
  }
  __device__ __forceinline__ static void store_staged(float* table, int32_t idx, const float (&w)[T::P], uint4* st) {
    const int L = threadIdx.x & 63;
    const StageMap<NQ> m(idx, L);
    store_passes<0>(reinterpret_cast<char*>(table), m, RowSrc{w}, st, L);
  }
  // row idx <- expand(s) (chunk state, T::A values)
  __device__ __forceinline__ static void store_state_staged(float* table, int32_t idx, const float* s, uint4* st) {
    const int L = threadIdx.x & 63;
    const StageMap<NQ> m(idx, L);
    store_passes<0>(reinterpret_cast<char*>(table), m, StateSrc{s}, st, L);
  }
};

// chunk ids of the shuffled output (4 bits per weight) in LDS, word w of lane L at
// cw[w * st + L] (st = the workgroup size; consecutive lanes -> consecutive banks)
template <class T>
struct ChunkPerm {
  static constexpr int NW = (T::P + 7) / 8;
  static_assert(T::A <= 16, "chunk ids are 4-bit");
  uint32_t* cw;
  int st = TBROW;  // LDS words between a lane's consecutive chunk-id words (= the workgroup size)
  __device__ uint32_t word(int w) const { return cw[w * st]; }
  __device__ int cid(int k) const { return (int)((cw[(k >> 3) * st] >> (4 * (k & 7))) & 15u); }
  // fisher_yates(perm, P, rng, id, step, P_AGGSHUF) applied to chunk(perm[k])
  __device__ void draw(const Rng& rng, uint64_t id, uint32_t step) const {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      uint32_t x = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * w + e < T::P) x |= (uint32_t)T::chunk_c(8 * w + e) << (4 * e);
      cw[w * st] = x;
    }
    U4 r{0, 0, 0, 0};
    int used = 4;
    uint32_t blk = 0;
    for (int i = T::P - 1; i > 0; --i) {
      if (used == 4) {
        r = rng.draw(id, step, P_AGGSHUF + (blk << 8));
        ++blk;
        used = 0;
      }
      const uint32_t x = used == 0 ? r.x : used == 1 ? r.y : used == 2 ? r.z : r.w;
      ++used;
      int j = (int)(u01(x) * (float)(i + 1));
      if (j > i) j = i;
      const int wi = i >> 3, wj = j >> 3, si = 4 * (i & 7), sj = 4 * (j & 7);
      const uint32_t xi = cw[wi * st], xj = cw[wj * st];
      const uint32_t d = ((xi >> si) ^ (xj >> sj)) & 15u;
      if (wi == wj) {
        cw[wi * st] = xi ^ (d << si) ^ (d << sj);
      } else {
        cw[wi * st] = xi ^ (d << si);
        cw[wj * st] = xj ^ (d << sj);
      }
    }
  }
};

// h[c] for a runtime chunk id c (A-way select, no dynamic register indexing)
template <class T>
__device__ __forceinline__ float pick(const float* h, int c) {
  float v = h[0];
#pragma unroll
  for (int q = 1; q < T::A; ++q) v = (c == q) ? h[q] : v;
  return v;
}
// w = expand(h) (chunk-constant) or its shuffled form h[chunk(perm[k])]
template <class T, bool SHUF>
__device__ __forceinline__ void expand_out(float (&w)[T::P], const float* h, const ChunkPerm<T>& cp) {
  if constexpr (SHUF) {
#pragma unroll
    for (int wd = 0; wd < ChunkPerm<T>::NW; ++wd) {
      const uint32_t x = cp.word(wd);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * wd + e < T::P) w[8 * wd + e] = pick<T>(h, (int)((x >> (4 * e)) & 15u));
    }
  } else {
#pragma unroll
    for (int k = 0; k < T::P; ++k) w[k] = h[T::chunk_c(k)];
  }
}
// every |expand'(h)[k] - w[k]| < eps (expand' = shuffled or plain)
template <class T, bool SHUF>
__device__ __forceinline__ bool close_out(const float (&w)[T::P], const float* h, float eps, const ChunkPerm<T>& cp) {
  bool ok = true;
  if constexpr (SHUF) {
#pragma unroll
    for (int wd = 0; wd < ChunkPerm<T>::NW; ++wd) {
      const uint32_t x = cp.word(wd);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * wd + e < T::P) ok &= !(fabsf(pick<T>(h, (int)((x >> (4 * e)) & 15u)) - w[8 * wd + e]) >= eps);
    }
  } else {
    ok = lrow_close_state<T>(w, h, eps);
  }
  return ok;
}
// chunk aggregation of expand'(h) (mean: double sums in index order, like g_aggregate of the
// materialised vector; without the shuffle the result is h itself, exactly)
template <class T, bool SHUF>
__device__ __forceinline__ void aggregate_out(const float* h, float* g, int aggregator, const ChunkPerm<T>& cp) {
  if constexpr (!SHUF) {
#pragma unroll
    for (int c = 0; c < T::A; ++c) g[c] = h[c];
  } else {
#pragma unroll
    for (int c = 0; c < T::A; ++c) {
      const int b = c * T::CS, e = (c == T::A - 1) ? T::P : b + T::CS;
      double acc = 0.0;
      float m = pick<T>(h, cp.cid(b));
      for (int k = b; k < e; ++k) {
        const float v = pick<T>(h, cp.cid(k));
        acc += (double)v;
        m = (aggregator == 1) ? (v > m ? v : m) : ((v > m && v != 0.0f) ? v : m);
      }
      g[c] = aggregator == 0 ? (float)(acc / (double)(e - b)) : m;
    }
  }
}
// census class of a register row (g_classify_w): f1 = apply(w, w), f2 = apply(w, f1), both
// with the same shuffle permutation (one ApplyCtx), rounded to the storage format
template <class T, class S, bool SHUF>
__device__ int8_t bclassify(const float (&w)[T::P], float eps, bool with_sec, int aggregator, const ChunkPerm<T>& cp) {
  bool fin = true;
#pragma unroll
  for (int k = 0; k < T::P; ++k) fin &= finitef(w[k]);
  if (!fin) return C_DIVERGENT;
  float g[T::A], h1[T::A], h2[T::A];
  lrow_aggregate<T>(w, g, aggregator);
  lmlp<T>(w, g, h1);
  BRow<T, S>::quant_a(h1);
  if (finite_all<T>(h1) && close_out<T, SHUF>(w, h1, eps, cp)) {
    bool zero = true;
#pragma unroll
    for (int k = 0; k < T::P; ++k) zero &= (-eps <= w[k]) && (w[k] <= eps);
    return zero ? C_FIX_ZERO : C_FIX_OTHER;
  }
  if (with_sec) {
    aggregate_out<T, SHUF>(h1, g, aggregator, cp);
    lmlp<T>(w, g, h2);
    BRow<T, S>::quant_a(h2);
    if (finite_all<T>(h2) && close_out<T, SHUF>(w, h2, eps, cp)) return C_FIX_SEC;
  }
  return C_OTHER;
}

// classify (+ histogram, + respawn count flag 64, + generation advance flag 512), attack,
// train and learn_from with any storage format and shuffler
template <class T, class S, bool SHUF, int OP>
__global__ __launch_bounds__(TBROW) void k_big_rows(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, S>;
  __shared__ uint32_t s_cw[SHUF ? ChunkPerm<T>::NW * TBROW : 1];
  __shared__ uint4 s_stg[(TBROW / 64) * R::G::WAVE_U4];
  uint4* st = s_stg + (threadIdx.x >> 6) * R::G::WAVE_U4;  // this wave's staging area
  const ChunkPerm<T> cp{s_cw + threadIdx.x};
  const int64_t p = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  const bool valid = p < a.n;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  float w[T::P];
  // rows move through the wave's LDS staging area (coalesced, see Stage): every lane takes
  // part in the transfers, lanes past n with row index -1
  if constexpr (OP == OP_CLASSIFY) {
    __shared__ uint32_t s_cnt[6];
    if (threadIdx.x < 6) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    int8_t k = -1;
    R::load_staged(a.W, valid ? (int32_t)p : -1, w, st);
    if (valid) {
      if constexpr (SHUF) cp.draw(rng, a.uid ? (uint64_t)a.uid[p] : (uint64_t)(a.lo + p), a.ctr);
      if constexpr (SHUF) k = bclassify<T, S, SHUF>(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, c.aggregator, cp);
      else k = sclassify<T, S>(w, RowSummary<T>(w), a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, c.aggregator);
      if (a.cls) a.cls[p] = k;
    }
    if (a.counts) {  // wave ballots -> LDS -> one atomic per (block, class)
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const unsigned long long m = __ballot(k == q);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_cnt[q], (uint32_t)__popcll(m));
      }
      if (a.flags & SRNN_F_COUNT_RESPAWNS) {
        const unsigned long long m = __ballot(valid && a.respawn[p] != 0);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_cnt[5], (uint32_t)__popcll(m));
      }
      __syncthreads();
      if (threadIdx.x < 6 && s_cnt[threadIdx.x] && (threadIdx.x < 5 || (a.flags & SRNN_F_COUNT_RESPAWNS)))
        atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
    }
    if ((a.flags & SRNN_F_GEN_ADVANCE) && blockIdx.x == 0 && threadIdx.x == 0) {
      if (a.gen_out) a.gen_out[0] = a.gen_ptr[0] + 1;
      else ((int32_t*)a.gen_ptr)[0] = a.gen_ptr[0] + 1;
    }
    return;
  }
  if (blockIdx.x * (int64_t)TBROW + (threadIdx.x & ~63) >= a.n) return;  // whole wave past n
  if constexpr (OP == OP_APPLY) {
    int32_t fi = -1, ti = -1, oi = -1;
    if (valid) {
      fi = (int32_t)(a.idx_f ? a.idx_f[p] : p);
      ti = (int32_t)(a.idx_t ? a.idx_t[p] : p);
      oi = (int32_t)(a.idx_o ? a.idx_o[p] : p);
    }
    float g[T::A], h[T::A];
    // target row (aggregated), then the attacker's row into the same registers
    R::load_staged(a.W, ti, w, st);
    lrow_aggregate<T>(w, g, c.aggregator);
    R::load_staged(a.W, fi, w, st);
    lmlp<T>(w, g, h);
    R::quant_a(h);
    if constexpr (SHUF) cp.draw(rng, a.uid ? (uint64_t)a.uid[ti < 0 ? 0 : ti] : (uint64_t)ti, a.ctr);
    expand_out<T, SHUF>(w, h, cp);
    R::store_staged(a.W2, oi, w, st);
  } else {  // OP_TRAIN / OP_LEARN (no randomness in an aggregating net's SGD step)
    float g[T::A];
    if constexpr (OP == OP_LEARN) {  // teacher row first, aggregated (same sums as stream_aggregate)
      R::load_staged(a.W2, valid ? (int32_t)(a.idx_t ? a.idx_t[p] : p) : -1, w, st);
      lrow_aggregate<T>(w, g, c.aggregator);
    }
    R::load_staged(a.W, valid ? (int32_t)p : -1, w, st);
    float loss = 0.f;
    for (int e = 0; e < a.epochs; ++e) {
      if constexpr (OP == OP_TRAIN) lrow_aggregate<T>(w, g, c.aggregator);
      loss = ltrain_step<T>(w, g, a.lr);
    }
    R::store_staged(a.W, valid ? (int32_t)p : -1, w, st);
    if (valid && a.loss) a.loss[p] = loss;
  }
}

// run_fixpoint phase 3, lane per row: rows that took steps <- expand(chunk state), written
// through the staging area (the wave-per-row k_big_fix3 issued one 1.1 KB row per wave:
// launch-bound, 3.6 TB/s)
template <class T>
__global__ __launch_bounds__(TBROW) void k_big_fix3_row(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, StF32>;
  __shared__ uint4 s_stg[(TBROW / 64) * R::G::WAVE_U4];
  const int64_t p = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  if (blockIdx.x * (int64_t)TBROW + (threadIdx.x & ~63) >= a.n) return;  // whole wave past n
  const float* state = reinterpret_cast<const float*>(a.temp);
  const int8_t* flag = reinterpret_cast<const int8_t*>(state + a.n * T::A);
  const bool on = p < a.n && flag[p] != 0;
  float st[T::A];
#pragma unroll
  for (int i = 0; i < T::A; ++i) st[i] = on ? state[p * T::A + i] : 0.f;
  R::store_state_staged(a.W, on ? (int32_t)p : -1, st, s_stg + (threadIdx.x >> 6) * R::G::WAVE_U4);
}

// init / perturb / respawn of big rows in any storage format (lane per particle)
template <class T, class S, int OP>
__global__ __launch_bounds__(256) void k_big_lane_s(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, S>;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  char* row = R::at(a.W, i);
  if constexpr (OP == OP_INIT) {
    R::init_row(row, rng, a.uid ? (uint64_t)a.uid[i] : (uint64_t)i);
  } else if constexpr (OP == OP_RESPAWN) {
    if (a.respawn[i] != 0) R::init_row(row, rng, respawn_key(a.gen_ptr ? a.gen_ptr[0] : a.gen, a.lo + i));
  } else {  // OP_PERTURB
    const uint64_t uid = a.uid ? (uint64_t)a.uid[i] : (uint64_t)i;
    float w[T::P];
    R::load(row, w);
    for (int k = 0; k < T::P; ++k) {
      const U4 u = rng.draw(uid, a.ctr * 1024u + (uint32_t)k, P_PERTURB);
      const double mag = (double)u01(u.y) * (double)a.eps;
      R::put(row, k, u01(u.x) < 0.5f ? (float)((double)w[k] + mag) : (float)((double)w[k] - mag));
    }
  }
}

// Synchronous soup generation of local row j (Item::soup_evolve / GItem::soup_evolve with
// the row in VGPRs): attacks received in ascending attacker-slot order (generation-start
// attacker rows), learn_from `severity` epochs on the teacher's aggregated generation-start
// row, `epochs` self-train steps, respawn flags (+ inline re-init).  Only one 280-float row
// is live at a time: the victim's aggregate is taken before the attacker's row is loaded
// into the same registers (an attack rewrites every weight of the victim).  Returns the
// respawn code; tk = the received row of a remote teacher (SRNN_F_X2).
template <class T, class S, bool SHUF>
__device__ __forceinline__ int8_t big_soup_one(const SrnnCfg& c, const SrnnArgs& a, const ChunkPerm<T>& cp,
                                               int64_t j, uint32_t tk) {
  using R = BRow<T, S>;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const int64_t g = a.lo + j;
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const bool x2 = (a.flags & SRNN_F_X2) != 0;
  // Attacks received: after the first one the victim's row is chunk-constant (its shuffled form:
  // a permutation of the chunk values), so the victim is carried as its 4-value state h and the
  // row registers hold only the current attacker's row; the victim's row is defined ONCE after the
  // attacks (expanded from h, or its generation-start row), so no 280-float array is carried
  // through the attack loop.  The same arithmetic: the aggregate of expand'(h) is h exactly
  // (shuffled: aggregate_out, the materialised vector's sums).
  float w[T::P];
  float h[T::A];
  bool attacked = false;
  uint32_t ctr = (uint32_t)gen * 1024u;
  for_each_attacker<false>(a, j, [&](uint32_t e, int64_t slot) {
    float gv[T::A];
    if (!attacked) {
      R::stream_aggregate(R::at(a.W2, j), gv, c.aggregator);
    } else if constexpr (SHUF) {
      aggregate_out<T, SHUF>(h, gv, c.aggregator, cp);  // cp: the previous attack's permutation
    } else {
#pragma unroll
      for (int q = 0; q < T::A; ++q) gv[q] = h[q];
    }
    const char* r = ent_row(a, e, R::RB);
    if (x2 && (int64_t)e >= a.n) x2_check(a, r, R::RB, slot, gen);
    R::load(r, w);
    lmlp<T>(w, gv, h);
    R::quant_a(h);
    if constexpr (SHUF) cp.draw(rng, (uint64_t)g, ctr);
    attacked = true;
    ctr += 1;
  });
  int64_t my_at, te;
  Item<Weightwise<1, 1>, StF32>::decision(a, g, gen, my_at, te);
  int8_t act = A_NONE;
  int64_t cpart = -1;
  if (my_at >= 0) act = A_ATTACKING, cpart = my_at;
  // learn_from (`severity` steps on the teacher's aggregate) then self-train (`epochs`
  // steps on the own aggregate) as ONE step loop: a single inlined SGD step keeps the
  // register allocation of the 280-float row to one copy
  float gt[T::A];
  int nlearn = 0;
  if (te >= 0) {
    const char* r = teacher_row(a, te, tk, R::RB);
    if (x2 && tk != SRNN_NIL) x2_check(a, r, R::RB, te, gen);
    R::stream_aggregate(r, gt, c.aggregator);
    nlearn = a.severity > 0 ? a.severity : 0;
    act = A_LEARN_FROM;
    cpart = te;
  }
  // the own row (the generation is SGD-bound: a per-lane load; staging it through LDS measured
  // slower, profiles/r2j_staged_rows_finish_par.md)
  if (attacked) expand_out<T, SHUF>(w, h, cp);
  else R::load(R::at(a.W2, j), w);
  if (a.epochs > 0) act = A_TRAIN_SELF, cpart = -1;
  const int nsteps = nlearn + (a.epochs > 0 ? a.epochs : 0);
  float loss = 0.f;
  for (int s = 0; s < nsteps; ++s) {
    float gs[T::A];
    if (s < nlearn) {
#pragma unroll
      for (int q = 0; q < T::A; ++q) gs[q] = gt[q];
    } else {
      lrow_aggregate<T>(w, gs, c.aggregator);
    }
    loss = ltrain_step<T>(w, gs, a.lr);
  }
  R::quant(w);  // the stored state decides respawn
  // any non-finite weight <=> NaN in sum(w * 0); all |w| <= eps <=> min / max within
  // (fminf / fmaxf skip NaNs: a NaN row is never a zero row, as in the per-weight test)
  // (8 independent partial chains: min / max / NaN propagation are order-free)
  float nz[8], lo[8], hi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) nz[q] = 0.f, lo[q] = w[0], hi[q] = w[0];
#pragma unroll
  for (int k = 0; k < T::P; ++k) {
    nz[k & 7] = fmaf(w[k], 0.f, nz[k & 7]);
    lo[k & 7] = fminf(lo[k & 7], w[k]);
    hi[k & 7] = fmaxf(hi[k & 7], w[k]);
  }
#pragma unroll
  for (int q = 1; q < 8; ++q) nz[0] += nz[q], lo[0] = fminf(lo[0], lo[q]), hi[0] = fmaxf(hi[0], hi[q]);
  const bool bad = !finitef(nz[0]);
  const bool zero = !bad && (-a.eps <= lo[0]) && (hi[0] <= a.eps);
  int8_t rsp = 0;
  if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && bad) rsp = 1;
  else if ((a.flags & SRNN_F_REMOVE_ZERO) && zero) rsp = 2;
  if (rsp && (a.flags & SRNN_F_RESPAWN_INLINE)) R::init_row(R::at(a.W, j), rng, respawn_key(gen, g));  // newborn
  else R::store(R::at(a.W, j), w);
  if (a.action) a.action[j] = act;
  if (a.counterpart) a.counterpart[j] = cpart;
  if (a.loss) a.loss[j] = loss;
  if (a.respawn) a.respawn[j] = rsp;
  return rsp;
}

// OP_SOUP_EVOLVE of big nets: rows of this workgroup (single rank / all-gather: 64-row
// ballots or per-row flags; SRNN_F_X2 local: minus the remote-dependent rows, block stats
// by atomics) or, with SRNN_F_X2_REMOTE, the remote-dependent list (grid-stride)
template <class T, class S, bool SHUF>
__global__ __launch_bounds__(TBROW) void k_big_soup_evolve(SrnnCfg c, SrnnArgs a) {
  __shared__ uint32_t s_cw[SHUF ? ChunkPerm<T>::NW * TBROW : 1];
  const ChunkPerm<T> cp{s_cw + threadIdx.x};
  const bool x2 = (a.flags & SRNN_F_X2) != 0;
  const bool remote = x2 && (a.flags & SRNN_F_X2_REMOTE);
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  // ONE call site of the inlined particle step for both forms (two inlined copies doubled the
  // kernel's code: 19.6k vs 13.6k lines of ISA)
  const int64_t cnt = remote ? (int64_t) * (volatile const int32_t*)a.x_rcount : 0;
  int64_t q = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  for (;;) {
    if (remote && q - threadIdx.x >= cnt) break;  // (workgroup-uniform)
    int64_t j = q;
    uint32_t tk = SRNN_NIL;
    bool on;
    if (remote) {
      on = q < cnt;
      if (on) j = a.x_rlist[2 * q], tk = a.x_rlist[2 * q + 1];
    } else {
      on = j < a.n && !(x2 && x2_dep(a, j));
    }
    const bool rs = on ? big_soup_one<T, S, SHUF>(c, a, cp, j, tk) != 0 : false;
    if (remote) {
      if (on) bs_publish_lane(bs, j, rs, -1);
      q += (int64_t)gridDim.x * TBROW;
      continue;
    }
    if (x2) {
      const int64_t wd = (j >> 6) * 2 + (threadIdx.x & 63);
      if ((threadIdx.x & 63) < 2 && wd * 32 < a.n) a.x_dep[wd] = 0u;
      bs_publish_wave(bs, j >> 6, rs, -1);
    } else if (a.flags & SRNN_F_ROW_FLAGS) {
      if (j < a.n && a.rowflags) a.rowflags[j] = rs ? 1 : 0;
    } else if (a.ballots) {
      const unsigned long long m = __ballot(rs);
      if ((threadIdx.x & 63) == 0) a.ballots[j >> 6] = m;
    }
    return;
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(a.x_ctl + 3, 1) == (int32_t)gridDim.x - 1) {
    *a.x_rcount = 0;
    a.x_ctl[3] = 0;
  }
}

// Single-rank respawn of big nets (k_respawn_seq): one workgroup scans the 64-row ballots
// in slot order, assigns the newborns' uids, re-initialises their rows, advances next_uid
// and the generation counter, zeroes the census histogram.
template <class T, class S>
__global__ __launch_bounds__(TBR) void k_big_respawn_seq(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, S>;
  __shared__ int32_t s_wave[TBR / 64];
  const unsigned long long* masks = a.ballots;
  const int64_t nb = (a.n + 63) / 64;
  const int64_t ch = (nb + TBR - 1) / TBR;
  const int64_t b0 = (int64_t)threadIdx.x * ch;
  const int64_t b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t cnt = 0;
  for (int64_t b = b0; b < b1; ++b) cnt += __popcll(masks[b]);
  int32_t total;
  const int32_t incl = block_incl_scan<TBR>(cnt, s_wave, &total);
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  int64_t k = base + incl - cnt;
  for (int64_t b = b0; b < b1 && cnt; ++b) {
    unsigned long long m = masks[b];
    while (m) {
      const int bit = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int64_t r = b * 64 + bit;
      a.uid_out[r] = k++;
      if (!(a.flags & SRNN_F_RESPAWN_INLINE)) R::init_row(R::at(a.W, r), rng, respawn_key(gen, a.lo + r));  // else inline
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.uid_base[0] = base + total;
    if (a.gen_out) a.gen_out[0] = gen + 1;
    else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = gen + 1;
  }
  if (a.counts && threadIdx.x < 5) a.counts[threadIdx.x] = 0;
}

// ------------------------------------------------------------------ reference order
// The reference's in-place, index-ordered generation (code/soup.py:51-87) of a big
// aggregating net on the continuation scheduler of srnn_ordered.h (plan / mark / count / run
// are shape independent; this is the turn and the close).  Recompute depth 1: an unstored
// attack output A(j) is its attacker's forward on its victim's aggregate, and an aggregating
// net's output is chunk-constant (shuffled: a permutation of the chunk values), so a version
// read is either a streamed row or a 4-value chunk state -- the turn's own row is the only
// 280-float array (as in big_soup_one).  Every step is the serial loop's (the runtime-shape
// engine's soup_seq_one: attack keyed (attacker, gen*1024+1), learn_from `severity` steps on
// the teacher's aggregate, `epochs` self-train steps, respawn_key(gen, k)) in the same
// arithmetic order, so the generation equals OP_SOUP_SEQ bitwise whatever order its turns run in.
template <class T, class S, bool SHUF>
struct BigOrd : ord::OrdSched<1> {
  using R = BRow<T, S>;
  using Sched = ord::OrdSched<1>;
  __device__ static float wget(const char* row, int k) {
    if constexpr (S::ID == 0) return reinterpret_cast<const float*>(row)[k];
    else return S::dec(reinterpret_cast<const uint16_t*>(row)[k]);
  }
  // lmlp with the weights read from a row in memory (same operation order)
  template <int L>
  __device__ static void smlp_rec(const char* row, float* x) {
    constexpr int I = T::rows(L), O = T::cols(L), OFF = T::off(L);
    float y[T::MAXW];
#pragma unroll
    for (int j = 0; j < O; ++j) {
      float acc = x[0] * wget(row, OFF + j);
#pragma unroll
      for (int i = 1; i < I; ++i) acc = fmaf(x[i], wget(row, OFF + i * O + j), acc);
      y[j] = acc;
    }
#pragma unroll
    for (int j = 0; j < O; ++j) x[j] = y[j];
    if constexpr (L < T::D) smlp_rec<L + 1>(row, x);
  }
  __device__ static void smlp(const char* row, const float* g, float* h) {
    float x[T::MAXW];
#pragma unroll
    for (int i = 0; i < T::A; ++i) x[i] = g[i];
    smlp_rec<0>(row, x);
#pragma unroll
    for (int i = 0; i < T::A; ++i) h[i] = x[i];
  }
  // the row of a stored version (E(j) in W, a stored A(j) in W3, the generation start in W2)
  __device__ static const char* vrow(const SrnnArgs& a, int32_t code) {
    if (code >= 0) return R::at((code & 1) ? a.W : a.W3, (int64_t)(code >> 1));
    return R::at(a.W2, -(int64_t)code - 1);
  }
  __device__ static Rng rng(const SrnnArgs& a) { return Rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)}; }
  // chunk state of the unstored attack output A(j): the attacker's forward on its victim's aggregate
  __device__ static void attack_state(const SrnnCfg& c, const SrnnArgs& a, int64_t j, float* h) {
    const int32_t* sj = ord::src_of(a, j);
    float gv[T::A];
    R::stream_aggregate(vrow(a, sj[1] == ord::SRC_SELF ? sj[0] : sj[1]), gv, c.aggregator);
    smlp(vrow(a, sj[0]), gv, h);
    R::quant_a(h);
  }
  // aggregate of the output expand'(h) of attacker j (no shuffle: h itself, exactly)
  __device__ static void state_agg(const SrnnCfg& c, const SrnnArgs& a, int64_t j, int32_t gen,
                                   const ChunkPerm<T>& cp, const float* h, float* g) {
    if constexpr (SHUF) {
      cp.draw(rng(a), (uint64_t)j, (uint32_t)gen * 1024u + 1u);
      aggregate_out<T, SHUF>(h, g, c.aggregator, cp);
    } else {
#pragma unroll
      for (int q = 0; q < T::A; ++q) g[q] = h[q];
    }
  }
  __device__ static void agg_version(const SrnnCfg& c, const SrnnArgs& a, int32_t code, int32_t gen,
                                     const ChunkPerm<T>& cp, float* g) {
    if (ord::is_A(code) && !ord::stored(a, code >> 1)) {
      float h[T::A];
      attack_state(c, a, code >> 1, h);
      state_agg(c, a, code >> 1, gen, cp, h, g);
    } else {
      R::stream_aggregate(vrow(a, code), g, c.aggregator);
    }
  }
  __device__ static void load_version(const SrnnCfg& c, const SrnnArgs& a, int32_t code, int32_t gen,
                                      const ChunkPerm<T>& cp, float (&w)[T::P]) {
    if (ord::is_A(code) && !ord::stored(a, code >> 1)) {
      float h[T::A];
      attack_state(c, a, code >> 1, h);
      if constexpr (SHUF) cp.draw(rng(a), (uint64_t)(code >> 1), (uint32_t)gen * 1024u + 1u);
      expand_out<T, SHUF>(w, h, cp);
    } else {
      R::load(vrow(a, code), w);
    }
  }
  // this lane's stores of a row are complete before it reads the row back
  __device__ static void own_row_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // a stored attack output, written weight by weight from its chunk state
  __device__ static void store_state(char* row, const float* h, const ChunkPerm<T>& cp) {
    for (int k = 0; k < T::P; ++k) R::put(row, k, pick<T>(h, SHUF ? cp.cid(k) : T::chunk(k)));
    for (int k = T::P; k < T::PP; ++k) R::put(row, k, 0.f);
  }

  __device__ static void turn(const SrnnCfg& c, const SrnnArgs& a, int64_t k, int32_t gen, const ChunkPerm<T>& cp) {
    const int32_t* s = ord::src_of(a, k);
    int64_t at, te;
    Sched::Dec::decision(a, k, gen, at, te);
    const bool attack = at >= 0 && ord::needs_A(a, k, s);
    // the aggregates of the versions this turn reads that do not depend on its own row first
    // (streamed rows and chunk-state forwards: their loads never compete with the 280-float
    // row for registers)
    float gv[T::A], gt[T::A];
    if (attack && at != k) agg_version(c, a, s[1], gen, cp, gv);
    if (te >= 0 && s[2] != ord::SRC_SELF && s[2] != ord::SRC_ATK) agg_version(c, a, s[2], gen, cp, gt);
    // the own row is read from memory until the training: an unstored attack output is
    // materialised into this turn's E slot (W row k: nothing reads it before the turn ends), a
    // self-attack's output too -- the 280 registers of the row are defined once, by one load
    char* ek = R::at(a.W, k);
    const char* p0 = vrow(a, s[0]);
    if (ord::is_A(s[0]) && !ord::stored(a, s[0] >> 1)) {
      float h[T::A];
      attack_state(c, a, s[0] >> 1, h);
      if constexpr (SHUF) cp.draw(rng(a), (uint64_t)(s[0] >> 1), (uint32_t)gen * 1024u + 1u);
      store_state(ek, h, cp);
      own_row_fence();
      p0 = ek;
    }
    int8_t act = A_NONE;
    int64_t cpart = -1;
    float ho[T::A];  // the chunk state of A(k)
    if (at >= 0) {  // 1. attack: the victim's row becomes f_k(victim)
      if (attack) {
        if (at == k) R::stream_aggregate(p0, gv, c.aggregator);
        smlp(p0, gv, ho);
        R::quant_a(ho);
        if constexpr (SHUF) cp.draw(rng(a), (uint64_t)k, (uint32_t)gen * 1024u + 1u);
        if (ord::stored(a, k)) store_state(R::at(a.W3, k), ho, cp);
        if (at == k) {
          store_state(ek, ho, cp);
          own_row_fence();
          p0 = ek;
        }
      }
      act = A_ATTACKING;
      cpart = at;
    }
    float w[T::P];
    R::load(p0, w);
    // 2. learn_from (`severity` steps on the teacher's aggregate), 3. self-train (`epochs` steps
    // on the own aggregate): one step loop, one register copy of the row (big_soup_one)
    int nlearn = 0;
    if (te >= 0) {
      if (s[2] == ord::SRC_SELF) lrow_aggregate<T>(w, gt, c.aggregator);
      else if (s[2] == ord::SRC_ATK) state_agg(c, a, k, gen, cp, ho, gt);
      nlearn = a.severity > 0 ? a.severity : 0;
      act = A_LEARN_FROM;
      cpart = te;
    }
    if (a.epochs > 0) act = A_TRAIN_SELF, cpart = -1;
    const int nsteps = nlearn + (a.epochs > 0 ? a.epochs : 0);
    float loss = 0.f;
    for (int st = 0; st < nsteps; ++st) {
      float gs[T::A];
      if (st < nlearn) {
#pragma unroll
        for (int q = 0; q < T::A; ++q) gs[q] = gt[q];
      } else {
        lrow_aggregate<T>(w, gs, c.aggregator);
      }
      loss = ltrain_step<T>(w, gs, a.lr);
    }
    R::quant(w);  // 4. respawn: the stored state decides (tests of big_soup_one)
    float nz[8], lo[8], hi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) nz[q] = 0.f, lo[q] = w[0], hi[q] = w[0];
#pragma unroll
    for (int i = 0; i < T::P; ++i) {
      nz[i & 7] = fmaf(w[i], 0.f, nz[i & 7]);
      lo[i & 7] = fminf(lo[i & 7], w[i]);
      hi[i & 7] = fmaxf(hi[i & 7], w[i]);
    }
#pragma unroll
    for (int q = 1; q < 8; ++q) nz[0] += nz[q], lo[0] = fminf(lo[0], lo[q]), hi[0] = fmaxf(hi[0], hi[q]);
    const bool bad = !finitef(nz[0]);
    const bool zero = !bad && (-a.eps <= lo[0]) && (hi[0] <= a.eps);
    int8_t rsp = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && bad) rsp = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && zero) rsp = 2;
    if (a.traj) R::store(R::at(a.traj, k), w);  // recording: the state before any respawn
    if (rsp) R::init_row(R::at(a.W, k), rng(a), respawn_key(gen, k));  // E(k): a newborn
    else R::store(R::at(a.W, k), w);                                      // E(k)
    if (a.action) a.action[k] = act;
    if (a.counterpart) a.counterpart[k] = cpart;
    if (a.loss) a.loss[k] = loss;
    if (a.respawn) a.respawn[k] = rsp;
  }
};
// the run policy of k_ord_run: the chunk ids of the shuffled outputs in LDS (stride TBROW)
template <class T, class S, bool SHUF>
struct BigOrdPol {
  static constexpr bool SHADOW = false;  // (the turn's staged reads are wave-cooperative)
  static constexpr bool CENSUS = false;  // (its census stays in the close)
  static constexpr int RB = 1;  // the plan's recompute depth (big nets)
  using PT = void;              // no permutation table (an aggregating net's SGD step has one sample)
  struct Shared {
    uint32_t cw[SHUF ? ChunkPerm<T>::NW * TB : 1];
  };
  __device__ static void turn(const SrnnCfg& c, const SrnnArgs& a, int64_t k, int32_t gen, Shared& sh, int64_t) {
    BigOrd<T, S, SHUF>::turn(c, a, k, gen, ChunkPerm<T>{sh.cw + threadIdx.x, TB});
  }
};
// final rows (the last attack after a row's own turn, else its E version), the next
// generation's lists, census of the stored rows, block stats (two-phase, as k_ord_close)
template <class T, class S, bool SHUF>
__global__ __launch_bounds__(TB) void k_ordbig_close(SrnnCfg c, SrnnArgs a) {
  using R = BRow<T, S>;
  using Dec = ord::OrdSched<1>::Dec;
  __shared__ uint32_t s_cw[SHUF ? ChunkPerm<T>::NW * TB : 1];
  const ChunkPerm<T> cp{s_cw + threadIdx.x, TB};
  const int64_t gb = blockIdx.x;
  const int64_t r = gb * TB + threadIdx.x;
  const int lane = threadIdx.x;
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const bool census = !SHUF && (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  if ((a.flags & SRNN_F_ORD_INPLAN) && gb == 0 && threadIdx.x == 0) a.o_ctl[ord::BARW] = 0;
  bool rs = false;
  int8_t k = -1;
  // the E rows through the wave's staging area (coalesced passes, as the synchronous soup's
  // census: a lane-per-row load touches 64 rows 1120 B apart per instruction)
  __shared__ uint4 s_stg[R::G::WAVE_U4];
  float w[T::P];
  R::load_staged(a.W, r < a.n ? (int32_t)r : -1, w, s_stg);
  if (r < a.n) {
    if (a.o_src[4 * r + 3] < 0) atomicOr(a.o_ctl + ord::ERRW, ord::ERR_NOT_RUN);  // never ran: a scheduling bug
    const int64_t ja = ord::last_attacker_before(a, r, a.n);
    a.heads[r] = SRNN_NIL;  // consumed: NIL for the generation after next
    if (ja > r) {  // attacked after its own turn: the last attack's output
      BigOrd<T, S, SHUF>::load_version(c, a, ord::code_A(ja), gen, cp, w);
      R::store(R::at(a.W, r), w);
    }
    rs = a.respawn[r] != 0;
    if (!(a.flags & SRNN_F_ORD_PLANNED)) {  // (planned ahead: the next OP_ORD_PLAN links them)
      int64_t at, te;
      Dec::decision(a, r, gen + 1, at, te);
      if (at >= 0) Dec::link(a.heads_next, a.nexts_next, at, (uint32_t)r);
    }
    if (census) k = sclassify<T, S>(w, RowSummary<T>(w), a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, c.aggregator);
  }
  if ((a.flags & SRNN_F_GEN_COUNTS) && gb == 0 && lane == 0) Dec::set_gen(a, gen + 1);
  const unsigned long long m = __ballot(rs);
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(k == q));
  if (lane == 0) {
    unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
    unsigned long long* mine = bs + gb * 4;
    mine[0] = m;
    mine[1] = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
    mine[2] = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
    mine[3] = (unsigned long long)cnt[4];
    if ((a.flags & SRNN_F_BORN_TOTAL) && m) atomicAdd(bs + ((a.n + TB - 1) / TB) * 4, (unsigned long long)__popcll(m));
  }
  // SRNN_F_ORD_SYNC: the launch ends (and the next run starts) once the next generation's plan is done
  if ((a.flags & SRNN_F_ORD_SYNC) && gb == 0 && lane == 0)
    ord::sync_wait(a.o_sync, ord::SYNC_CLOSE, ord::SYNC_PLAN, a.o_ctl + ord::ERRW);
}
// OP_SOUP_ORDERED of a big aggregating net (device): soup_ordered's launch sequence with this
// family's run policy and close (no permutation table: an aggregating net's SGD step has one
// sample); the finish (uids, census, counter) follows unless the caller batches it
template <class T, class S, bool SHUF>
int big_soup_ordered(const SrnnCfg& c, const SrnnArgs& a) {
  const bool planned = (a.flags & SRNN_F_ORD_PLANNED) != 0;
  if (!ord_single_table(a)) return -5;
  if (!a.W || !a.W2 || !a.W3 || !a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts ||
      (!planned && (!a.heads_next || !a.nexts_next)) || !a.respawn || !(a.flags & SRNN_F_TWO_PHASE) || !a.temp) {
    set_error("ordered soup generation needs W, W2, W3, o_src, o_list, o_ctl, the attack lists (both unless "
              "planned ahead), respawn and two-phase block stats (temp)");
    return -5;
  }
  if (!ord_inplan_ok(a) || !ord_sync_ok(a)) return -5;
  if (a.o_census_temp) {
    set_error("big ordered generation: no census in the run launch (o_census_temp)");
    return -5;
  }
  const int64_t nb = (a.n + TB - 1) / TB;
  if (nb <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  if (!planned) ord_plan_dev<1, void>(c, a, false);
  SrnnArgs ra = ord_run_args(a, nb);
  // (no head start for the critical roots by default: a 1M soup's bulk is the generation's work, and
  // delaying its first round cost 0.5-1.5 %, profiles/r6a r6n)
  ra.o_bulk_delay = std::min(1000, std::max(0, knob(SRNN_KNOB_ORD_BULK_DELAY, 0)));
  hipLaunchKernelGGL((k_ord_run<BigOrdPol<T, S, SHUF>>), dim3((unsigned)ord_run_grid(ra, nb)), dim3(TB), 0, st, c, ra);
  hipLaunchKernelGGL((k_ordbig_close<T, S, SHUF>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  if (!(a.flags & SRNN_F_GEN_COUNTS)) {
    constexpr int FNT = SRNN_FINISH_NT;
    hipLaunchKernelGGL((k_gen_finish<Weightwise<1, 1>, StF32, FNT>), dim3(1), dim3(FNT), 0, st, a, (int32_t)nb);
  }
  return 0;
}

// ops of the big nets that take any storage format / shuffler (everything a soup needs)
template <class T, class S, bool SHUF>
int big_run_s(int op, const SrnnCfg& c, const SrnnArgs& a) {
  hipStream_t st = (hipStream_t)a.stream;
  const unsigned gl = (unsigned)((a.n + 255) / 256), g64 = (unsigned)((a.n + TBROW - 1) / TBROW);
  switch (op) {
    case OP_INIT: hipLaunchKernelGGL((k_big_lane_s<T, S, OP_INIT>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_PERTURB: hipLaunchKernelGGL((k_big_lane_s<T, S, OP_PERTURB>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_RESPAWN: hipLaunchKernelGGL((k_big_lane_s<T, S, OP_RESPAWN>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_APPLY: hipLaunchKernelGGL((k_big_rows<T, S, SHUF, OP_APPLY>), dim3(g64), dim3(TBROW), 0, st, c, a); break;
    case OP_CLASSIFY:
      hipLaunchKernelGGL((k_big_rows<T, S, SHUF, OP_CLASSIFY>), dim3(g64), dim3(TBROW), 0, st, c, a);
      break;
    case OP_TRAIN: hipLaunchKernelGGL((k_big_rows<T, S, SHUF, OP_TRAIN>), dim3(g64), dim3(TBROW), 0, st, c, a); break;
    case OP_LEARN: hipLaunchKernelGGL((k_big_rows<T, S, SHUF, OP_LEARN>), dim3(g64), dim3(TBROW), 0, st, c, a); break;
    case OP_SOUP_EVOLVE: {
      unsigned g = g64;
      if ((a.flags & SRNN_F_X2) && (a.flags & SRNN_F_X2_REMOTE)) {  // bounded grid over the remote list
        const int64_t rb = (x2_remote_bound(a) + TBROW - 1) / TBROW;
        g = (unsigned)(rb < X2_REMOTE_WAVES / 4 ? rb : X2_REMOTE_WAVES / 4);
      }
      hipLaunchKernelGGL((k_big_soup_evolve<T, S, SHUF>), dim3(g), dim3(TBROW), 0, st, c, a);
      break;
    }
    case OP_RESPAWN_SEQ: hipLaunchKernelGGL((k_big_respawn_seq<T, S>), dim3(1), dim3(TBR), 0, st, c, a); break;
    case OP_SOUP_ORDERED: {
      const int r = big_soup_ordered<T, S, SHUF>(c, a);
      if (r) return r;
      break;
    }
    case OP_ORD_PLAN:  // (shape independent, recompute depth 1: soup_ord_plan's device path)
      if (!ord_single_table(a)) return -5;
      if (!a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts) {
        set_error("ordered generation plan needs o_src, o_list, o_ctl and the planned generation's attack lists");
        return -5;
      }
      if ((a.flags & SRNN_F_ORD_SYNC) && (!a.o_sync || !(a.flags & SRNN_F_ORD_NEXT))) {
        set_error("SRNN_F_ORD_SYNC: a device plan of the next generation with the o_sync counters");
        return -5;
      }
      ord_plan_dev<1, void>(c, a, true);
      break;
    case OP_SOUP_DECIDE: {
      // decisions are shape independent: every global slot
      if (a.n_total <= 0) return 0;
      hipLaunchKernelGGL((k_op<Weightwise<1, 1>, OP_SOUP_DECIDE, StF32>), dim3((unsigned)((a.n_total + TB - 1) / TB)),
                         dim3(TB), 0, st, SrnnCfg{}, a);
      break;
    }
    default: set_error("op not supported for big aggregating nets"); return -5;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// true when big_run serves (op, storage, shuffler); the rest goes to the runtime-shape engine
constexpr bool big_serves(int op, int dtype, int shuffler) {
  if (op == OP_INIT || op == OP_PERTURB || op == OP_RESPAWN || op == OP_APPLY || op == OP_CLASSIFY ||
      op == OP_TRAIN || op == OP_LEARN || op == OP_SOUP_EVOLVE || op == OP_RESPAWN_SEQ || op == OP_SOUP_DECIDE ||
      op == OP_SOUP_ORDERED || op == OP_ORD_PLAN)
    return true;
  return op == OP_RUN_FIXPOINT && dtype == 0 && shuffler == 0;
}

template <class T>
int big_run(int op, const SrnnCfg& c, const SrnnArgs& a) {
  if (!a.dev) {
    set_error("wave-per-particle nets run on the GPU only (use a smaller shape on the host)");
    return -5;
  }
  if (!big_serves(op, c.dtype, c.shuffler)) {
    set_error("op not served by the big-net kernels (runtime-shape engine)");
    return -5;
  }
  // lane-per-particle row kernels (default) or the wave-per-particle ones (SRNN_BIG_WAVE=1,
  // fp32 tables without shuffle only)
  const bool row_kernels = knob(SRNN_KNOB_BIG_WAVE, 0) != 1;
  const bool wave_op = !row_kernels && (op == OP_APPLY || op == OP_CLASSIFY || op == OP_TRAIN || op == OP_LEARN);
  if (op != OP_RUN_FIXPOINT && !(wave_op && c.dtype == 0 && c.shuffler == 0)) {
    if (a.n <= 0 && op != OP_SOUP_DECIDE) return 0;
    const bool sh = c.shuffler != 0;
#ifndef SRNN_BIG_FAST  // (register-allocation experiments: fp32 instantiations only)
    if (c.dtype == 1) return sh ? big_run_s<T, StBF16, true>(op, c, a) : big_run_s<T, StBF16, false>(op, c, a);
    if (c.dtype == 2) return sh ? big_run_s<T, StF16, true>(op, c, a) : big_run_s<T, StF16, false>(op, c, a);
#endif
    return sh ? big_run_s<T, StF32, true>(op, c, a) : big_run_s<T, StF32, false>(op, c, a);
  }
  hipStream_t st = (hipStream_t)a.stream;
  if (a.n <= 0) return 0;
  const unsigned gw = (unsigned)((a.n + BW - 1) / BW), gl = (unsigned)((a.n + 255) / 256);
  const unsigned g64 = (unsigned)((a.n + TBROW - 1) / TBROW);
  switch (op) {
    case OP_INIT: hipLaunchKernelGGL((k_big_lane<T, OP_INIT>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_PERTURB: hipLaunchKernelGGL((k_big_lane<T, OP_PERTURB>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_APPLY:
      if (row_kernels) hipLaunchKernelGGL((k_big_row<T, OP_APPLY>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big<T, OP_APPLY>), dim3(gw), dim3(TBB), 0, st, c, a);
      break;
    case OP_RUN_FIXPOINT:
      if (!a.temp || a.temp_bytes < a.n * (T::A * 4 + 1)) {
        set_error("run_fixpoint on wave-per-particle nets needs temp >= n*(4*aggregates+1) bytes");
        return -5;
      }
      if (row_kernels) hipLaunchKernelGGL((k_big_fix1_row<T>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big_fix1<T>), dim3(gw), dim3(TBB), 0, st, c, a);
      hipLaunchKernelGGL((k_big_fix2<T>), dim3(gl), dim3(256), 0, st, c, a);
      if (row_kernels) hipLaunchKernelGGL((k_big_fix3_row<T>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big_fix3<T>), dim3(gw), dim3(TBB), 0, st, c, a);
      break;
    case OP_CLASSIFY:
      if (row_kernels) hipLaunchKernelGGL((k_big_row<T, OP_CLASSIFY>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big<T, OP_CLASSIFY>), dim3(gw), dim3(TBB), 0, st, c, a);
      break;
    case OP_TRAIN:
      if (row_kernels) hipLaunchKernelGGL((k_big_row<T, OP_TRAIN>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big<T, OP_TRAIN>), dim3(gw), dim3(TBB), 0, st, c, a);
      break;
    case OP_LEARN:
      if (row_kernels) hipLaunchKernelGGL((k_big_row<T, OP_LEARN>), dim3(g64), dim3(TBROW), 0, st, c, a);
      else hipLaunchKernelGGL((k_big<T, OP_LEARN>), dim3(gw), dim3(TBB), 0, st, c, a);
      break;
    default: set_error("op not supported for wave-per-particle nets"); return -5;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

}  // namespace srnn
