// srnn_bignet.hip — wave-per-particle kernels for Aggregating nets too large for the
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
#include "srnn_kernels.h"
#include <cstdlib>

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
      const bool with_sec = (a.flags & 8) != 0;
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
  const bool with_sec = (a.flags & 8) != 0;
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
        if (a.flags & 8) {
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

// run_fixpoint phase 1 with the row in VGPRs (same decisions as k_big_fix1)
template <class T>
__global__ __launch_bounds__(TBROW) void k_big_fix1_row(SrnnCfg c, SrnnArgs a) {
  const int64_t p = (int64_t)blockIdx.x * TBROW + threadIdx.x;
  if (p >= a.n) return;
  float* state = reinterpret_cast<float*>(a.temp);
  int8_t* flag = reinterpret_cast<int8_t*>(state + a.n * T::A);
  float w[T::P];
  lrow_load<T>(a.W + p * T::PP, w);
  bool stop = a.steps <= 0;
  if (!stop && a.early_exit) {
    bool fin = true;
#pragma unroll
    for (int k = 0; k < T::P; ++k) fin &= finitef(w[k]);
    stop = !fin;
  }
  float g[T::A], h[T::A];
  if (!stop) {
    lrow_aggregate<T>(w, g, c.aggregator);
    lmlp<T>(w, g, h);
    if (a.early_exit && finite_all<T>(h) && lrow_close_state<T>(w, h, a.eps)) stop = true;
  }
  if (stop) {  // no step taken: the row is unchanged, classify the general weights
    flag[p] = 0;
    if (a.nsteps) a.nsteps[p] = 0;
    if (a.cls) a.cls[p] = lclassify<T>(w, a.eps, (a.flags & 8) != 0, c.aggregator);
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
      k = lclassify<T>(w, a.eps, (a.flags & 8) != 0, c.aggregator);
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

template <class T>
int big_run(int op, const SrnnCfg& c, const SrnnArgs& a) {
  if (!a.dev) {
    set_error("wave-per-particle nets run on the GPU only (use a smaller shape on the host)");
    return -5;
  }
  if (c.shuffler != 0 && op != OP_INIT && op != OP_PERTURB && op != OP_TRAIN && op != OP_LEARN) {
    set_error("wave-per-particle aggregating nets: shuffle_random is not supported");
    return -5;
  }
  hipStream_t st = (hipStream_t)a.stream;
  if (a.n <= 0) return 0;
  const unsigned gw = (unsigned)((a.n + BW - 1) / BW), gl = (unsigned)((a.n + 255) / 256);
  const unsigned g64 = (unsigned)((a.n + TBROW - 1) / TBROW);
  // lane-per-particle row kernels (default) or the wave-per-particle ones (SRNN_BIG_WAVE=1)
  const char* wave_env = std::getenv("SRNN_BIG_WAVE");
  const bool row_kernels = !(wave_env && wave_env[0] == '1');
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
      hipLaunchKernelGGL((k_big_fix3<T>), dim3(gw), dim3(TBB), 0, st, c, a);
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

using AGGB_4_10_3 = srnn::AggBig<4, 10, 3>;
using AGGB_4_8_2 = srnn::AggBig<4, 8, 2>;
using AGGB_4_16_2 = srnn::AggBig<4, 16, 2>;

#define SRNN_TRY_BIG(T, W_, D_, A_)                                              \
  if (c->width == (W_) && c->depth == (D_) && c->aggregates == (A_)) {           \
    if (c->p != T::P || c->pp != T::PP) {                                        \
      srnn::set_error("layout mismatch (p/pp) for instantiated shape");          \
      return -4;                                                                 \
    }                                                                            \
    if (op < 0) return 0;                                                        \
    return srnn::big_run<T>(op, *c, *a);                                         \
  }

extern "C" int srnn_dispatch_aggbig(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY_BIG(AGGB_4_10_3, 10, 3, 4)
  SRNN_TRY_BIG(AGGB_4_8_2, 8, 2, 4)
  SRNN_TRY_BIG(AGGB_4_16_2, 16, 2, 4)
  return 1;
}
