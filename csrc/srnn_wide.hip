// srnn_wide.hip — MFMA kernels for wide Weightwise nets (width 16 / 32).
//
// Self-application of a Weightwise net evaluates the SAME MLP 4 -> W -> ... -> W -> 1 at
// all P weight-points of the target (reference code/network.py:265-279): per particle
// that is a real GEMM chain  X[P x 4] . A0[4 x W] . A1[W x W] ... . AD[W x 1]  with the
// particle's own weights as the B operands.  One wave owns one particle and streams the
// points in 16-row tiles through v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf
// chain, bit-identical to the VALU lane-per-particle kernels' dense_fwd):
//
//   layer 0   K = 4  : one MFMA per 16-column tile; A = (target weight, 3 coordinates)
//   layer l   K = W  : W/4 chained MFMAs per column tile; the accumulator tile is
//                      re-fragmented through a [16][W+1] LDS tile (odd stride: no bank
//                      conflicts on the column reads)
//   output    N = 1  : VALU dot products (4 lanes per row + shuffles)
//
// The B fragments of every layer are loaded once per application and stay in VGPRs for
// all P/16 row tiles.  The particle's weights, the target and the output live in LDS.
#include "srnn_kernels.h"

namespace srnn {

constexpr int WBW = 4;  // waves (particles) per block
constexpr int WTB = 64 * WBW;

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int W_, int D_>
struct WWWide {
  static constexpr int W = W_, D = D_;
  static_assert(W % 16 == 0, "MFMA weightwise path needs width % 16 == 0");
  using Net = MLP<4, W, D, 1>;
  static constexpr int P = Net::P;
  static constexpr int PP = (P + 3) & ~3;
  static constexpr int NT = (P + 15) / 16;  // row tiles
  static constexpr int NU = W / 16;         // column tiles
  static constexpr int NK = W / 4;          // k-steps of a hidden layer
  static constexpr int NL = D + 1;
  static constexpr int TS = W + 1;          // LDS tile row stride
  static constexpr int off(int l) { return Net::off(l); }
  static constexpr int rows(int l) { return l == 0 ? 4 : W; }
  static constexpr int cols(int l) { return l == D ? 1 : W; }
  // normalised coordinate q (0 layer, 1 cell, 2 position) of flat weight p
  // (reference normalize_id, code/network.py:216-220)
  __device__ static float coord(int p, int q) {
    int l = 0;
#pragma unroll
    for (int k = 1; k < NL; ++k) l = (p >= off(k)) ? k : l;
    const int o = off(l), r = rows(l), c = cols(l);
    const int rel = p - o, i = rel / c, j = rel - i * c;
    const int v = q == 0 ? l : (q == 1 ? i : j);
    const int m = q == 0 ? NL - 1 : (q == 1 ? r - 1 : c - 1);
    return m > 1 ? (float)v / (float)m : (float)v;
  }
};

template <class T>
struct WideLds {
  float f[T::PP];                // applying net's weights
  float t[T::PP];                // target weights
  float o[T::PP];                // output weights
  float tile[16 * T::TS];        // accumulator tile re-fragmentation
};

template <class T>
struct BFrags {
  float b0[T::NU];                       // layer 0: B[k = lane>>4][j = 16u + (lane&15)]
  float bh[T::D > 1 ? T::D - 1 : 1][T::NK][T::NU];  // hidden layers
  float aout[T::W];                      // output layer column (kept replicated)
};

template <class T>
__device__ void load_bfrags(const float* __restrict__ f, BFrags<T>& B, int lane) {
  const int k = lane >> 4, j = lane & 15;
#pragma unroll
  for (int u = 0; u < T::NU; ++u) B.b0[u] = f[T::off(0) + k * T::W + 16 * u + j];
#pragma unroll
  for (int h = 1; h < T::D; ++h)
#pragma unroll
    for (int kk = 0; kk < T::NK; ++kk)
#pragma unroll
      for (int u = 0; u < T::NU; ++u) B.bh[h - 1][kk][u] = f[T::off(h) + (4 * kk + k) * T::W + 16 * u + j];
#pragma unroll
  for (int q = 0; q < T::W; ++q) B.aout[q] = f[T::off(T::D) + q];
}

// out[p] = f(point p of target t) for every p; B holds the applying net.
template <class T>
__device__ void wide_apply(const BFrags<T>& B, const float* __restrict__ t, float* __restrict__ out, float* tile,
                           int lane) {
  const int i16 = lane & 15, k4 = lane >> 4;
  for (int tt = 0; tt < T::NT; ++tt) {
    const int p = 16 * tt + i16;
    float a0 = 0.f;
    if (p < T::P) a0 = (k4 == 0) ? t[p] : T::coord(p, k4 - 1);
    f32x4 acc[T::NU];
#pragma unroll
    for (int u = 0; u < T::NU; ++u) {
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, B.b0[u], z, 0, 0, 0);
    }
#pragma unroll
    for (int h = 1; h < T::D; ++h) {
      // accumulator tile -> LDS [row][col]
#pragma unroll
      for (int u = 0; u < T::NU; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) tile[(4 * k4 + r) * T::TS + 16 * u + i16] = acc[u][r];
      __builtin_amdgcn_wave_barrier();
      float af[T::NK];
#pragma unroll
      for (int kk = 0; kk < T::NK; ++kk) af[kk] = tile[i16 * T::TS + 4 * kk + k4];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < T::NU; ++u) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[0], B.bh[h - 1][0][u], z, 0, 0, 0);
#pragma unroll
        for (int kk = 1; kk < T::NK; ++kk)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[kk], B.bh[h - 1][kk][u], acc[u], 0, 0, 0);
      }
    }
    // output layer on the VALU: row = lane & 15, 4 lanes per row split the W columns
#pragma unroll
    for (int u = 0; u < T::NU; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(4 * k4 + r) * T::TS + 16 * u + i16] = acc[u][r];
    __builtin_amdgcn_wave_barrier();
    // k-ordered chain over all W columns (same order as the VALU kernels): lanes 0..15
    if (lane < 16 && p < T::P) {
      const float* row = tile + i16 * T::TS;
      float y = row[0] * B.aout[0];
#pragma unroll
      for (int q = 1; q < T::W; ++q) y = fmaf(row[q], B.aout[q], y);
      out[p] = y;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <class T>
__device__ bool lds_all_finite(const float* v, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) ok &= finitef(v[k]);
  return __ballot(!ok) == 0ull;
}
template <class T>
__device__ bool lds_all_close(const float* a, const float* b, float eps, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) ok &= !(fabsf(a[k] - b[k]) >= eps);
  return __ballot(!ok) == 0ull;
}
template <class T>
__device__ bool lds_all_zero(const float* a, float eps, int lane) {
  bool ok = true;
  for (int k = lane; k < T::P; k += 64) ok &= (-eps <= a[k]) && (a[k] <= eps);
  return __ballot(!ok) == 0ull;
}
template <class T>
__device__ void lds_load(float* __restrict__ d, const float* __restrict__ row, int lane) {
  const float4* r4 = reinterpret_cast<const float4*>(row);
  float4* d4 = reinterpret_cast<float4*>(d);
  for (int q = lane; q < T::PP / 4; q += 64) d4[q] = r4[q];
}
template <class T>
__device__ void lds_store(float* __restrict__ row, const float* __restrict__ s, int lane) {
  float4* r4 = reinterpret_cast<float4*>(row);
  const float4* s4 = reinterpret_cast<const float4*>(s);
  for (int q = lane; q < T::PP / 4; q += 64) {
    float4 v = s4[q];
    if (4 * q + 3 >= T::P) {  // keep the row padding zero
      if (4 * q + 0 >= T::P) v.x = 0.f;
      if (4 * q + 1 >= T::P) v.y = 0.f;
      if (4 * q + 2 >= T::P) v.z = 0.f;
      if (4 * q + 3 >= T::P) v.w = 0.f;
    }
    r4[q] = v;
  }
}

// classification of the weights in L.f (L.t, L.o as scratch)
template <class T>
__device__ int8_t wide_classify(WideLds<T>& L, float eps, bool with_sec, int lane) {
  if (!lds_all_finite<T>(L.f, lane)) return C_DIVERGENT;
  BFrags<T> B;
  load_bfrags<T>(L.f, B, lane);
  wide_apply<T>(B, L.f, L.o, L.tile, lane);
  __builtin_amdgcn_wave_barrier();
  if (lds_all_finite<T>(L.o, lane) && lds_all_close<T>(L.o, L.f, eps, lane))
    return lds_all_zero<T>(L.f, eps, lane) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    wide_apply<T>(B, L.o, L.t, L.tile, lane);
    __builtin_amdgcn_wave_barrier();
    if (lds_all_finite<T>(L.t, lane) && lds_all_close<T>(L.t, L.f, eps, lane)) return C_FIX_SEC;
  }
  return C_OTHER;
}

template <class T, int OP>
__global__ __launch_bounds__(WTB) void k_wide(SrnnCfg c, SrnnArgs a) {
  __shared__ WideLds<T> lds[WBW];
  __shared__ uint32_t s_cnt[5];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * WBW + wv;
  WideLds<T>& L = lds[wv];
  if (OP == OP_CLASSIFY && threadIdx.x < 5) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  int8_t cls = -1;
  if (p < a.n) {
    if constexpr (OP == OP_APPLY) {
      const int64_t fi = a.idx_f ? a.idx_f[p] : p, ti = a.idx_t ? a.idx_t[p] : p, oi = a.idx_o ? a.idx_o[p] : p;
      lds_load<T>(L.f, a.W + fi * T::PP, lane);
      lds_load<T>(L.t, a.W + ti * T::PP, lane);
      __builtin_amdgcn_wave_barrier();
      BFrags<T> B;
      load_bfrags<T>(L.f, B, lane);
      wide_apply<T>(B, L.t, L.o, L.tile, lane);
      __builtin_amdgcn_wave_barrier();
      lds_store<T>(a.W2 + oi * T::PP, L.o, lane);
    } else if constexpr (OP == OP_RUN_FIXPOINT) {
      lds_load<T>(L.f, a.W + p * T::PP, lane);
      __builtin_amdgcn_wave_barrier();
      int s = 0;
      for (; s < a.steps; ++s) {
        if (a.early_exit && !lds_all_finite<T>(L.f, lane)) break;
        BFrags<T> B;
        load_bfrags<T>(L.f, B, lane);
        wide_apply<T>(B, L.f, L.o, L.tile, lane);
        __builtin_amdgcn_wave_barrier();
        if (a.early_exit && lds_all_finite<T>(L.o, lane) && lds_all_close<T>(L.o, L.f, a.eps, lane)) break;
        for (int k = lane; k < T::PP; k += 64) L.f[k] = L.o[k];
        __builtin_amdgcn_wave_barrier();
      }
      lds_store<T>(a.W + p * T::PP, L.f, lane);
      if (a.nsteps && lane == 0) a.nsteps[p] = s;
      if (a.cls) {
        cls = wide_classify<T>(L, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, lane);
        if (lane == 0) a.cls[p] = cls;
      }
    } else if constexpr (OP == OP_CLASSIFY) {
      lds_load<T>(L.f, a.W + p * T::PP, lane);
      __builtin_amdgcn_wave_barrier();
      cls = wide_classify<T>(L, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, lane);
      if (a.cls && lane == 0) a.cls[p] = cls;
    }
  }
  if constexpr (OP == OP_CLASSIFY) {
    if (a.counts && lane == 0 && cls >= 0) atomicAdd(&s_cnt[cls], 1u);
    __syncthreads();
    if (a.counts && threadIdx.x < 5 && s_cnt[threadIdx.x]) atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
  }
}

template <class T>
__global__ __launch_bounds__(256) void k_wide_init(SrnnCfg c, SrnnArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  float* row = a.W + i * T::PP;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const uint64_t uid = a.uid ? (uint64_t)a.uid[i] : (uint64_t)i;
#pragma unroll
  for (int l = 0; l < T::NL; ++l) glorot_fill(row, T::off(l), T::rows(l), T::cols(l), rng, uid);
  for (int k = T::P; k < T::PP; ++k) row[k] = 0.f;
}

template <class T>
int wide_run(int op, const SrnnCfg& c, const SrnnArgs& a) {
  if (!a.dev) {
    set_error("wide weightwise nets (MFMA path) run on the GPU only");
    return -5;
  }
  if (a.n <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  const unsigned gw = (unsigned)((a.n + WBW - 1) / WBW), gl = (unsigned)((a.n + 255) / 256);
  switch (op) {
    case OP_INIT: hipLaunchKernelGGL((k_wide_init<T>), dim3(gl), dim3(256), 0, st, c, a); break;
    case OP_APPLY: hipLaunchKernelGGL((k_wide<T, OP_APPLY>), dim3(gw), dim3(WTB), 0, st, c, a); break;
    case OP_RUN_FIXPOINT: hipLaunchKernelGGL((k_wide<T, OP_RUN_FIXPOINT>), dim3(gw), dim3(WTB), 0, st, c, a); break;
    case OP_CLASSIFY: hipLaunchKernelGGL((k_wide<T, OP_CLASSIFY>), dim3(gw), dim3(WTB), 0, st, c, a); break;
    default: set_error("op not supported by the MFMA weightwise path (apply / run_fixpoint / classify / init)"); return -5;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

}  // namespace srnn

using WWW_16_2 = srnn::WWWide<16, 2>;
using WWW_16_3 = srnn::WWWide<16, 3>;
using WWW_32_2 = srnn::WWWide<32, 2>;

#define SRNN_TRY_WIDE(T, W_, D_)                                                 \
  if (c->width == (W_) && c->depth == (D_)) {                                    \
    if (c->p != T::P || c->pp != T::PP) {                                        \
      srnn::set_error("layout mismatch (p/pp) for instantiated shape");          \
      return -4;                                                                 \
    }                                                                            \
    if (op < 0) return 0;                                                        \
    return srnn::wide_run<T>(op, *c, *a);                                        \
  }

extern "C" int srnn_dispatch_wwwide(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY_WIDE(WWW_16_2, 16, 2)
  SRNN_TRY_WIDE(WWW_16_3, 16, 3)
  SRNN_TRY_WIDE(WWW_32_2, 32, 2)
  return 1;
}
