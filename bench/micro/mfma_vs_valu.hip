// mfma_vs_valu.hip — does v_mfma_f32_4x4x1_16b_f32 beat lane-per-particle VALU code on the
// tiny per-particle nets?  ("benchmark it against the VALU
// lane-per-particle path before committing, and show rocprof MFMA/VALU counters for both")
//
// (a) WeightwiseNeuralNetwork(2, 2) self-application (BASELINE config 2): every particle
//     maps each of its 14 weights, presented as the point (w, layer, cell, weight-id),
//     through its own 4 -> 2 -> 2 -> 1 linear net; `steps` applications in a row.
//     VALU: one lane per particle, 14 weights in VGPRs, 14 MACs per point.
//     MFMA: 16 lanes per particle, one point per lane; the 16 4x4 blocks of one
//     v_mfma_f32_4x4x1_16b_f32 are (particle, group of 4 points) x (4 units), A = the
//     particle's weights (gathered with ds_bpermute each step: the weights change every
//     application), B = the points' features, K = 1 per instruction (fp32 products,
//     accumulated in the same order as the VALU fma chain).
// (b) Aggregating(4, 10, 3) forward (the GEMV chain 4 -> 10 -> 10 -> 10 -> 4, P = 280) of
//     self-application on the aggregate state, chained `steps` times.
//     VALU: one lane per particle, the 280 weights in VGPRs/AGPRs.
//     MFMA: 5 particles per wave, blocks = (particle, group of 4 units), A = weights held
//     per lane (static), B = the broadcast input element (ds_bpermute from the block that
//     produced it).
//
// Output: one JSON line per kernel (time per launch, particle-steps/s) and the max
// relative difference of the MFMA result from the VALU result after a few steps.
// Profile: rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES ... -- ./mfma_vs_valu
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ (a) WW(2,2)
// point features of weight p: (w_p, layer id, cell id, weight id), normalised like the
// reference's compute_all_weight_points (constants; their values do not change the cost)
__constant__ float c_feat[16][3];

__device__ __forceinline__ float ww_net(const float* w, float x0, float x1, float x2, float x3) {
  // layer 1: kernel [4][2] at w[0..7] (flat index 2k + u)
  float h0 = x0 * w[0];
  h0 = fmaf(x1, w[2], h0);
  h0 = fmaf(x2, w[4], h0);
  h0 = fmaf(x3, w[6], h0);
  float h1 = x0 * w[1];
  h1 = fmaf(x1, w[3], h1);
  h1 = fmaf(x2, w[5], h1);
  h1 = fmaf(x3, w[7], h1);
  // layer 2: [2][2] at w[8..11]
  float g0 = h0 * w[8];
  g0 = fmaf(h1, w[10], g0);
  float g1 = h0 * w[9];
  g1 = fmaf(h1, w[11], g1);
  // layer 3: [2][1] at w[12..13]
  float y = g0 * w[12];
  return fmaf(g1, w[13], y);
}

__global__ __launch_bounds__(64) void ww_valu(float* W, int n, int steps) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  float w[14], o[14];
#pragma unroll
  for (int p = 0; p < 14; ++p) w[p] = W[(size_t)i * 16 + p];
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int p = 0; p < 14; ++p) o[p] = ww_net(w, w[p], c_feat[p][0], c_feat[p][1], c_feat[p][2]);
#pragma unroll
    for (int p = 0; p < 14; ++p) w[p] = o[p];
  }
#pragma unroll
  for (int p = 0; p < 14; ++p) W[(size_t)i * 16 + p] = w[p];
}

__device__ __forceinline__ float bperm(int src_lane, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

// 16 lanes per particle: lane t of the group owns point t (t < 14).  Block b = lane / 4
// covers points 4g .. 4g + 3 of particle q (g = (lane / 4) % 4).  D[b][i][j] sits in lane
// 4b + j, accumulator register i (units along i, points along j), so a layer's output for
// the lane's own point is in its own registers -- only the weights move between lanes.
__global__ __launch_bounds__(64) void ww_mfma(float* W, int n, int steps) {
  const int lane = threadIdx.x;
  const int t = lane & 15, q = lane >> 4, i4 = lane & 3;
  const int part = blockIdx.x * 4 + q;
  const bool live = part < n && t < 14;
  float w = live ? W[(size_t)part * 16 + t] : 0.f;
  const float f1 = c_feat[t][0], f2 = c_feat[t][1], f3 = c_feat[t][2];
  const int base = q * 16;
  for (int s = 0; s < steps; ++s) {
    // A operands: lane 4b + i needs unit i's weight for input k; units >= 2 (>= 1 at the
    // output) are padding
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const float feats[4] = {w, f1, f2, f3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a = bperm(base + 2 * k + (i4 & 1), w);
      a = i4 < 2 ? a : 0.f;
      acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a, feats[k], acc, 0, 0, 0);
    }
    f4 acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float a = bperm(base + 8 + 2 * k + (i4 & 1), w);
      a = i4 < 2 ? a : 0.f;
      acc2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, acc[k], acc2, 0, 0, 0);
    }
    f4 acc3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float a = bperm(base + 12 + k, w);
      a = i4 == 0 ? a : 0.f;
      acc3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, acc2[k], acc3, 0, 0, 0);
    }
    w = t < 14 ? acc3[0] : 0.f;
  }
  if (live) W[(size_t)part * 16 + t] = w;
}

// ------------------------------------------------------------------ (b) Agg(4,10,3) GEMV chain
// flat layout (Keras): L0 [4][10] at 0, L1 [10][10] at 40, L2 [10][10] at 140, L3 [10][4] at 240
constexpr int AP = 280;

__global__ __launch_bounds__(64) void agg_valu(const float* Wt, float* X, int n, int steps) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  float w[AP];
  const float4* src = reinterpret_cast<const float4*>(Wt + (size_t)i * AP);
#pragma unroll
  for (int k = 0; k < AP / 4; ++k) {
    const float4 v = src[k];
    w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
  }
  float x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = X[(size_t)i * 4 + k];
  for (int s = 0; s < steps; ++s) {
    float h[10], g[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      float y = x[0] * w[u];
#pragma unroll
      for (int k = 1; k < 4; ++k) y = fmaf(x[k], w[k * 10 + u], y);
      h[u] = y;
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      float y = h[0] * w[40 + u];
#pragma unroll
      for (int k = 1; k < 10; ++k) y = fmaf(h[k], w[40 + k * 10 + u], y);
      g[u] = y;
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      float y = g[0] * w[140 + u];
#pragma unroll
      for (int k = 1; k < 10; ++k) y = fmaf(g[k], w[140 + k * 10 + u], y);
      h[u] = y;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float y = h[0] * w[240 + u];
#pragma unroll
      for (int k = 1; k < 10; ++k) y = fmaf(h[k], w[240 + k * 4 + u], y);
      x[u] = y;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) X[(size_t)i * 4 + k] = x[k];
}

// 5 particles per wave: block b = 3 q + ug (q < 5, ug < 3: units 4ug .. 4ug + 3 of 10),
// block 15 idle.  Lane 4b + i keeps column (4ug + i) of every layer's kernel in registers
// (34 floats); the input element k is broadcast to the block's lanes with ds_bpermute from
// the block that produced it (block (q, k / 4), accumulator register k % 4).
template <int K, int O, int OFF>
__device__ __forceinline__ f4 agg_layer(const float (&wcol)[K], const f4 in, int qbase, int j) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float b = bperm(4 * (qbase + k / 4) + j, in[k % 4]);
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(wcol[k], b, acc, 0, 0, 0);
  }
  return acc;
}

__global__ __launch_bounds__(64) void agg_mfma(const float* Wt, float* X, int n, int steps) {
  const int lane = threadIdx.x;
  const int b = lane >> 2, i = lane & 3;
  const int q = b / 3, ug = b % 3;
  const int part = blockIdx.x * 5 + q;
  const bool live = b < 15 && part < n;
  const int u = 4 * ug + i;  // this lane's unit (column)
  float w0[4], w1[10], w2[10], w3[10];
  const float* row = Wt + (size_t)(live ? part : 0) * AP;
#pragma unroll
  for (int k = 0; k < 4; ++k) w0[k] = (live && u < 10) ? row[k * 10 + u] : 0.f;
#pragma unroll
  for (int k = 0; k < 10; ++k) w1[k] = (live && u < 10) ? row[40 + k * 10 + u] : 0.f;
#pragma unroll
  for (int k = 0; k < 10; ++k) w2[k] = (live && u < 10) ? row[140 + k * 10 + u] : 0.f;
#pragma unroll
  for (int k = 0; k < 10; ++k) w3[k] = (live && u < 4) ? row[240 + k * 4 + u] : 0.f;
  const int qbase = 3 * (b < 15 ? q : 0);
  // input: the aggregate state lives in block (q, 0), registers 0..3 (any lane j)
  f4 x = {0.f, 0.f, 0.f, 0.f};
  if (live && ug == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = X[(size_t)part * 4 + k];
  const int j = i;
  for (int s = 0; s < steps; ++s) {
    const f4 h = agg_layer<4, 10, 0>(w0, x, qbase, j);
    const f4 g = agg_layer<10, 10, 40>(w1, h, qbase, j);
    const f4 h2 = agg_layer<10, 10, 140>(w2, g, qbase, j);
    x = agg_layer<10, 4, 240>(w3, h2, qbase, j);
  }
  if (live && ug == 0 && i == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) X[(size_t)part * 4 + k] = x[k];
}

// ------------------------------------------------------------------ host
static float urand(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((s >> 40) & 0xFFFFFF) / 16777216.f;
}

template <class F>
static float time_ms(F&& launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const int na = argc > 1 ? std::atoi(argv[1]) : 100000;
  const int nb = argc > 2 ? std::atoi(argv[2]) : 1000000;
  const int steps = argc > 3 ? std::atoi(argv[3]) : 100;
  const int reps = 5;
  uint64_t seed = 12345;
  // (a) point features: layer / cell / weight ids of the 14 weights, normalised
  float feat[16][3] = {};
  {
    const int lay[3][2] = {{4, 2}, {2, 2}, {2, 1}};
    int p = 0;
    for (int l = 0; l < 3; ++l)
      for (int c = 0; c < lay[l][0]; ++c)
        for (int u = 0; u < lay[l][1]; ++u, ++p) {
          feat[p][0] = l / 2.f;
          feat[p][1] = lay[l][0] > 1 ? c / float(lay[l][0] - 1) : 0.f;
          feat[p][2] = lay[l][1] > 1 ? u / float(lay[l][1] - 1) : 0.f;
        }
  }
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_feat), feat, sizeof(feat)));
  std::vector<float> ha((size_t)na * 16, 0.f);
  for (int i = 0; i < na; ++i)
    for (int p = 0; p < 14; ++p) ha[(size_t)i * 16 + p] = (urand(seed) * 2.f - 1.f) * 0.9f;
  float *dA, *dB;
  CK(hipMalloc(&dA, ha.size() * 4));
  CK(hipMalloc(&dB, ha.size() * 4));
  // correctness after 3 applications
  auto run_a = [&](bool mfma, float* d, int st) {
    if (mfma) hipLaunchKernelGGL(ww_mfma, dim3((na + 3) / 4), dim3(64), 0, 0, d, na, st);
    else hipLaunchKernelGGL(ww_valu, dim3((na + 63) / 64), dim3(64), 0, 0, d, na, st);
  };
  CK(hipMemcpy(dA, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  run_a(false, dA, 3);
  run_a(true, dB, 3);
  CK(hipDeviceSynchronize());
  std::vector<float> ra(ha.size()), rb(ha.size());
  CK(hipMemcpy(ra.data(), dA, ha.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rb.data(), dB, ha.size() * 4, hipMemcpyDeviceToHost));
  double maxrel = 0;
  size_t nbit = 0, ncmp = 0;
  for (size_t k = 0; k < ra.size(); ++k) {
    if (!std::isfinite(ra[k]) || !std::isfinite(rb[k])) continue;
    ++ncmp;
    nbit += ra[k] == rb[k];
    maxrel = std::max(maxrel, (double)std::fabs(ra[k] - rb[k]) / (std::fabs(ra[k]) + 1e-6));
  }
  std::printf("{\"case\": \"ww22_check\", \"steps\": 3, \"max_rel_diff\": %.3e, \"bitwise_equal_frac\": %.4f}\n",
              maxrel, ncmp ? (double)nbit / ncmp : 0.0);
  for (int m = 0; m < 2; ++m) {
    const float ms = time_ms([&] {
      CK(hipMemcpyAsync(dA, ha.data(), 0, hipMemcpyHostToDevice));
      run_a(m == 1, dA, steps);
    }, reps);
    std::printf("{\"case\": \"ww22_self_apply\", \"kernel\": \"%s\", \"n\": %d, \"steps\": %d, \"ms\": %.4f, "
                "\"particle_steps_per_s\": %.4e}\n",
                m ? "mfma_4x4x1_16b" : "valu_lane_per_particle", na, steps, ms, (double)na * steps / (ms * 1e-3));
  }
  CK(hipFree(dA));
  CK(hipFree(dB));

  // (b) Agg(4,10,3) forward chain
  std::vector<float> hw((size_t)nb * AP), hx((size_t)nb * 4);
  for (auto& v : hw) v = (urand(seed) * 2.f - 1.f) * 0.55f;  // ~unit gain per 10-wide layer
  for (auto& v : hx) v = urand(seed) * 2.f - 1.f;
  float *dW, *dX1, *dX2;
  CK(hipMalloc(&dW, hw.size() * 4));
  CK(hipMalloc(&dX1, hx.size() * 4));
  CK(hipMalloc(&dX2, hx.size() * 4));
  CK(hipMemcpy(dW, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  auto run_b = [&](bool mfma, float* x, int st) {
    if (mfma) hipLaunchKernelGGL(agg_mfma, dim3((nb + 4) / 5), dim3(64), 0, 0, dW, x, nb, st);
    else hipLaunchKernelGGL(agg_valu, dim3((nb + 63) / 64), dim3(64), 0, 0, dW, x, nb, st);
  };
  CK(hipMemcpy(dX1, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dX2, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  run_b(false, dX1, 3);
  run_b(true, dX2, 3);
  CK(hipDeviceSynchronize());
  std::vector<float> xa(hx.size()), xb(hx.size());
  CK(hipMemcpy(xa.data(), dX1, hx.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(xb.data(), dX2, hx.size() * 4, hipMemcpyDeviceToHost));
  maxrel = 0, nbit = 0, ncmp = 0;
  for (size_t k = 0; k < xa.size(); ++k) {
    if (!std::isfinite(xa[k]) || !std::isfinite(xb[k])) continue;
    ++ncmp;
    nbit += xa[k] == xb[k];
    maxrel = std::max(maxrel, (double)std::fabs(xa[k] - xb[k]) / (std::fabs(xa[k]) + 1e-6));
  }
  std::printf("{\"case\": \"agg4_10_3_check\", \"steps\": 3, \"max_rel_diff\": %.3e, \"bitwise_equal_frac\": %.4f}\n",
              maxrel, ncmp ? (double)nbit / ncmp : 0.0);
  for (int m = 0; m < 2; ++m) {
    const float ms = time_ms([&] { run_b(m == 1, dX1, steps); }, reps);
    std::printf("{\"case\": \"agg4_10_3_forward_chain\", \"kernel\": \"%s\", \"n\": %d, \"steps\": %d, \"ms\": %.4f, "
                "\"particle_steps_per_s\": %.4e}\n",
                m ? "mfma_4x4x1_16b" : "valu_lane_per_particle", nb, steps, ms, (double)nb * steps / (ms * 1e-3));
  }
  CK(hipFree(dW));
  CK(hipFree(dX1));
  CK(hipFree(dX2));
  return 0;
}
