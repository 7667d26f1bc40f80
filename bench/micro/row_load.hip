// Row-load micro-benchmark for the P = 280 lane-per-particle kernels (srnn_bignet.h): how
// fast can 64 lanes of a wave get 64 rows of 1120 bytes each into their registers?
//
//   stream   coalesced read of the table (1 KB per wave instruction), per-lane partial sums:
//            the read-bandwidth ceiling
//   lane     every lane loads its own row with 70 global_load_dwordx4 (the current kernels):
//            each wave instruction touches 64 cache lines 1120 B apart
//   lane_nt  the same with non-temporal loads
//   lds      the wave's 64 rows are read in 4 passes of 18 float4 per row, coalesced
//            (a wave instruction covers ~3.6 row segments of 288 B), staged through LDS with a
//            19-float4 row pitch (conflict-free ds_read_b128), then each lane reads its row
//   lds2     lds with the next pass's loads issued before the current pass is staged
//
// Each variant writes one float per row (sum of the row) and is checked against `lane`.
// Output: one JSON line per variant.  Build: hipcc -O3 --offload-arch=gfx950 row_load.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int P4 = 70;   // float4 per row (P = 280)
constexpr int TB = 256;  // 4 waves
constexpr int PITCH = 19;  // float4 pitch of a staged row segment (76 dwords: 12 L mod 64 distinct)

__global__ __launch_bounds__(TB) void k_stream(const float4* __restrict__ W, float* __restrict__ out, int64_t n) {
  // wave w of the grid reads the same 64-row block as the other variants, coalesced
  const int64_t wave = ((int64_t)blockIdx.x * TB + threadIdx.x) >> 6;
  const int L = threadIdx.x & 63;
  const int64_t r0 = wave * 64;
  if (r0 >= n) return;
  const int64_t nf4 = (n - r0 < 64 ? n - r0 : 64) * P4;
  const float4* b = W + r0 * P4;
  float s = 0.f;
#pragma unroll 10
  for (int k = 0; k < P4; ++k) {
    const int64_t t = (int64_t)k * 64 + L;
    if (t < nf4) {
      const float4 v = b[t];
      s += v.x + v.y + v.z + v.w;
    }
  }
  if (r0 + L < n) out[r0 + L] = s;  // not the row sum: bandwidth only
}

template <bool NT>
__global__ __launch_bounds__(TB) void k_lane(const float4* __restrict__ W, float* __restrict__ out, int64_t n) {
  const int64_t p = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (p >= n) return;
  const float4* r = W + p * P4;
  float4 v[P4];
#pragma unroll
  for (int q = 0; q < P4; ++q) {
    if constexpr (NT) {
      const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(r) + q);
      v[q] = make_float4(t.x, t.y, t.z, t.w);
    } else {
      v[q] = r[q];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < P4; ++q) s += (v[q].x + v[q].y) + (v[q].z + v[q].w);
  out[p] = s;
}

// pass s covers float4 [Q s, Q s + Q) of every row (the last pass: what is left), staged with
// an LDS row pitch of Q + 1 float4 (Q even: 4 (Q + 1) dwords, an odd multiple of 4 -> the 16
// lanes of a ds_read_b128 quarter-wave hit distinct 4-bank groups)
template <int Q>
__global__ __launch_bounds__(TB) void k_lds(const float4* __restrict__ W, float* __restrict__ out, int64_t n) {
  constexpr int PI = Q + 1, NPASS = (P4 + Q - 1) / Q;
  __shared__ float4 s_st[4 * 64 * PI];
  const int wv = threadIdx.x >> 6, L = threadIdx.x & 63;
  float4* st = s_st + wv * 64 * PI;
  const int64_t r0 = ((int64_t)blockIdx.x * TB) + wv * 64;
  const int64_t p = r0 + L;
  if (r0 >= n) return;
  const int nr = n - r0 < 64 ? (int)(n - r0) : 64;
  const float4* blk = W + r0 * P4;
  // piece k of a pass: row (64 k + L) / Q, float4 (64 k + L) % Q of the pass
  int off[Q], lo[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    const int t = k * 64 + L, r = t / Q, f = t - r * Q;
    off[k] = r < nr ? r * P4 + f : -1;
    lo[k] = r * PI + f;
  }
  float sum = 0.f;  // streaming consumer (same summation order as k_lane)
#pragma unroll 1
  for (int s = 0; s < NPASS; ++s) {
    const int len = P4 - Q * s < Q ? P4 - Q * s : Q;
    float4 b[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      const bool ok = off[k] >= 0 && (off[k] % P4) < len;
      b[k] = blk[ok ? off[k] + Q * s : 0];
    }
#pragma unroll
    for (int k = 0; k < Q; ++k) st[lo[k]] = b[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (q < len) {
        const float4 v = st[L * PI + q];
        sum += (v.x + v.y) + (v.z + v.w);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (p < n) out[p] = sum;
}

__global__ void k_fill(float* W, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) W[i] = (float)((i * 2654435761ull >> 7) & 1023) * (1.0f / 1024.0f);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
  float4* W;
  float *o_ref, *o;
  CK(hipMalloc(&W, n * P4 * sizeof(float4)));
  CK(hipMalloc(&o_ref, n * sizeof(float)));
  CK(hipMalloc(&o, n * sizeof(float)));
  const int64_t nf = n * P4 * 4;
  k_fill<<<(nf + 255) / 256, 256>>>(reinterpret_cast<float*>(W), nf);
  const int grid = (int)((n + TB - 1) / TB);
  k_lane<false><<<grid, TB>>>(W, o_ref, n);
  CK(hipDeviceSynchronize());
  std::vector<float> ref(n), got(n);
  CK(hipMemcpy(ref.data(), o_ref, n * sizeof(float), hipMemcpyDeviceToHost));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)n * P4 * 16;
  auto run = [&](const char* name, auto launch, bool check) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    int bad = 0;
    if (check) {
      CK(hipMemcpy(got.data(), o, n * sizeof(float), hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < n; ++i) bad += got[i] != ref[i];
    }
    std::printf("{\"variant\": \"%s\", \"n\": %lld, \"ms\": %.4f, \"TBps\": %.3f, \"mismatch\": %d}\n", name,
                (long long)n, best, bytes / (best * 1e-3) / 1e12, bad);
  };
  run("stream", [&] { k_stream<<<grid, TB>>>(W, o, n); }, false);
  run("lane", [&] { k_lane<false><<<grid, TB>>>(W, o, n); }, true);
  run("lane_nt", [&] { k_lane<true><<<grid, TB>>>(W, o, n); }, true);
  run("lds_q18", [&] { k_lds<18><<<grid, TB>>>(W, o, n); }, true);
  run("lds_q8", [&] { k_lds<8><<<grid, TB>>>(W, o, n); }, true);
  run("lds_q12", [&] { k_lds<12><<<grid, TB>>>(W, o, n); }, true);
  run("lds_q24", [&] { k_lds<24><<<grid, TB>>>(W, o, n); }, true);
  CK(hipFree(W));
  CK(hipFree(o_ref));
  CK(hipFree(o));
  return 0;
}
