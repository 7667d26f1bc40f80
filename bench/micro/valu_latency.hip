// VALU issue / dependency-latency probe (gfx950): cycles per instruction for one and two
// waves per SIMD, dependent vs independent chains, scalar fma vs v_pk_fma_f32.
// hipcc --offload-arch=gfx950 -O3 -o valu_latency valu_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CHAINS>
__global__ void k_fma(float* out, int iters, float a, float b) {
  float x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 64 / CHAINS; ++r)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fmaf(x[c], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_pk(float* out, int iters, float a, float b) {
  f2 x[CHAINS];
  f2 av = {a, a * 0.5f}, bv = {b, b * 0.25f};
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = f2{threadIdx.x * 1e-3f + c, (float)c};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 64 / CHAINS; ++r)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c].x + x[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
float time_ms(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int dev = 0, clk = 0, cus = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int simds = cus * 4, iters = 2000;
  float* out;
  hipMalloc(&out, sizeof(float) * simds * 64 * 8);
  printf("{\"clock_khz\": %d, \"cus\": %d}\n", clk, cus);
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int waves = simds * wps;  // 64-thread blocks, round-robin over SIMDs
    auto run = [&](const char* name, auto kern) {
      float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, out, iters, 0.999f, 1e-3f); });
      double instr_per_wave = (double)iters * 64;
      double cyc = ms * 1e-3 * clk * 1e3 / (instr_per_wave * wps);
      printf("{\"waves_per_simd\": %d, \"kernel\": \"%s\", \"ms\": %.4f, \"cycles_per_instr_per_simd\": %.2f}\n", wps,
             name, ms, cyc);
    };
    run("fma_dep1", k_fma<1>);
    run("fma_chains4", k_fma<4>);
    run("fma_chains16", k_fma<16>);
    run("pk_dep1", k_pk<1>);
    run("pk_chains4", k_pk<4>);
    run("pk_chains16", k_pk<16>);
  }
  hipFree(out);
  return 0;
}
