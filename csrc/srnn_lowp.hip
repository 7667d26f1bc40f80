// 16-bit weight tables: bf16 / fp16 storage with fp32 arithmetic (SURVEY §7.7,
// BASELINE.json configs #2 "10k-particle weightwise self-application, bf16" and #5
// "mixed learn+attack soup, fp16").  Same per-item code as the fp32 kernels
// (srnn_kernels.h); rows are 2 bytes per weight, read/written as 8-byte quads, and every
// application result is rounded to the storage format before it is used or compared.
#include "srnn_kernels.h"

using LP_WW_2_2 = srnn::Weightwise<2, 2>;
using LP_AGG_4_2_2 = srnn::Aggregating<4, 2, 2>;

extern "C" int srnn_dispatch_lowp(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (c->kind == 0) {
    SRNN_TRY_LOWP(LP_WW_2_2, 2, 2, 0)
  } else if (c->kind == 1) {
    SRNN_TRY_LOWP(LP_AGG_4_2_2, 2, 2, 4)
  }
  return 1;
}

// Storage encoding of fp32 values as the kernels perform it (dtype 1 = bf16, 2 = fp16), for
// the numerics test of the device rounding against the host formula.
template <class S>
__global__ void k_storage_encode(const float* __restrict__ x, uint16_t* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = S::enc(x[i]);
}

extern "C" int srnn_storage_encode(const float* x, void* out, int64_t n, int dtype, void* stream) {
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 1)
    hipLaunchKernelGGL(k_storage_encode<srnn::StBF16>, grid, block, 0, st, x, (uint16_t*)out, n);
  else if (dtype == 2)
    hipLaunchKernelGGL(k_storage_encode<srnn::StF16>, grid, block, 0, st, x, (uint16_t*)out, n);
  else
    return 1;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
