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
