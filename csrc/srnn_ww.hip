// Weightwise shapes instantiated for the population kernels (reference default (2,2);
// code/network.py:222-230).  Add a line to support another (width, depth).
#include "srnn_kernels.h"

extern "C" int srnn_dispatch_wwwide(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_ww22(int op, const SrnnCfg* c, const SrnnArgs* a);  // srnn_ww22.hip

using WW_1_1 = srnn::Weightwise<1, 1>;
using WW_2_1 = srnn::Weightwise<2, 1>;
using WW_2_3 = srnn::Weightwise<2, 3>;
using WW_3_2 = srnn::Weightwise<3, 2>;
using WW_4_2 = srnn::Weightwise<4, 2>;
using WW_4_3 = srnn::Weightwise<4, 3>;
using WW_8_2 = srnn::Weightwise<8, 2>;

extern "C" int srnn_dispatch_ww(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (c->width == 2 && c->depth == 2 && c->aggregates == 0) return srnn_dispatch_ww22(op, c, a);
  SRNN_TRY(WW_1_1, 1, 1, 0)
  SRNN_TRY(WW_2_1, 2, 1, 0)
  SRNN_TRY(WW_2_3, 2, 3, 0)
  SRNN_TRY(WW_3_2, 3, 2, 0)
  SRNN_TRY(WW_4_2, 4, 2, 0)
  SRNN_TRY(WW_4_3, 4, 3, 0)
  SRNN_TRY(WW_8_2, 8, 2, 0)
  return srnn_dispatch_wwwide(op, c, a);  // width 16/32: MFMA wave-per-particle path
}
