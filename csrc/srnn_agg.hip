// Aggregating shapes instantiated for the population kernels (reference default
// (aggregates=4, width=2, depth=2); code/network.py:324-333).
#include "srnn_kernels.h"

using AGG_4_2_2 = srnn::Aggregating<4, 2, 2>;
using AGG_2_2_2 = srnn::Aggregating<2, 2, 2>;
using AGG_4_2_3 = srnn::Aggregating<4, 2, 3>;
using AGG_4_4_2 = srnn::Aggregating<4, 4, 2>;

extern "C" int srnn_dispatch_agg(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY(AGG_4_2_2, 2, 2, 4)
  SRNN_TRY(AGG_2_2_2, 2, 2, 2)
  SRNN_TRY(AGG_4_2_3, 2, 3, 4)
  SRNN_TRY(AGG_4_4_2, 4, 2, 4)
  return 1;
}
