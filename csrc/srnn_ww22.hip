// Weightwise(2, 2) -- the reference's default net and the headline soup's -- in its own
// translation unit (its lane, lane-pair and reference-order kernels are the ones that change
// most often; one file per shape keeps `make -j` rebuilds parallel).
#include "srnn_kernels.h"

using WW_2_2 = srnn::Weightwise<2, 2>;

extern "C" int srnn_dispatch_ww22(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY(WW_2_2, 2, 2, 0)
  return 1;
}
