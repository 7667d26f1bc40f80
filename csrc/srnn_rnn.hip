// Recurrent shapes instantiated for the population kernels (reference default
// (width=2, depth=2); code/network.py:526-535).
#include "srnn_kernels.h"

using RNN_1_1 = srnn::Recurrent<1, 1>;
using RNN_2_1 = srnn::Recurrent<2, 1>;
using RNN_2_2 = srnn::Recurrent<2, 2>;
using RNN_2_3 = srnn::Recurrent<2, 3>;
using RNN_4_2 = srnn::Recurrent<4, 2>;

extern "C" int srnn_dispatch_rnn(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY(RNN_2_2, 2, 2, 0)
  SRNN_TRY(RNN_1_1, 1, 1, 0)
  SRNN_TRY(RNN_2_1, 2, 1, 0)
  SRNN_TRY(RNN_2_3, 2, 3, 0)
  SRNN_TRY(RNN_4_2, 4, 2, 0)
  return 1;
}
