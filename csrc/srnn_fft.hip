// FFT-reduction shapes (defined real-valued semantics, see srnn_core.h FFTNet;
// reference code/network.py:442-521).
#include "srnn_kernels.h"

using FFT_4_2_2 = srnn::FFTNet<4, 2, 2>;
using FFT_2_2_2 = srnn::FFTNet<2, 2, 2>;

extern "C" int srnn_dispatch_fft(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY(FFT_4_2_2, 2, 2, 4)
  SRNN_TRY(FFT_2_2_2, 2, 2, 2)
  return 1;
}
