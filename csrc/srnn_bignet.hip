// srnn_bignet.hip — dispatch of the big aggregating nets (kernels: srnn_bignet.h, one
// shape per srnn_bignet_<a>_<w>_<d>.hip)
#include "srnn_bignet.h"

extern "C" int srnn_big_4_10_3(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_big_4_8_2(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_big_4_16_2(int op, const SrnnCfg* c, const SrnnArgs* a);

#define SRNN_TRY_BIG(FN, W_, D_, A_)                                                   \
  if (c->width == (W_) && c->depth == (D_) && c->aggregates == (A_)) {                 \
    using T = srnn::AggBig<A_, W_, D_>;                                                \
    if (c->p != T::P || c->pp != T::PP) {                                              \
      srnn::set_error("layout mismatch (p/pp) for instantiated shape");                \
      return -4;                                                                       \
    }                                                                                  \
    if (op < 0) return 0;                                                              \
    return FN(op, c, a);                                                               \
  }

extern "C" int srnn_aggbig_serves(int op, int dtype, int shuffler) { return srnn::big_serves(op, dtype, shuffler) ? 1 : 0; }

extern "C" int srnn_dispatch_aggbig(int op, const SrnnCfg* c, const SrnnArgs* a) {
  SRNN_TRY_BIG(srnn_big_4_10_3, 10, 3, 4)
  SRNN_TRY_BIG(srnn_big_4_8_2, 8, 2, 4)
  SRNN_TRY_BIG(srnn_big_4_16_2, 16, 2, 4)
  return 1;
}
