// AggBig<4, 8, 2>: every big-net operator of srnn_bignet.h for this shape (its own
// translation unit so the shapes compile in parallel)
#include "srnn_bignet.h"

extern "C" int srnn_big_4_8_2(int op, const SrnnCfg* c, const SrnnArgs* a) {
  return srnn::big_run<srnn::AggBig<4, 8, 2>>(op, *c, *a);
}
