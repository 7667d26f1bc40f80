// Dispatchers not linked into the sanitizer self-test (shape "not instantiated").
#include "../srnn_abi.h"
extern "C" int srnn_dispatch_rnn(int, const SrnnCfg*, const SrnnArgs*) { return 1; }
extern "C" int srnn_dispatch_fft(int, const SrnnCfg*, const SrnnArgs*) { return 1; }
extern "C" int srnn_dispatch_aggbig(int, const SrnnCfg*, const SrnnArgs*) { return 1; }
extern "C" int srnn_dispatch_lowp(int, const SrnnCfg*, const SrnnArgs*) { return 1; }
extern "C" int srnn_dispatch_wwwide(int, const SrnnCfg*, const SrnnArgs*) { return 1; }
