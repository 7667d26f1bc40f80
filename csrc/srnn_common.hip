// srnn_common.hip — ABI entry points, error handling and device scans of libsrnn.so.
#include "srnn_kernels.h"
#include <hipcub/hipcub.hpp>
#include <cstring>
#include <cstdlib>
#include <string>
#include <dlfcn.h>

namespace srnn {
static thread_local std::string g_err;
void set_error(const char* msg) { g_err = msg ? msg : ""; }
}  // namespace srnn

extern "C" int srnn_dispatch_ww(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_agg(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_rnn(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_fft(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_aggbig(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_dispatch_lowp(int op, const SrnnCfg* c, const SrnnArgs* a);

__global__ void k_scan_tail(int32_t* out, const int32_t* in, int64_t n) {
  // out[0] = 0 (inclusive scan was written to out+1)
  out[0] = 0;
  (void)in;
  (void)n;
}

// ---- tracing / checking hooks, read once from the environment:
//   SRNN_ROCTX=1       one roctx range per operator launch (rocprofv3 --marker-trace),
//                      roctx resolved with dlopen (no link dependency)
//   SRNN_SYNC_CHECK=1  synchronise the stream after every device operator and report a
//                      fault at the operator that caused it (like HIP_LAUNCH_BLOCKING)
namespace {
typedef int (*push_fn)(const char*);
typedef int (*pop_fn)();
struct Hooks {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  bool sync = false;
  Hooks() {
    const char* r = std::getenv("SRNN_ROCTX");
    if (r && r[0] == '1') {
      const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                            "libroctx64.so"};
      for (const char* l : libs) {
        void* h = dlopen(l, RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        push = (push_fn)dlsym(h, "roctxRangePushA");
        pop = (pop_fn)dlsym(h, "roctxRangePop");
        if (push && pop) break;
        push = nullptr;
        pop = nullptr;
      }
    }
    const char* sc = std::getenv("SRNN_SYNC_CHECK");
    sync = sc && sc[0] == '1';
  }
};
const Hooks& hooks() {
  static Hooks h;
  return h;
}
const char* op_name(int op) {
  static const char* names[] = {"srnn:init",       "srnn:apply",        "srnn:run_fixpoint", "srnn:train",
                                "srnn:learn",      "srnn:classify",     "srnn:perturb",      "srnn:soup_decide",
                                "srnn:respawn_seq", "srnn:soup_evolve", "srnn:scan",         "srnn:respawn",
                                "srnn:vary_run",   "srnn:soup_pack",    "srnn:soup_unpack",  "srnn:uid_assign",
                                "srnn:soup_gen"};
  return (op >= 0 && op < (int)(sizeof(names) / sizeof(names[0]))) ? names[op] : "srnn:op";
}
}  // namespace

static int dispatch(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (c->dtype != 0) {
    if (c->dtype != 1 && c->dtype != 2) {
      srnn::set_error("unknown weight-table dtype");
      return -1;
    }
    return srnn_dispatch_lowp(op, c, a);
  }
  switch (c->kind) {
    case 0: return srnn_dispatch_ww(op, c, a);
    case 1: {
      int r = srnn_dispatch_agg(op, c, a);
      return r == 1 ? srnn_dispatch_aggbig(op, c, a) : r;
    }
    case 2: return srnn_dispatch_rnn(op, c, a);
    case 3: return srnn_dispatch_fft(op, c, a);
    default: srnn::set_error("unknown network kind"); return -1;
  }
}

extern "C" {

int srnn_abi_version() { return 11; }

const char* srnn_last_error() { return srnn::g_err.c_str(); }

int srnn_has_config(const SrnnCfg* cfg) {
  int r = dispatch(-1, cfg, nullptr);
  return r == 0 ? 1 : 0;
}

int64_t srnn_scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return (int64_t)bytes;
}

int srnn_run(int op, const SrnnCfg* cfg, const SrnnArgs* a) {
  srnn::set_error("");
  if (op == OP_SCAN) {
    // i32d[0] = 0, i32d[k+1] = sum_{q<=k} i32c[q]
    if (!a->dev) {
      int64_t acc = 0;
      a->i32d[0] = 0;
      for (int64_t k = 0; k < a->n; ++k) {
        acc += a->i32c[k];
        a->i32d[k + 1] = (int32_t)acc;
      }
      return 0;
    }
    hipStream_t st = (hipStream_t)a->stream;
    if (a->n > 0) {
      size_t bytes = (size_t)a->temp_bytes;
      hipError_t e = hipcub::DeviceScan::InclusiveSum(a->temp, bytes, a->i32c, a->i32d + 1, (int)a->n, st);
      if (e != hipSuccess) {
        srnn::set_error(hipGetErrorString(e));
        return -3;
      }
    }
    hipLaunchKernelGGL(k_scan_tail, dim3(1), dim3(1), 0, st, a->i32d, a->i32c, a->n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      srnn::set_error(hipGetErrorString(e));
      return -3;
    }
    return 0;
  }
  const Hooks& h = hooks();
  if (h.push) h.push(op_name(op));
  int r = dispatch(op, cfg, a);
  if (r == 1) srnn::set_error("network shape not instantiated in libsrnn (add it to csrc/srnn_<kind>.hip)");
  if (r == 0 && h.sync && a->dev) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing((hipStream_t)a->stream, &cs);
    if (cs == hipStreamCaptureStatusNone) {
      hipError_t e = hipStreamSynchronize((hipStream_t)a->stream);
      if (e == hipSuccess) e = hipGetLastError();
      if (e != hipSuccess) {
        std::string m = std::string(op_name(op)) + ": " + hipGetErrorString(e);
        srnn::set_error(m.c_str());
        r = -5;
      }
    }
  }
  if (h.pop) h.pop();
  return r;
}

}  // extern "C"
