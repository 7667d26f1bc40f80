// srnn_common.hip — ABI entry points, error handling and device scans of libsrnn.so.
#include "srnn_kernels.h"
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
extern "C" int srnn_aggbig_serves(int op, int dtype, int shuffler);
extern "C" int srnn_dispatch_lowp(int op, const SrnnCfg* c, const SrnnArgs* a);

extern "C" int srnn_dispatch_generic(int op, const SrnnCfg* c, const SrnnArgs* a);
extern "C" int srnn_x2_run(int op, const SrnnCfg* c, const SrnnArgs* a);

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
  switch (op) {
    case OP_INIT: return "srnn:init";
    case OP_APPLY: return "srnn:apply";
    case OP_RUN_FIXPOINT: return "srnn:run_fixpoint";
    case OP_TRAIN: return "srnn:train";
    case OP_LEARN: return "srnn:learn";
    case OP_CLASSIFY: return "srnn:classify";
    case OP_PERTURB: return "srnn:perturb";
    case OP_SOUP_DECIDE: return "srnn:soup_decide";
    case OP_RESPAWN_SEQ: return "srnn:respawn_seq";
    case OP_SOUP_EVOLVE: return "srnn:soup_evolve";
    case OP_RESPAWN: return "srnn:respawn";
    case OP_VARY_RUN: return "srnn:vary_run";
    case OP_UID_ASSIGN: return "srnn:uid_assign";
    case OP_SOUP_GEN: return "srnn:soup_gen";
    case OP_GEN_FINISH: return "srnn:gen_finish";
    case OP_SOUP_SEQ: return "srnn:soup_seq";
    case OP_X2_PACK: return "srnn:x2_pack";
    case OP_X2_POST: return "srnn:x2_post";
    case OP_SOUP_ORDERED: return "srnn:soup_ordered";
    case OP_SOUP_ORDERED_SH: return "srnn:soup_ordered_sh";
    case OP_ORD_PLAN: return "srnn:ord_plan";
    case OP_ORD_CENSUS: return "srnn:ord_census";
    default: return "srnn:op";
  }
}
}  // namespace

// Specialised (templated) paths first; 1 = shape not instantiated, 2 = op / host execution
// not provided by the specialised path: both fall through to the runtime-shape engine.
static int dispatch_special(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (c->dtype != 0) {
    if (c->dtype != 1 && c->dtype != 2) {
      srnn::set_error("unknown weight-table dtype");
      return -1;
    }
    const int r = srnn_dispatch_lowp(op, c, a);
    // big aggregating nets take every storage format in their own row kernels
    return (r == 1 && c->kind == 1) ? srnn_dispatch_aggbig(op, c, a) : r;
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

// ---- execution knobs (srnn_abi.h SrnnKnob; config.py ExecConfig): environment variable if
// set (read on every query: A/B tests flip it between calls), else the value set through the
// API, else the built-in default
namespace {
const char* const g_knob_env[SRNN_KNOB_COUNT] = {"SRNN_FORCE_GENERIC", "SRNN_RNN_WAVE", "SRNN_RNN_SPEC",
                                                 "SRNN_RNN_SOUP",      "SRNN_WW_WAVE",  "SRNN_BIG_WAVE",
                                                 "SRNN_FIX_GROUP",     "SRNN_SOUP_LANES", "SRNN_ORD_CRIT",
                                                 "SRNN_ORD_QUEUE",     "SRNN_ORD_SHADOW", "SRNN_ORD_BULK_DELAY"};
// (every knob starts at -1 = its built-in default)
int g_knob[SRNN_KNOB_COUNT] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
static_assert(sizeof(g_knob) / sizeof(g_knob[0]) == SRNN_KNOB_COUNT && SRNN_KNOB_COUNT == 12, "one -1 per knob");
}  // namespace
namespace srnn {
int knob(int id, int dflt) {
  if (id < 0 || id >= SRNN_KNOB_COUNT) return dflt;
  const char* e = std::getenv(g_knob_env[id]);
  if (e && *e) return std::atoi(e);
  return g_knob[id] >= 0 ? g_knob[id] : dflt;
}
}  // namespace srnn
static bool force_generic() { return srnn::knob(SRNN_KNOB_FORCE_GENERIC, 0) == 1; }

// which engine serves (op, cfg, host/device): 0 specialised, 1 generic, -1 none
static int route(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (!force_generic()) {
    SrnnArgs probe{};
    probe.dev = a ? a->dev : 1;
    const int r = dispatch_special(-1, c, &probe);
    if (r == 0) {
      // instantiated: does the specialised path provide this op (on this side)?
      const int k = c->kind == 1 && c->p > 64 ? 1 : (c->kind == 0 && c->width >= 16 ? 2 : 0);
      if (k == 0) return 0;  // lane-per-particle templates: every op, host and device
      const bool host = a && !a->dev;
      if (host) return 1;  // wave-per-particle paths are GPU only
      if (k == 1 && srnn_aggbig_serves(op, c->dtype, c->shuffler)) return 0;
      if (k == 2 && (op == OP_INIT || op == OP_APPLY || op == OP_RUN_FIXPOINT || op == OP_CLASSIFY)) return 0;
      return 1;
    }
    if (r < 0 && r != -1) return -1;  // layout mismatch etc.
  }
  return srnn_dispatch_generic(-1, c, a) == 0 ? 1 : -1;
}

static int dispatch(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (op < 0) return route(0, c, a) >= 0 ? 0 : 1;
  const int r = route(op, c, a);
  if (r == 0) return dispatch_special(op, c, a);
  if (r == 1) {
    const int g = srnn_dispatch_generic(op, c, a);
    if (g == 2) {
      srnn::set_error("op not supported for this network shape (fused soup generations need an instantiated shape)");
      return -1;
    }
    return g;
  }
  return 1;
}

// Device scratch of the generic engine when the caller passes none: one grow-only buffer
// per device (allocated outside graph captures: the first eager call sizes it).
static void* g_scratch[64] = {nullptr};
static int64_t g_scratch_bytes[64] = {0};

static int with_scratch(int op, const SrnnCfg* c, const SrnnArgs* a) {
  if (!a->dev || a->scratch || route(op, c, a) != 1 || op == OP_SOUP_DECIDE)
    return dispatch(op, c, a);
  const int64_t want = srnn_generic_scratch_bytes(c, a->n, 65536);
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (want > g_scratch_bytes[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing((hipStream_t)a->stream, &cs);
    if (cs != hipStreamCaptureStatusNone) {
      srnn::set_error("generic engine: scratch must be allocated before graph capture (pass SrnnArgs.scratch)");
      return -5;
    }
    if (g_scratch[dev]) {
      (void)hipDeviceSynchronize();
      (void)hipFree(g_scratch[dev]);
      g_scratch[dev] = nullptr;
      g_scratch_bytes[dev] = 0;
    }
    if (hipMalloc(&g_scratch[dev], (size_t)want) != hipSuccess) {
      srnn::set_error("generic engine: scratch allocation failed");
      return -3;
    }
    g_scratch_bytes[dev] = want;
  }
  SrnnArgs b = *a;
  b.scratch = g_scratch[dev];
  b.scratch_bytes = g_scratch_bytes[dev];
  return dispatch(op, c, &b);
}

// ---- do two streams run concurrently?  (SRNN_F_ORD_SYNC graphs order their two streams by device
// counters: a profiler that serialises kernels -- rocprofv3 --pmc -- or two streams that share a
// hardware queue would turn every wait into a timeout.)  The waiter on `side` spins (bounded by
// `timeout_us` of the 100 MHz real-time clock) for the flag the setter on `main` raises; f[1]:
// 1 seen, 2 timed out.
__global__ void k_stream_probe_wait(int32_t* f, int64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1) {
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) {
      __hip_atomic_store(f + 1, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(f + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_stream_probe_set(int32_t* f) {
  if (threadIdx.x == 0) __hip_atomic_store(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

extern "C" {

int srnn_abi_version() { return 31; }

int srnn_stream_probe(int32_t* flag, void* side, void* main_stream, int64_t timeout_us) {
  hipLaunchKernelGGL(k_stream_probe_wait, dim3(1), dim3(64), 0, (hipStream_t)side, flag, timeout_us * 100);
  hipLaunchKernelGGL(k_stream_probe_set, dim3(1), dim3(64), 0, (hipStream_t)main_stream, flag);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    srnn::set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}


// layout check of the ctypes mirror (ops/_lib.py): sizeof(SrnnArgs) / sizeof(SrnnCfg)
int64_t srnn_args_size() { return (int64_t)sizeof(SrnnArgs); }
int64_t srnn_cfg_size() { return (int64_t)sizeof(SrnnCfg); }

const char* srnn_last_error() { return srnn::g_err.c_str(); }

int srnn_has_config(const SrnnCfg* cfg) {
  SrnnArgs probe{};
  probe.dev = 0;
  return route(0, cfg, &probe) >= 0 ? 1 : 0;
}

void srnn_set_force_generic(int on) { srnn_set_knob(SRNN_KNOB_FORCE_GENERIC, on ? 1 : 0); }
void srnn_set_knob(int id, int value) {
  if (id >= 0 && id < SRNN_KNOB_COUNT) g_knob[id] = value < 0 ? -1 : value;
}
int srnn_get_knob(int id) { return srnn::knob(id, -1); }

int srnn_is_generic(const SrnnCfg* cfg, int op) {
  SrnnArgs probe{};
  probe.dev = 1;
  return route(op, cfg, &probe) == 1 ? 1 : 0;
}

// 1 when `op` of this configuration has an implementation on the host (dev 0) / device (dev 1)
int srnn_supports(const SrnnCfg* cfg, int op, int dev) {
  SrnnArgs probe{};
  probe.dev = dev;
  const int r = route(op, cfg, &probe);
  if (r == 0) return 1;
  return r == 1 && srnn_generic_op_supported(op, dev) ? 1 : 0;
}

int srnn_run(int op, const SrnnCfg* cfg, const SrnnArgs* a) {
  srnn::set_error("");
  const Hooks& h = hooks();
  if (op == OP_X2_PACK || op == OP_X2_POST || op == OP_UID_ASSIGN) {
    // the exchange protocol is shape independent (srnn_shard.hip)
    if (h.push) h.push(op_name(op));
    const int r = srnn_x2_run(op, cfg, a);
    if (h.pop) h.pop();
    return r;
  }
  if (h.push) h.push(op_name(op));
  int r = with_scratch(op, cfg, a);
  if (r == 1) srnn::set_error("not a valid network shape for libsrnn");
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
