// srnn_comm.cpp — native RCCL communicator of libsrnn.
//
// The sharded soup issues its per-generation collective (the row / stats all-to-all) and
// the stats all-gather through its OWN RCCL communicator on the caller's HIP stream, so
// the collective can sit inside a captured hipGraph next to the HIP kernels without any
// framework bookkeeping (torch's process-group watchdog queries the events of its work
// items and faults when one of them was recorded by a capturing stream).  torch.distributed
// is used only for launch and rendezvous: rank 0's ncclUniqueId is broadcast through it.
//
// librccl is resolved at run time with dlopen: by default the copy the running process
// already loaded (torch's), otherwise $SRNN_RCCL_LIB or /opt/rocm/lib/librccl.so — one RCCL
// instance per process, no link-time dependency.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace srnn {
void set_error(const char* msg);
}

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*all_to_all)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;      // optional: introspection
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
  std::string path;
};

std::mutex g_mu;
Rccl g_rccl;

template <class F>
bool sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

bool load(const char* hint) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_rccl.h) return true;
  const char* env = std::getenv("SRNN_RCCL_LIB");
  const char* cands[] = {hint, env, "librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"};
  for (const char* c : cands) {
    if (!c || !*c) continue;
    // prefer a copy that is already loaded (torch's): RTLD_NOLOAD first
    void* h = dlopen(c, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
    if (!h) h = dlopen(c, RTLD_NOW | RTLD_GLOBAL);
    if (!h) continue;
    Rccl r;
    r.h = h;
    bool ok = sym(h, "ncclGetUniqueId", r.get_unique_id) && sym(h, "ncclCommInitRank", r.comm_init_rank) &&
              sym(h, "ncclCommDestroy", r.comm_destroy) && sym(h, "ncclCommAbort", r.comm_abort) &&
              sym(h, "ncclCommGetAsyncError", r.async_error) && sym(h, "ncclAllToAll", r.all_to_all) &&
              sym(h, "ncclAllGather", r.all_gather) && sym(h, "ncclAllReduce", r.all_reduce) &&
              sym(h, "ncclGetErrorString", r.error_string);
    if (!ok) continue;
    sym(h, "ncclCommCount", r.comm_count);
    sym(h, "ncclCommUserRank", r.comm_user_rank);
    r.path = c;
    g_rccl = r;
    return true;
  }
  srnn::set_error("librccl not found (set SRNN_RCCL_LIB)");
  return false;
}

int check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  std::string m = std::string(what) + ": " + (g_rccl.error_string ? g_rccl.error_string(r) : "rccl error");
  srnn::set_error(m.c_str());
  return -10 - (int)r;
}

}  // namespace

extern "C" {

// 1 if RCCL could be loaded (optionally from `lib_hint`, e.g. torch's librccl path)
int srnn_comm_available(const char* lib_hint) { return load(lib_hint) ? 1 : 0; }

const char* srnn_comm_library() { return g_rccl.h ? g_rccl.path.c_str() : ""; }

int srnn_comm_unique_id(const char* lib_hint, uint8_t* out, int out_bytes) {
  if (!load(lib_hint)) return -1;
  if (out_bytes < (int)sizeof(ncclUniqueId)) {
    srnn::set_error("unique id buffer too small");
    return -2;
  }
  ncclUniqueId id;
  int r = check(g_rccl.get_unique_id(&id), "ncclGetUniqueId");
  if (r) return r;
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(ncclUniqueId);
}

// communicator of `rank` among `world` on HIP device `device`; *out receives the handle
int srnn_comm_init(const char* lib_hint, const uint8_t* id_bytes, int world, int rank, int device, void** out) {
  if (!load(lib_hint)) return -1;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    srnn::set_error(hipGetErrorString(e));
    return -3;
  }
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t comm = nullptr;
  int r = check(g_rccl.comm_init_rank(&comm, world, id, rank), "ncclCommInitRank");
  if (r) return r;
  *out = comm;
  return 0;
}

int srnn_comm_destroy(void* comm, int abort) {
  if (!comm || !g_rccl.h) return 0;
  return check(abort ? g_rccl.comm_abort((ncclComm_t)comm) : g_rccl.comm_destroy((ncclComm_t)comm),
               abort ? "ncclCommAbort" : "ncclCommDestroy");
}

// 0 = healthy; otherwise the communicator's asynchronous error (failure detection)
int srnn_comm_async_error(void* comm) {
  if (!comm || !g_rccl.h) return 0;
  ncclResult_t a = ncclSuccess;
  int r = check(g_rccl.async_error((ncclComm_t)comm, &a), "ncclCommGetAsyncError");
  if (r) return r;
  return check(a, "async");
}

// ranks of the communicator and this process's rank in it, as RCCL reports them
// (ncclCommCount / ncclCommUserRank): the bench prints them so a run shows that RCCL saw N ranks
int srnn_comm_count(void* comm) {
  if (!comm || !g_rccl.comm_count) return -1;
  int n = -1;
  return check(g_rccl.comm_count((ncclComm_t)comm, &n), "ncclCommCount") ? -1 : n;
}
int srnn_comm_user_rank(void* comm) {
  if (!comm || !g_rccl.comm_user_rank) return -1;
  int r = -1;
  return check(g_rccl.comm_user_rank((ncclComm_t)comm, &r), "ncclCommUserRank") ? -1 : r;
}

// equal-split all-to-all of `bytes_per_peer` bytes per destination (4-byte granules)
int srnn_comm_all_to_all(void* comm, const void* send, void* recv, int64_t bytes_per_peer, void* stream) {
  if (bytes_per_peer % 4) {
    srnn::set_error("all-to-all block must be a multiple of 4 bytes");
    return -2;
  }
  return check(g_rccl.all_to_all(send, recv, (size_t)(bytes_per_peer / 4), ncclInt32, (ncclComm_t)comm,
                                 (hipStream_t)stream),
               "ncclAllToAll");
}

int srnn_comm_all_gather(void* comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream) {
  return check(g_rccl.all_gather(send, recv, (size_t)bytes_per_rank, ncclUint8, (ncclComm_t)comm, (hipStream_t)stream),
               "ncclAllGather");
}

// sum all-reduce of int64 (class histograms)
int srnn_comm_all_reduce_i64(void* comm, const void* send, void* recv, int64_t count, void* stream) {
  return check(g_rccl.all_reduce(send, recv, (size_t)count, ncclInt64, ncclSum, (ncclComm_t)comm, (hipStream_t)stream),
               "ncclAllReduce");
}

}  // extern "C"
