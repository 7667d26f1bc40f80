// srnn_abi.h — C ABI of libsrnn.so (mirrored by ctypes structures in
// self_replicating_neural_networks_amd/ops/_lib.py; keep the field order in sync).
#pragma once
#include <stdint.h>

extern "C" {

struct SrnnCfg {
  int32_t kind;        // 0 weightwise, 1 aggregating, 2 recurrent, 3 fft
  int32_t width;
  int32_t depth;
  int32_t aggregates;
  int32_t aggregator;  // 0 mean, 1 max, 2 max with the reference's and/or quirk
  int32_t shuffler;    // 0 none, 1 random
  int32_t pp;          // padded row stride (floats)
  int32_t p;           // weights per particle
  int32_t dtype;       // weight-table storage: 0 fp32, 1 bf16, 2 fp16 (arithmetic is fp32)
};

struct SrnnArgs {
  int64_t n;            // work items (rows) of this call
  int64_t n_total;      // soup: global population size
  int64_t lo;           // soup: first global slot owned by this rank
  int32_t steps;        // fixpoint run: step limit
  int32_t epochs;       // train: epochs; soup: train count
  int32_t severity;     // soup: learn_from_severity
  int32_t early_exit;   // fixpoint run: stop at fixpoint / divergence
  int32_t flags;        // bit0 shuffle, bit1 remove_divergent, bit2 remove_zero, bit3 fix_sec, bit4 per-row respawn flags, bit5 respawn inline, bit6 count respawns in counts[5], bit7 recvbuf is the all-gathered table,
                        // bit8 uid_assign reads the per-rank stats from the exchange's stats rows, bit9 classify advances *gen_ptr,
                        // bit10 fused generation computes the census, bit16 asynchronous finish (OP_SOUP_GEN
                        // advances the generation counter itself and leaves the finish to OP_GEN_FINISH),
                        // bit17 precomputed SGD permutations (perm_cur / perm_next, helper waves),
                        // bit18 OP_GEN_FINISH is a batch of `steps` generations (block stats ring in temp,
                        // temp_bytes per generation; census = optional [steps][6] history)
  int32_t gen;          // soup generation (time)
  float eps;
  float lr;
  float attacking_rate;
  float learn_from_rate;
  uint64_t seed;
  uint32_t ctr;         // op counter for per-particle random streams
  uint32_t pad0;
  float* W;             // rows [n][pp] (in/out)
  float* W2;            // second table (source rows / output rows)
  float* traj;          // fixpoint run trajectory [(steps+1)][n][pp] or null
  const int64_t* idx_f; // apply: applying-net row per item (null = identity)
  const int64_t* idx_t; // apply: target row per item (null = identity)
  const int64_t* idx_o; // apply: output row per item (null = identity)
  const int64_t* uid;   // per-row uid (keys random streams); null -> row index
  int8_t* cls;          // per-row class
  int32_t* nsteps;      // per-row steps taken
  float* loss;          // per-row loss
  uint64_t* counts;     // [5] class histogram (atomic adds)
  int32_t* i32a;        // soup: attack target per global slot
  int32_t* i32b;        // soup: teacher per global slot
  int32_t* i32c;        // soup: per-local-victim attack count; later respawn flags as int32
  int32_t* i32d;        // soup: exclusive offsets [n+1]
  int32_t* i32e;        // soup: fill cursor per local victim
  int32_t* i32f;        // soup: attacker list (CSR payload)
  int64_t* uid_out;     // respawn: uid column to update
  const int64_t* uid_base;  // respawn: device scalar, first uid for this rank
  const int32_t* gen_ptr;   // soup: device scalar generation (graph replay); null -> gen
  int64_t segment;          // soup: >0 -> independent sub-soups of this many slots (partners chosen inside)
  int32_t world;            // soup: ranks sharing the population (<= 1: unsharded)
  int32_t rank;
  int64_t cap;              // soup: rows per destination rank in the exchange buffers
  float* sendbuf;           // [world][cap][pp + 4]: row, then (slot, generation) tags
  const float* recvbuf;     // [world][cap][pp + 4]
  int32_t* need;            // [n] bitmask of the ranks that need local row j this generation
  int32_t* sendcnt;         // [world] rows packed per destination
  int32_t* rmap;            // [n_total] received row index of a remote slot
  int32_t* ovf;             // [1] exchange overflow flag
  const int64_t* stats;     // [world][6] gathered (class counts[5], respawns) per rank
  int64_t* census;          // [5] global class counts (written by OP_UID_ASSIGN)
  int8_t* action;       // soup: action code per local row
  int64_t* counterpart; // soup: counterpart slot per local row
  int8_t* respawn;      // soup: 0 none, 1 divergent_dead, 2 zweo_dead
  void* temp;           // scratch for device scans
  int64_t temp_bytes;
  int32_t dev;          // 0 host (CPU tensors), 1 device (HIP)
  int32_t pad1;
  void* stream;         // hipStream_t for dev == 1
  int32_t* gen_out;     // soup: where "advance the generation" writes gen + 1 (null -> *gen_ptr in
                        // place).  The engine keeps a 2-slot ring indexed by the ping-pong parity
                        // so a kernel can advance the counter while its other blocks still read it.
  void* scratch;        // generic (runtime-shape) engine: per-lane vectors, element-major; null ->
  int64_t scratch_bytes;  // the library's own cached device buffer (not inside a graph capture)
  // fused single-rank generation with precomputed shuffles (flag 131072): the SGD
  // permutations of generation gen are in perm_cur[k][n] (k < perm_e: learn epochs then
  // train epochs), helper waves fill perm_next for gen + 1; helper_ctl = work-queue head +
  // per-SIMD main-wave counts of this parity (re-armed by the finish kernel)
  uint64_t* perm_cur;
  uint64_t* perm_next;
  int32_t* helper_ctl;
  int32_t perm_e;
  int32_t helpers;      // helper workgroups appended to the generation grid
  // sharded fused generation with the post-exchange work folded in (flag 524288): the
  // respawn ballots of the PREVIOUS generation (block stats, u64[4] per 64 rows; temp holds
  // this generation's) and the counter the unpack workgroups bump for the generation waves
  void* temp2;
  int32_t* xdone;
};

enum SrnnOp {
  OP_INIT = 0,          // W[i] = fresh particle keyed by uid[i]
  OP_APPLY = 1,         // W2[idx_o[i]] = f_{W[idx_f[i]]}(W[idx_t[i]])
  OP_RUN_FIXPOINT = 2,  // run_net semantics per row (in place), cls + nsteps (+traj)
  OP_TRAIN = 3,         // `epochs` self-train epochs (in place), loss
  OP_LEARN = 4,         // `epochs` epochs on samples of W2[idx_t[i]], loss
  OP_CLASSIFY = 5,      // cls + counts
  OP_PERTURB = 6,       // W[i] +-= U(0,1) * eps, p=1/2 each (known-fixpoint variation)
  OP_SOUP_DECIDE = 7,   // per global slot: decisions; attacks on local victims linked (i32e head, i32f next)
  OP_RESPAWN_SEQ = 8,   // single rank: scan respawn flags, new uids from *uid_base (updated), re-init, ++*gen_ptr
  OP_SOUP_EVOLVE = 9,   // fused attack -> learn -> train -> respawn flags for local rows
  OP_SCAN = 10,         // i32d[0..n] = exclusive scan of i32c[0..n)
  OP_RESPAWN = 11,      // rows with respawn != 0: uid_out = *uid_base + i32d[i], fresh weights
  OP_VARY_RUN = 12,     // known-fixpoint variation run: nsteps = time to vergence, loss = time as fixpoint
  OP_SOUP_PACK = 13,    // sharded soup: stats rows + local rows needed by other ranks -> sendbuf (tagged)
  OP_SOUP_UNPACK = 14,  // sharded soup: index the received rows (rmap), reset sendcnt
  OP_SOUP_GEN = 16,     // fused generation: evolve + next decisions + census (+ finish; flag 32768: the
                        // finish launch also packs the next all-to-all = OP_SOUP_PACK)
  OP_SOUP_PERMS = 18,   // fill perm_next with the SGD permutations of generation *gen_ptr (first generation)
  OP_SOUP_SEQ = 19,     // host: `steps` sequential (Gauss-Seidel, in-place, index-order) soup generations
  OP_GEN_FINISH = 17,   // single rank, flag 65536: census + newborn uids of the generation whose block
                        // stats are in temp (the finish half of OP_SOUP_GEN, on a side stream)
  OP_UID_ASSIGN = 15,   // sharded soup: uids of the previous generation's newborns from the per-rank stats
                        // (flag 16384: the same launch also indexes the received rows = OP_SOUP_UNPACK)
};

int srnn_abi_version();  // 14
int srnn_has_config(const SrnnCfg* cfg);
int srnn_run(int op, const SrnnCfg* cfg, const SrnnArgs* args);
const char* srnn_last_error();
int64_t srnn_scan_temp_bytes(int64_t n);
int srnn_is_generic(const SrnnCfg* cfg, int op);
void srnn_set_force_generic(int on);  // 1: this op of this config runs on the generic engine
int64_t srnn_generic_scratch_bytes(const SrnnCfg* cfg, int64_t n, int64_t max_lanes);
}
