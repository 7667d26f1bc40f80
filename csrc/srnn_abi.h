// srnn_abi.h — C ABI of libsrnn.so (mirrored by ctypes structures in
// self_replicating_neural_networks_amd/ops/_lib.py; keep the field order and the flag
// values in sync).
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

// ---- SrnnArgs.flags bits (one meaning each; SRNN_F_* below, FLAG_* in ops/_lib.py)
enum SrnnFlag : uint32_t {
  SRNN_F_SHUFFLE = 1u << 0,          // SGD sample order shuffled per epoch (Keras fit shuffle=True)
  SRNN_F_REMOVE_DIVERGENT = 1u << 1, // soup: respawn divergent particles (reference code/soup.py:77-80)
  SRNN_F_REMOVE_ZERO = 1u << 2,      // soup: respawn zero particles (code/soup.py:81-86)
  SRNN_F_FIX_SEC = 1u << 3,          // classification tests second-order fixpoints too
  SRNN_F_ROW_FLAGS = 1u << 4,        // evolve: per-row respawn flags (rowflags[n]) instead of 64-row ballots
  SRNN_F_RESPAWN_INLINE = 1u << 5,   // evolve re-initialises newborn rows itself
  SRNN_F_COUNT_RESPAWNS = 1u << 6,   // classify: respawns of this generation into counts[5]
  SRNN_F_FULL_TABLE = 1u << 7,       // sharded all-gather: recvbuf is the gathered [n_total] table
  SRNN_F_X2_PRIME = 1u << 8,         // X2 pack / post: first exchange (decisions of THIS generation, no rows)
  SRNN_F_GEN_ADVANCE = 1u << 9,      // classify advances the generation counter
  SRNN_F_FUSED_CENSUS = 1u << 10,    // the generation kernel classifies its stored rows (census)
  SRNN_F_TWO_PHASE = 1u << 11,       // fused generation: block stats for a separate finish launch
  SRNN_F_MASKS_BS = 1u << 12,        // uid assignment reads ballots from block stats (u64[4] per block)
  SRNN_F_GEN_COUNTS = 1u << 13,      // fused generation advances the counter itself (finish follows later)
  SRNN_F_FINISH_BATCH = 1u << 14,    // OP_GEN_FINISH: a ring of `steps` generations' block stats
  SRNN_F_BORN_TOTAL = 1u << 15,      // fused generation adds its newborn count after its block stats
  SRNN_F_X2 = 1u << 16,              // sharded all-to-all exchange (srnn_shard.hip): list entries >= n are
                                     // received rows, teachers of remote learners come from rlist
  SRNN_F_X2_REMOTE = 1u << 17,       // X2 evolve: the remote-dependent slots of rlist (else: the local slots)
  SRNN_F_X2_FINISH_ONLY = 1u << 18,  // X2 pack: only the finish of the last generation (flush)
  SRNN_F_X2_BOTH = 1u << 20,         // X2 evolve (with X2_REMOTE): one launch of n/64 waves for the whole
                                     // generation, the lanes of remote-dependent slots take the remote
                                     // list's entries -- the single-stream generation
  SRNN_F_X2_POST_FUSED = 1u << 21,   // X2 evolve with X2_BOTH: its first workgroups run the post of this
                                     // generation's exchange (block stats of the last one in temp2)
  SRNN_F_X2_PRIO = 1u << 19,         // X2 pack / post / remote evolve: raised wave issue priority (the
                                     // exchange chain wins the SIMDs it shares with the local evolve)
  SRNN_F_ORD_CRIT = 1u << 22,        // ordered run: turns in the run order of k_ord_order (internal: set by
                                     // the library from SRNN_KNOB_ORD_CRIT)
  SRNN_F_ORD_QUEUE = 1u << 24,       // ordered run: continuations through the generation's ready queue
                                     // (internal: set by the library from SRNN_KNOB_ORD_QUEUE)
  SRNN_F_PTAB_READY = 1u << 23,      // ptab already holds this generation's permutations (built by the
                                     // sharded pack): the generation launch does not rebuild them
  SRNN_F_ORD_PLANNED = 1u << 25,     // OP_SOUP_ORDERED: o_src / o_list / o_ctl / ptab already hold this
                                     // generation's plan (OP_ORD_PLAN, issued one generation ahead): no
                                     // planning launches, and the close consumes this generation's lists
                                     // without linking the next one's (the next OP_ORD_PLAN links them)
  SRNN_F_ORD_NEXT = 1u << 26,        // OP_ORD_PLAN: plan generation gen + 1 (the one after the generation
                                     // in flight) instead of gen
  SRNN_F_ORD_SYNC = 1u << 27,        // OP_ORD_PLAN (next) / OP_SOUP_ORDERED (planned): the plan and the
                                     // generation are ordered by the o_sync counters instead of stream
                                     // events (two hipGraphs on two streams, no cross-queue edge): the
                                     // plan waits until the run of the generation before it has started
                                     // (its close is done) and counts itself done; the close waits for
                                     // the next generation's plan (bounded: ~2 s, then an error bit)
  SRNN_F_ORD_INPLAN = 1u << 28,      // OP_SOUP_ORDERED (planned): the run launch's last o_plan_groups workgroups build
                                     // the NEXT generation's plan into o_src_next / o_list_next /
                                     // o_ctl_next / ptab_next and the lists heads_next / nexts_next while
                                     // this generation's turns run (one launch, no second stream)
  SRNN_F_ORD_CENSUS_LATER = 1u << 29, // OP_SOUP_ORDERED: the close writes the final rows, respawn ballots and
                                     // the counter only; the census of the final rows (block-stat class
                                     // counts) is OP_ORD_CENSUS's, issued on the side stream beside the
                                     // next generation
};

// Attack-list entries (uint32, SRNN_NIL ends a list).  Single rank: the attacker's row
// (= its slot).  SRNN_F_FULL_TABLE: the attacker's global slot.  SRNN_F_X2: e < n is the
// local row e, e >= n the received row e - n (its slot in x_rslot[e - n]).
#define SRNN_NIL 0xFFFFFFFFu

struct SrnnArgs {
  int64_t n;            // work items (rows) of this call
  int64_t n_total;      // soup: global population size
  int64_t lo;           // soup: first global slot owned by this rank
  int32_t steps;        // fixpoint run: step limit; batched finish: generations
  int32_t epochs;       // train: epochs; soup: train count
  int32_t severity;     // soup: learn_from_severity
  int32_t early_exit;   // fixpoint run: stop at fixpoint / divergence
  uint32_t flags;       // SrnnFlag bits
  int32_t gen;          // soup generation (time) when gen_ptr is null
  float eps;
  float lr;
  float attacking_rate;
  float learn_from_rate;
  uint64_t seed;
  uint32_t ctr;         // op counter for per-particle random streams
  uint32_t x_emul;      // X2 pack at world 1 only (timing model of R ranks): a Philox-keyed
                        // fraction x_emul / 2^32 of the local slots is marked remote-dependent
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
  uint64_t* counts;     // [6] class histogram (atomic adds) + respawns
  // ---- soup: decisions and attack lists
  uint32_t* heads;      // [n] first attacker entry of each local victim this generation (consumed -> NIL)
  uint32_t* nexts;      // entry -> next entry of the same victim
  uint32_t* heads_next; // fused generation / X2 pack+post: the NEXT generation's lists
  uint32_t* nexts_next;
  int64_t* dec_at;      // OP_SOUP_DECIDE: attack target per global slot (diagnostics, optional)
  int64_t* dec_te;      // OP_SOUP_DECIDE: teacher per global slot (diagnostics, optional)
  unsigned long long* ballots;  // evolve: respawn ballot per 64-row block (u64[nb])
  int32_t* rowflags;    // evolve with SRNN_F_ROW_FLAGS: respawn flag per row
  int32_t* done;        // fused generation / parallel batched finish: done counter (last-wave hand-off)
  int64_t* uid_out;     // respawn: uid column to update
  int64_t* uid_base;    // respawn: device scalar, next uid (advanced in place)
  const int32_t* gen_ptr;   // soup: device scalar generation (graph replay); null -> gen
  int32_t* gen_out;     // soup: where "advance the generation" writes gen + 1 (null -> *gen_ptr in
                        // place): a 2-slot ring indexed by the ping-pong parity
  int64_t segment;      // soup: >0 -> independent sub-soups of this many slots (partners chosen inside)
  int32_t world;        // soup: ranks sharing the population (<= 1: unsharded)
  int32_t rank;
  // ---- sharded soup exchange (srnn_shard.hip).  SRNN_F_FULL_TABLE: recvbuf = the gathered
  // table, stats = [world][6].  SRNN_F_X2: one all-to-all per generation; per peer a block of
  // x_blk bytes = header (int64[X2_HDR]) + x_cr rows of (row, int64 slot, int32 gen, pad) +
  // x_cn notices (int64 attacker, int64 victim) + x_cq requests (int64 teacher)
  int64_t x_cr, x_cn, x_cq, x_blk;
  char* sendbuf;
  const char* recvbuf;
  const int64_t* stats;       // FULL_TABLE: [world][6] gathered (class counts[5], respawns) per rank
  int64_t* census;            // [5] global class counts of the previous generation
  int32_t* err;               // [1] exchange error bits: 1 capacity overflow, 4 row tag mismatch
  // ---- X2 per-generation state ("this" = the generation being evolved / exchanged, "next" =
  // the one whose decisions pack and post prepare; the engine swaps them by parity)
  uint32_t* x_dep;            // [ceil(n/32)] remote-dependent bits of this generation (read, reset)
  uint32_t* x_dep_next;       // the next generation's (set by pack / post)
  uint32_t* x_rlist;          // [2n] (row, teacher recv row or NIL) of this generation's remote slots
  uint32_t* x_rlist_next;
  int32_t* x_rcount;          // [1] entries of x_rlist (zeroed by the remote evolve's last wave)
  int32_t* x_rcount_next;
  int64_t* x_rslot;           // [world * x_cr] attacker slot of received row k (this generation)
  int64_t* x_rslot_next;
  uint32_t* x_satt;           // [world * x_cn] local attacker rows noticed to each peer for this generation
  uint32_t* x_satt_next;
  int32_t* x_cno;             // [world] notices sent per peer for this generation (zeroed by post)
  int32_t* x_cno_next;
  int32_t* x_crq;             // [world] requests sent per peer for this generation (zeroed by post)
  int32_t* x_crq_next;
  uint32_t* x_srep;           // [world * x_cq] local rows requested by each peer (this generation)
  int32_t* x_nsrep;           // [world]
  int64_t* x_part;            // [x_groups][6] finish partials (born, census[5]) per workgroup
  int32_t* x_ctl;             // [8] last-workgroup tickets (re-armed by their last workgroup): 0 pack
                              // finish, 2 post uids, 3 evolve waves
  int32_t x_groups;           // finish / uid workgroups
  int32_t pad2;
  int32_t* x_hpre;            // [ceil(n/64)] (SRNN_F_X2_BOTH generations) remote-dependent slots before
                              // each 64-row block within its finish workgroup's range (pack)
  int32_t* x_hgrp;            // [x_groups] ... before each finish workgroup's range (pack)
  void* temp2;                // SRNN_F_X2_POST_FUSED: the previous generation's block stats (post's temp)
  int8_t* action;       // soup: action code per local row (optional)
  int64_t* counterpart; // soup: counterpart slot per local row (optional)
  int8_t* respawn;      // soup: 0 none, 1 divergent_dead, 2 zweo_dead
  void* temp;           // block stats u64[4] per 64-row block (ballot, census): the fused generation /
                        // X2 evolve write them, the finish / X2 pack + post read them
  int64_t temp_bytes;
  int32_t dev;          // 0 host (CPU tensors), 1 device (HIP)
  int32_t pad1;
  void* stream;         // hipStream_t for dev == 1
  void* scratch;        // generic (runtime-shape) engine: per-lane vectors, element-major; null ->
  int64_t scratch_bytes;  // the library's own cached device buffer (not inside a graph capture)
  // ---- ordered (reference-order) generation, OP_SOUP_ORDERED (srnn_ordered.h)
  float* W3;            // [n][pp] attack outputs A(k) of this generation
  int32_t* o_src;       // [n][4] source versions of each turn's reads + its level | [n] stored-attack
                        // flags | [n] consumer-list heads | [ord::rec_total(n)][32] pending records |
                        // [ord::rec_total(n)] critical list (producers of later turns) |
                        // [ord::rec_total(n)] ready queue (records in the order they became ready)
  int32_t* o_list;      // [n] the pending record of each turn (-1: no producer)
  int32_t* o_ctl;       // [ord::CTL_WORDS = 166] record / critical-list counts per partition, ready-queue
                        // head and tail, max level
                        // (host), error bits (sticky: the plan kernel clears every word but that one)
  int32_t o_levels;     // dependency levels the host path reports one by one (1..16; the device
                        // schedules turns by continuation, not by level)
  int32_t pad3;
  // ---- precomputed SGD epoch permutations of a soup generation (nibble Weightwise nets, shuffle
  // on): [severity + epochs][n] uint64, epoch e of local row j at ptab[e * n + j] (counter
  // gen * 1024 + 512 + e); filled by the generation's own k_perm_table launch.  null: inline
  uint64_t* ptab;
  // ---- ordered generation trace (debug, SoupEngine.ordered_trace): [n][2] s_memrealtime (100 MHz,
  // chip-wide) at the start and the end (after its publish) of each turn on the device.  null: off
  uint64_t* o_trace;
  // ---- the reference-order generation sharded over ranks (OP_SOUP_ORDERED_SH): this rank's turns
  // [o_lo, o_hi) of the n global ones (every other field in the global view: n = n_total, lo = 0)
  int64_t o_lo, o_hi;
  // ---- SRNN_F_ORD_INPLAN: the plan set of the next generation (see o_src / o_list / o_ctl / ptab) and
  // the number of workgroups of the run launch that build it
  int32_t* o_src_next;
  int32_t* o_list_next;
  int32_t* o_ctl_next;
  uint64_t* ptab_next;
  int32_t o_plan_groups;
  int32_t o_bulk_delay;  // (internal, SRNN_KNOB_ORD_BULK_DELAY) us the run's turn waves wait before their first turn
  // ---- SRNN_F_ORD_SYNC: 4 monotonic int32 counters shared by the main and the side stream:
  // runs started, plans gated, plans done, closes waited (srnn_ordered.h ord::SYNC_*)
  int32_t* o_sync;
  // ---- (internal, set by the library from SRNN_KNOB_ORD_SHADOW) shadow lanes of a reference-order run
  int32_t o_shadow;
  int32_t pad5;
  // ---- OP_SOUP_ORDERED (device, lane nets): the block stats of the PREVIOUS generation, whose close
  // ran with SRNN_F_ORD_CENSUS_LATER: extra workgroups of this generation's run launch classify its
  // final rows (this generation's W2) into them.  null: none
  uint64_t* o_census_temp;
};

#define SRNN_X2_HDR 12  // int64 header words of an X2 exchange block (see srnn_shard.hip)

enum SrnnOp {
  OP_INIT = 0,          // W[i] = fresh particle keyed by uid[i]
  OP_APPLY = 1,         // W2[idx_o[i]] = f_{W[idx_f[i]]}(W[idx_t[i]])
  OP_RUN_FIXPOINT = 2,  // run_net semantics per row (in place), cls + nsteps (+traj)
  OP_TRAIN = 3,         // `epochs` self-train epochs (in place), loss
  OP_LEARN = 4,         // `epochs` epochs on samples of W2[idx_t[i]], loss
  OP_CLASSIFY = 5,      // cls + counts
  OP_PERTURB = 6,       // W[i] +-= U(0,1) * eps, p=1/2 each (known-fixpoint variation)
  OP_SOUP_DECIDE = 7,   // per global slot: decisions; attacks on local victims linked (heads, nexts)
  OP_RESPAWN_SEQ = 8,   // single rank: scan respawn ballots, new uids from *uid_base, re-init, ++gen
  OP_SOUP_EVOLVE = 9,   // attack -> learn -> train -> respawn flags for local rows (X2: local / remote slots)
  OP_RESPAWN = 11,      // rows with respawn != 0: fresh weights
  OP_VARY_RUN = 12,     // known-fixpoint variation run: nsteps = time to vergence, loss = time as fixpoint
  OP_UID_ASSIGN = 15,   // sharded all-gather soup: uids of the previous generation's newborns from stats
  OP_SOUP_GEN = 16,     // fused single-rank generation: evolve + next decisions + census (+ finish)
  OP_GEN_FINISH = 17,   // single rank: census + newborn uids of generations whose block stats are in temp
  OP_SOUP_SEQ = 19,     // `steps` sequential (Gauss-Seidel, in-place, index-order) soup generations
  OP_X2_PACK = 20,      // sharded all-to-all soup: finish of the previous generation + next decisions
                        // (links, notices, requests) + the rows of this generation's exchange
  OP_X2_POST = 21,      // after the all-to-all: uids of the previous generation's newborns, global
                        // census, received notices linked for the next generation, requests kept
  OP_SOUP_ORDERED = 22, // one reference-order (sequential, in-place) generation scheduled by its
                        // dependency DAG: bitwise OP_SOUP_SEQ, every turn as soon as its producers
                        // are done (srnn_ordered.h)
  OP_SOUP_ORDERED_SH = 23, // one phase (steps) of a reference-order generation sharded over ranks:
                           // 0 plan + levels of every turn, 1 run this rank's turns of level
                           // o_levels, 2 pack their outputs, 3 unpack the gathered outputs, 4 close
                           // this rank's rows, 5 link the next generation's attacks
                           // (srnn_ordered_sh.h)
  OP_ORD_CENSUS = 25,   // the census of a reference-order generation's final rows (W) into the class counts
                        // of its two-phase block stats (temp), after a close with SRNN_F_ORD_CENSUS_LATER
  OP_ORD_PLAN = 24,     // the plan of a single-rank reference-order generation into o_src / o_list /
                        // o_ctl / ptab: its attack lists linked into heads / nexts (NIL on entry),
                        // source versions, stored-output marks, pending records + consumer lists
                        // (device) or levels (host), the critical turns' permutations.  Weight
                        // independent: issued on a side stream while the previous generation runs
};

int srnn_abi_version();  // 31
int64_t srnn_args_size();  // sizeof(SrnnArgs): the ctypes mirror checks its layout against it
int64_t srnn_cfg_size();
int srnn_has_config(const SrnnCfg* cfg);
int srnn_run(int op, const SrnnCfg* cfg, const SrnnArgs* args);
const char* srnn_last_error();
int srnn_is_generic(const SrnnCfg* cfg, int op);
int srnn_supports(const SrnnCfg* cfg, int op, int dev);  // 1: op has a host (0) / device (1) path
int srnn_generic_op_supported(int op, int dev);
void srnn_set_force_generic(int on);  // 1: this op of this config runs on the generic engine
// Execution knobs (config.py ExecConfig): which kernel family serves an op.  A value set here
// is used unless the knob's environment variable is set (the variable overrides: A/B runs);
// -1 = unset (built-in default).  srnn_get_knob returns the value in force.
enum SrnnKnob {
  SRNN_KNOB_FORCE_GENERIC = 0,  // SRNN_FORCE_GENERIC: every op on the runtime-shape engine (default 0)
  SRNN_KNOB_RNN_WAVE = 1,       // SRNN_RNN_WAVE: wide Recurrent nets wave per particle (default 1)
  SRNN_KNOB_RNN_SPEC = 2,       // SRNN_RNN_SPEC: width/depth-specialised Recurrent wave kernels (default 1)
  SRNN_KNOB_RNN_SOUP = 3,       // SRNN_RNN_SOUP: wide Recurrent soup generations wave per particle (default 1)
  SRNN_KNOB_WW_WAVE = 4,        // SRNN_WW_WAVE: wide Weightwise training lanes-per-particle waves (default 1)
  SRNN_KNOB_BIG_WAVE = 5,       // SRNN_BIG_WAVE: P = 280 nets on the wave kernels instead of row kernels (default 0)
  SRNN_KNOB_FIX_GROUP = 6,      // SRNN_FIX_GROUP: 16-lane run_fixpoint (1), lane (0), by population size (-1)
  SRNN_KNOB_SOUP_LANES = 7,     // SRNN_SOUP_LANES: lanes per particle of WW(2,2) soup generations (0 = by size)
  SRNN_KNOB_ORD_CRIT = 8,       // SRNN_ORD_CRIT: reference-order generations run the producers of later turns
                                // first, at raised wave priority (default 1)
  SRNN_KNOB_ORD_QUEUE = 9,      // SRNN_ORD_QUEUE: reference-order continuations through one ready queue
                                //   (1) or run by the producers' waves (0, default: measured faster)
  SRNN_KNOB_ORD_SHADOW = 10,    // SRNN_ORD_SHADOW: a reference-order round with at most this many turns in a
                                //   wave runs each on several lanes (the idle lanes repeat a busy lane's
                                //   turn; 0: off; default 32)
  SRNN_KNOB_ORD_BULK_DELAY = 11, // SRNN_ORD_BULK_DELAY: microseconds a reference-order run's turn waves (not the
                                 //   critical-list waves) wait before their first turn (default 12)
  SRNN_KNOB_COUNT = 12
};
void srnn_set_knob(int knob, int value);
int srnn_get_knob(int knob);
// launches a waiter on stream `side` (bounded: timeout_us) and a setter on `main_stream`; after both
// finished flag[1] is 1 when the two streams ran concurrently, 2 when the waiter timed out
int srnn_stream_probe(int32_t* flag, void* side, void* main_stream, int64_t timeout_us);
int64_t srnn_generic_scratch_bytes(const SrnnCfg* cfg, int64_t n, int64_t max_lanes);
}
