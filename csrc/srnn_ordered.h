// srnn_ordered.h — the reference's sequential, in-place soup generation on the GPU
// (OP_SOUP_ORDERED), bitwise equal to the serial loop (Item::soup_seq_one / OP_SOUP_SEQ).
// Included by srnn_kernels.h inside namespace srnn.
//
// Reference Soup.evolve (code/soup.py:51-87) visits particles in index order and updates
// the table IN PLACE: particle k sees every change made by particles < k in the same
// generation.  Read literally that is a serial loop; but the decisions of a
// generation are a pure function of (seed, slot, generation), so its whole dependency
// structure is known before any weight is touched:
//
//   turn k reads   its own row at turn start   = the last write to row k before k
//                  the victim's row (attack)   = the last write to row at_k before k
//                  the teacher's row (learn)   = the last write to row te_k before k
//                                                (or k's own / just-attacked row)
//   turn k writes  A(k) = f_k(victim)          (the attack output, row at_k)
//                  E(k) = k's row at turn end  (after learn / train / respawn)
//
// Writes to a row r happen at "times" j (A(j) for each attacker j of r) and r + 1/2 (E(r)).
// Keeping every written version (E(j) in W row j, the generation start in W2) removes the
// write-after-read hazards, so only read-after-write edges remain: turn k depends on the
// turns that produced the versions it reads.  An attack output A(j) is cheap (one forward
// of 14 points for WW(2,2), against 20 epochs of SGD for the turn), so it is not an edge by
// itself: a turn that reads A(j) recomputes it from A(j)'s own inputs (up to RB nested
// attack outputs deep), and only the attack outputs past that depth are stored (W3 row j,
// flagged by k_ord_mark).  A turn then waits only for the TRAINING of the turns it reads;
// the DAG is shallow (100k particles: 95 % of the turns have no producer, 4.8 % are one hop
// deep, ~170 two, a handful three).  A generation on the device runs as
//
//   k_ord_plan    per turn: decisions, the source version of each of its reads (src codes)
//   k_ord_mark    per turn / row: flags the attack outputs reached past the recompute depth
//   k_ord_count   per turn: its producers; a turn with producers becomes a pending record
//                 {turn, producers, remaining count} and is pushed onto every producer's
//                 consumer list (lock-free: no turn runs in this launch, so the lists are
//                 complete before any is walked)
//   k_ord_ptab    the pending records' epoch permutations (with a table)
//   k_ord_run     ONE launch for every turn: a lane runs its own turn if it has no producer;
//                 a lane that finishes a turn with consumers releases its rows and counts
//                 down each consumer's record -- the lane whose decrement reaches zero runs
//                 that consumer next, right away (continuation scheduling: a dependent turn
//                 starts when ITS producers are done, not when a level launch could start it;
//                 no workgroup ever waits for another, no level launches, no tail)
//   k_ord_close   per row: its final version (a row attacked after its own turn ends the
//                 generation as that attack's output), census class, the next generation's
//                 decisions linked, block stats for the finish (newborn uids in slot order)
//
// Every turn runs the serial loop's per-particle code with the same Philox streams (attack
// keyed (k, gen*1024+1), SGD (k, gen*1024+512), newborn init respawn_key(gen, k)), and a
// recomputed attack output is the same function of the same versions, so a generation
// equals OP_SOUP_SEQ bitwise whatever order its turns run in (tests/test_ordered_soup.py,
// host and device).  The host path runs the same DAG level by level.
#pragma once

namespace ord {

// src codes: >= 0 a version written this generation (2j: A(j), 2j+1: E(j) in W); -(r+1): the
// generation-start row r (W2); SELF: the turn's own current row (s[1]: a self-attack, s[2]:
// learn_from itself); ATK: its own attack output (learn_from its victim); NONE: no such read
constexpr int32_t SRC_SELF = INT32_MIN;
constexpr int32_t SRC_ATK = INT32_MIN + 1;
constexpr int32_t SRC_NONE = INT32_MIN + 2;
constexpr int MAX_LEVELS = 16;  // dependency levels reported one by one (deeper: one bin)
// o_ctl words: [MAXLW] deepest level (host path), [ERRW] error bits -- STICKY: set by any
// generation, never cleared by the next one (ERR_* below; SoupEngine.ORD_ERRORS lists them),
// [PART0 + p] records (pending turns) of
// partition p, [CRIT0 + p] producers of later turns in partition p (the producer's block mod
// NPART; k_ord_count appends a producer when its first consumer registers)
constexpr int MAXLW = 17, ERRW = 18;
constexpr int32_t ERR_UNSTORED = 2;  // an attack output past the recompute depth left unstored (marking bug)
constexpr int32_t ERR_NOT_RUN = 4;   // a turn that never ran (scheduling bug)
constexpr int32_t ERR_QUEUE = 8;     // a ready-queue entry never written (scheduling bug)
constexpr int32_t ERR_PACK = 16;     // sharded: a level's records overflowed the send buffer (sizing bug)
constexpr int32_t ERR_PLAN_BARRIER = 64;  // a plan workgroup gave up at a phase barrier (scheduling bug)
constexpr int32_t ERR_SYNC = 128;    // SRNN_F_ORD_SYNC: a wait on the other stream gave up after ~2 s
// (32: set by the engine -- a one-rank timing model of a sharded generation ran 1/R of the turns)
// o_sync counters (SRNN_F_ORD_SYNC): runs started, plans gated, plans done, closes that waited
constexpr int SYNC_RUN = 0, SYNC_GATE = 1, SYNC_PLAN = 2, SYNC_CLOSE = 3, SYNC_WORDS = 4;
// pending records (and the run order) live in NPART partitions (partition p: the workgroups
// b = p mod NPART, appended by one counter each: no chip-wide contended counter)
constexpr int NPART = 64, PART0 = 2 * MAX_LEVELS + 3;
constexpr int CRIT0 = PART0 + NPART;
// [QH], [QT]: head / tail of the generation's ready queue (SRNN_F_ORD_QUEUE); [BARW]: the arrivals
// at the phase barriers of the workgroups that build this set's plan inside the previous
// generation's run launch (SRNN_F_ORD_INPLAN; zeroed by the close of the generation that used it)
constexpr int QH = CRIT0 + NPART, QT = QH + 1, BARW = QT + 1;
constexpr int CTL_WORDS = BARW + 1;
// o_src layout: [n][4] {own, victim, teacher, level} | [n] stored flags of A(j) | [n] consumer-list
// heads (pending records reading E(j) / A(j), EMPTY-terminated) | [rec_total(n)][REC] pending
// records | [rec_total(n)] the critical list (producers of later turns; partition p: the producers
// of blocks b = p mod NPART, rec_cap(n) slots) | [rec_total(n)] the ready queue (records whose
// producers are all done, in the order they became ready; EMPTY until written);
// o_list: [n] the record of each pending turn (-1: none)
constexpr int NPROD = 12;  // producers of one turn: 3 reads x 2^RB leaves
constexpr int REC = 32;    // record words: {turn, np, producers[NPROD], count, ready-next, next[NPROD], -}
constexpr int R_PROD = 2, R_CNT = R_PROD + NPROD, R_RDY = R_CNT + 1, R_NEXT = R_RDY + 1;
constexpr int32_t EMPTY = -1;
static_assert(R_NEXT + NPROD <= REC, "record layout");

// the generation a plan is for: the one in flight, or -- SRNN_F_ORD_NEXT, OP_ORD_PLAN issued one
// generation ahead on a side stream -- the one after it
SRNN_HD int32_t plan_gen(const SrnnArgs& a) {
  return (a.gen_ptr ? a.gen_ptr[0] : a.gen) + ((a.flags & SRNN_F_ORD_NEXT) ? 1 : 0);
}

// epochs a turn trains (learn_from severity + self-train): the permutation-table row length
SRNN_HD int32_t table_epochs(const SrnnArgs& a) {
  return (a.severity > 0 ? a.severity : 0) + (a.epochs > 0 ? a.epochs : 0);
}

SRNN_HD int32_t code_A(int64_t j) { return (int32_t)(2 * j); }
SRNN_HD int32_t code_E(int64_t j) { return (int32_t)(2 * j + 1); }
SRNN_HD int32_t code_G(int64_t r) { return (int32_t)(-(r + 1)); }
SRNN_HD bool is_A(int32_t c) { return c >= 0 && !(c & 1); }
// a read of a row version (not NONE / SELF / ATK)
SRNN_HD bool is_row(int32_t c) { return c > SRC_NONE; }

// the last attacker j < k of row r this generation (-1: none); the list is unordered
SRNN_HD int64_t last_attacker_before(const SrnnArgs& a, int64_t r, int64_t k) {
  int64_t best = -1;
  for (uint32_t e = a.heads[r]; e != SRNN_NIL; e = a.nexts[e]) {
    const int64_t j = (int64_t)e;
    if (j < k && j > best) best = j;
  }
  return best;
}
// the version of row r that turn k reads (before any write of its own): the latest of
// A(j) (time j, j an attacker of r) and E(r) (time r + 1/2) strictly before time k
SRNN_HD int32_t latest(const SrnnArgs& a, int64_t r, int64_t k) {
  const int64_t ja = last_attacker_before(a, r, k);
  if (r < k && ja <= r) return code_E(r);
  return ja >= 0 ? code_A(ja) : code_G(r);
}

SRNN_HD const int32_t* src_of(const SrnnArgs& a, int64_t k) { return a.o_src + 4 * k; }
SRNN_HD int32_t* cons_head(const SrnnArgs& a) { return a.o_src + 5 * a.n; }
SRNN_HD int32_t* pend(const SrnnArgs& a, int64_t q) { return a.o_src + 6 * a.n + REC * q; }
// records per partition (each count workgroup of TB turns appends to its partition only)
SRNN_HD int64_t rec_cap(int64_t n) { return ((n + TB - 1) / TB + NPART - 1) / NPART * TB; }
SRNN_HD int64_t rec_total(int64_t n) { return NPART * rec_cap(n); }
SRNN_HD bool stored(const SrnnArgs& a, int64_t j) { return a.o_src[4 * a.n + j] != 0; }
SRNN_HD int32_t* run_order(const SrnnArgs& a) { return a.o_src + 6 * a.n + REC * rec_total(a.n); }
SRNN_HD int32_t* ready_queue(const SrnnArgs& a) { return a.o_src + 6 * a.n + (REC + 1) * rec_total(a.n); }
// turn k computes A(k): it attacked, and the attack output is its own row (self-attack),
// its teacher (learn_from the victim) or read by a turn past the recompute depth
SRNN_HD bool needs_A(const SrnnArgs& a, int64_t k, const int32_t* s) {
  return s[1] != SRC_NONE && (s[1] == SRC_SELF || s[2] == SRC_ATK || stored(a, k));
}

// flag every attack output that the recompute of version `code` (budget B) reaches at depth B
template <int B>
SRNN_HD void mark_version(const SrnnArgs& a, int32_t code) {
  if (!is_A(code)) return;
  const int64_t j = code >> 1;
  if constexpr (B == 0) {
    a.o_src[4 * a.n + j] = 1;
  } else {
    const int32_t* sj = src_of(a, j);
    mark_version<B - 1>(a, sj[0]);
    if (sj[1] != SRC_SELF) mark_version<B - 1>(a, sj[1]);
  }
}
// the turns whose outputs the materialisation of `code` (budget B) reads; error on an
// unstored attack output at depth B
template <int B>
SRNN_HD void collect(const SrnnArgs& a, int32_t code, int32_t* pr, int& np, bool& bad) {
  if (code < 0) return;
  const int64_t j = code >> 1;
  if ((code & 1) || stored(a, j)) {
    if (pr) pr[np] = (int32_t)j;  // (nullptr: count only)
    ++np;
    return;
  }
  if constexpr (B == 0) {
    bad = true;
  } else {
    const int32_t* sj = src_of(a, j);
    collect<B - 1>(a, sj[0], pr, np, bad);
    if (sj[1] != SRC_SELF) collect<B - 1>(a, sj[1], pr, np, bad);
  }
}

// the schedule of a generation for recompute depth RB (shape independent: decisions, version
// codes, the stored-output marks and the producer lists of the turns)
template <int RB_>
struct OrdSched {
  static constexpr int RB = RB_;
  using Dec = Item<Weightwise<1, 1>, StF32>;  // decisions are shape independent

  // src codes of turn k (generation gen) -> o_src[k] = {own, victim, teacher, level = -1};
  // its stored flag cleared, its consumer list emptied, no record
  SRNN_HD static void plan(const SrnnArgs& a, int64_t k, int32_t gen) {
    int64_t at, te;
    Dec::decision(a, k, gen, at, te);
    int32_t* s = a.o_src + 4 * k;
    s[0] = latest(a, k, k);
    s[1] = at < 0 ? SRC_NONE : at == k ? SRC_SELF : latest(a, at, k);
    if (te < 0) s[2] = SRC_NONE;
    else if (te == k) s[2] = SRC_SELF;
    else if (te == at) s[2] = SRC_ATK;
    else s[2] = latest(a, te, k);
    s[3] = -1;
    a.o_src[4 * a.n + k] = 0;
    cons_head(a)[k] = EMPTY;
    if (a.o_list) a.o_list[k] = -1;
  }

  // the attack outputs turn k and the close of row k reach past the recompute depth (every
  // attacker's victim read is walked: whether A(k) is needed depends on these flags)
  SRNN_HD static void mark(const SrnnArgs& a, int64_t k) {
    const int32_t* s = src_of(a, k);
    mark_version<RB>(a, s[0]);
    if (is_row(s[1])) mark_version<RB>(a, s[1]);
    if (is_row(s[2])) mark_version<RB>(a, s[2]);
    const int64_t ja = last_attacker_before(a, k, a.n);
    if (ja > k) mark_version<RB>(a, code_A(ja));
  }

  // the turns turn k waits for (after mark; a producer may appear more than once)
  SRNN_HD static int producers(const SrnnArgs& a, int64_t k, int32_t* pr, bool& bad) {
    const int32_t* s = src_of(a, k);
    int np = 0;
    collect<RB>(a, s[0], pr, np, bad);
    if (needs_A(a, k, s) && is_row(s[1])) collect<RB>(a, s[1], pr, np, bad);
    if (is_row(s[2])) collect<RB>(a, s[2], pr, np, bad);
    return np;
  }
};

// recompute depth of the attack outputs: two nested outputs for the small nets, one for the rest
// (each level doubles the inlined forwards of a read; the big aggregating nets: srnn_bignet.h)
template <class Net>
constexpr int ord_rb() {
  return Net::P <= 20 ? 2 : 1;
}

// fine turn trace (diagnostic build, -DSRNN_ORD_TRACE_FINE): s_memrealtime at the phases of a
// turn into o_trace[10k + i] (0 start, 1 own row, 2 attack, 3 teacher row, 4 learn_from epochs,
// 5 self-train, 6 stores, 7 published); the shipped build records 0 and 7 only ([2k], [2k + 1])
// (8, 9: the shader-clock counter s_memtime at the self-train's start and end: the clock the chain
// ran at is their difference over the real-time one)
// (10: the permutation-table row the turn trained with, -1: drawn inline; 11: spare; 12..35: the
// start of each self-train epoch)
#if defined(__HIP_DEVICE_COMPILE__) && defined(SRNN_ORD_TRACE_FINE)
#define SRNN_ORD_STAMP(a, k, i)                                                        \
  if ((a).o_trace) {                                                                   \
    (a).o_trace[36 * (k) + (i)] = __builtin_amdgcn_s_memrealtime();                   \
    if ((i) == 4 || (i) == 5) (a).o_trace[36 * (k) + 4 + (i)] = __builtin_amdgcn_s_memtime(); \
  }
#define SRNN_ORD_NOTE(a, k, i, v) \
  if ((a).o_trace) (a).o_trace[36 * (k) + (i)] = (uint64_t)(v)
constexpr int TRACE_SLOTS = 36, TRACE_END = 7;
#else
#define SRNN_ORD_STAMP(a, k, i)
#define SRNN_ORD_NOTE(a, k, i, v)
constexpr int TRACE_SLOTS = 2, TRACE_END = 1;
#endif

template <class Net, class S>
struct Ord : OrdSched<ord_rb<Net>()> {
  using I = Item<Net, S>;
  using Sched = OrdSched<ord_rb<Net>()>;
  static constexpr int P = Net::P;
  static constexpr int RB = Sched::RB;

  SRNN_HD static void read_version(const SrnnArgs& a, int32_t code, float* w) {
    if (code >= 0) {
      const int64_t j = code >> 1;
      I::load((code & 1) ? I::rowp(a.W, j) : I::rowp(a.W3, j), w);
    } else {
      I::load(I::rowp(a.W2, (int64_t)(-(int64_t)code - 1)), w);
    }
  }

  // version `code` into w: a stored version is loaded, an unstored attack output A(j) is
  // recomputed as f_j(victim) from its own two reads (ap(x, t, o, j): the attack's forward)
  template <int B, class AP>
  SRNN_HD static void mat(const SrnnArgs& a, int32_t code, float* w, const AP& ap) {
    if constexpr (B > 0) {
      if (is_A(code) && !stored(a, code >> 1)) {
        const int64_t j = code >> 1;
        const int32_t* sj = src_of(a, j);
        float x[P], t[P];
        mat<B - 1>(a, sj[0], x, ap);
        if (sj[1] == SRC_SELF) I::copy(t, x);
        else mat<B - 1>(a, sj[1], t, ap);
        ap(x, t, w, j);
        I::q(w);
        return;
      }
    }
    read_version(a, code, w);
  }

  // turn k: the serial loop's particle step (soup_seq_one) reading the versions of its plan
  // (prow >= 0: the turn's epoch permutations are row prow of k_ord_ptab's table, stride
  // 2 rec_total; else drawn inline)
  SRNN_HD static void turn(const SrnnCfg& c, const SrnnArgs& a, int64_t k, int32_t gen, float4* samp, uint8_t* perm,
                           int64_t prow = -1) {
    const int32_t* s = a.o_src + 4 * k;
    int64_t at, te;
    I::decision(a, k, gen, at, te);
    auto ap = [&](const float* x, const float* t, float* o, int64_t j) {
      Net::apply(x, t, o, I::actx(a, c, (uint64_t)j, (uint32_t)gen * 1024u + 1u, perm));
    };
    float w[P], f[P], o[P];
    mat<RB>(a, s[0], w, ap);
    SRNN_ORD_STAMP(a, k, 1);
    int8_t act = A_NONE;
    int64_t cp = -1;
    if (at >= 0) {  // 1. attack: the victim's row becomes f_k(victim) (A(k))
      if (needs_A(a, k, s)) {
        if (at == k) I::copy(f, w);
        else mat<RB>(a, s[1], f, ap);
        ap(w, f, o, k);
        I::q(o);
        if (stored(a, k)) I::store(I::rowp(a.W3, k), o);
        if (at == k) I::copy(w, o);
      }
      act = A_ATTACKING;
      cp = at;
    }
    SRNN_ORD_STAMP(a, k, 2);
    TrainCtx tc;
    tc.lr = a.lr;
    tc.rng = I::rng(a);
    tc.uid = (uint64_t)k;
    tc.ctr = (uint32_t)gen * 1024u + 512u;
    tc.samp = samp;
    tc.perm = perm;
    tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
    tc.stride = SAMP_STRIDE;
    tc.aggregator = c.aggregator;
    if (a.ptab && a.dev && prow >= 0) {  // precomputed by k_ord_ptab: the turn's epochs side by side
      tc.ptab = a.ptab + prow * (int64_t)table_epochs(a);
      tc.pstride = 1;
      tc.pbase = tc.ctr;
    }
    SRNN_ORD_NOTE(a, k, 10, tc.ptab ? prow : -1);
#if defined(SRNN_ORD_TRACE_FINE) && defined(__HIP_DEVICE_COMPILE__)
    // where the turn runs: HW_ID (wave slot, SIMD, CU, SH, SE) | XCC_ID << 32
    SRNN_ORD_NOTE(a, k, 11, ((uint64_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)));
#endif
#if defined(SRNN_ORD_TRACE_FINE)
    tc.etrace = a.o_trace ? a.o_trace + 36 * k + 12 : nullptr;
#endif
    float loss = 0.f;
    if (te >= 0) {  // 2. learn_from the teacher's current row
      if (s[2] == SRC_SELF) I::copy(f, w);
      else if (s[2] == SRC_ATK) I::copy(f, o);
      else mat<RB>(a, s[2], f, ap);
      SRNN_ORD_STAMP(a, k, 3);
      if constexpr (Net::KIND == 0) {
        if (a.severity > 0) loss = Net::template train_epochs<false>(w, f, a.severity, tc);
      } else {
        for (int e = 0; e < a.severity; ++e) loss = Net::train_epoch(w, f, tc);
      }
      act = A_LEARN_FROM;
      cp = te;
    }
    SRNN_ORD_STAMP(a, k, 4);
    if (a.epochs > 0) {  // 3. self-train
      if constexpr (Net::KIND == 0) {
        loss = Net::template train_epochs<true>(w, f, a.epochs, tc);
      } else {
        for (int e = 0; e < a.epochs; ++e) {
          I::copy(f, w);
          loss = Net::train_epoch(w, f, tc);
        }
      }
      act = A_TRAIN_SELF;
      cp = -1;
    }
    SRNN_ORD_STAMP(a, k, 5);
    I::q(w);  // 4. respawn (the stored state decides; the zero test on the old particle)
    int8_t rs = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && is_diverged<P>(w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && is_zero<P>(w, a.eps)) rs = 2;
    if (a.traj) I::store(I::rowp(a.traj, k), w);  // recording: the state before any respawn
    if (rs) Net::init(w, I::rng(a), respawn_key(gen, k));
    I::store(I::rowp(a.W, k), w);  // E(k)
    if (a.action) a.action[k] = act;
    if (a.counterpart) a.counterpart[k] = cp;
    if (a.loss) a.loss[k] = loss;
    if (a.respawn) a.respawn[k] = rs;
    SRNN_ORD_STAMP(a, k, 6);
  }

  // row r after the generation: the last attack after its own turn, else E(r) (in W);
  // consumes r's attack list.  w receives the final row as a reload would see it (ROW = false:
  // only a recomputed final row is written, nothing is loaded -- the census comes later).
  template <bool ROW = true>
  SRNN_HD static void close_row(const SrnnCfg& c, const SrnnArgs& a, int64_t r, int32_t gen, uint8_t* perm, float* w) {
    const int64_t ja = last_attacker_before(a, r, a.n);
    a.heads[r] = SRNN_NIL;  // consumed: NIL for the generation after next
    if (ja > r) {
      auto ap = [&](const float* x, const float* t, float* o, int64_t j) {
        Net::apply(x, t, o, I::actx(a, c, (uint64_t)j, (uint32_t)gen * 1024u + 1u, perm));
      };
      mat<RB>(a, code_A(ja), w, ap);
      I::store(I::rowp(a.W, r), w);
    } else if constexpr (ROW) {
      I::load(I::rowp(a.W, r), w);
    }
  }
};

// the distinct entries of pr[0..np) moved to its front (order of first appearance)
SRNN_HD int dedupe(int32_t* pr, int np) {
  int m = 0;
  for (int q = 0; q < np; ++q) {
    bool seen = false;
    for (int t = 0; t < m; ++t) seen = seen || pr[t] == pr[q];
    if (!seen) pr[m++] = pr[q];
  }
  return m;
}

__device__ __forceinline__ int32_t ld_level(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_level(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave-aggregated append: this lane's position among the wave's `want` lanes after one
// atomicAdd on ctr (every lane of the wave calls it)
__device__ __forceinline__ int32_t wave_append(int32_t* ctr, bool want) {
  const unsigned long long m = __ballot(want);
  if (!m) return -1;
  const int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1;
  int32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (int32_t)__popcll(m));
  base = __shfl(base, leader);
  return want ? base + (int32_t)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}
__device__ __forceinline__ int32_t wave_sum(int32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Turn `k` is done: publish it to its consumers (pending records pushed onto its list by
// k_ord_count).  Its rows were stored with plain stores; they are drained and released at
// agent scope (the consumers may run on any CU / XCD) BEFORE the counts go down.  Every
// record whose count this lane takes to zero joins the lane's ready list (linked through the
// records' R_RDY words, `nready` long); k_ord_run shares the lists out over its wave.
// ROWS = false (level propagation only): nothing but the producer's level -- an agent-scope atomic
// store -- is handed over, so its completion (vmcnt) before the decrements replaces the release.
// PRIVATE (the ready-queue run, where a lane keeps the first record it made ready): a turn with ONE
// consumer whose only producer it is hands that consumer to itself -- nothing the turn wrote is
// read by another lane of this launch -- so the drain and the release are skipped and `priv` tells
// the caller that the continuation needs no acquire either (the chains of a generation's deep
// tail are such links: a release + an acquire is ~3 us of a ~33 us link, profiles/r6*).
template <bool ROWS = true, bool PRIVATE = false>
__device__ __forceinline__ void publish(const SrnnArgs& a, int64_t k, int32_t& ready, int32_t& nready, bool& priv) {
  priv = false;
  const int32_t h = cons_head(a)[k];
  if (h == EMPTY) return;
  if constexpr (PRIVATE) {
    const int32_t* r0 = pend(a, h);
    priv = r0[1] == 1 && r0[R_NEXT] == EMPTY;
  }
  if (!priv) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (ROWS) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (kept: ROCm 7.2 may drop the fence's own wait)
    }
  }
  for (int32_t q = h; q != EMPTY;) {
    int32_t* rec = pend(a, q);
    const int np = rec[1];
    int s = 0;
    for (int t = 0; t < np; ++t)
      if (rec[R_PROD + t] == (int32_t)k) s = t;
    const int32_t nxt = rec[R_NEXT + s];
    if (__hip_atomic_fetch_add(rec + R_CNT, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
      rec[R_RDY] = ready;
      ready = q;
      ++nready;
    }
    q = nxt;
  }
}
template <bool ROWS = true>
__device__ __forceinline__ void publish(const SrnnArgs& a, int64_t k, int32_t& ready, int32_t& nready) {
  bool priv;
  publish<ROWS, false>(a, k, ready, nready, priv);
}

}  // namespace ord

// (link / plan / mark / count: shape independent, one instantiation per recompute depth).  Each
// phase is a per-item (or per-64-item chunk) body, run by its own launch (OP_ORD_PLAN) or by the
// plan workgroups of a run launch (SRNN_F_ORD_INPLAN, ord_plan_group below).
namespace ord {
// the planned generation's attack lists: row r joins its victim's list (the lists are NIL on entry:
// the close two generations before consumed them)
template <int RB>
__device__ __forceinline__ void link_item(const SrnnArgs& a, int64_t r) {
  using Dec = typename OrdSched<RB>::Dec;
  int64_t at, te;
  Dec::decision(a, r, plan_gen(a), at, te);
  if (at >= 0) Dec::link(a.heads, a.nexts, at, (uint32_t)r);
}
template <int RB>
__device__ __forceinline__ void plan_item(const SrnnArgs& a, int64_t k) {
  OrdSched<RB>::plan(a, k, plan_gen(a));
  ready_queue(a)[k] = EMPTY;  // (at most one queue entry per pending turn: < n)
}
// every turn of 64-turn chunk `ci` counts its producers; a turn with producers becomes a pending
// record of the chunk's partition (producers written straight into the record, deduplicated) and
// is pushed onto each producer's consumer list.  No turn runs before the lists are complete.
// (One wave per chunk: the record slots are appended wave-wide.)
template <int RB>
__device__ __forceinline__ void count_chunk(const SrnnArgs& a, int64_t ci) {
  using O = OrdSched<RB>;
  const int lane = threadIdx.x & 63;
  const int64_t k = ci * TB + lane;
  const bool valid = k < a.n;
  int np = 0;
  bool bad = false;
  if (valid) np = O::producers(a, k, nullptr, bad);
  if (bad) atomicOr(a.o_ctl + ERRW, ERR_UNSTORED);
  const bool pd = valid && np > 0;
  const int part = (int)(ci % NPART);
  const int32_t i = wave_append(a.o_ctl + PART0 + part, pd);
  if (pd) {
    const int64_t q = part * rec_cap(a.n) + i;
    int32_t* rec = pend(a, q);
    bool bad2 = false;
    int32_t* pr = rec + R_PROD;
    const int m = dedupe(pr, O::producers(a, k, pr, bad2));
    rec[0] = (int32_t)k;
    rec[1] = m;
    rec[R_CNT] = m;
    a.o_list[k] = (int32_t)q;
    int32_t* heads = cons_head(a);
    for (int s = 0; s < m; ++s) {
      const int32_t old = atomicExch(heads + pr[s], (int32_t)q);
      rec[R_NEXT + s] = old;
      if (old == EMPTY && (a.flags & SRNN_F_ORD_CRIT)) {  // pr[s]'s first consumer: a critical turn
        const int pp = (int)((pr[s] / TB) % NPART);
        const int32_t pos = atomicAdd(a.o_ctl + CRIT0 + pp, 1);
        run_order(a)[pp * rec_cap(a.n) + pos] = pr[s];
      }
    }
  }
}
// the epoch permutations of the turns on the generation's critical paths, drawn in parallel instead
// of on their latency-bound chains: the pending records (rows q < rec_total) and the roots that have
// consumers (row rec_total + their run-order slot).  Task y = (group, partition, epoch pair); items
// i0, i0 + step, ... of the partition's entries.  A row's E words are side by side
// (ptab[row * E + e]): the chain that reads them one epoch ahead touches one cache line / page per
// turn -- with the epochs 2 rec_total words apart (~1.6 MB at 100k) every epoch's word was its own
// page walk, ~0.5 us of stall per epoch (profiles/r6*).
template <class Net>
__device__ __forceinline__ void ptab_task(const SrnnArgs& a, int32_t E, int y, int64_t i0, int64_t step) {
  constexpr int P = Net::P;
  const int npair = (E + 1) / 2;
  const int grp = y / (NPART * npair);  // 0: records, 1: critical roots
  const int part = (y / npair) % NPART, p = y % npair;
  const int64_t cnt = ld_level(a.o_ctl + (grp ? CRIT0 : PART0) + part), q0 = part * rec_cap(a.n);
  const int32_t gen = plan_gen(a);
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const uint32_t c0 = (uint32_t)gen * 1024u + 512u + 2u * (uint32_t)p;  // even: one draw, two epochs
  for (int64_t i = i0; i < cnt; i += step) {
    const int64_t q = q0 + i;
    const int64_t k = grp ? run_order(a)[q] : pend(a, q)[0];
    const int64_t row = grp ? rec_total(a.n) + q : q;
    const U4 r = perm_draw(rng, (uint64_t)(a.lo + k), c0, P_SHUFFLE);
    a.ptab[row * E + 2 * p] = perm_from_bits<P>(perm_bits(r, c0));
    if (2 * p + 1 < E) a.ptab[row * E + 2 * p + 1] = perm_from_bits<P>(perm_bits(r, c0 + 1u));
  }
}
}  // namespace ord

template <int RB>
__global__ __launch_bounds__(TB) void k_ord_link(SrnnArgs a) {
  const int64_t r = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (r < a.n) ord::link_item<RB>(a, r);
}

template <int RB>
__global__ __launch_bounds__(TB) void k_ord_plan(SrnnCfg, SrnnArgs a) {
  const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
  // control words for the next launches (the error word is sticky: never cleared here)
  if (blockIdx.x == 0)
    for (int w = threadIdx.x; w < ord::CTL_WORDS; w += TB)
      if (w != ord::ERRW) a.o_ctl[w] = 0;
  if (k < a.n) ord::plan_item<RB>(a, k);
}

template <int RB>
__global__ __launch_bounds__(TB) void k_ord_mark(SrnnCfg, SrnnArgs a) {
  const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (k < a.n) ord::OrdSched<RB>::mark(a, k);
}

template <int RB>
__global__ __launch_bounds__(TB) void k_ord_count(SrnnCfg, SrnnArgs a) {
  ord::count_chunk<RB>(a, blockIdx.x);
}

// workgroup row y = (group, partition, pair), grid-stride over the partition's entries
template <class Net>
__global__ __launch_bounds__(TB) void k_ord_ptab(SrnnArgs a, int32_t E) {
  ord::ptab_task<Net>(a, E, (int)blockIdx.y, (int64_t)blockIdx.x * TB + threadIdx.x, (int64_t)gridDim.x * TB);
}

// ptab tasks of a plan: (records + critical roots) x partitions x epoch pairs
SRNN_HD int ord_ptab_rows(const SrnnArgs& a, int32_t E) {
  return ((a.flags & SRNN_F_ORD_CRIT) ? 2 : 1) * ord::NPART * ((E + 1) / 2);
}

namespace ord {
// all plan workgroups of a run launch have finished the phase: arrivals counted on the plan set's
// BARW word.  The phase's stores are released before the arrival and the other workgroups' are
// acquired after the wait.  Bounded: a barrier still short after ~2^24 polls (~1 s) sets
// ERR_PLAN_BARRIER and lets the workgroup go on -- a wrong plan instead of a launch that never ends.
// (Only plan workgroups wait here, only on each other, and they are the launch's last workgroups:
// every turn workgroup is dispatched before them and never waits on them.)
__device__ __forceinline__ void plan_barrier(int32_t* bar, int32_t target, int32_t* errw) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if ((threadIdx.x & 63) == 0) {
    __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int32_t polls = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++polls < (1 << 24))
      __builtin_amdgcn_s_sleep(4);
    if (polls >= (1 << 24)) atomicOr(errw, ERR_PLAN_BARRIER);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// SRNN_F_ORD_SYNC (one thread): count `mine` up by one (its own counter, touched by this stream only)
// and wait until the other stream's counter `other` has reached it.  Bounded by the shader's real-time
// clock (100 MHz): after ~2 s the wait sets ERR_SYNC and gives up -- a wrong generation, reported,
// instead of a launch that never ends (e.g. two streams that landed on one hardware queue).
__device__ __forceinline__ void sync_wait(int32_t* sync, int mine, int other, int32_t* errw) {
  const int32_t t = __hip_atomic_load(sync + mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __hip_atomic_store(sync + mine, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int32_t)(__hip_atomic_load(sync + other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - t) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      atomicOr(errw, ERR_SYNC);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
}  // namespace ord

// SRNN_F_ORD_SYNC, side stream: before a plan overwrites its set, the run of the generation before it
// has started -- so that generation's predecessor, the last user of the set, has closed
template <int D = 0>  // (a template: one weak definition across the translation units)
__global__ void k_ord_gate(SrnnArgs a) {
  if (threadIdx.x == 0) ord::sync_wait(a.o_sync, ord::SYNC_GATE, ord::SYNC_RUN, a.o_ctl + ord::ERRW);
}
// ... and after its last phase, the plan counts itself done (its launches' stores released first)
template <int D = 0>
__global__ void k_ord_signal(SrnnArgs a) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(a.o_sync + ord::SYNC_PLAN, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

namespace ord {
// SRNN_F_ORD_INPLAN: plan workgroup w of G builds the NEXT generation's plan (the *_next buffers and
// lists) while this generation's turns run -- link, plan, mark, count, permutations, the phases
// separated by plan_barrier -- instead of launches on a second stream, whose cross-queue
// dependencies cost ~10 us of idle queue per generation inside a hipGraph (profiles/r6a).
template <int RB, class PT>
__device__ void plan_group(const SrnnArgs& a, int64_t w, int64_t G) {
  SrnnArgs pa = a;
  pa.o_src = a.o_src_next;
  pa.o_list = a.o_list_next;
  pa.o_ctl = a.o_ctl_next;
  pa.ptab = a.ptab_next;
  pa.heads = a.heads_next;
  pa.nexts = a.nexts_next;
  pa.flags |= SRNN_F_ORD_NEXT;
  const int lane = threadIdx.x & 63;
  const int64_t nb = (a.n + TB - 1) / TB;
  int32_t* bar = pa.o_ctl + BARW;
  int32_t* errw = pa.o_ctl + ERRW;
  if (w == 0)  // the plan's control words (the sticky error word and the barrier counter excepted)
    for (int i = lane; i < CTL_WORDS; i += 64)
      if (i != ERRW && i != BARW) pa.o_ctl[i] = 0;
  for (int64_t ci = w; ci < nb; ci += G)
    if (ci * TB + lane < a.n) link_item<RB>(pa, ci * TB + lane);
  plan_barrier(bar, (int32_t)G, errw);
  for (int64_t ci = w; ci < nb; ci += G)
    if (ci * TB + lane < a.n) plan_item<RB>(pa, ci * TB + lane);
  plan_barrier(bar, (int32_t)(2 * G), errw);
  for (int64_t ci = w; ci < nb; ci += G)
    if (ci * TB + lane < a.n) OrdSched<RB>::mark(pa, ci * TB + lane);
  plan_barrier(bar, (int32_t)(3 * G), errw);
  for (int64_t ci = w; ci < nb; ci += G) count_chunk<RB>(pa, ci);
  if constexpr (!std::is_void_v<PT>) {
    const int32_t E = table_epochs(pa);
    if (pa.ptab && (pa.flags & SRNN_F_SHUFFLE) && E > 0) {
      plan_barrier(bar, (int32_t)(4 * G), errw);
      const int Y = ord_ptab_rows(pa, E);
      for (int64_t y = w; y < Y; y += G) ptab_task<PT>(pa, E, (int)y, lane, 64);
    }
  }
}
}  // namespace ord

// the g-th entry of the critical list (-1: past its end) and its slot; the wave's exclusive prefix
// of the partitions' counts in s_c (64 partitions = one per lane)
__device__ __forceinline__ int64_t ord_crit_at(const SrnnArgs& a, int64_t g, int32_t* s_c, int64_t& slot) {
  const int lane = threadIdx.x & 63;
  const int32_t c = ord::ld_level(a.o_ctl + ord::CRIT0 + lane);
  int32_t ic = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t v = __shfl_up(ic, off);
    if (lane >= off) ic += v;
  }
  s_c[lane] = ic - c;
  const int64_t C = __shfl(ic, 63);
  __syncthreads();
  slot = -1;
  if (g >= C) return -1;
  int p = 0;  // the last partition whose prefix is <= g (a partition with entries)
#pragma unroll
  for (int step = 32; step > 0; step >>= 1)
    if (s_c[p + step] <= g) p += step;
  slot = p * ord::rec_cap(a.n) + (g - s_c[p]);
  return ord::run_order(a)[slot];
}

// every turn of the generation.  A lane first runs a turn without producers: turn k (or, with
// the run order, the k-th of it: producers of later turns first, their waves at raised priority,
// their permutations from the table).  Then the wave works in rounds: the records its lanes made
// ready (each lane's list) are gathered into LDS and handed out one per lane -- a producer whose
// row several turns read does not run those turns one after another -- each run as a
// continuation (raised priority, permutations from the table) at level 1 + its deepest
// producer's.  The wave ends when no lane has a ready record left.
// (Pol: the turn of a net family and its LDS -- OrdLanePol below, the big aggregating nets'
// in srnn_bignet.h; the schedule itself is shape independent)
// the class counts of the 64-row block gb of final rows W into its block stats (words 1..3; the
// close wrote the respawn ballot, word 0): the census of a close with SRNN_F_ORD_CENSUS_LATER, by
// k_ord_census or by extra workgroups of the next generation's run launch (o_census_temp)
template <class Net, class S>
__device__ void ord_census_block(const SrnnCfg& c, const SrnnArgs& a, const float* W, uint64_t* temp, int64_t gb,
                                 uint8_t* perm) {
  using I = Item<Net, S>;
  const int lane = threadIdx.x & 63;
  const int64_t r = gb * TB + lane;
  int8_t k = -1;
  if (r < a.n) {
    float w[Net::P];
    I::load(I::rowp(W, r), w);
    k = I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, I::actx(a, c, (uint64_t)r, 0x7FFFFFF0u, perm));
  }
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(k == q));
  if (lane == 0) {
    uint64_t* mine = temp + gb * 4;
    mine[1] = (uint64_t)cnt[0] | ((uint64_t)cnt[1] << 32);
    mine[2] = (uint64_t)cnt[2] | ((uint64_t)cnt[3] << 32);
    mine[3] = (uint64_t)cnt[4];
  }
}

template <class Net, class S>
struct OrdLanePol {
  static constexpr bool SHADOW = true;
  static constexpr bool CENSUS = true;  // extra run workgroups may take the previous close's census  // a turn is one lane's: idle lanes may repeat it (k_ord_run)
  static constexpr int SAMP = samp_slots<Net>();
  static constexpr int PERM = (Net::P + 4) & ~3;
  static constexpr int RB = ord::Ord<Net, S>::RB;  // the plan's recompute depth
  using PT = std::conditional_t<(Net::KIND == 0 && Net::P <= 16), Net, void>;  // the permutation-table net
  struct Shared {
    float4 samp[TB * SAMP];
    uint8_t perm[TB * PERM];
  };
  __device__ static void turn(const SrnnCfg& c, const SrnnArgs& a, int64_t k, int32_t gen, Shared& sh, int64_t prow) {
    const int lane = threadIdx.x;
    ord::Ord<Net, S>::turn(c, a, k, gen, samp_lane<Net>(sh.samp, lane), sh.perm + lane * PERM, prow);
  }
  // the previous generation's census: its final rows are this generation's start rows W2
  __device__ static void census(const SrnnCfg& c, const SrnnArgs& a, int64_t gb, Shared& sh) {
    ord_census_block<Net, S>(c, a, a.W2, a.o_census_temp, gb, sh.perm + threadIdx.x * PERM);
  }
};
template <class Pol>
__global__ __launch_bounds__(TB) void k_ord_run(SrnnCfg c, SrnnArgs a) {
  __shared__ typename Pol::Shared s_sh;
  __shared__ int32_t s_q[TB];
  const int lane = threadIdx.x;
  // (SRNN_F_ORD_SYNC: this run has started, so the close before it is done -- the side stream's plan
  // of the next generation may overwrite that close's plan set)
  if ((a.flags & SRNN_F_ORD_SYNC) && blockIdx.x == 0 && lane == 0)
    __hip_atomic_fetch_add(a.o_sync + ord::SYNC_RUN, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  int64_t cur = -1, prow = -1;
  bool raised = false;
  // with the critical list: its waves first (the grid's first a.x_groups workgroups), at raised
  // priority, permutations from the table; then every other turn without producers in index order;
  // with SRNN_F_ORD_INPLAN the last a.o_plan_groups workgroups build the next generation's plan
  // (dispatched after the turn workgroups: measured faster than before them, profiles/r6a r6o)
  // (with o_census_temp, the ncen workgroups after the turn workgroups take the previous close's census)
  const int64_t ncw = (a.flags & SRNN_F_ORD_CRIT) ? a.x_groups : 0;
  const int64_t nturn = ncw + (a.n + TB - 1) / TB;
  const int64_t ncen = a.o_census_temp ? (a.n + TB - 1) / TB : 0;
  const int64_t bid = blockIdx.x;
  if ((a.flags & SRNN_F_ORD_INPLAN) && bid >= nturn + ncen) {
    ord::plan_group<Pol::RB, typename Pol::PT>(a, bid - nturn - ncen, a.o_plan_groups);
    return;
  }
  if constexpr (Pol::CENSUS) {
    if (bid >= nturn && bid < nturn + ncen) {
      Pol::census(c, a, bid - nturn, s_sh);
      return;
    }
  }
  if (bid < ncw) {
    __shared__ int32_t s_c[64];
    int64_t slot = -1;
    cur = ord_crit_at(a, (int64_t)blockIdx.x * TB + lane, s_c, slot);
    if (cur >= 0 && a.o_list[cur] >= 0) cur = -1;  // a producer with producers of its own: a continuation
    if (cur >= 0) prow = ord::rec_total(a.n) + slot;
    if (__ballot(cur >= 0)) {
      __builtin_amdgcn_s_setprio(2);
      raised = true;
    }
  } else {
    const int64_t k = (bid - ncw) * TB + lane;
    if (k < a.n && a.o_list[k] < 0 && !(ncw && ord::cons_head(a)[k] != ord::EMPTY)) cur = k;
    // (SRNN_KNOB_ORD_BULK_DELAY: the critical roots first, at full clock -- only the first residency
    // round of turn waves waits: a soup of many rounds (1M big-net turns) would pay it per round)
    if (a.o_bulk_delay > 0 && bid - ncw < 2048) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)a.o_bulk_delay * 100u) __builtin_amdgcn_s_sleep(16);
    }
  }
  if (cur >= 0) ord::st_level(a.o_src + 4 * cur + 3, 0);
  int32_t ready = ord::EMPTY, nready = 0, curlvl = 0;  // (curlvl: the level of this lane's turn)
  const bool queue = (a.flags & SRNN_F_ORD_QUEUE) != 0;
  for (;;) {
    bool priv = false;  // this lane's next turn is its private continuation (no acquire needed)
    int32_t lvl = 0;    // this lane's turn's level
    int32_t keep = ord::EMPTY;  // (ready-queue run) the first record this lane made ready
    // shadow lanes (a.o_shadow, SRNN_KNOB_ORD_SHADOW): in a round of at most o_shadow turns, every
    // idle lane repeats a busy lane's turn -- the same reads, the same arithmetic, the same values
    // stored to the same addresses -- and publishes nothing.  A lone lane's SGD chain runs ~15-35 %
    // slower per epoch than a full wave's (profiles/r6a r6o-r6p); the chain links of a generation
    // are mostly lone kept continuations.
    bool shadow = false;
    if constexpr (Pol::SHADOW) {
      const unsigned long long busy = __ballot(cur >= 0);
      const int nbusy = (int)__popcll(busy);
      if (nbusy > 0 && nbusy < TB && nbusy <= a.o_shadow) {  // (wave uniform)
        unsigned long long m = busy;
        for (int i = lane % nbusy; i > 0; --i) m &= m - 1;
        const int src = cur >= 0 ? lane : (int)__ffsll((long long)m) - 1;
        const int64_t c2 = __shfl(cur, src), p2 = __shfl(prow, src);
        if (cur < 0) {
          cur = c2;
          prow = p2;
          shadow = true;
        }
        // (a shadow reads rows its owner lane may have written in an earlier round of this wave)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      }
    }
    if (cur >= 0) {
      const uint64_t t0 = a.o_trace ? __builtin_amdgcn_s_memrealtime() : 0;
      Pol::turn(c, a, cur, gen, s_sh, prow);
      if (!shadow) {
        if (queue) ord::publish<true, true>(a, cur, ready, nready, priv);
        else ord::publish(a, cur, ready, nready);
        lvl = curlvl;
        if (a.o_trace) {
          a.o_trace[ord::TRACE_SLOTS * cur] = t0;
          a.o_trace[ord::TRACE_SLOTS * cur + ord::TRACE_END] = __builtin_amdgcn_s_memrealtime();
        }
      }
    }
    if (a.flags & SRNN_F_ORD_QUEUE) {
      // the generation's ready queue.  The first record a lane made ready is that lane's own next
      // turn (the continuation stays on the producer's lane: a chain of dependent turns pays no
      // queue round trips); the lane's other ready records are appended (one counter add per
      // wave), then the wave claims entries for its free lanes, whoever made them ready -- every
      // continuation round runs a full wave of turns instead of the few its own producers freed.
      // A record is appended by a wave that claims afterwards (a wave never leaves while a lane
      // still has a kept turn), so none is left behind when the others have left; a claimed slot
      // is written right after its tail add (the spin is short).
      int32_t* qa = ord::ready_queue(a);
      if (nready > 0) {
        keep = ready;
        if (--nready > 0) ready = ord::pend(a, keep)[ord::R_RDY];
      }
      const int32_t total = ord::wave_sum(nready);
      if (total) {
        int32_t pre = nready;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int32_t v = __shfl_up(pre, off);
          if (lane >= off) pre += v;
        }
        pre -= nready;
        int32_t base = 0;
        if (lane == 0) base = __hip_atomic_fetch_add(a.o_ctl + ord::QT, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        base = __shfl(base, 0);
        for (int32_t t = base + pre; nready > 0; ++t) {
          ord::st_level(qa + t, ready);
          ready = ord::pend(a, ready)[ord::R_RDY];
          --nready;
        }
      }
      const unsigned long long kept = __ballot(keep != ord::EMPTY);
      const int32_t room = TB - (int32_t)__popcll(kept);
      int32_t qb = 0, m = 0;
      if (lane == 0 && room > 0) {
        for (;;) {
          int32_t h = ord::ld_level(a.o_ctl + ord::QH);
          const int32_t avail = ord::ld_level(a.o_ctl + ord::QT) - h;
          if (avail <= 0) break;
          const int32_t want = avail < room ? avail : room;
          if (__hip_atomic_compare_exchange_strong(a.o_ctl + ord::QH, &h, h + want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)) {
            qb = h;
            m = want;
            break;
          }
        }
      }
      qb = __shfl(qb, 0);
      m = __shfl(m, 0);
      if (m == 0 && !kept) break;
      cur = -1;
      prow = keep;
      // the claimed entries go to the lanes without a kept turn, in lane order
      const int32_t slot = (int32_t)__popcll(~kept & ((1ull << lane) - 1ull));
      if (keep == ord::EMPTY && slot < m) {
        // (bounded: a slot still unwritten after ~2^24 polls is a scheduling bug -- error bit 8
        // and the entry skipped, rather than a wave that never ends)
        int32_t q, polls = 0;
        while ((q = ord::ld_level(qa + qb + slot)) == ord::EMPTY && ++polls < (1 << 24)) __builtin_amdgcn_s_sleep(1);
        if (q == ord::EMPTY) atomicOr(a.o_ctl + ord::ERRW, ord::ERR_QUEUE);
        else prow = q;
      }
      // the producers' rows (released before their decrements) are visible after an acquire; a
      // wave whose every continuation is private skips it (its lanes read only what they wrote)
      if (__ballot(prow >= 0 && !(priv && keep == prow))) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (prow >= 0) cur = ord::pend(a, prow)[0];
    } else {
    // the wave's ready records, one per lane (the rest stay in their lists for the next round)
    const int32_t total = ord::wave_sum(nready);
    if (total == 0) break;
    int32_t pre = nready;  // exclusive prefix of the list lengths
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t v = __shfl_up(pre, off);
      if (lane >= off) pre += v;
    }
    pre -= nready;
    for (int32_t t = pre; t < TB && nready > 0; ++t) {
      s_q[t] = ready;
      ready = ord::pend(a, ready)[ord::R_RDY];
      --nready;
    }
    __syncthreads();
    cur = -1;
    prow = -1;
    if (lane < total) {
      const int32_t q = s_q[lane];
      const int32_t* rec = ord::pend(a, q);
      cur = rec[0];
      prow = q;
    }
    __syncthreads();  // (s_q is refilled next round)
    // the producers' rows (released before their decrements) are visible after this
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!raised) {
      __builtin_amdgcn_s_setprio(2);
      raised = true;
    }
    if (cur >= 0) {
      int32_t lv = lvl;  // (a private continuation's one producer is this lane's last turn)
      if (!(priv && keep == prow)) {
        const int32_t* rec = ord::pend(a, prow);
        lv = 0;
        for (int t = 0; t < rec[1]; ++t) {
          const int32_t lp = ord::ld_level(a.o_src + 4 * (int64_t)rec[ord::R_PROD + t] + 3);
          lv = lv > lp ? lv : lp;
        }
      }
      ord::st_level(a.o_src + 4 * cur + 3, lv + 1);
      curlvl = lv + 1;
    }
  }
}

// final rows, census, next decisions, block stats (the fused generation's two-phase form:
// k_gen_finish / the batched finish number the newborns afterwards)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_close(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t gb = blockIdx.x;
  const int64_t r = gb * TB + threadIdx.x;
  const int lane = threadIdx.x;
  uint8_t* perm = s_perm + lane * PERM;
  const int32_t gen = I::gen_of(a);
  const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
  // (in-run planning: this set's barrier counter is free for the plan two generations on)
  if ((a.flags & SRNN_F_ORD_INPLAN) && gb == 0 && lane == 0) a.o_ctl[ord::BARW] = 0;
  bool rs = false;
  int8_t k = -1;
  const bool later = (a.flags & SRNN_F_ORD_CENSUS_LATER) != 0;  // the census: k_ord_census, beside the next run
  if (r < a.n) {
    if (a.o_src[4 * r + 3] < 0) atomicOr(a.o_ctl + ord::ERRW, ord::ERR_NOT_RUN);  // never ran: a scheduling bug
    float w[Net::P];
    if (later) ord::Ord<Net, S>::template close_row<false>(c, a, r, gen, perm, w);
    else ord::Ord<Net, S>::close_row(c, a, r, gen, perm, w);
    rs = a.respawn[r] != 0;
    if (!(a.flags & SRNN_F_ORD_PLANNED)) {  // (planned ahead: the next OP_ORD_PLAN links them)
      int64_t at, te;
      I::decision(a, r, gen + 1, at, te);
      if (at >= 0) I::link(a.heads_next, a.nexts_next, at, (uint32_t)r);
    }
    if (census && !later)
      k = I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, I::actx(a, c, (uint64_t)r, 0x7FFFFFF0u, perm));
  }
  if ((a.flags & SRNN_F_GEN_COUNTS) && gb == 0 && lane == 0) I::set_gen(a, gen + 1);
  const unsigned long long m = __ballot(rs);
  uint32_t cnt[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) cnt[q] = (uint32_t)__popcll(__ballot(k == q));
  if (lane == 0) {
    unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
    unsigned long long* mine = bs + gb * 4;
    mine[0] = m;
    mine[1] = (unsigned long long)cnt[0] | ((unsigned long long)cnt[1] << 32);
    mine[2] = (unsigned long long)cnt[2] | ((unsigned long long)cnt[3] << 32);
    mine[3] = (unsigned long long)cnt[4];
    if ((a.flags & SRNN_F_BORN_TOTAL) && m) atomicAdd(bs + ((a.n + TB - 1) / TB) * 4, (unsigned long long)__popcll(m));
  }
  // SRNN_F_ORD_SYNC: the launch ends (and the next run starts) once the next generation's plan is done
  if ((a.flags & SRNN_F_ORD_SYNC) && gb == 0 && lane == 0)
    ord::sync_wait(a.o_sync, ord::SYNC_CLOSE, ord::SYNC_PLAN, a.o_ctl + ord::ERRW);
}

// the census of the final rows after a close with SRNN_F_ORD_CENSUS_LATER: the class counts of each
// 64-row block into its block stats (words 1..3; the close wrote the respawn ballot, word 0)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_census(SrnnCfg c, SrnnArgs a) {
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ uint8_t s_perm[TB * PERM];
  ord_census_block<Net, S>(c, a, a.W, reinterpret_cast<uint64_t*>(a.temp), blockIdx.x, s_perm + threadIdx.x * PERM);
}

template <class Net, class S>
int soup_ord_census(const SrnnCfg& c, const SrnnArgs& a) {
  if (!a.dev || !a.W || !a.temp || a.n < 0) {
    set_error("ordered census: device, final rows W and the generation's block stats (temp)");
    return -5;
  }
  const int64_t nb = (a.n + TB - 1) / TB;
  if (nb <= 0) return 0;
  hipLaunchKernelGGL((k_ord_census<Net, S>), dim3((unsigned)nb), dim3(TB), 0, (hipStream_t)a.stream, c, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

#include "srnn_pair.h"

// The plan of a reference-order generation (o_src / o_list / o_ctl / ptab): weight independent --
// decisions are a pure function of (seed, slot, generation) -- so the engine issues it one
// generation ahead (OP_ORD_PLAN with SRNN_F_ORD_NEXT) on a side stream, beside the generation in
// flight, whose run launch leaves most of the chip idle behind its few dependent chains; the
// generation itself (SRNN_F_ORD_PLANNED) is then run + close.  `link`: the planned generation's
// attack lists are linked into heads / nexts first (else they are this generation's, linked by
// the previous close).

// the run (and count) launch's scheduling flags from the knobs, and the critical-list waves: the
// list holds at most one entry per pending record's producer slot; waves past its end return
// the run launch's workgroups: critical-list waves, turn waves, plan workgroups (SRNN_F_ORD_INPLAN)
inline int64_t ord_run_grid(const SrnnArgs& ra, int64_t nb) {
  return nb + ((ra.flags & SRNN_F_ORD_CRIT) ? ra.x_groups : 0) + ((ra.flags & SRNN_F_ORD_INPLAN) ? ra.o_plan_groups : 0) +
         (ra.o_census_temp ? nb : 0);
}
// SRNN_F_ORD_INPLAN needs the next plan set, its lists and 1..4096 plan workgroups
inline bool ord_inplan_ok(const SrnnArgs& a) {
  if (!(a.flags & SRNN_F_ORD_INPLAN)) return true;
  if (!(a.flags & SRNN_F_ORD_PLANNED) || !a.o_src_next || !a.o_list_next || !a.o_ctl_next || !a.heads_next ||
      !a.nexts_next || a.o_plan_groups < 1 || a.o_plan_groups > 4096) {
    set_error("in-run planning (SRNN_F_ORD_INPLAN) needs a planned generation, the next plan set (o_src_next, "
              "o_list_next, o_ctl_next), the next attack lists and 1..4096 plan workgroups");
    return false;
  }
  return true;
}
// SRNN_F_ORD_SYNC on a generation: device, planned ahead (by a synchronised plan), the counters
inline bool ord_sync_ok(const SrnnArgs& a) {
  if (!(a.flags & SRNN_F_ORD_SYNC)) return true;
  if (!a.dev || !a.o_sync || !(a.flags & SRNN_F_ORD_PLANNED) || (a.flags & SRNN_F_ORD_INPLAN)) {
    set_error("SRNN_F_ORD_SYNC: a device generation planned ahead on the side stream, with the o_sync counters");
    return false;
  }
  return true;
}
// the next generation's plan arguments of an in-run planning generation (host path)
inline SrnnArgs ord_next_plan_args(const SrnnArgs& a) {
  SrnnArgs pa = a;
  pa.o_src = a.o_src_next;
  pa.o_list = a.o_list_next;
  pa.o_ctl = a.o_ctl_next;
  pa.ptab = a.ptab_next;
  pa.heads = a.heads_next;
  pa.nexts = a.nexts_next;
  pa.flags |= SRNN_F_ORD_NEXT;
  return pa;
}

inline SrnnArgs ord_run_args(const SrnnArgs& a, int64_t nb) {
  SrnnArgs ra = a;
  // (defaults measured, profiles/r6a r6q-r6r: per-wave lists 0.173 ms vs the ready queue 0.296; shadow
  // lanes in rounds of <= 32 turns 0.160-0.162, <= 16 0.161-0.162, <= 63 0.163-0.165, off 0.172-0.173)
  if (knob(SRNN_KNOB_ORD_QUEUE, 0) != 0) ra.flags |= SRNN_F_ORD_QUEUE;
  ra.o_shadow = std::max(0, knob(SRNN_KNOB_ORD_SHADOW, 32));
  // (the turn waves start 12 us after the critical-list waves: the roots' SGD chains run their first
  // epochs before the bulk pulls the clock down; measured 0: 0.163-0.164 ms, 6: 0.160-0.162, 10:
  // 0.158-0.161, 14: 0.159-0.160, 20: 0.159-0.160, 35: 0.164, profiles/r6a r6i-r6j)
  ra.o_bulk_delay = std::min(1000, std::max(0, knob(SRNN_KNOB_ORD_BULK_DELAY, 12)));
  if (knob(SRNN_KNOB_ORD_CRIT, 1) != 0) {
    ra.flags |= SRNN_F_ORD_CRIT;
    ra.x_groups = (int32_t)std::min<int64_t>(nb, (ord::rec_total(a.n) + TB - 1) / TB);
  }
  return ra;
}

// device: [link ->] plan -> mark -> count (records, consumer lists, critical list) -> the
// critical turns' epoch permutations (PT: the nibble Weightwise net of the table, void: none)
template <int RB, class PT>
void ord_plan_dev(const SrnnCfg& c, const SrnnArgs& a, bool link) {
  const int64_t nb = (a.n + TB - 1) / TB;
  if (nb <= 0) return;
  hipStream_t st = (hipStream_t)a.stream;
  const bool sync = link && (a.flags & SRNN_F_ORD_SYNC);
  if (sync) hipLaunchKernelGGL(k_ord_gate<0>, dim3(1), dim3(64), 0, st, a);
  if (link) hipLaunchKernelGGL((k_ord_link<RB>), dim3((unsigned)nb), dim3(TB), 0, st, a);
  hipLaunchKernelGGL((k_ord_plan<RB>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  hipLaunchKernelGGL((k_ord_mark<RB>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  const SrnnArgs ra = ord_run_args(a, nb);
  hipLaunchKernelGGL((k_ord_count<RB>), dim3((unsigned)nb), dim3(TB), 0, st, c, ra);
  if constexpr (!std::is_void_v<PT>) {
    const int32_t E = ord::table_epochs(a);
    if (a.ptab && (a.flags & SRNN_F_SHUFFLE) && E > 0) {
      const int64_t est = std::max<int64_t>(a.n / 12 / ord::NPART, 1);
      hipLaunchKernelGGL((k_ord_ptab<PT>), dim3((unsigned)((est + TB - 1) / TB), (unsigned)ord_ptab_rows(ra, E)), dim3(TB),
                         0, st, ra, E);
    }
  }
  if (sync) hipLaunchKernelGGL(k_ord_signal<0>, dim3(1), dim3(64), 0, st, a);
}

// host: [link ->] plan -> mark -> every turn's level (producers precede their consumers in index
// order); o_ctl[MAXLW] the deepest level
template <int RB>
void ord_plan_host(const SrnnArgs& a, bool link) {
  using O = ord::OrdSched<RB>;
  const int32_t gen = ord::plan_gen(a);
  for (int w = 0; w < ord::CTL_WORDS; ++w)
    if (w != ord::ERRW) a.o_ctl[w] = 0;
  if (link)
    for (int64_t r = 0; r < a.n; ++r) {
      int64_t at, te;
      O::Dec::decision(a, r, gen, at, te);
      if (at >= 0) {
        a.nexts[r] = a.heads[at];
        a.heads[at] = (uint32_t)r;
      }
    }
  host_parallel(a.n, [&](int64_t k) { O::plan(a, k, gen); });
  for (int64_t k = 0; k < a.n; ++k) O::mark(a, k);
  int32_t maxl = 0;
  for (int64_t k = 0; k < a.n; ++k) {
    int32_t pr[ord::NPROD];
    bool bad = false;
    const int np = O::producers(a, k, pr, bad);
    if (bad) a.o_ctl[ord::ERRW] |= ord::ERR_UNSTORED;
    int32_t lv = 0;
    for (int q = 0; q < np; ++q) lv = std::max(lv, a.o_src[4 * (int64_t)pr[q] + 3] + 1);
    a.o_src[4 * k + 3] = lv;
    maxl = std::max(maxl, lv);
  }
  a.o_ctl[ord::MAXLW] = maxl;
}

// a single unsharded table of < 2^30 rows (int32 version codes)
inline bool ord_single_table(const SrnnArgs& a) {
  if (a.world > 1 || a.lo != 0 || a.n_total != a.n || a.n >= (int64_t)(1 << 30)) {
    set_error("ordered soup generation: one unsharded table of < 2^30 rows");
    return false;
  }
  return true;
}

// OP_ORD_PLAN of a lane-template net (the big aggregating nets: srnn_bignet.h)
template <class Net, class S>
int soup_ord_plan(const SrnnCfg& c, const SrnnArgs& a) {
  constexpr int RB = ord::Ord<Net, S>::RB;
  if (!ord_single_table(a)) return -5;
  if (!a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts) {
    set_error("ordered generation plan needs o_src, o_list, o_ctl and the planned generation's (NIL) attack lists");
    return -5;
  }
  if ((a.flags & SRNN_F_ORD_SYNC) && (!a.dev || !a.o_sync || !(a.flags & SRNN_F_ORD_NEXT))) {
    set_error("SRNN_F_ORD_SYNC: a device plan of the next generation with the o_sync counters");
    return -5;
  }
  if (!a.dev) {
    ord_plan_host<RB>(a, true);
    return 0;
  }
  using PT = std::conditional_t<(Net::KIND == 0 && Net::P <= 16), Net, void>;
  ord_plan_dev<RB, PT>(c, a, true);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// OP_SOUP_ORDERED: one sequential (reference-order) generation of a single-rank table.
// W2: generation-start rows, W: the generation's rows (E versions, then the final table),
// W3: the stored attack outputs, o_src (layout above), o_list [n], o_ctl [CTL_WORDS],
// o_levels: dependency levels the host path runs as separate passes (the rest: one pass per
// level as well; the device schedules by continuation and ignores it);
// heads / nexts: this generation's attack lists (consumed), heads_next / nexts_next: the
// next generation's (linked here, unless SRNN_F_ORD_PLANNED: the plan was built ahead by
// OP_ORD_PLAN, which links its own lists).  Device: the block stats of the two-phase fused
// generation in temp (SRNN_F_TWO_PHASE); host: the finish inline (uids, census, counter).
template <class Net, class S>
int soup_ordered(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  using O = ord::Ord<Net, S>;
  const bool planned = (a.flags & SRNN_F_ORD_PLANNED) != 0;
  if (!ord_single_table(a)) return -5;
  if (!a.W || !a.W2 || !a.W3 || !a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts ||
      (!planned && (!a.heads_next || !a.nexts_next)) || !a.respawn || a.o_levels < 1 ||
      a.o_levels > ord::MAX_LEVELS) {
    set_error("ordered soup generation needs W, W2, W3, o_src, o_list, o_ctl, the attack lists (both unless "
              "planned ahead), respawn and 1 <= o_levels <= 16");
    return -5;
  }
  if (!ord_inplan_ok(a) || !ord_sync_ok(a)) return -5;
  if (!a.dev) {
    const int32_t gen = I::gen_of(a);
    if (!planned) ord_plan_host<O::RB>(a, false);
    // levels in index order (every producer precedes its consumer)
    std::vector<std::vector<int64_t>> lists;
    for (int64_t k = 0; k < a.n; ++k) {
      const int32_t lv = a.o_src[4 * k + 3];
      if ((size_t)lv >= lists.size()) lists.resize((size_t)lv + 1);
      lists[(size_t)lv].push_back(k);
    }
    for (const auto& li : lists)
      host_parallel((int64_t)li.size(), [&](int64_t q) {
        float4 samp[Net::P + 1];
        uint8_t perm[Net::P + 4];
        O::turn(c, a, li[(size_t)q], gen, samp, perm);
      });
    std::vector<int8_t> ks((size_t)a.n, (int8_t)-1);
    const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
    host_parallel(a.n, [&](int64_t r) {
      float w[Net::P];
      uint8_t perm[Net::P + 4];
      O::close_row(c, a, r, gen, perm, w);
      if (census)
        ks[(size_t)r] = I::classify_w(w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0,
                                      I::actx(a, c, (uint64_t)r, 0x7FFFFFF0u, perm));
    });
    if (!planned)
      for (int64_t r = 0; r < a.n; ++r) {
        int64_t at, te;
        I::decision(a, r, gen + 1, at, te);
        if (at >= 0) {
          a.nexts_next[r] = a.heads_next[at];
          a.heads_next[at] = (uint32_t)r;
        }
      }
    uint64_t cs[5] = {0, 0, 0, 0, 0};
    for (int64_t r = 0; r < a.n; ++r)
      if (ks[(size_t)r] >= 0) cs[ks[(size_t)r]]++;
    int64_t u = a.uid_base ? a.uid_base[0] : 0, total = 0;
    for (int64_t r = 0; r < a.n; ++r)
      if (a.respawn[r]) {
        if (a.uid_out) a.uid_out[r] = u;
        ++u;
        ++total;
      }
    if (a.uid_base) a.uid_base[0] = u;
    I::set_gen(a, gen + 1);
    if (a.counts) {
      for (int q = 0; q < 5; ++q) a.counts[q] = census ? cs[q] : 0;
      a.counts[5] = (uint64_t)total;
    }
    if (a.flags & SRNN_F_ORD_INPLAN) ord_plan_host<O::RB>(ord_next_plan_args(a), true);  // the next plan
    return 0;
  }
  if (!(a.flags & SRNN_F_TWO_PHASE) || !a.temp) {
    set_error("device ordered soup generation: two-phase block stats (temp) needed");
    return -5;
  }
  const int64_t nb = (a.n + TB - 1) / TB;
  if (nb <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  using PT = std::conditional_t<(Net::KIND == 0 && Net::P <= 16), Net, void>;
  if (!planned) ord_plan_dev<O::RB, PT>(c, a, false);
  const SrnnArgs ra = ord_run_args(a, nb);
  hipLaunchKernelGGL((k_ord_run<OrdLanePol<Net, S>>), dim3((unsigned)ord_run_grid(ra, nb)), dim3(TB), 0, st, c, ra);
  hipLaunchKernelGGL((k_ord_close<Net, S>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  if (!(a.flags & SRNN_F_GEN_COUNTS)) {
    constexpr int FNT = SRNN_FINISH_NT;
    hipLaunchKernelGGL((k_gen_finish<Net, S, FNT>), dim3(1), dim3(FNT), 0, st, a, (int32_t)nb);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

#include "srnn_ordered_sh.h"
