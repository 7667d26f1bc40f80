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
// the DAG is shallow (100k particles: 95 % level 0, 4.8 % level 1, ~160 turns at level 2,
// a handful at 3; storing every A(j) gives 86 / 12.5 / 1.6 % and 5-6 levels), so a
// generation runs as
//
//   k_ord_plan    per turn: decisions, the source version of each of its reads (src codes)
//   k_ord_mark    per turn / row: flags the attack outputs reached past the recompute depth
//   k_ord_level0  per turn: its producers; none -> the turn runs now (level 0), else a pending
//                 record {turn, producers} in the workgroup's partition
//   k_ord_ptab    the pending records' epoch permutations (with a table)
//   k_ord_level   L = 1..C-1: a pass over the pending records -- a record whose producers all
//                 ran at levels < L runs now (WW(2,2): on a lane pair); no level is computed
//                 ahead, no DFS
//   k_ord_tail    the records still pending after level C-1, in rounds (fence + barrier per
//                 round): the last workgroup of launch C-1 to finish, or its own launch (C = 1)
//   k_ord_close   per row: its final version (a row attacked after its own turn ends the
//                 generation as that attack's output), census class, the next generation's
//                 decisions linked, block stats for the finish (newborn uids in slot order)
//
// Every turn runs the serial loop's per-particle code with the same Philox streams (attack
// keyed (k, gen*1024+1), SGD (k, gen*1024+512), newborn init respawn_key(gen, k)), and a
// recomputed attack output is the same function of the same versions, so a generation
// equals OP_SOUP_SEQ bitwise (tests/test_ordered_soup.py, host and device).  No workgroup
// waits for another: levels are separated by kernel boundaries, the tail's rounds by one
// wave's own barrier.
#pragma once

namespace ord {

// src codes: >= 0 a version written this generation (2j: A(j), 2j+1: E(j) in W); -(r+1): the
// generation-start row r (W2); SELF: the turn's own current row (s[1]: a self-attack, s[2]:
// learn_from itself); ATK: its own attack output (learn_from its victim); NONE: no such read
constexpr int32_t SRC_SELF = INT32_MIN;
constexpr int32_t SRC_ATK = INT32_MIN + 1;
constexpr int32_t SRC_NONE = INT32_MIN + 2;
constexpr int MAX_LEVELS = 16;  // parallel level launches per generation (the rest: the tail)
// o_ctl words: [TAILW] turns run by the tail, [MAXLW] max level, [ERRW] error bits (2: an
// unstored attack output past the recompute depth -- a marking bug, 4: the tail found no
// runnable turn among the pending ones), [REM0 + L] turns still pending after level launch L
// (turns run at level L = REM(L-1) - REM(L), level 0: n - REM(0)), [PART0 + p] records of
// partition p
constexpr int TICKW = 0;  // the last parallel level launch's workgroup tickets
constexpr int TAILW = MAX_LEVELS, MAXLW = MAX_LEVELS + 1, ERRW = MAX_LEVELS + 2, REM0 = MAX_LEVELS + 3;
// pending records live in NPART partitions (partition p: the level-0 workgroups b = p mod NPART,
// appended by one counter each at PART0 + p: no chip-wide contended counter)
constexpr int NPART = 64, PART0 = 2 * MAX_LEVELS + 3;
constexpr int CTL_WORDS = PART0 + NPART;
// o_src layout: [n][4] {own, victim, teacher, level} | [n] stored flags of A(j) |
// [rec_total(n)][16] pending records {turn, producer count, producers...}; o_list: [n] the
// tail's records
constexpr int NPROD = 12;  // producers of one turn: 3 reads x 2^RB leaves
constexpr int REC = 16;

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
SRNN_HD int32_t* pend(const SrnnArgs& a, int64_t q) { return a.o_src + 5 * a.n + REC * q; }
// records per partition (each level-0 workgroup of TB turns appends to its partition only)
SRNN_HD int64_t rec_cap(int64_t n) { return ((n + TB - 1) / TB + NPART - 1) / NPART * TB; }
SRNN_HD int64_t rec_total(int64_t n) { return NPART * rec_cap(n); }
SRNN_HD bool stored(const SrnnArgs& a, int64_t j) { return a.o_src[4 * a.n + j] != 0; }
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

template <class Net, class S>
struct Ord {
  using I = Item<Net, S>;
  static constexpr int P = Net::P;
  // recompute depth of the attack outputs: two nested outputs for the small nets, one for
  // the rest (each level doubles the inlined forwards of a read)
  static constexpr int RB = P <= 20 ? 2 : 1;

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

  // src codes of turn k (generation gen) -> o_src[k] = {own, victim, teacher, level = -1};
  // its stored flag cleared
  SRNN_HD static void plan(const SrnnArgs& a, int64_t k, int32_t gen) {
    int64_t at, te;
    I::decision(a, k, gen, at, te);
    int32_t* s = a.o_src + 4 * k;
    s[0] = latest(a, k, k);
    s[1] = at < 0 ? SRC_NONE : at == k ? SRC_SELF : latest(a, at, k);
    if (te < 0) s[2] = SRC_NONE;
    else if (te == k) s[2] = SRC_SELF;
    else if (te == at) s[2] = SRC_ATK;
    else s[2] = latest(a, te, k);
    s[3] = -1;
    a.o_src[4 * a.n + k] = 0;
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

  // the turns turn k waits for (after mark)
  SRNN_HD static int producers(const SrnnArgs& a, int64_t k, int32_t* pr, bool& bad) {
    const int32_t* s = src_of(a, k);
    int np = 0;
    collect<RB>(a, s[0], pr, np, bad);
    if (needs_A(a, k, s) && is_row(s[1])) collect<RB>(a, s[1], pr, np, bad);
    if (is_row(s[2])) collect<RB>(a, s[2], pr, np, bad);
    return np;
  }

  // turn k: the serial loop's particle step (soup_seq_one) reading the versions of its plan
  // (prow >= 0: the turn's epoch permutations are row prow of the pending records' table, stride
  // rec_total; else drawn inline)
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
    if (a.ptab && a.dev && prow >= 0) {  // precomputed by the level-0 launch
      tc.ptab = a.ptab + prow;
      tc.pstride = rec_total(a.n);
      tc.pbase = tc.ctr;
    }
    float loss = 0.f;
    if (te >= 0) {  // 2. learn_from the teacher's current row
      if (s[2] == SRC_SELF) I::copy(f, w);
      else if (s[2] == SRC_ATK) I::copy(f, o);
      else mat<RB>(a, s[2], f, ap);
      if constexpr (Net::KIND == 0) {
        if (a.severity > 0) loss = Net::template train_epochs<false>(w, f, a.severity, tc);
      } else {
        for (int e = 0; e < a.severity; ++e) loss = Net::train_epoch(w, f, tc);
      }
      act = A_LEARN_FROM;
      cp = te;
    }
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
  }

  // row r after the generation: the last attack after its own turn, else E(r) (in W);
  // consumes r's attack list.  w receives the final row as a reload would see it.
  SRNN_HD static void close_row(const SrnnCfg& c, const SrnnArgs& a, int64_t r, int32_t gen, uint8_t* perm, float* w) {
    const int64_t ja = last_attacker_before(a, r, a.n);
    a.heads[r] = SRNN_NIL;  // consumed: NIL for the generation after next
    if (ja > r) {
      auto ap = [&](const float* x, const float* t, float* o, int64_t j) {
        Net::apply(x, t, o, I::actx(a, c, (uint64_t)j, (uint32_t)gen * 1024u + 1u, perm));
      };
      mat<RB>(a, code_A(ja), w, ap);
      I::store(I::rowp(a.W, r), w);
    } else {
      I::load(I::rowp(a.W, r), w);
    }
  }
};

__device__ __forceinline__ int32_t ld_level(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_level(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_ctl(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all producers of pending record rec have levels in [0, L)
__device__ __forceinline__ bool ready(const SrnnArgs& a, const int32_t* rec, int32_t L) {
  const int np = rec[1];
  bool ok = true;
  for (int q = 0; q < np; ++q) {
    const int32_t lp = ld_level(a.o_src + 4 * (int64_t)rec[2 + q] + 3);
    ok = ok && lp >= 0 && lp < L;
  }
  return ok;
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

// level launch L >= 1 over the pending records, TPT threads per turn (1: lane, 2: pair),
// workgroup b on partition b mod NPART: a record whose producers all have levels < L runs now
// (its level becomes L); the others stay pending (REM(L), a fire-and-forget count; the last
// parallel launch also lists them for the tail).  run(k, q): turn k of record q.
template <int TPT, class F>
__device__ __forceinline__ void pending_pass(const SrnnArgs& a, int32_t L, F&& run) {
  if (ld_ctl(a.o_ctl + REM0 + L - 1) == 0) return;  // nothing left: REM(L) stays 0
  const bool last = L == a.o_levels - 1;
  const int part = (int)(blockIdx.x % NPART);
  const int64_t bpp = gridDim.x / NPART, j = blockIdx.x / NPART;
  const int64_t cnt = ld_ctl(a.o_ctl + PART0 + part), q0 = part * rec_cap(a.n);
  const int slots = (int)blockDim.x / TPT, slot = (int)threadIdx.x / TPT, sub = (int)threadIdx.x % TPT;
  int32_t ex = 0, nleft = 0;
  for (int64_t base = j * slots; base < cnt; base += bpp * slots) {
    const int64_t i = base + slot, q = q0 + i;
    bool left = false;
    if (i < cnt) {
      const int32_t* rec = pend(a, q);
      const int64_t k = rec[0];
      if (ld_level(a.o_src + 4 * k + 3) < 0) {
        if (ready(a, rec, L)) {
          run(k, q);
          if (sub == 0) {
            st_level(a.o_src + 4 * k + 3, L);
            ++ex;
          }
        } else {
          left = sub == 0;
        }
      }
    }
    if (last) {
      const int32_t pos = wave_append(a.o_ctl + REM0 + L, left);
      if (left) a.o_list[pos] = (int32_t)q;  // the tail's list
    } else {
      nleft += left;
    }
  }
  nleft = wave_sum(nleft);
  ex = wave_sum(ex);
  if ((threadIdx.x & 63) == 0) {
    if (nleft) atomicAdd(a.o_ctl + REM0 + L, nleft);
    if (ex) atomicMax(a.o_ctl + MAXLW, L);
  }
}

// levels >= C in one workgroup, round by round over the tail's records (C = 1: every pending
// record, partition by partition): the rows a round writes are released before the barrier
// and the L1 is invalidated after it.  A round that runs nothing while turns are left (no DAG:
// a bug) sets error bit 4 and stops -- never a hang.
template <int TPT, class F>
__device__ __forceinline__ void tail_rounds(const SrnnArgs& a, F&& run) {
  const int C = a.o_levels;
  const int64_t T = ld_ctl(a.o_ctl + REM0 + C - 1);
  if (T == 0) return;
  __shared__ int32_t s_cnt[2];
  const int slots = (int)blockDim.x / TPT, slot = (int)threadIdx.x / TPT, sub = (int)threadIdx.x % TPT;
  const int64_t cap = rec_cap(a.n);
  for (int32_t lv = C;; ++lv) {
    if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0;
    __syncthreads();
    int32_t ex = 0, left = 0;
    auto visit = [&](int64_t q) {
      const int32_t* rec = pend(a, q);
      const int64_t k = rec[0];
      if (ld_level(a.o_src + 4 * k + 3) < 0) {
        if (ready(a, rec, lv)) {
          run(k, q);
          if (sub == 0) {
            st_level(a.o_src + 4 * k + 3, lv);
            ++ex;
          }
        } else if (sub == 0) {
          ++left;
        }
      }
    };
    if (C > 1) {
      for (int64_t i0 = 0; i0 < T; i0 += slots)
        if (i0 + slot < T) visit(a.o_list[i0 + slot]);
    } else {
      for (int p = 0; p < NPART; ++p) {
        const int64_t cnt = ld_ctl(a.o_ctl + PART0 + p);
        for (int64_t i0 = 0; i0 < cnt; i0 += slots)
          if (i0 + slot < cnt) visit(p * cap + i0 + slot);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (ex) atomicAdd(&s_cnt[0], ex);
    if (left) atomicAdd(&s_cnt[1], left);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int32_t ext = s_cnt[0], lt = s_cnt[1];
    if (threadIdx.x == 0 && ext) {
      a.o_ctl[TAILW] += ext;
      a.o_ctl[MAXLW] = lv;
    }
    if (lt == 0) break;
    if (ext == 0) {
      if (threadIdx.x == 0) atomicOr(a.o_ctl + ERRW, 4);
      break;
    }
    __syncthreads();  // s_cnt is reset by the next round
  }
}

// the last parallel level launch (L = C-1 >= 1) runs the tail in its LAST workgroup to finish
// (a ticket, no waiting): every other workgroup's turns are released before its ticket, so
// the tail's rounds see them -- one launch less per generation
template <int TPT, class F>
__device__ __forceinline__ void level_then_tail(const SrnnArgs& a, int32_t L, F&& run) {
  pending_pass<TPT>(a, L, run);
  if (L != a.o_levels - 1) return;
  __shared__ int32_t s_last;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(a.o_ctl + TICKW, 1) == (int32_t)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  tail_rounds<TPT>(a, run);
}

}  // namespace ord

template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_plan(SrnnCfg, SrnnArgs a) {
  const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < ord::CTL_WORDS) a.o_ctl[threadIdx.x] = 0;  // read from the next launch on
  if (blockIdx.x == 0 && threadIdx.x + TB < ord::CTL_WORDS) a.o_ctl[threadIdx.x + TB] = 0;
  if (k < a.n) ord::Ord<Net, S>::plan(a, k, Item<Net, S>::gen_of(a));
}

template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_mark(SrnnCfg, SrnnArgs a) {
  const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (k < a.n) ord::Ord<Net, S>::mark(a, k);
}

// level 0: every turn counts its producers; a turn without any runs now (permutations drawn
// inline), the others become pending records of this workgroup's partition (producers written
// straight into the record)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_level0(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  using O = ord::Ord<Net, S>;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int lane = threadIdx.x;
  const int64_t k = (int64_t)blockIdx.x * TB + lane;
  const bool valid = k < a.n;
  const int32_t gen = I::gen_of(a);
  int np = 0;
  bool bad = false;
  if (valid) np = O::producers(a, k, nullptr, bad);
  if (bad) atomicOr(a.o_ctl + ord::ERRW, 2);
  const bool pend = valid && np > 0;
  const int part = (int)(blockIdx.x % ord::NPART);
  const int32_t i = ord::wave_append(a.o_ctl + ord::PART0 + part, pend);
  if (pend) {
    const int64_t q = part * ord::rec_cap(a.n) + i;
    int32_t* rec = ord::pend(a, q);
    rec[0] = (int32_t)k;
    bool bad2 = false;
    rec[1] = O::producers(a, k, rec + 2, bad2);
  } else if (valid) {
    ord::st_level(a.o_src + 4 * k + 3, 0);
    O::turn(c, a, k, gen, samp_lane<Net>(s_samp, lane), s_perm + lane * PERM);
  }
  const int32_t npend = ord::wave_sum(pend ? 1 : 0);
  if (lane == 0 && npend) atomicAdd(a.o_ctl + ord::REM0, npend);  // fire and forget
}

// the epoch permutations of the pending records (their turns run on the latency-bound level
// launches, where an inline draw sits on the chain): thread (record, epoch pair), workgroup
// row y = partition * pairs + pair, grid-stride over the partition's records
template <class Net>
__global__ __launch_bounds__(TB) void k_ord_ptab(SrnnArgs a, int32_t E) {
  constexpr int P = Net::P;
  const int npair = (E + 1) / 2;
  const int part = (int)blockIdx.y / npair, p = (int)blockIdx.y % npair;
  const int64_t cnt = ord::ld_ctl(a.o_ctl + ord::PART0 + part), q0 = part * ord::rec_cap(a.n);
  const int64_t stride = ord::rec_total(a.n);
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const Rng rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)};
  const uint32_t c0 = (uint32_t)gen * 1024u + 512u + 2u * (uint32_t)p;  // even: one draw, two epochs
  for (int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * TB) {
    const int64_t q = q0 + i, k = ord::pend(a, q)[0];
    const U4 r = perm_draw(rng, (uint64_t)(a.lo + k), c0, P_SHUFFLE);
    a.ptab[2 * p * stride + q] = perm_from_bits<P>(perm_bits(r, c0));
    if (2 * p + 1 < E) a.ptab[(2 * p + 1) * stride + q] = perm_from_bits<P>(perm_bits(r, c0 + 1u));
  }
}

// levels 1..C-1: a pass over the pending records
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_level(SrnnCfg c, SrnnArgs a, int32_t L) {
  using I = Item<Net, S>;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int lane = threadIdx.x;
  const int32_t gen = I::gen_of(a);
  float4* samp = samp_lane<Net>(s_samp, lane);
  uint8_t* perm = s_perm + lane * PERM;
  ord::level_then_tail<1>(a, L, [&](int64_t k, int64_t q) { ord::Ord<Net, S>::turn(c, a, k, gen, samp, perm, q); });
}

// levels >= C: one wave
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ord_tail(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int lane = threadIdx.x;
  const int32_t gen = I::gen_of(a);
  float4* samp = samp_lane<Net>(s_samp, lane);
  uint8_t* perm = s_perm + lane * PERM;
  ord::tail_rounds<1>(a, [&](int64_t k, int64_t q) { ord::Ord<Net, S>::turn(c, a, k, gen, samp, perm, q); });
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
  bool rs = false;
  int8_t k = -1;
  if (r < a.n) {
    float w[Net::P];
    ord::Ord<Net, S>::close_row(c, a, r, gen, perm, w);
    rs = a.respawn[r] != 0;
    int64_t at, te;
    I::decision(a, r, gen + 1, at, te);
    if (at >= 0) I::link(a.heads_next, a.nexts_next, at, (uint32_t)r);
    if (census)
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
}

#include "srnn_pair.h"

// OP_SOUP_ORDERED: one sequential (reference-order) generation of a single-rank table.
// W2: generation-start rows, W: the generation's rows (E versions, then the final table),
// W3: the stored attack outputs, o_src [n][4] + [n] stored flags, o_list [(C+1) n], o_ctl [CTL_WORDS], o_levels = C;
// heads / nexts: this generation's attack lists (consumed), heads_next / nexts_next: the
// next generation's (linked here).  Device: the block stats of the two-phase fused
// generation in temp (SRNN_F_TWO_PHASE); host: the finish inline (uids, census, counter).
template <class Net, class S>
int soup_ordered(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  using O = ord::Ord<Net, S>;
  if (a.world > 1 || a.lo != 0 || a.n_total != a.n || a.n >= (int64_t)(1 << 30)) {
    set_error("ordered soup generation: one unsharded table of < 2^30 rows");
    return -5;
  }
  if (!a.W || !a.W2 || !a.W3 || !a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts || !a.heads_next ||
      !a.nexts_next || !a.respawn || a.o_levels < 1 || a.o_levels > ord::MAX_LEVELS) {
    set_error("ordered soup generation needs W, W2, W3, o_src, o_list, o_ctl, both attack lists, respawn and "
              "1 <= o_levels <= 16");
    return -5;
  }
  const int32_t C = a.o_levels;
  if (!a.dev) {
    const int32_t gen = I::gen_of(a);
    for (int w = 0; w < ord::CTL_WORDS; ++w) a.o_ctl[w] = 0;
    host_parallel(a.n, [&](int64_t k) { O::plan(a, k, gen); });
    for (int64_t k = 0; k < a.n; ++k) O::mark(a, k);
    // levels in index order (every producer precedes its consumer)
    std::vector<std::vector<int64_t>> lists((size_t)C + 1);
    int32_t maxl = 0;
    for (int64_t k = 0; k < a.n; ++k) {
      int32_t* s = a.o_src + 4 * k;
      int32_t pr[ord::NPROD];
      bool bad = false;
      const int np = O::producers(a, k, pr, bad);
      if (bad) a.o_ctl[ord::ERRW] |= 2;
      int32_t lv = 0;
      for (int q = 0; q < np; ++q) lv = std::max(lv, a.o_src[4 * (int64_t)pr[q] + 3] + 1);
      s[3] = lv;
      maxl = std::max(maxl, lv);
      lists[(size_t)std::min(lv, C)].push_back(k);
    }
    // the device's control words: turns pending after each parallel level, the tail's count
    int64_t rem = a.n;
    for (int32_t L = 0; L < C; ++L) {
      rem -= (int64_t)lists[(size_t)L].size();
      a.o_ctl[ord::REM0 + L] = (int32_t)rem;
    }
    a.o_ctl[ord::TAILW] = (int32_t)lists[(size_t)C].size();
    a.o_ctl[ord::MAXLW] = maxl;
    auto run_turn = [&](int64_t k) {
      float4 samp[Net::P + 1];
      uint8_t perm[Net::P + 4];
      O::turn(c, a, k, gen, samp, perm);
    };
    for (int32_t L = 0; L < C; ++L) {
      const auto& li = lists[(size_t)L];
      host_parallel((int64_t)li.size(), [&](int64_t q) { run_turn(li[(size_t)q]); });
    }
    for (int32_t L = C; L <= maxl; ++L) {  // the tail, level by level
      std::vector<int64_t> li;
      for (int64_t k : lists[(size_t)C])
        if (a.o_src[4 * k + 3] == L) li.push_back(k);
      host_parallel((int64_t)li.size(), [&](int64_t q) { run_turn(li[(size_t)q]); });
    }
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
    return 0;
  }
  if (!(a.flags & SRNN_F_TWO_PHASE) || !a.temp) {
    set_error("device ordered soup generation: two-phase block stats (temp) needed");
    return -5;
  }
  const int64_t nb = (a.n + TB - 1) / TB;
  if (nb <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  hipLaunchKernelGGL((k_ord_plan<Net, S>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  hipLaunchKernelGGL((k_ord_mark<Net, S>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  constexpr bool ww22 = std::is_same_v<Net, Weightwise<2, 2>>;
  hipLaunchKernelGGL((k_ord_level0<Net, S>), dim3((unsigned)nb), dim3(TB), 0, st, c, a);
  if constexpr (Net::KIND == 0 && Net::P <= 16) {
    const int32_t E = (a.severity > 0 ? a.severity : 0) + (a.epochs > 0 ? a.epochs : 0);
    if (a.ptab && (a.flags & SRNN_F_SHUFFLE) && E > 0) {
      const int64_t est = std::max<int64_t>(a.n / 12 / ord::NPART, 1);
      hipLaunchKernelGGL((k_ord_ptab<Net>), dim3((unsigned)((est + TB - 1) / TB), (unsigned)(ord::NPART * ((E + 1) / 2))),
                         dim3(TB), 0, st, a, E);
    }
  }
  // levels >= 1 pass over the pending records (~5 % of the turns at the reference's rates, most
  // of them level 1): per partition, workgroups covering 8 % of its share in one pass (grid-
  // stride beyond); WW(2,2) on lane pairs (latency-bound: srnn_pair.h)
  const int64_t est = std::max<int64_t>(a.n / 12 / ord::NPART, 1);
  bool pairs = false;
  if constexpr (ww22) pairs = use_pairs(a.n / 20);
  for (int32_t L = 1; L < C; ++L) {
    if (pairs) {
      if constexpr (ww22) {
        const int64_t bpp = (est + 63) / 64;
        hipLaunchKernelGGL((k_ord_level2<S>), dim3((unsigned)(bpp * ord::NPART)), dim3(pair::TBW), 0, st, c, a, L);
      }
    } else {
      const int64_t bpp = (est + TB - 1) / TB;
      hipLaunchKernelGGL((k_ord_level<Net, S>), dim3((unsigned)(bpp * ord::NPART)), dim3(TB), 0, st, c, a, L);
    }
  }
  if (C == 1) {  // (C >= 2: the last level launch runs the tail in its last workgroup)
    if (pairs) {
      if constexpr (ww22) hipLaunchKernelGGL((k_ord_tail2<S>), dim3(1), dim3(pair::TBW), 0, st, c, a);
    } else {
      hipLaunchKernelGGL((k_ord_tail<Net, S>), dim3(1), dim3(TB), 0, st, c, a);
    }
  }
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
