// srnn_ordered_sh.h — the reference's sequential, in-place soup generation sharded over R ranks
// (OP_SOUP_ORDERED_SH), bitwise equal to the single-rank generation (srnn_ordered.h) and to the
// serial loop.  Included by srnn_ordered.h inside namespace srnn.
//
// Every rank plans the WHOLE generation (decisions are a pure function of (seed, slot,
// generation); the plan, the attack-output marks and the dependency DAG are replicated, a few
// int32 per turn), but runs only its own turns [o_lo, o_hi).  The generation-start rows come
// from an all-gather of every rank's rows; then the DAG is run level by level: each rank runs its
// turns of level L, packs their outputs (E(k) and, where later turns read it past the recompute
// depth, A(k)), and one all-gather gives every rank every output of level L before any turn of
// level L+1 -- which reads only versions of levels < L+1 -- starts.  Each turn reads exactly the
// versions it reads on one rank, so the generation is bitwise the same for any rank count
// (tests/test_ordered_sharded.py).  Phases (SrnnArgs.steps), in the global view (n = n_total,
// lo = 0; W2 the gathered generation-start table, W / W3 the version tables of all rows):
//
//   0 PLAN    plan + mark + count of every turn, then every turn's level (propagated along the
//             consumer lists without running anything); o_ctl[MAXLW] the deepest level
//   1 LEVEL   this rank's turns whose level is o_levels
//   2 PACK    their outputs as exchange records {slot, E row, A row} (x_ctl[0] counts them)
//   3 UNPACK  the gathered records of every rank (recvbuf, x_blk records) into W / W3
//   4 CLOSE   this rank's rows: final version (a later attacker's output, recomputed) into W,
//             per-row respawn flags (rowflags, local) for the uid assignment
//   5 LINK    every slot: this generation's attack lists consumed, the next one's linked
//
// The caller (SoupEngine) runs the collectives between the phases and the census / uid
// assignment of the all-gather exchange after them (OP_CLASSIFY, OP_UID_ASSIGN).
#pragma once

namespace ordsh {
constexpr int PLAN = 0, LEVEL = 1, PACK = 2, UNPACK = 3, CLOSE = 4, LINK = 5;
// exchange record: int64 slot (-1: empty) + pad to 16 bytes | E row | A row (rows 16-byte aligned:
// the row loads / stores are 16-byte vector accesses)
constexpr int64_t HDR = 16;
template <class I>
constexpr int64_t rec_bytes() {
  return HDR + 2 * (int64_t)I::RB;
}
}  // namespace ordsh

// levels of every turn without running any: a root (no producer) is level 0 and counts its
// consumers down; the lane that takes a record to zero sets its level (1 + its deepest
// producer's) and counts that turn's consumers down in turn.  Levels are agent-scope atomics,
// drained before the decrements (ord::publish<false>: no rows handed over, no release).
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_levels(SrnnArgs a) {
  const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
  int32_t ready = ord::EMPTY, nready = 0, maxl = 0;
  if (k < a.n && a.o_list[k] < 0) {
    ord::st_level(a.o_src + 4 * k + 3, 0);
    ord::publish<false>(a, k, ready, nready);
  }
  while (ready != ord::EMPTY) {
    const int32_t q = ready;
    const int32_t* rec = ord::pend(a, q);
    ready = rec[ord::R_RDY];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    int32_t lv = 0;
    for (int t = 0; t < rec[1]; ++t) {
      const int32_t lp = ord::ld_level(a.o_src + 4 * (int64_t)rec[ord::R_PROD + t] + 3);
      lv = lv > lp ? lv : lp;
    }
    const int64_t kk = rec[0];
    ord::st_level(a.o_src + 4 * kk + 3, lv + 1);
    maxl = maxl > lv + 1 ? maxl : lv + 1;
    ord::publish<false>(a, kk, ready, nready);
  }
  if (maxl) atomicMax(a.o_ctl + ord::MAXLW, maxl);
}

// this rank's turns of level L (lane per own turn; a wave without one returns at once).  A wave
// with at most a.o_shadow of them (the deep levels are sparse) runs each on several lanes: the idle
// lanes repeat a busy lane's turn -- identical values to identical addresses -- as k_ord_run's
// shadow lanes (a lone lane's SGD chain is ~16 % slower than a full wave's, profiles/r6a)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_level(SrnnCfg c, SrnnArgs a, int32_t L) {
  using I = Item<Net, S>;
  constexpr int SAMP = samp_slots<Net>();
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ float4 s_samp[TB * SAMP];
  __shared__ uint8_t s_perm[TB * PERM];
  const int lane = threadIdx.x;
  int64_t k = a.o_lo + (int64_t)blockIdx.x * TB + lane;
  bool mine = k < a.o_hi && a.o_src[4 * k + 3] == L;
  const unsigned long long busy = __ballot(mine);
  if (!busy) return;
  const int nbusy = (int)__popcll(busy);
  if (nbusy < TB && nbusy <= a.o_shadow) {  // (wave uniform)
    unsigned long long m = busy;
    for (int i = lane % nbusy; i > 0; --i) m &= m - 1;
    const int src = mine ? lane : (int)__ffsll((long long)m) - 1;
    k = __shfl(k, src);
    mine = true;
  }
  if (mine) ord::Ord<Net, S>::turn(c, a, k, I::gen_of(a), samp_lane<Net>(s_samp, lane), s_perm + lane * PERM);
}

// records of this rank's level-L outputs (append order is irrelevant: records carry their slot)
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_pack(SrnnArgs a, int32_t L) {
  using I = Item<Net, S>;
  constexpr int64_t RECB = ordsh::rec_bytes<I>();
  const int64_t k = a.o_lo + (int64_t)blockIdx.x * TB + threadIdx.x;
  const bool mine = k < a.o_hi && a.o_src[4 * k + 3] == L;
  const int32_t pos = ord::wave_append(a.x_ctl, mine);
  if (!mine) return;
  if ((int64_t)pos >= a.x_blk) {  // the caller sized the buffer for this level: a bug
    atomicOr(a.o_ctl + ord::ERRW, ord::ERR_PACK);
    return;
  }
  char* r = reinterpret_cast<char*>(a.sendbuf) + (int64_t)pos * RECB;
  *reinterpret_cast<int64_t*>(r) = k;
  float w[Net::P];
  I::load(I::rowp(a.W, k), w);
  I::store(r + ordsh::HDR, w);
  if (ord::stored(a, k)) {
    I::load(I::rowp(a.W3, k), w);
    I::store(r + ordsh::HDR + I::RB, w);
  }
}

// the gathered records (every rank's, this rank's included: the same bytes) into W / W3
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_unpack(SrnnArgs a, int64_t nrec) {
  using I = Item<Net, S>;
  constexpr int64_t RECB = ordsh::rec_bytes<I>();
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.x_ctl[0] = 0;  // the next level's pack counter
  if (i >= nrec) return;
  const char* r = reinterpret_cast<const char*>(a.recvbuf) + i * RECB;
  const int64_t k = *reinterpret_cast<const int64_t*>(r);
  if (k < 0 || k >= a.n || (k >= a.o_lo && k < a.o_hi)) return;
  float w[Net::P];
  I::load(r + ordsh::HDR, w);
  I::store(I::rowp(a.W, k), w);
  if (ord::stored(a, k)) {
    I::load(r + ordsh::HDR + I::RB, w);
    I::store(I::rowp(a.W3, k), w);
  }
}

// this rank's rows: final version into W, respawn flag for the uid assignment
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_close(SrnnCfg c, SrnnArgs a) {
  using I = Item<Net, S>;
  constexpr int PERM = (Net::P + 4) & ~3;
  __shared__ uint8_t s_perm[TB * PERM];
  const int64_t r = a.o_lo + (int64_t)blockIdx.x * TB + threadIdx.x;
  if (r >= a.o_hi) return;
  if (a.o_src[4 * r + 3] < 0) atomicOr(a.o_ctl + ord::ERRW, ord::ERR_NOT_RUN);
  float w[Net::P];
  ord::Ord<Net, S>::close_row(c, a, r, I::gen_of(a), s_perm + threadIdx.x * PERM, w);
  if (a.rowflags) a.rowflags[r] = a.respawn[r] != 0;
}

// every slot: this generation's attack list consumed, the next generation's decision linked
template <class Net, class S>
__global__ __launch_bounds__(TB) void k_ordsh_link(SrnnArgs a) {
  using I = Item<Net, S>;
  const int64_t r = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (r >= a.n) return;
  a.heads[r] = SRNN_NIL;
  int64_t at, te;
  I::decision(a, r, I::gen_of(a) + 1, at, te);
  if (at >= 0) I::link(a.heads_next, a.nexts_next, at, (uint32_t)r);
}

template <class Net, class S>
int soup_ordered_sh(const SrnnCfg& c, const SrnnArgs& a) {
  using I = Item<Net, S>;
  using O = ord::Ord<Net, S>;
  constexpr int64_t RECB = ordsh::rec_bytes<I>();
  const int phase = a.steps;
  if (a.lo != 0 || a.n_total != a.n || a.n >= (int64_t)(1 << 30) || a.o_lo < 0 || a.o_hi < a.o_lo || a.o_hi > a.n) {
    set_error("sharded ordered generation: the global view (lo 0, n = n_total < 2^30) and 0 <= o_lo <= o_hi <= n");
    return -5;
  }
  if (!a.W || !a.W2 || !a.W3 || !a.o_src || !a.o_list || !a.o_ctl || !a.heads || !a.nexts || !a.respawn ||
      phase < ordsh::PLAN || phase > ordsh::LINK) {
    set_error("sharded ordered generation needs W, W2, W3, o_src, o_list, o_ctl, the attack lists, respawn and a "
              "phase 0..5");
    return -5;
  }
  if ((phase == ordsh::PACK && (!a.sendbuf || !a.x_ctl)) || (phase == ordsh::UNPACK && (!a.recvbuf || !a.x_ctl)) ||
      (phase == ordsh::LINK && (!a.heads_next || !a.nexts_next))) {
    set_error("sharded ordered generation: pack needs sendbuf + x_ctl, unpack recvbuf + x_ctl, link the next lists");
    return -5;
  }
  const int32_t gen = I::gen_of(a);
  const int32_t L = a.o_levels;
  const int64_t own = a.o_hi - a.o_lo;
  const int64_t nrec = phase == ordsh::UNPACK ? (int64_t)a.world * a.x_blk : 0;
  if (!a.dev) {
    switch (phase) {
      case ordsh::PLAN:
        ord_plan_host<O::RB>(a, false);
        return 0;
      case ordsh::LEVEL: {
        std::vector<int64_t> li;
        for (int64_t k = a.o_lo; k < a.o_hi; ++k)
          if (a.o_src[4 * k + 3] == L) li.push_back(k);
        host_parallel((int64_t)li.size(), [&](int64_t q) {
          float4 samp[Net::P + 1];
          uint8_t perm[Net::P + 4];
          O::turn(c, a, li[(size_t)q], gen, samp, perm);
        });
        return 0;
      }
      case ordsh::PACK: {
        int64_t pos = 0;
        for (int64_t k = a.o_lo; k < a.o_hi; ++k) {
          if (a.o_src[4 * k + 3] != L) continue;
          if (pos >= a.x_blk) {
            a.o_ctl[ord::ERRW] |= ord::ERR_PACK;
            break;
          }
          char* r = reinterpret_cast<char*>(a.sendbuf) + pos * RECB;
          *reinterpret_cast<int64_t*>(r) = k;
          float w[Net::P];
          I::load(I::rowp(a.W, k), w);
          I::store(r + ordsh::HDR, w);
          if (ord::stored(a, k)) {
            I::load(I::rowp(a.W3, k), w);
            I::store(r + ordsh::HDR + I::RB, w);
          }
          ++pos;
        }
        a.x_ctl[0] = (int32_t)pos;
        return 0;
      }
      case ordsh::UNPACK: {
        host_parallel(nrec, [&](int64_t i) {
          const char* r = reinterpret_cast<const char*>(a.recvbuf) + i * RECB;
          const int64_t k = *reinterpret_cast<const int64_t*>(r);
          if (k < 0 || k >= a.n || (k >= a.o_lo && k < a.o_hi)) return;
          float w[Net::P];
          I::load(r + ordsh::HDR, w);
          I::store(I::rowp(a.W, k), w);
          if (ord::stored(a, k)) {
            I::load(r + ordsh::HDR + I::RB, w);
            I::store(I::rowp(a.W3, k), w);
          }
        });
        a.x_ctl[0] = 0;
        return 0;
      }
      case ordsh::CLOSE: {
        host_parallel(own, [&](int64_t i) {
          const int64_t r = a.o_lo + i;
          float w[Net::P];
          uint8_t perm[Net::P + 4];
          O::close_row(c, a, r, gen, perm, w);
          if (a.rowflags) a.rowflags[r] = a.respawn[r] != 0;
        });
        return 0;
      }
      default: {  // LINK
        for (int64_t r = 0; r < a.n; ++r) a.heads[r] = SRNN_NIL;
        for (int64_t r = 0; r < a.n; ++r) {
          int64_t at, te;
          I::decision(a, r, gen + 1, at, te);
          if (at >= 0) {
            a.nexts_next[r] = a.heads_next[at];
            a.heads_next[at] = (uint32_t)r;
          }
        }
        return 0;
      }
    }
  }
  hipStream_t st = (hipStream_t)a.stream;
  const unsigned nb = (unsigned)((a.n + TB - 1) / TB), nbo = (unsigned)std::max<int64_t>((own + TB - 1) / TB, 1);
  switch (phase) {
    case ordsh::PLAN:
      hipLaunchKernelGGL((k_ord_plan<O::RB>), dim3(nb), dim3(TB), 0, st, c, a);
      hipLaunchKernelGGL((k_ord_mark<O::RB>), dim3(nb), dim3(TB), 0, st, c, a);
      hipLaunchKernelGGL((k_ord_count<O::RB>), dim3(nb), dim3(TB), 0, st, c, a);
      hipLaunchKernelGGL((k_ordsh_levels<Net, S>), dim3(nb), dim3(TB), 0, st, a);
      break;
    case ordsh::LEVEL:
      {
        SrnnArgs la = a;
        la.o_shadow = std::max(0, knob(SRNN_KNOB_ORD_SHADOW, 32));
        hipLaunchKernelGGL((k_ordsh_level<Net, S>), dim3(nbo), dim3(TB), 0, st, c, la, L);
      }
      break;
    case ordsh::PACK:
      hipLaunchKernelGGL((k_ordsh_pack<Net, S>), dim3(nbo), dim3(TB), 0, st, a, L);
      break;
    case ordsh::UNPACK:
      hipLaunchKernelGGL((k_ordsh_unpack<Net, S>), dim3((unsigned)std::max<int64_t>((nrec + TB - 1) / TB, 1)), dim3(TB),
                         0, st, a, nrec);
      break;
    case ordsh::CLOSE:
      hipLaunchKernelGGL((k_ordsh_close<Net, S>), dim3(nbo), dim3(TB), 0, st, c, a);
      break;
    default:
      hipLaunchKernelGGL((k_ordsh_link<Net, S>), dim3(nb), dim3(TB), 0, st, a);
      break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}
