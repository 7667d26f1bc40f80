// srnn_shard.hip — the sharded soup's exchange protocol (shape independent).
//
// One process per GPU owns a contiguous shard [lo, lo + n) of ONE global soup (reference
// Soup.evolve, code/soup.py:51-87: partners uniform over the whole population).  A
// generation t needs, on the rank of victim v, the generation-start rows of v's attackers,
// and on the rank of learner l, the row of l's teacher.  Every rank decides only its OWN
// slots (O(local) work and memory, int64 slots), one generation ahead:
//
//   pack_t   finish of generation t-1 (census, newborn count: this rank's stats) ->
//            exchange header; the decisions of t+1 for the local slots: attacks on local
//            victims linked into the t+1 lists, attacks on remote victims -> NOTICES
//            (attacker, victim) to the victim's rank, remote teachers -> REQUESTS to the
//            teacher's rank; the rows of exchange t: the rows requested in exchange t-1
//            (replies) and the attacker rows noticed in exchange t-1
//   all-to-all (one collective per generation; RCCL over xGMI, on a comm stream)
//   post_t   uids of generation t-1's newborns (rank prefix from the headers), global
//            census; received notices linked into the t+1 lists (entries n + received row
//            of exchange t+1, whose position both sides know), received requests kept for
//            pack_{t+1}
//   evolve_t local slots (no remote attacker / teacher) run beside the all-to-all;
//            remote-dependent slots (x_rlist) after post_t
//
// Block of the exchange from rank r to rank q (x_blk bytes):
//   header int64[12]  0..4 census of t-1, 5 newborns of t-1, 6 stats valid, 7 generation t,
//                     8 reply rows, 9 attack rows (10, 11 unused)
//   x_cr rows         replies first (in q's request order), then attack rows (in r's notice
//                     order); each row = table row + (int64 slot, int64 generation) tag
//   x_cn notices      (int64 attacker slot, int64 victim slot), -1 after the last one
//   x_cq requests     int64 teacher slot, -1 after the last one
// The notice / request areas are appended densely by atomic counters and terminated by the
// -1 sentinel (no count to publish: no workgroup waits for the others); the sender's post
// clears its own areas back to -1 once the exchange has left.
// Capacity overflows set err bit 1 (the generation is invalid; the engine raises on every
// rank), tag or range mismatches set err bit 4.
#include "srnn_kernels.h"

namespace srnn {
namespace {

enum : int { H_CENSUS = 0, H_BORN = 5, H_VALID = 6, H_GEN = 7, H_NREP = 8, H_NATT = 9 };
static_assert(SRNN_X2_HDR == 12, "header words");
constexpr int XT = 256;  // threads per workgroup

struct X2Geom {
  int64_t rb, xb;
  SRNN_HD char* blk(char* base, const SrnnArgs& a, int q) const { return base + (int64_t)q * a.x_blk; }
  SRNN_HD const char* blk(const char* base, const SrnnArgs& a, int q) const { return base + (int64_t)q * a.x_blk; }
  SRNN_HD int64_t* hdr(char* b) const { return reinterpret_cast<int64_t*>(b); }
  SRNN_HD const int64_t* hdr(const char* b) const { return reinterpret_cast<const int64_t*>(b); }
  SRNN_HD char* row(char* b, int64_t pos) const { return b + X2_HB + pos * xb; }
  SRNN_HD int64_t* notice(char* b, const SrnnArgs& a, int64_t k) const {
    return reinterpret_cast<int64_t*>(b + X2_HB + a.x_cr * xb) + 2 * k;
  }
  SRNN_HD const int64_t* notice(const char* b, const SrnnArgs& a, int64_t k) const {
    return reinterpret_cast<const int64_t*>(b + X2_HB + a.x_cr * xb) + 2 * k;
  }
  SRNN_HD int64_t* request(char* b, const SrnnArgs& a, int64_t k) const {
    return reinterpret_cast<int64_t*>(b + X2_HB + a.x_cr * xb + a.x_cn * 16) + k;
  }
  SRNN_HD const int64_t* request(const char* b, const SrnnArgs& a, int64_t k) const {
    return reinterpret_cast<const int64_t*>(b + X2_HB + a.x_cr * xb + a.x_cn * 16) + k;
  }
};
SRNN_HD X2Geom geom(const SrnnCfg& c) {
  X2Geom g;
  g.rb = (int64_t)c.pp * (c.dtype == 0 ? 4 : 2);
  g.xb = x2_xb(g.rb);
  return g;
}

SRNN_HD int32_t gen_of(const SrnnArgs& a) { return a.gen_ptr ? a.gen_ptr[0] : a.gen; }
SRNN_HD int32_t atomic_add(int32_t* p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}
SRNN_HD uint32_t atomic_or_u32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicOr(p, v);
#else
  return __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}
using Dec = Item<Weightwise<1, 1>, StF32>;  // decisions / links are shape independent

// slot i (local row) becomes remote-dependent in the next generation; the first marker
// appends it to the next generation's remote list with its teacher's received row
SRNN_HD void mark_remote(const SrnnArgs& a, int64_t i, uint32_t tk) {
  const uint32_t bit = 1u << (i & 31);
  const uint32_t old = atomic_or_u32(a.x_dep_next + (i >> 5), bit);
  if (old & bit) return;
  const int32_t c = atomic_add(a.x_rcount_next, 1);
  a.x_rlist_next[2 * (int64_t)c] = (uint32_t)i;
  a.x_rlist_next[2 * (int64_t)c + 1] = tk;
}

// timing model of R ranks on one GPU (x_emul, world 1 only): a hashed fraction x_emul / 2^32 of
// the slots goes through the remote list (same results: their rows are local)
SRNN_HD bool emul_hit(int64_t g, int32_t dgen, uint32_t x) {
  uint64_t h = (uint64_t)g * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)dgen * 0xBF58476D1CE4E5B9ull);
  h ^= h >> 31;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 29;
  return (uint32_t)(h >> 32) < x;
}

// What pack decides for one local slot: a local attack to link, a notice or request to append
// for a peer rank, a remote-dependence mark (the teacher's reply row is known only once the
// request has its position).
struct PackDec {
  int64_t g, at, te;
  int32_t qa, qt;   // owner ranks of victim / teacher (-1: none)
  bool mark;        // emulated remote dependence (no teacher row)
};
SRNN_HD PackDec pack_decision(const SrnnArgs& a, int64_t i, int32_t dgen) {
  PackDec d;
  d.g = a.lo + i;
  Dec::decision(a, d.g, dgen, d.at, d.te);
  d.qa = d.at >= 0 ? (a.world > 1 ? shard_of(d.at, a.n_total, a.world) : 0) : -1;
  d.qt = d.te >= 0 ? (a.world > 1 ? shard_of(d.te, a.n_total, a.world) : 0) : -1;
  if (d.qt == a.rank) d.qt = -1;  // a local teacher needs nothing
  d.mark = a.x_emul && a.world == 1 && emul_hit(d.g, dgen, a.x_emul);
  return d;
}
// a notice (slot k of peer q's area) and a request (slot k) once their positions are known
SRNN_HD void put_notice(const SrnnArgs& a, const X2Geom& G, int64_t i, const PackDec& d, int32_t k) {
  if (k < a.x_cn) {
    int64_t* nt = G.notice(G.blk(a.sendbuf, a, d.qa), a, k);
    nt[0] = d.g;
    nt[1] = d.at;
    a.x_satt_next[(int64_t)d.qa * a.x_cn + k] = (uint32_t)i;
  } else {
    err_or(a.err, 1);
  }
}
SRNN_HD bool put_request(const SrnnArgs& a, const X2Geom& G, const PackDec& d, int32_t k) {
  if (k < a.x_cq) {
    *G.request(G.blk(a.sendbuf, a, d.qt), a, k) = d.te;
    return true;
  }
  err_or(a.err, 1);
  return false;
}

// decisions of local row i for the next generation dgen (pack; host form: one slot at a time)
SRNN_HD void pack_decide(const SrnnArgs& a, const X2Geom& G, int64_t i, int32_t dgen) {
  const PackDec d = pack_decision(a, i, dgen);
  if (d.qa == a.rank) Dec::link(a.heads_next, a.nexts_next, d.at - a.lo, (uint32_t)i);
  else if (d.qa >= 0) put_notice(a, G, i, d, atomic_add(a.x_cno_next + d.qa, 1));
  if (d.qt >= 0) {
    const int32_t k = atomic_add(a.x_crq_next + d.qt, 1);
    // the reply comes back as row k of q's block in the next exchange
    if (put_request(a, G, d, k)) mark_remote(a, i, (uint32_t)((int64_t)d.qt * a.x_cr + k));
  }
  if (d.mark) mark_remote(a, i, SRNN_NIL);
}

// row copy idx of the exchange (peer q): replies (k < x_cq) then noticed attackers
SRNN_HD void pack_row(const SrnnArgs& a, const X2Geom& G, int64_t idx, int32_t gen) {
  const int64_t per = a.x_cq + a.x_cn;
  const int q = (int)(idx / per);
  const int64_t k = idx - (int64_t)q * per;
  const int64_t nrep = a.x_nsrep[q];
  int64_t src, pos;
  if (k < a.x_cq) {
    if (k >= nrep) return;
    src = a.x_srep[(int64_t)q * a.x_cq + k];
    pos = k;
  } else {
    const int64_t k2 = k - a.x_cq;
    if (k2 >= a.x_cno[q]) return;
    src = a.x_satt[(int64_t)q * a.x_cn + k2];
    pos = nrep + k2;
  }
  if (pos >= a.x_cr || src < 0 || src >= a.n) {
    err_or(a.err, 1);
    return;
  }
  const char* s = reinterpret_cast<const char*>(a.W2) + src * G.rb;
  char* d = G.row(G.blk(a.sendbuf, a, q), pos);
  const uint2* s2 = reinterpret_cast<const uint2*>(s);
  uint2* d2 = reinterpret_cast<uint2*>(d);
  for (int64_t w = 0; w < G.rb / 8; ++w) d2[w] = s2[w];
  int64_t* tag = reinterpret_cast<int64_t*>(d + G.rb);
  tag[0] = a.lo + src;
  tag[1] = gen;
}

// the header words of every peer block that the finish owns
SRNN_HD void write_stats(const SrnnArgs& a, const X2Geom& G, const int64_t* tot, int32_t gen) {
  for (int q = 0; q < a.world; ++q) {
    int64_t* h = G.hdr(G.blk(a.sendbuf, a, q));
    for (int w = 0; w < 6; ++w) h[w] = tot[w];
    h[H_VALID] = 1;
    h[H_GEN] = gen;
    h[H_NREP] = a.x_nsrep ? a.x_nsrep[q] : 0;
    h[H_NATT] = a.x_cno ? (a.x_cno[q] < a.x_cn ? a.x_cno[q] : a.x_cn) : 0;
  }
}
// stats word w of rank r: the gathered array (flush, all-gather exchange) or the header of
// r's block in the exchange just received (zeros when not valid)
SRNN_HD int64_t stat_of(const SrnnArgs& a, const X2Geom& G, int r, int w) {
  if (a.stats) return a.stats[r * 6 + w];
  const int64_t* h = G.hdr(G.blk(a.recvbuf, a, r));
  return h[H_VALID] ? h[w] : 0;
}

// received notice k of peer q -> the next generation's list of its victim; this rank's own
// sent notice k to q is cleared back to the sentinel (the exchange has left)
// (returns the victim's local row, which becomes remote-dependent; -1: nothing received)
SRNN_HD int64_t post_notice(const SrnnArgs& a, const X2Geom& G, int q, int64_t k) {
  int64_t* mine = G.notice(G.blk(a.sendbuf, a, q), a, k);
  mine[0] = -1;
  mine[1] = -1;
  const int64_t* nt = G.notice(G.blk(a.recvbuf, a, q), a, k);
  const int64_t aslot = nt[0], v = nt[1];
  if (v < 0) return -1;  // past the last notice
  const int64_t nreq = a.x_crq_next[q] < a.x_cq ? a.x_crq_next[q] : a.x_cq;
  const int64_t pos = nreq + k;  // after the replies to my requests to q
  if (pos >= a.x_cr) {
    err_or(a.err, 1);
    return -1;
  }
  if (v < a.lo || v >= a.lo + a.n) {
    err_or(a.err, 4);
    return -1;
  }
  const int64_t rk = (int64_t)q * a.x_cr + pos;
  a.x_rslot_next[rk] = aslot;
  Dec::link(a.heads_next, a.nexts_next, v - a.lo, (uint32_t)(a.n + rk));
  return v - a.lo;
}
// received request k of peer q -> a row to reply with next generation; the last valid
// request's thread (or thread 0 when there is none) stores the count
SRNN_HD void post_request(const SrnnArgs& a, const X2Geom& G, int q, int64_t k) {
  *G.request(G.blk(a.sendbuf, a, q), a, k) = -1;
  const char* b = G.blk(a.recvbuf, a, q);
  const int64_t te = *G.request(b, a, k);
  if (te < 0) {
    if (k == 0) a.x_nsrep[q] = 0;
    return;
  }
  if (k + 1 == a.x_cq || *G.request(b, a, k + 1) < 0) a.x_nsrep[q] = (int32_t)(k + 1);
  if (te < a.lo || te >= a.lo + a.n) {
    err_or(a.err, 4);
    return;
  }
  a.x_srep[(int64_t)q * a.x_cq + k] = (uint32_t)(te - a.lo);
}

// ============================================================================ device
__device__ __forceinline__ int64_t wg_sum(int64_t v, int64_t* s_red) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t t = 0;
  for (int w = 0; w < XT / 64; ++w) t += s_red[w];
  __syncthreads();
  return t;
}
// one atomic per WORKGROUP on a shared counter (same-address device atomics serialise: a
// generation's thousands of notices / requests / remote marks would queue on a few counters):
// this lane's position among the wanting lanes of the workgroup, -1 when it wants none.  Every
// thread of the workgroup calls it (two barriers); s: XT / 64 + 1 ints of LDS
__device__ __forceinline__ int32_t block_reserve(int32_t* ctr, bool want, int32_t* s) {
  const unsigned long long m = __ballot(want);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s[wv] = (int32_t)__popcll(m);
  __syncthreads();
  int32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < XT / 64; ++w) {
    pre += w < wv ? s[w] : 0;
    tot += s[w];
  }
  if (threadIdx.x == 0 && tot) s[XT / 64] = atomicAdd(ctr, tot);
  __syncthreads();
  const int32_t base = s[XT / 64];
  __syncthreads();  // s is reused by the next call
  return want ? base + pre + (int32_t)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}
// mark_remote with the list positions reserved once per workgroup (every thread calls it)
__device__ __forceinline__ void mark_remote_block(const SrnnArgs& a, int64_t i, uint32_t tk, bool want, int32_t* s) {
  bool first = false;
  if (want) {
    const uint32_t bit = 1u << (i & 31);
    first = !(atomicOr(a.x_dep_next + (i >> 5), bit) & bit);
  }
  const int32_t c = block_reserve(a.x_rcount_next, first, s);
  if (first) {
    a.x_rlist_next[2 * (int64_t)c] = (uint32_t)i;
    a.x_rlist_next[2 * (int64_t)c + 1] = tk;
  }
}
// pack_decide for a whole workgroup: notice / request / list positions reserved per workgroup
// and peer
__device__ void pack_decide_block(const SrnnArgs& a, const X2Geom& G, int64_t i, bool on, int32_t dgen, int32_t* s) {
  PackDec d;
  d.qa = d.qt = -1;
  d.mark = false;
  if (on) d = pack_decision(a, i, dgen);
  if (d.qa == a.rank) Dec::link(a.heads_next, a.nexts_next, d.at - a.lo, (uint32_t)i);
  const bool notice = d.qa >= 0 && d.qa != a.rank, request = d.qt >= 0;
  int32_t kn = -1, kq = -1;
  if (a.world <= 16) {
    for (int q = 0; q < a.world; ++q) {
      if (q == a.rank) continue;
      const int32_t r1 = block_reserve(a.x_cno_next + q, notice && d.qa == q, s);
      const int32_t r2 = block_reserve(a.x_crq_next + q, request && d.qt == q, s);
      kn = r1 >= 0 ? r1 : kn;
      kq = r2 >= 0 ? r2 : kq;
    }
  } else {
    if (notice) kn = atomicAdd(a.x_cno_next + d.qa, 1);
    if (request) kq = atomicAdd(a.x_crq_next + d.qt, 1);
  }
  if (notice) put_notice(a, G, i, d, kn);
  bool mark = d.mark;  // (emulated marks exist at world 1 only, where there are no requests)
  uint32_t tk = SRNN_NIL;
  if (request && put_request(a, G, d, kq)) {
    mark = true;
    tk = (uint32_t)((int64_t)d.qt * a.x_cr + kq);  // the reply: row kq of q's next block
  }
  mark_remote_block(a, i, tk, mark, s);
}

// block range of finish / uid workgroup g (the same split in pack and post)
SRNN_HD void wg_range(const SrnnArgs& a, int64_t g, int64_t& b0, int64_t& b1) {
  const int64_t nb = (a.n + 63) / 64, per = (nb + a.x_groups - 1) / a.x_groups;
  b0 = g * per < nb ? g * per : nb;
  b1 = b0 + per < nb ? b0 + per : nb;
}

__global__ __launch_bounds__(XT) void k_x2_pack(SrnnCfg c, SrnnArgs a) {
  if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
  const X2Geom G = geom(c);
  const int32_t gen = gen_of(a);
  const bool prime = (a.flags & SRNN_F_X2_PRIME) != 0, fin_only = (a.flags & SRNN_F_X2_FINISH_ONLY) != 0;
  const int64_t nd = fin_only ? 0 : (a.n + XT - 1) / XT;
  __shared__ int64_t s_red[XT / 64];
  __shared__ int32_t s_last;
  __shared__ int32_t s_hw[XT / 64];
  if ((int64_t)blockIdx.x < a.x_groups) {
    // ---- finish of generation t-1: this workgroup's blocks -> partial (born, census)
    int64_t b0, b1;
    wg_range(a, blockIdx.x, b0, b1);
    const unsigned long long* bs = reinterpret_cast<const unsigned long long*>(a.temp);
    int64_t v[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t b = b0 + threadIdx.x; b < b1; b += XT) {
      const unsigned long long* st = bs + b * 4;
      v[0] += __popcll(st[0]);
      v[1] += (uint32_t)st[1];
      v[2] += (uint32_t)(st[1] >> 32);
      v[3] += (uint32_t)st[2];
      v[4] += (uint32_t)(st[2] >> 32);
      v[5] += (uint32_t)st[3];
    }
    for (int w = 0; w < 6; ++w) v[w] = wg_sum(v[w], s_red);
    if (a.x_hpre) {
      // remote-dependent slots (holes) per 64-row block of THIS generation (bits final since
      // pack / post of the last one): exclusive prefix inside the workgroup's range -> x_hpre,
      // its total -> x_hgrp (scanned by the last workgroup); the single-launch evolve's waves
      // map their holes onto the remote list with them
      const int64_t nw = (a.n + 31) / 32;
      int32_t carry = 0;
      for (int64_t c0 = b0; c0 < b1; c0 += XT) {
        const int64_t b = c0 + threadIdx.x;
        int32_t h = 0;
        if (b < b1) h = __popc(a.x_dep[2 * b]) + (2 * b + 1 < nw ? __popc(a.x_dep[2 * b + 1]) : 0);
        int32_t tot;
        const int32_t incl = block_incl_scan<XT, int32_t>(h, s_hw, &tot);
        if (b < b1) a.x_hpre[b] = carry + incl - h;
        carry += tot;
        __syncthreads();
      }
      if (threadIdx.x == 0) __hip_atomic_store(a.x_hgrp + blockIdx.x, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
      // partials leave L2 at once (sc1 stores: other XCDs read them), drained before the ticket
      for (int w = 0; w < 6; ++w)
        __hip_atomic_store(a.x_part + blockIdx.x * 6 + w, v[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_last = atomicAdd(a.x_ctl + 0, 1) == a.x_groups - 1;
    }
    __syncthreads();
    if (!s_last) return;
    // the last workgroup sums every workgroup's partials: one device-scope load round trip per
    // thread (a serial walk by one thread costs one round trip per workgroup)
    int64_t pv[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t g = threadIdx.x; g < a.x_groups; g += XT)
      for (int w = 0; w < 6; ++w) pv[w] += __hip_atomic_load(a.x_part + g * 6 + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int w = 0; w < 6; ++w) pv[w] = wg_sum(pv[w], s_red);
    if (a.x_hpre) {  // exclusive prefix of the workgroups' hole totals, in place
      int32_t carry = 0;
      for (int64_t c0 = 0; c0 < a.x_groups; c0 += XT) {
        const int64_t g = c0 + threadIdx.x;
        const int32_t h =
            g < a.x_groups ? __hip_atomic_load(a.x_hgrp + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        int32_t tot;
        const int32_t incl = block_incl_scan<XT, int32_t>(h, s_hw, &tot);
        if (g < a.x_groups) a.x_hgrp[g] = carry + incl - h;
        carry += tot;
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) {
      int64_t tot[6];  // census[5], born
      tot[5] = pv[0];
      for (int w = 0; w < 5; ++w) tot[w] = pv[1 + w];
      if (a.counts) {  // census accumulated by a classify launch (nets without a fused census)
        for (int w = 0; w < 5; ++w) tot[w] += (int64_t)a.counts[w];
        for (int w = 0; w < 6; ++w) a.counts[w] = 0;
      }
      write_stats(a, G, tot, gen);
      a.x_ctl[0] = 0;
    }
    return;
  }
  if ((int64_t)blockIdx.x < a.x_groups + nd) {
    // ---- decisions of the next generation (PRIME: of this one) for the local slots
    const int64_t i = ((int64_t)blockIdx.x - a.x_groups) * XT + threadIdx.x;
    __shared__ int32_t s_res[XT / 64 + 1];
    pack_decide_block(a, G, i, i < a.n, prime ? gen : gen + 1, s_res);
    return;
  }
  // ---- rows of this generation's exchange
  const int64_t idx = ((int64_t)blockIdx.x - a.x_groups - nd) * XT + threadIdx.x;
  if (idx < (int64_t)a.world * (a.x_cq + a.x_cn)) pack_row(a, G, idx, gen);
}

__global__ __launch_bounds__(XT) void k_x2_post(SrnnCfg c, SrnnArgs a) {
  if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
  const X2Geom G = geom(c);
  const bool fin_only = (a.flags & SRNN_F_X2_FINISH_ONLY) != 0;
  __shared__ int64_t s_pre, s_tot, s_base;
  if ((int64_t)blockIdx.x < a.x_groups) {
    // ---- uids of generation t-1's newborns, in slot order across ranks and workgroups
    if (threadIdx.x == 0) {
      int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
      for (int r = 0; r < a.world; ++r) {
        const int64_t k = stat_of(a, G, r, 5);
        if (r < a.rank) pre += k;
        tot += k;
        for (int w = 0; w < 5; ++w) cen[w] += stat_of(a, G, r, w);
      }
      for (int w = 0; w < 5; ++w) all += cen[w];
      if (blockIdx.x == 0 && a.census && all > 0)
        for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
      for (int64_t g = 0; g < (int64_t)blockIdx.x; ++g) pre += a.x_part[g * 6];
      s_pre = pre;
      s_tot = tot;
      s_base = *(volatile const int64_t*)a.uid_base;
      if (blockIdx.x == 0 && !fin_only) {  // this generation's notice / request counters are spent
        for (int q = 0; q < a.world; ++q) a.x_cno[q] = 0, a.x_crq[q] = 0;
        // the generation counter of the next generation (the other ring slot: nothing of
        // this generation reads it)
        if (!(a.flags & SRNN_F_X2_PRIME)) Dec::set_gen(a, gen_of(a) + 1);
      }
    }
    __syncthreads();
    int64_t b0, b1;
    wg_range(a, blockIdx.x, b0, b1);
    const int64_t ch = (b1 - b0 + XT - 1) / XT;
    const int64_t t0 = b0 + threadIdx.x * ch < b1 ? b0 + threadIdx.x * ch : b1;
    const int64_t t1 = t0 + ch < b1 ? t0 + ch : b1;
    unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
    int64_t cnt = 0;
    for (int64_t b = t0; b < t1; ++b) cnt += __popcll(bs[b * 4]);
    int64_t wave_tot;
    __shared__ int64_t s_wave[XT / 64];
    const int64_t incl = block_incl_scan<XT, int64_t>(cnt, s_wave, &wave_tot);
    int64_t u = s_base + s_pre + incl - cnt;
    for (int64_t b = t0; b < t1; ++b) {
      unsigned long long m = bs[b * 4];
      while (m) {
        const int bit = __ffsll((long long)m) - 1;
        m &= m - 1;
        a.uid_out[b * 64 + bit] = u++;
      }
      bs[b * 4] = 0ull;  // the block stats are free for generation t+1
      bs[b * 4 + 1] = 0ull;
      bs[b * 4 + 2] = 0ull;
      bs[b * 4 + 3] = 0ull;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // every workgroup read next_uid before its ticket: the last one may overwrite it
      if (atomicAdd(a.x_ctl + 2, 1) == a.x_groups - 1) {
        a.uid_base[0] = s_base + s_tot;
        a.x_ctl[2] = 0;
      }
    }
    return;
  }
  if (fin_only) return;
  const int64_t nn = ((int64_t)a.world * a.x_cn + XT - 1) / XT;
  if ((int64_t)blockIdx.x < a.x_groups + nn) {
    const int64_t idx = ((int64_t)blockIdx.x - a.x_groups) * XT + threadIdx.x;
    const int64_t v = idx < (int64_t)a.world * a.x_cn ? post_notice(a, G, (int)(idx / a.x_cn), idx % a.x_cn) : -1;
    __shared__ int32_t s_res[XT / 64 + 1];
    mark_remote_block(a, v, SRNN_NIL, v >= 0, s_res);
    return;
  }
  const int64_t idx = ((int64_t)blockIdx.x - a.x_groups - nn) * XT + threadIdx.x;
  if (idx < (int64_t)a.world * a.x_cq) post_request(a, G, (int)(idx / a.x_cq), idx % a.x_cq);
}

// ============================================================================ host
void host_pack(const SrnnCfg& c, const SrnnArgs& a) {
  const X2Geom G = geom(c);
  const int32_t gen = gen_of(a);
  const bool prime = (a.flags & SRNN_F_X2_PRIME) != 0;
  const unsigned long long* bs = reinterpret_cast<const unsigned long long*>(a.temp);
  int64_t tot[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t g = 0; g < a.x_groups; ++g) {
    int64_t b0, b1, v[6] = {0, 0, 0, 0, 0, 0};
    wg_range(a, g, b0, b1);
    for (int64_t b = b0; b < b1; ++b) {
      const unsigned long long* st = bs + b * 4;
      v[0] += __builtin_popcountll(st[0]);
      v[1] += (uint32_t)st[1];
      v[2] += (uint32_t)(st[1] >> 32);
      v[3] += (uint32_t)st[2];
      v[4] += (uint32_t)(st[2] >> 32);
      v[5] += (uint32_t)st[3];
    }
    for (int w = 0; w < 6; ++w) a.x_part[g * 6 + w] = v[w];
    tot[5] += v[0];
    for (int w = 0; w < 5; ++w) tot[w] += v[1 + w];
  }
  if (a.counts) {
    for (int w = 0; w < 5; ++w) tot[w] += (int64_t)a.counts[w];
    for (int w = 0; w < 6; ++w) a.counts[w] = 0;
  }
  write_stats(a, G, tot, gen);
  if (a.flags & SRNN_F_X2_FINISH_ONLY) return;
  for (int64_t i = 0; i < a.n; ++i) pack_decide(a, G, i, prime ? gen : gen + 1);
  const int64_t rows = (int64_t)a.world * (a.x_cq + a.x_cn);
  for (int64_t idx = 0; idx < rows; ++idx) pack_row(a, G, idx, gen);
}

void host_post(const SrnnCfg& c, const SrnnArgs& a) {
  const X2Geom G = geom(c);
  int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
  for (int r = 0; r < a.world; ++r) {
    const int64_t k = stat_of(a, G, r, 5);
    if (r < a.rank) pre += k;
    tot += k;
    for (int w = 0; w < 5; ++w) cen[w] += stat_of(a, G, r, w);
  }
  for (int w = 0; w < 5; ++w) all += cen[w];
  if (a.census && all > 0)
    for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
  unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
  int64_t u = a.uid_base[0] + pre;
  const int64_t nb = (a.n + 63) / 64;
  for (int64_t b = 0; b < nb; ++b) {
    unsigned long long m = bs[b * 4];
    while (m) {
      const int bit = __builtin_ctzll(m);
      m &= m - 1;
      a.uid_out[b * 64 + bit] = u++;
    }
    for (int w = 0; w < 4; ++w) bs[b * 4 + w] = 0ull;
  }
  a.uid_base[0] += tot;
  if (a.flags & SRNN_F_X2_FINISH_ONLY) return;
  for (int q = 0; q < a.world; ++q) a.x_cno[q] = 0, a.x_crq[q] = 0;
  if (!(a.flags & SRNN_F_X2_PRIME)) Dec::set_gen(a, gen_of(a) + 1);
  for (int q = 0; q < a.world; ++q)
    for (int64_t k = 0; k < a.x_cn; ++k) {
      const int64_t v = post_notice(a, G, q, k);
      if (v >= 0) mark_remote(a, v, SRNN_NIL);
    }
  for (int q = 0; q < a.world; ++q)
    for (int64_t k = 0; k < a.x_cq; ++k) post_request(a, G, q, k);
}

// uids of the previous generation's newborns for the all-gather exchange: per-rank stats
// in a.stats ([world][6]), per-row respawn flags (rowflags, consumed)
void host_uid_assign(const SrnnArgs& a) {
  int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
  for (int r = 0; r < a.world; ++r) {
    const int64_t k = a.stats[r * 6 + 5];
    if (r < a.rank) pre += k;
    tot += k;
    for (int w = 0; w < 5; ++w) cen[w] += a.stats[r * 6 + w];
  }
  for (int w = 0; w < 5; ++w) all += cen[w];
  if (a.census && all > 0)
    for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
  int64_t k = a.uid_base[0] + pre;
  for (int64_t i = 0; i < a.n; ++i)
    if (a.rowflags[i]) {
      a.uid_out[i] = k++;
      a.rowflags[i] = 0;
    }
  a.uid_base[0] += tot;
  if (a.counts)
    for (int w = 0; w < 6; ++w) a.counts[w] = 0;
}
constexpr int TBU = 1024;
__global__ __launch_bounds__(TBU) void k_uid_assign(SrnnArgs a) {
  __shared__ int32_t s_wave[TBU / 64];
  __shared__ int64_t s_prefix, s_total;
  if (threadIdx.x == 0) {
    int64_t pre = 0, tot = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
    for (int r = 0; r < a.world; ++r) {
      const int64_t k = a.stats[r * 6 + 5];
      if (r < a.rank) pre += k;
      tot += k;
      for (int w = 0; w < 5; ++w) cen[w] += a.stats[r * 6 + w];
    }
    for (int w = 0; w < 5; ++w) all += cen[w];
    s_prefix = pre;
    s_total = tot;
    if (a.census && all > 0)
      for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
  }
  // per-row flags: thread t walks rows [t*ch, (t+1)*ch)
  const int64_t ch = (a.n + TBU - 1) / TBU;
  const int64_t r0 = (int64_t)threadIdx.x * ch < a.n ? (int64_t)threadIdx.x * ch : a.n;
  const int64_t r1 = r0 + ch < a.n ? r0 + ch : a.n;
  int32_t cnt = 0;
  for (int64_t i = r0; i < r1; ++i) cnt += a.rowflags[i] != 0;
  int32_t total_local;
  const int32_t incl = block_incl_scan<TBU>(cnt, s_wave, &total_local);  // barrier inside
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t k = base + s_prefix + incl - cnt;
  for (int64_t i = r0; i < r1 && cnt; ++i)
    if (a.rowflags[i]) {
      a.uid_out[i] = k++;
      a.rowflags[i] = 0;
    }
  __syncthreads();
  if (threadIdx.x == 0) a.uid_base[0] = base + s_total;
  if (a.counts && threadIdx.x < 6) a.counts[threadIdx.x] = 0;
}

int check(hipError_t e) {
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

}  // namespace
}  // namespace srnn

// OP_X2_PACK / OP_X2_POST / OP_UID_ASSIGN: shape independent (row bytes from the config)
extern "C" int srnn_x2_run(int op, const SrnnCfg* c, const SrnnArgs* a) {
  using namespace srnn;
  if (op == OP_UID_ASSIGN) {
    if (!a->stats || !a->rowflags || !a->uid_out || !a->uid_base) {
      set_error("uid assignment needs stats, rowflags, uid_out and uid_base");
      return -5;
    }
    if (!a->dev) {
      host_uid_assign(*a);
      return 0;
    }
    hipLaunchKernelGGL(k_uid_assign, dim3(1), dim3(TBU), 0, (hipStream_t)a->stream, *a);
    return check(hipGetLastError());
  }
  if (a->world < 1 || a->world > 1024 || a->x_groups < 1 || a->x_cr < 1 || a->x_blk < X2_HB || !a->sendbuf ||
      !a->x_part || !a->x_ctl || !a->temp || !a->uid_base) {
    set_error("X2 exchange: world, x_groups, capacities, buffers, partials, tickets and block stats needed");
    return -5;
  }
  const X2Geom G = geom(*c);
  if (a->x_blk < X2_HB + a->x_cr * G.xb + a->x_cn * 16 + a->x_cq * 8) {
    set_error("X2 exchange: x_blk smaller than header + rows + notices + requests");
    return -5;
  }
  if (a->n + (int64_t)a->world * a->x_cr >= (int64_t)SRNN_NIL) {
    set_error("X2 exchange: local rows + received rows must stay below 2^32 - 1 list entries");
    return -5;
  }
  const bool fin_only = (a->flags & SRNN_F_X2_FINISH_ONLY) != 0;
  if (op == OP_X2_PACK) {
    if (!fin_only && (!a->x_cno_next || !a->x_crq_next || !a->x_satt_next || !a->heads_next || !a->nexts_next ||
                      !a->x_dep_next || !a->x_rlist_next || !a->x_rcount_next || !a->x_nsrep || !a->x_srep ||
                      !a->x_cno || !a->x_satt || !a->W2)) {
      set_error("X2 pack: next-generation lists / counters and this generation's send lists needed");
      return -5;
    }
    if (!a->dev) {
      host_pack(*c, *a);
      return 0;
    }
    const int64_t nd = fin_only ? 0 : (a->n + XT - 1) / XT;
    const bool prime = (a->flags & SRNN_F_X2_PRIME) != 0;
    const int64_t nr = (fin_only || prime) ? 0 : ((int64_t)a->world * (a->x_cq + a->x_cn) + XT - 1) / XT;
    const int64_t grid = a->x_groups + nd + nr;
    if (grid > 0x7fffffffLL) {
      set_error("grid too large");
      return -2;
    }
    hipLaunchKernelGGL(k_x2_pack, dim3((unsigned)grid), dim3(XT), 0, (hipStream_t)a->stream, *c, *a);
    return check(hipGetLastError());
  }
  if (op == OP_X2_POST) {
    if (!a->recvbuf && !a->stats) {
      set_error("X2 post: the received exchange (or gathered stats) needed");
      return -5;
    }
    if (!fin_only && (!a->x_crq_next || !a->x_rslot_next || !a->heads_next || !a->nexts_next || !a->x_dep_next ||
                      !a->x_rlist_next || !a->x_rcount_next || !a->x_nsrep || !a->x_srep || !a->x_cno || !a->x_crq)) {
      set_error("X2 post: next-generation lists and request buffers needed");
      return -5;
    }
    if (!a->dev) {
      host_post(*c, *a);
      return 0;
    }
    const int64_t nn = fin_only ? 0 : ((int64_t)a->world * a->x_cn + XT - 1) / XT;
    const int64_t nq = fin_only ? 0 : ((int64_t)a->world * a->x_cq + XT - 1) / XT;
    hipLaunchKernelGGL(k_x2_post, dim3((unsigned)(a->x_groups + nn + nq)), dim3(XT), 0, (hipStream_t)a->stream, *c,
                       *a);
    return check(hipGetLastError());
  }
  set_error("srnn_x2_run: unknown op");
  return -1;
}
