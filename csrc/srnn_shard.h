// srnn_shard.h -- the sharded soup's exchange protocol: geometry of an exchange block and the
// per-slot / per-row steps of pack and post (csrc/srnn_shard.hip has the kernels and the host
// path).  A fragment included INSIDE namespace srnn by srnn_kernels.h, after Item<>: the
// single-launch X2 evolve (SRNN_F_X2_POST_FUSED) runs post's workgroups itself.
#pragma once

namespace x2 {
enum : int { H_CENSUS = 0, H_BORN = 5, H_VALID = 6, H_GEN = 7, H_NREP = 8, H_NATT = 9 };
static_assert(SRNN_X2_HDR == 12, "header words");
constexpr int XT = 256;  // threads per workgroup of pack / post
constexpr int X2_LDS_PEERS = 256;  // ranks whose notice / request positions are reserved in LDS

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

// the header words of peer q's block that the finish owns
SRNN_HD void write_stats_peer(const SrnnArgs& a, const X2Geom& G, int q, const int64_t* tot, int32_t gen) {
  int64_t* h = G.hdr(G.blk(a.sendbuf, a, q));
  for (int w = 0; w < 6; ++w) h[w] = tot[w];
  h[H_VALID] = 1;
  h[H_GEN] = gen;
  h[H_NREP] = a.x_nsrep ? a.x_nsrep[q] : 0;
  h[H_NATT] = a.x_cno ? (a.x_cno[q] < a.x_cn ? a.x_cno[q] : a.x_cn) : 0;
}
SRNN_HD void write_stats(const SrnnArgs& a, const X2Geom& G, const int64_t* tot, int32_t gen) {
  for (int q = 0; q < a.world; ++q) write_stats_peer(a, G, q, tot, gen);
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
template <int NT = XT>
__device__ __forceinline__ int32_t block_reserve(int32_t* ctr, bool want, int32_t* s) {
  const unsigned long long m = __ballot(want);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s[wv] = (int32_t)__popcll(m);
  __syncthreads();
  int32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    pre += w < wv ? s[w] : 0;
    tot += s[w];
  }
  if (threadIdx.x == 0 && tot) s[NT / 64] = atomicAdd(ctr, tot);
  __syncthreads();
  const int32_t base = s[NT / 64];
  __syncthreads();  // s is reused by the next call
  return want ? base + pre + (int32_t)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}
// mark_remote with the list positions reserved once per workgroup (every thread calls it)
template <int NT = XT>
__device__ __forceinline__ void mark_remote_block(const SrnnArgs& a, int64_t i, uint32_t tk, bool want, int32_t* s) {
  bool first = false;
  if (want) {
    const uint32_t bit = 1u << (i & 31);
    first = !(atomicOr(a.x_dep_next + (i >> 5), bit) & bit);
  }
  const int32_t c = block_reserve<NT>(a.x_rcount_next, first, s);
  if (first) {
    a.x_rlist_next[2 * (int64_t)c] = (uint32_t)i;
    a.x_rlist_next[2 * (int64_t)c + 1] = tk;
  }
}
// pack_decide for a whole workgroup: notice / request / list positions reserved per workgroup
// and peer
__device__ __forceinline__ void pack_decide_block(const SrnnArgs& a, const X2Geom& G, int64_t i, bool on, int32_t dgen, int32_t* s) {
  PackDec d;
  d.qa = d.qt = -1;
  d.mark = false;
  if (on) d = pack_decision(a, i, dgen);
  if (d.qa == a.rank) Dec::link(a.heads_next, a.nexts_next, d.at - a.lo, (uint32_t)i);
  const bool notice = d.qa >= 0 && d.qa != a.rank, request = d.qt >= 0;
  int32_t kn = -1, kq = -1;
  if (a.world > 1 && a.world <= X2_LDS_PEERS) {
    // per-peer positions: LDS atomics inside the workgroup, then ONE device atomic per peer and
    // counter (three barriers whatever the rank count)
    __shared__ int32_t s_cn[X2_LDS_PEERS], s_cq[X2_LDS_PEERS];
    for (int q = threadIdx.x; q < a.world; q += XT) s_cn[q] = 0, s_cq[q] = 0;
    __syncthreads();
    const int32_t ln = notice ? atomicAdd(&s_cn[d.qa], 1) : -1;
    const int32_t lq = request ? atomicAdd(&s_cq[d.qt], 1) : -1;
    __syncthreads();
    for (int q = threadIdx.x; q < a.world; q += XT) {
      const int32_t cn = s_cn[q], cq = s_cq[q];
      s_cn[q] = cn ? atomicAdd(a.x_cno_next + q, cn) : 0;
      s_cq[q] = cq ? atomicAdd(a.x_crq_next + q, cq) : 0;
    }
    __syncthreads();
    if (notice) kn = s_cn[d.qa] + ln;
    if (request) kq = s_cq[d.qt] + lq;
  } else if (a.world > 1) {
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

// post of an exchange, workgroup `blk` of NT threads (k_x2_post: NT = XT; the single-launch
// evolve's first workgroups: NT = 64).  Roles by workgroup: x_groups uid workgroups (uids of
// the previous generation's newborns in slot order, its block stats `bs` zeroed), notice
// workgroups, request workgroups.
template <int NT>
SRNN_HD int64_t post_blocks(const SrnnArgs& a) {
  if (a.flags & SRNN_F_X2_FINISH_ONLY) return a.x_groups;
  return a.x_groups + ((int64_t)a.world * a.x_cn + NT - 1) / NT + ((int64_t)a.world * a.x_cq + NT - 1) / NT;
}
template <int NT>
__device__ __forceinline__ void post_block(const X2Geom& G, const SrnnArgs& a, unsigned long long* bs, int64_t blk) {
  const bool fin_only = (a.flags & SRNN_F_X2_FINISH_ONLY) != 0;
  __shared__ int64_t s_pre, s_tot, s_base;
  __shared__ int64_t s_wave[NT / 64];
  __shared__ int32_t s_res[NT / 64 + 1];
  if (blk < a.x_groups) {
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
      if (blk == 0 && a.census && all > 0)
        for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
      for (int64_t g = 0; g < blk; ++g) pre += a.x_part[g * 6];
      s_pre = pre;
      s_tot = tot;
      s_base = *(volatile const int64_t*)a.uid_base;
      if (blk == 0 && !fin_only) {  // this generation's notice / request counters are spent
        for (int q = 0; q < a.world; ++q) a.x_cno[q] = 0, a.x_crq[q] = 0;
        // the generation counter of the next generation (the other ring slot: nothing of
        // this generation reads it)
        if (!(a.flags & SRNN_F_X2_PRIME)) Dec::set_gen(a, gen_of(a) + 1);
      }
    }
    __syncthreads();
    int64_t b0, b1;
    wg_range(a, blk, b0, b1);
    const int64_t ch = (b1 - b0 + NT - 1) / NT;
    const int64_t t0 = b0 + threadIdx.x * ch < b1 ? b0 + threadIdx.x * ch : b1;
    const int64_t t1 = t0 + ch < b1 ? t0 + ch : b1;
    int64_t cnt = 0;
    for (int64_t b = t0; b < t1; ++b) cnt += __popcll(bs[b * 4]);
    int64_t wave_tot;
    const int64_t incl = block_incl_scan<NT, int64_t>(cnt, s_wave, &wave_tot);
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
  const int64_t nn = ((int64_t)a.world * a.x_cn + NT - 1) / NT;
  if (blk < a.x_groups + nn) {
    const int64_t idx = (blk - a.x_groups) * NT + threadIdx.x;
    const int64_t v = idx < (int64_t)a.world * a.x_cn ? post_notice(a, G, (int)(idx / a.x_cn), idx % a.x_cn) : -1;
    mark_remote_block<NT>(a, v, SRNN_NIL, v >= 0, s_res);
    return;
  }
  const int64_t idx = (blk - a.x_groups - nn) * NT + threadIdx.x;
  if (idx < (int64_t)a.world * a.x_cq) post_request(a, G, (int)(idx / a.x_cq), idx % a.x_cq);
}
}  // namespace x2
