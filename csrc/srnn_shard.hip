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

using namespace x2;

// The finish of generation t-1 in ONE workgroup (no ticket, no second pass): its block stats
// (popcount of the respawn ballots, class counts) -> this rank's totals in every peer's header,
// the newborns per finish group -> x_part[g * 6] (post's uid workgroups start from them), and
// the remote-dependent slots of THIS generation per 64-row block (x_dep bits, final since the
// last post) -> x_hpre[b] = holes before block b, x_hgrp = 0 (the single-launch evolve's waves
// map their holes onto the remote list with x_hpre[b] + x_hgrp[g]).  One load round trip, LDS
// reductions, stores: the ticketed form (x_groups workgroups, partials through memory, a last
// workgroup summing them) was a chain of ~7 dependent memory round trips, ~9.6 us per
// generation on the sharded critical path (profiles/r5e_*).
constexpr int X2_MAX_GROUPS = 1024;
__device__ void pack_finish_wg(const SrnnArgs& a, const X2Geom& G, int32_t gen) {
  __shared__ int64_t s_red[XT / 64][6];
  __shared__ int32_t s_hw[XT / 64];
  __shared__ int32_t s_born[X2_MAX_GROUPS];
  const int t = threadIdx.x;
  for (int64_t g = t; g < a.x_groups; g += XT) s_born[g] = 0;
  int64_t v[6] = {0, 0, 0, 0, 0, 0};  // born, census[5]
  if (a.counts && t == 0) {
    // census accumulated by a classify launch (nets without a fused census): read and cleared
    // by this thread alone, before anything waits
    for (int w = 0; w < 5; ++w) v[1 + w] = (int64_t)a.counts[w];
    for (int w = 0; w < 6; ++w) a.counts[w] = 0;
  }
  __syncthreads();
  const unsigned long long* bs = reinterpret_cast<const unsigned long long*>(a.temp);
  const int64_t nb = (a.n + 63) / 64, per = (nb + a.x_groups - 1) / a.x_groups, nw = (a.n + 31) / 32;
  int32_t carry = 0;
  for (int64_t c0 = 0; c0 < nb; c0 += XT) {
    const int64_t b = c0 + t;
    int32_t h = 0;
    if (b < nb) {
      const unsigned long long* st = bs + b * 4;
      const unsigned long long m = st[0], c01 = st[1], c23 = st[2], c4 = st[3];
      if (a.x_hpre) h = __popc(a.x_dep[2 * b]) + (2 * b + 1 < nw ? __popc(a.x_dep[2 * b + 1]) : 0);
      const int32_t born = __popcll(m);
      v[0] += born;
      v[1] += (uint32_t)c01;
      v[2] += (uint32_t)(c01 >> 32);
      v[3] += (uint32_t)c23;
      v[4] += (uint32_t)(c23 >> 32);
      v[5] += (uint32_t)c4;
      if (born) atomicAdd(&s_born[b / per], born);
    }
    if (a.x_hpre) {
      int32_t tot;
      const int32_t incl = block_incl_scan<XT, int32_t>(h, s_hw, &tot);
      if (b < nb) a.x_hpre[b] = carry + incl - h;
      carry += tot;
      __syncthreads();  // s_hw is reused by the next chunk
    }
  }
  // the six totals in one exchange (wave shuffles, one barrier; s_born complete after it too)
#pragma unroll
  for (int w = 0; w < 6; ++w)
    for (int off = 32; off > 0; off >>= 1) v[w] += __shfl_xor(v[w], off);
  if ((t & 63) == 0)
    for (int w = 0; w < 6; ++w) s_red[t >> 6][w] = v[w];
  __syncthreads();
  int64_t tot[6] = {0, 0, 0, 0, 0, 0};  // census[5], born
  for (int q = 0; q < XT / 64; ++q) {
    tot[5] += s_red[q][0];
    for (int w = 0; w < 5; ++w) tot[w] += s_red[q][1 + w];
  }
  for (int64_t g = t; g < a.x_groups; g += XT) {
    a.x_part[g * 6] = s_born[g];
    if (a.x_hpre) a.x_hgrp[g] = 0;
  }
  for (int q = t; q < a.world; q += XT) write_stats_peer(a, G, q, tot, gen);
}

__global__ __launch_bounds__(XT) void k_x2_pack(SrnnCfg c, SrnnArgs a) {
  if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
  const X2Geom G = geom(c);
  const int32_t gen = gen_of(a);
  const bool prime = (a.flags & SRNN_F_X2_PRIME) != 0, fin_only = (a.flags & SRNN_F_X2_FINISH_ONLY) != 0;
  const int64_t nd = fin_only ? 0 : (a.n + XT - 1) / XT;
  const int64_t nr = (fin_only || prime) ? 0 : ((int64_t)a.world * (a.x_cq + a.x_cn) + XT - 1) / XT;
  if (blockIdx.x == 0) {  // ---- finish of generation t-1
    pack_finish_wg(a, G, gen);
    return;
  }
  const int64_t blk = (int64_t)blockIdx.x - 1;
  if (blk < nd) {
    // ---- decisions of the next generation (PRIME: of this one) for the local slots
    const int64_t i = blk * XT + threadIdx.x;
    __shared__ int32_t s_res[XT / 64 + 1];
    pack_decide_block(a, G, i, i < a.n, prime ? gen : gen + 1, s_res);
    return;
  }
  if (blk < nd + nr) {  // ---- rows of this generation's exchange
    const int64_t idx = (blk - nd) * XT + threadIdx.x;
    if (idx < (int64_t)a.world * (a.x_cq + a.x_cn)) pack_row(a, G, idx, gen);
    return;
  }
  // ---- this generation's SGD epoch permutations (SrnnArgs::ptab, nibble Weightwise nets):
  // the table launch of the generation kernel folded into pack (pack_ptab_blocks)
  const int64_t tb = (a.n + XT - 1) / XT, q = blk - nd - nr, p = q / tb;
  const int64_t row = (q - p * tb) * XT + threadIdx.x;
  if (row < a.n) perm_table_entry(a, c.p, row, (int32_t)p, gen, (a.severity > 0 ? a.severity : 0) + (a.epochs > 0 ? a.epochs : 0));
}

__global__ __launch_bounds__(XT) void k_x2_post(SrnnCfg c, SrnnArgs a) {
  if (a.flags & SRNN_F_X2_PRIO) __builtin_amdgcn_s_setprio(3);
  post_block<XT>(geom(c), a, reinterpret_cast<unsigned long long*>(a.temp), blockIdx.x);
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
  // per-row flags in tiles of TBU * UR rows: thread t takes rows [tile + t*UR, +UR) (the wave's
  // loads cover consecutive memory), one block scan per tile numbers them in slot order (the
  // per-thread walk of n / TBU rows took 61 us at 100k rows, profiles/r5e_*)
  constexpr int UR = 8;
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  int64_t k = base;  // (s_prefix added after the first scan's barrier)
  bool first = true;
  for (int64_t t0 = 0; t0 < a.n; t0 += (int64_t)TBU * UR) {
    const int64_t r0 = t0 + (int64_t)threadIdx.x * UR;
    int32_t f[UR];
    int32_t cnt = 0;
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      f[u] = r0 + u < a.n ? a.rowflags[r0 + u] : 0;
      cnt += f[u] != 0;
    }
    int32_t tile_total;
    const int32_t incl = block_incl_scan<TBU>(cnt, s_wave, &tile_total);  // barrier inside
    if (first) k += s_prefix, first = false;
    int64_t u0 = k + incl - cnt;
#pragma unroll
    for (int u = 0; u < UR; ++u)
      if (f[u]) {
        a.uid_out[r0 + u] = u0++;
        a.rowflags[r0 + u] = 0;
      }
    k += tile_total;
    __syncthreads();  // s_wave is reused by the next tile
  }
  __syncthreads();
  if (threadIdx.x == 0) a.uid_base[0] = base + s_total;
  if (a.counts && threadIdx.x < 6) a.counts[threadIdx.x] = 0;
}

// The same assignment over the whole grid in two launches (SrnnArgs::temp: int32 count per
// UCH-row chunk, then int64 this rank's first uid): chunk counts (workgroup 0 also takes the
// census and the rank's uid base and advances next_uid), then every chunk numbers its flagged
// rows after the prefix of the chunks before it.  The one-workgroup form walks n rows in
// sequence (60 us at 100k rows, profiles/r5q_*).
constexpr int UCH = 4 * TBU;
SRNN_HD int64_t uid_chunks(int64_t n) { return (n + UCH - 1) / UCH; }
SRNN_HD int64_t uid_temp_bytes(int64_t n) { return ((uid_chunks(n) * 4 + 7) / 8) * 8 + 8; }
__device__ __forceinline__ int64_t* uid_first(const SrnnArgs& a) {
  return reinterpret_cast<int64_t*>(reinterpret_cast<char*>(a.temp) + ((uid_chunks(a.n) * 4 + 7) / 8) * 8);
}
__device__ __forceinline__ int32_t block_sum_tbu(int32_t v, int32_t* s_wave) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = v;
  __syncthreads();
  int32_t t = 0;
  for (int w = 0; w < TBU / 64; ++w) t += s_wave[w];
  return t;
}
__global__ __launch_bounds__(TBU) void k_uid_count(SrnnArgs a) {
  __shared__ int32_t s_wave[TBU / 64];
  const int64_t r0 = (int64_t)blockIdx.x * UCH + (int64_t)threadIdx.x * 4;
  int32_t c = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) c += (r0 + u < a.n && a.rowflags[r0 + u] != 0) ? 1 : 0;
  const int32_t tot = block_sum_tbu(c, s_wave);
  if (threadIdx.x == 0) reinterpret_cast<int32_t*>(a.temp)[blockIdx.x] = tot;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int64_t pre = 0, all_born = 0, cen[5] = {0, 0, 0, 0, 0}, all = 0;
    for (int r = 0; r < a.world; ++r) {
      const int64_t k = a.stats[r * 6 + 5];
      if (r < a.rank) pre += k;
      all_born += k;
      for (int w = 0; w < 5; ++w) cen[w] += a.stats[r * 6 + w];
    }
    for (int w = 0; w < 5; ++w) all += cen[w];
    if (a.census && all > 0)
      for (int w = 0; w < 5; ++w) a.census[w] = cen[w];
    const int64_t base = a.uid_base[0];
    *uid_first(a) = base + pre;
    a.uid_base[0] = base + all_born;
    if (a.counts)
      for (int w = 0; w < 6; ++w) a.counts[w] = 0;
  }
}
__global__ __launch_bounds__(TBU) void k_uid_write(SrnnArgs a) {
  __shared__ int32_t s_wave[TBU / 64];
  const int32_t* cnt = reinterpret_cast<const int32_t*>(a.temp);
  int32_t p = 0;  // flagged rows of the chunks before this one
  for (int64_t j = threadIdx.x; j < (int64_t)blockIdx.x; j += TBU) p += cnt[j];
  const int64_t before = block_sum_tbu(p, s_wave);
  __syncthreads();  // s_wave is reused by the scan
  const int64_t r0 = (int64_t)blockIdx.x * UCH + (int64_t)threadIdx.x * 4;
  int32_t f[4], c = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f[u] = r0 + u < a.n ? a.rowflags[r0 + u] : 0;
    c += f[u] != 0;
  }
  int32_t tot;
  const int32_t incl = block_incl_scan<TBU>(c, s_wave, &tot);
  int64_t k = *uid_first(a) + before + incl - c;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (f[u]) {
      a.uid_out[r0 + u] = k++;
      a.rowflags[r0 + u] = 0;
    }
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
    if (a->temp && a->temp_bytes >= uid_temp_bytes(a->n) && a->n > UCH) {  // the grid-wide form
      const unsigned g = (unsigned)uid_chunks(a->n);
      hipLaunchKernelGGL(k_uid_count, dim3(g), dim3(TBU), 0, (hipStream_t)a->stream, *a);
      hipLaunchKernelGGL(k_uid_write, dim3(g), dim3(TBU), 0, (hipStream_t)a->stream, *a);
      return check(hipGetLastError());
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
    if (a->x_groups > X2_MAX_GROUPS) {
      set_error("X2 pack: at most 1024 finish groups");
      return -5;
    }
    const int64_t nd = fin_only ? 0 : (a->n + XT - 1) / XT;
    const bool prime = (a->flags & SRNN_F_X2_PRIME) != 0;
    const int64_t nr = (fin_only || prime) ? 0 : ((int64_t)a->world * (a->x_cq + a->x_cn) + XT - 1) / XT;
    const int64_t grid = 1 + nd + nr + ((fin_only || prime) ? 0 : pack_ptab_blocks(*c, *a, XT));
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
