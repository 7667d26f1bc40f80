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
