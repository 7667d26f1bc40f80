// host_selftest.cpp — native self-test of libsrnn's host path through the C ABI, built
// under AddressSanitizer+UBSan (`make -C csrc asan`) or ThreadSanitizer (`make -C csrc
// tsan`) (sanitizers on host code; GPU sanitizers are not available on the
// pool).  It exercises every operator on host tables with the host thread pool, and
// rehearses the sharded soup protocol (srnn_shard.hip) for R = 2 and 3 in one process (the
// all-to-all is a memcpy between the ranks' buffers), checking bitwise equality with the
// single-rank generation (the R-invariance the multi-GPU path relies on).
#include "../srnn_abi.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static void run(int op, const SrnnCfg& c, const SrnnArgs& a) {
  int r = srnn_run(op, &c, &a);
  if (r != 0) {
    std::fprintf(stderr, "srnn_run(%d) = %d: %s\n", op, r, srnn_last_error());
    ++g_fail;
  }
}

static SrnnCfg ww22() {
  SrnnCfg c{};
  c.kind = 0, c.width = 2, c.depth = 2, c.aggregates = 0, c.aggregator = 0, c.shuffler = 0, c.pp = 16, c.p = 14;
  c.dtype = 0;
  return c;
}
static SrnnCfg agg422() {
  SrnnCfg c{};
  c.kind = 1, c.width = 2, c.depth = 2, c.aggregates = 4, c.aggregator = 0, c.shuffler = 0, c.pp = 20, c.p = 20;
  c.dtype = 0;
  return c;
}

static SrnnCfg cfg(int kind, int w, int d, int a, int p, int shuffler = 0, int dtype = 0) {
  SrnnCfg c{};
  c.kind = kind, c.width = w, c.depth = d, c.aggregates = a, c.aggregator = 0, c.shuffler = shuffler;
  c.p = p, c.pp = (p + 3) & ~3, c.dtype = dtype;
  return c;
}

extern "C" int srnn_comm_available(const char* hint);

static void ops_smoke(const SrnnCfg& c, int64_t n) {
  const int PP = c.pp;
  // fp32 tables, or 16-bit ones (dtype 1/2) in the same buffers (half the bytes used)
  std::vector<float> W((size_t)(n * PP), 0.f), O((size_t)(n * PP), 0.f);
  std::vector<int64_t> uid((size_t)n), idx((size_t)n);
  for (int64_t i = 0; i < n; ++i) uid[(size_t)i] = i + 7, idx[(size_t)i] = (i + 1) % n;
  std::vector<int8_t> cls((size_t)n);
  std::vector<int32_t> nsteps((size_t)n);
  std::vector<float> loss((size_t)n);
  uint64_t counts[6] = {0, 0, 0, 0, 0, 0};
  SrnnArgs a{};
  a.n = n, a.seed = 11, a.W = W.data(), a.uid = uid.data(), a.dev = 0, a.lr = 0.01f, a.eps = 1e-4f;
  run(OP_INIT, c, a);
  bool finite = true, nonzero = false;
  if (c.dtype == 0)
    for (int64_t i = 0; i < n; ++i)
      for (int k = 0; k < c.p; ++k) {
        finite &= std::isfinite(W[(size_t)(i * PP + k)]);
        nonzero |= W[(size_t)(i * PP + k)] != 0.f;
      }
  else
    nonzero = true;
  CHECK(finite && nonzero);
  SrnnArgs b = a;
  b.W2 = O.data(), b.idx_f = idx.data();
  run(OP_APPLY, c, b);
  SrnnArgs t = a;
  t.epochs = 3, t.flags = SRNN_F_SHUFFLE, t.loss = loss.data();
  run(OP_TRAIN, c, t);
  SrnnArgs l = t;
  l.W2 = O.data(), l.idx_t = idx.data();
  run(OP_LEARN, c, l);
  SrnnArgs f = a;
  f.steps = 20, f.early_exit = 1, f.flags = SRNN_F_FIX_SEC, f.cls = cls.data(), f.nsteps = nsteps.data();
  run(OP_RUN_FIXPOINT, c, f);
  SrnnArgs k = a;
  k.flags = SRNN_F_FIX_SEC, k.cls = cls.data(), k.counts = counts;
  run(OP_CLASSIFY, c, k);
  CHECK((int64_t)(counts[0] + counts[1] + counts[2] + counts[3] + counts[4]) == n);
  SrnnArgs p = a;
  p.eps = 1e-3f;
  run(OP_PERTURB, c, p);
  SrnnArgs v = a;
  v.steps = 10, v.nsteps = nsteps.data(), v.loss = loss.data();
  run(OP_VARY_RUN, c, v);
}

// ---- one soup over R ranks (R = 1: the single-rank pipeline; R > 1: the sharded
// all-to-all protocol of srnn_shard.hip, the collective a memcpy between the ranks) -------
struct RankSoup {
  int64_t lo, hi, n;
  std::vector<float> buf[2];
  std::vector<int64_t> uid, census, next_uid, part, rslot[2], bstat[2];
  std::vector<uint32_t> heads[2], nexts[2], dep[2], rlist[2], satt[2], srep;
  std::vector<int32_t> rcount[2], cno[2], crq[2], nsrep, ctl, err, gen;
  std::vector<unsigned long long> ballots;
  std::vector<int8_t> action, respawn;
  std::vector<int64_t> counterpart;
  std::vector<float> loss;
  std::vector<char> sendbuf, recvbuf;
  std::vector<uint64_t> counts;
};

static std::vector<float> soup(int R, int64_t N, int gens, std::vector<int64_t>* uids_out, int64_t* next_out) {
  const SrnnCfg c = ww22();
  const int PP = c.pp;
  const int64_t XB = PP * 4 + 16;
  const int64_t cr = N, cn = N, cq = N;  // generous: no overflow
  const int64_t blk = ((SRNN_X2_HDR * 8 + cr * XB + cn * 16 + cq * 8) + 15) / 16 * 16;
  const int G = 2;
  std::vector<RankSoup> rk((size_t)R);
  for (int r = 0; r < R; ++r) {
    RankSoup& s = rk[(size_t)r];
    s.lo = r * N / R, s.hi = (r + 1) * N / R, s.n = s.hi - s.lo;
    const size_t nb = (size_t)((s.n + 63) / 64);
    for (int q = 0; q < 2; ++q) {
      s.buf[q].assign((size_t)(s.n * PP), 0.f);
      s.heads[q].assign((size_t)s.n, SRNN_NIL), s.nexts[q].assign((size_t)(s.n + R * cr), SRNN_NIL);
      s.dep[q].assign((size_t)(s.n / 32 + 1), 0u), s.rlist[q].assign((size_t)(2 * s.n + 2), 0u);
      s.rcount[q].assign(1, 0), s.rslot[q].assign((size_t)(R * cr), 0), s.satt[q].assign((size_t)(R * cn), 0u);
      s.cno[q].assign((size_t)R, 0), s.crq[q].assign((size_t)R, 0), s.bstat[q].assign(nb * 4, 0);
    }
    s.uid.resize((size_t)s.n);
    for (int64_t j = 0; j < s.n; ++j) s.uid[(size_t)j] = s.lo + j;
    s.srep.assign((size_t)(R * cq), 0u), s.nsrep.assign((size_t)R, 0), s.ctl.assign(8, 0), s.err.assign(1, 0);
    s.part.assign((size_t)(G * 6), 0), s.ballots.assign(nb + 1, 0ull);
    s.action.assign((size_t)s.n, 0), s.respawn.assign((size_t)s.n, 0), s.counterpart.assign((size_t)s.n, -1);
    s.census.assign(5, 0), s.next_uid.assign(1, N), s.loss.assign((size_t)s.n, 0.f);
    s.sendbuf.assign((size_t)(R * blk), (char)-1), s.recvbuf.assign((size_t)(R * blk), 0);  // -1: no notices
    s.gen.assign(2, 1), s.counts.assign(6, 0);
    SrnnArgs a{};
    a.n = s.n, a.seed = 5, a.W = s.buf[0].data(), a.uid = s.uid.data();
    run(OP_INIT, c, a);
  }
  int p = 0;
  auto args = [&](RankSoup& s) {
    SrnnArgs a{};
    a.n = s.n, a.n_total = N, a.lo = s.lo, a.seed = 5, a.lr = 0.01f, a.eps = 1e-4f;
    a.attacking_rate = 0.3f, a.learn_from_rate = 0.3f, a.epochs = 2, a.severity = 1;
    a.flags = SRNN_F_SHUFFLE | SRNN_F_REMOVE_DIVERGENT | SRNN_F_REMOVE_ZERO;
    a.gen_ptr = s.gen.data() + p, a.gen_out = s.gen.data() + (1 - p);
    a.W2 = s.buf[p].data(), a.W = s.buf[1 - p].data(), a.uid = s.uid.data();
    a.heads = s.heads[p].data(), a.nexts = s.nexts[p].data(), a.ballots = s.ballots.data();
    a.action = s.action.data(), a.counterpart = s.counterpart.data(), a.loss = s.loss.data();
    a.respawn = s.respawn.data(), a.uid_out = s.uid.data(), a.counts = s.counts.data(), a.uid_base = s.next_uid.data();
    return a;
  };
  auto xargs = [&](RankSoup& s, int r, int tp) {  // X2 fields, "this" = parity tp
    SrnnArgs a = args(s);
    const int q = 1 - tp;
    a.world = R, a.rank = r, a.x_cr = cr, a.x_cn = cn, a.x_cq = cq, a.x_blk = blk;
    a.sendbuf = s.sendbuf.data(), a.recvbuf = s.recvbuf.data(), a.census = s.census.data(), a.err = s.err.data();
    a.heads = s.heads[tp].data(), a.nexts = s.nexts[tp].data(), a.heads_next = s.heads[q].data();
    a.nexts_next = s.nexts[q].data(), a.x_dep = s.dep[tp].data(), a.x_dep_next = s.dep[q].data();
    a.x_rlist = s.rlist[tp].data(), a.x_rlist_next = s.rlist[q].data(), a.x_rcount = s.rcount[tp].data();
    a.x_rcount_next = s.rcount[q].data(), a.x_rslot = s.rslot[tp].data(), a.x_rslot_next = s.rslot[q].data();
    a.x_satt = s.satt[tp].data(), a.x_satt_next = s.satt[q].data(), a.x_cno = s.cno[tp].data();
    a.x_cno_next = s.cno[q].data(), a.x_crq = s.crq[tp].data(), a.x_crq_next = s.crq[q].data();
    a.x_srep = s.srep.data(), a.x_nsrep = s.nsrep.data(), a.x_part = s.part.data(), a.x_ctl = s.ctl.data();
    a.x_groups = G;
    return a;
  };
  auto all_to_all = [&]() {  // block d of rank s's sendbuf -> block s of rank d's recvbuf
    for (int src = 0; src < R; ++src)
      for (int dst = 0; dst < R; ++dst)
        std::memcpy(rk[(size_t)dst].recvbuf.data() + (size_t)src * blk, rk[(size_t)src].sendbuf.data() + (size_t)dst * blk,
                    (size_t)blk);
  };
  if (R > 1) {  // prime: this generation's notices / requests (pointers "next" = this parity)
    for (int r = 0; r < R; ++r) {
      RankSoup& s = rk[(size_t)r];
      SrnnArgs a = xargs(s, r, 1 - p);
      a.W2 = s.buf[p].data(), a.temp = s.bstat[1 - p].data(), a.gen_ptr = nullptr, a.gen = s.gen[(size_t)p];
      a.flags |= SRNN_F_X2_PRIME;
      run(OP_X2_PACK, c, a);
    }
    all_to_all();
    for (int r = 0; r < R; ++r) {
      RankSoup& s = rk[(size_t)r];
      SrnnArgs a = xargs(s, r, 1 - p);
      a.temp = s.bstat[1 - p].data(), a.gen_ptr = nullptr, a.gen = s.gen[(size_t)p];
      a.flags |= SRNN_F_X2_PRIME;
      run(OP_X2_POST, c, a);
    }
  }
  for (int g = 0; g < gens; ++g) {
    if (R == 1) {
      RankSoup& s = rk[0];
      SrnnArgs a = args(s);
      run(OP_SOUP_DECIDE, c, a);
      run(OP_SOUP_EVOLVE, c, a);
      run(OP_RESPAWN_SEQ, c, a);
    } else {
      for (int r = 0; r < R; ++r) {
        RankSoup& s = rk[(size_t)r];
        SrnnArgs a = xargs(s, r, p);
        a.temp = s.bstat[1 - p].data();
        run(OP_X2_PACK, c, a);
      }
      all_to_all();
      for (int r = 0; r < R; ++r) {
        RankSoup& s = rk[(size_t)r];
        SrnnArgs a = xargs(s, r, p);
        a.temp = s.bstat[1 - p].data();
        run(OP_X2_POST, c, a);
        SrnnArgs e = xargs(s, r, p);
        e.temp = s.bstat[p].data();
        e.flags |= SRNN_F_X2 | SRNN_F_RESPAWN_INLINE | SRNN_F_FUSED_CENSUS | SRNN_F_FIX_SEC;
        SrnnArgs rem = e;
        rem.flags |= SRNN_F_X2_REMOTE;
        run(OP_SOUP_EVOLVE, c, rem);
        run(OP_SOUP_EVOLVE, c, e);
        CHECK(s.err[0] == 0);
      }
    }
    p = 1 - p;
  }
  if (R > 1) {  // flush: finish-only pack -> stats all-gather -> uids of the last newborns
    std::vector<int64_t> all((size_t)(6 * R));
    for (int r = 0; r < R; ++r) {
      RankSoup& s = rk[(size_t)r];
      SrnnArgs a = xargs(s, r, p);
      a.temp = s.bstat[1 - p].data();
      a.flags |= SRNN_F_X2_FINISH_ONLY;
      run(OP_X2_PACK, c, a);
      std::memcpy(all.data() + r * 6, s.sendbuf.data(), 48);
    }
    for (int r = 0; r < R; ++r) {
      RankSoup& s = rk[(size_t)r];
      SrnnArgs a = xargs(s, r, p);
      a.temp = s.bstat[1 - p].data(), a.stats = all.data();
      a.flags |= SRNN_F_X2_FINISH_ONLY;
      run(OP_X2_POST, c, a);
      CHECK(s.census[0] + s.census[1] + s.census[2] + s.census[3] + s.census[4] == N);
    }
  }
  std::vector<float> W;
  uids_out->clear();
  for (int r = 0; r < R; ++r) {
    W.insert(W.end(), rk[(size_t)r].buf[p].begin(), rk[(size_t)r].buf[p].end());
    uids_out->insert(uids_out->end(), rk[(size_t)r].uid.begin(), rk[(size_t)r].uid.end());
  }
  *next_out = rk[0].next_uid[0];
  for (int r = 1; r < R; ++r) CHECK(rk[(size_t)r].next_uid[0] == *next_out);
  return W;
}

// ---- exact sequential soup (OP_SOUP_SEQ): K steps in one call == K calls of one step,
// recording on or off (pre-respawn rows in W2, counterpart uids) ----------------------------
static void seq_soup(const SrnnCfg& c, int64_t n, int steps) {
  std::vector<float> W[2], rows((size_t)(n * c.pp));
  std::vector<int64_t> uid[2], next[2], cp((size_t)n);
  std::vector<int32_t> gen[2];
  std::vector<int8_t> act((size_t)n), rs((size_t)n);
  std::vector<float> loss((size_t)n);
  for (int v = 0; v < 2; ++v) {
    W[v].assign((size_t)(n * c.pp), 0.f), uid[v].resize((size_t)n), next[v].assign(1, n), gen[v].assign(1, 1);
    for (int64_t j = 0; j < n; ++j) uid[v][(size_t)j] = j;
    SrnnArgs a{};
    a.n = n, a.seed = 11, a.W = W[v].data(), a.uid = uid[v].data();
    run(OP_INIT, c, a);
  }
  auto args = [&](int v) {
    SrnnArgs a{};
    a.n = a.n_total = n, a.seed = 11, a.lr = 0.01f, a.eps = 1e-4f;
    a.attacking_rate = 0.3f, a.learn_from_rate = 0.3f, a.epochs = 2, a.severity = 2;
    a.flags = SRNN_F_SHUFFLE | SRNN_F_REMOVE_DIVERGENT | SRNN_F_REMOVE_ZERO;
    a.W = W[v].data(), a.gen_ptr = gen[v].data(), a.uid_base = next[v].data(), a.uid_out = uid[v].data();
    a.action = act.data(), a.counterpart = cp.data(), a.loss = loss.data(), a.respawn = rs.data();
    return a;
  };
  SrnnArgs a = args(0);
  a.steps = steps;
  run(OP_SOUP_SEQ, c, a);
  for (int s = 0; s < steps; ++s) {
    SrnnArgs b = args(1);
    b.steps = 1, b.W2 = rows.data();
    std::vector<int64_t> before = uid[1];
    run(OP_SOUP_SEQ, c, b);
    // a particle's recorded state is its row after its own turn: later attackers may still
    // change the table row, so most (not all) surviving rows match it, the last one always
    int64_t bad_cp = 0, bad_uid = 0, same = 0, kept = 0;
    for (int64_t j = 0; j < n; ++j) {
      bad_cp += cp[(size_t)j] >= next[1][0];  // counterparts are uids that existed
      const bool eq = std::memcmp(&rows[(size_t)(j * c.pp)], &W[1][(size_t)(j * c.pp)], 4 * (size_t)c.pp) == 0;
      if (rs[(size_t)j]) bad_uid += uid[1][(size_t)j] == before[(size_t)j];
      else kept += 1, same += eq;
    }
    CHECK(bad_cp == 0 && bad_uid == 0 && 2 * same >= kept);
    CHECK(rs[(size_t)(n - 1)] || std::memcmp(&rows[(size_t)((n - 1) * c.pp)], &W[1][(size_t)((n - 1) * c.pp)], 4 * (size_t)c.pp) == 0);
  }
  CHECK(W[0] == W[1] && uid[0] == uid[1] && next[0] == next[1] && gen[0][0] == 1 + steps && gen[1][0] == 1 + steps);
}

// ---- reference-order generation (OP_SOUP_ORDERED): the plan inline, or built one generation
// ahead by OP_ORD_PLAN into the other of two plan sets (SRNN_F_ORD_PLANNED / _NEXT), both
// bitwise the serial loop (OP_SOUP_SEQ) ---------------------------------------------------------
static int64_t ord_words(int64_t n) {  // ops/_lib.py ord_src_words
  const int64_t rec = 64 * ((((n + 63) / 64) + 63) / 64) * 64;
  return 6 * n + 34 * rec;
}
// pipe 0: inline plan, 1: OP_ORD_PLAN one generation ahead, 2: the generation call plans the next one
static void ordered_soup(const SrnnCfg& c, int64_t n, int gens, int pipe) {
  const size_t R = (size_t)(n * c.pp);
  std::vector<float> seqW(R), buf[2] = {std::vector<float>(R), std::vector<float>(R)}, W3(R);
  std::vector<int64_t> suid((size_t)n), uid((size_t)n), snext(1, n), next(1, n), scp((size_t)n), cp((size_t)n);
  std::vector<int32_t> sgen(1, 1), ring = {1, 1}, osrc[2], olist[2], octl[2];
  std::vector<uint32_t> heads[2], nexts[2];
  std::vector<int8_t> sact((size_t)n), act((size_t)n), srs((size_t)n), rs((size_t)n);
  std::vector<float> sloss((size_t)n), loss((size_t)n);
  std::vector<uint64_t> counts(6, 0);
  for (int q = 0; q < 2; ++q) {
    osrc[q].assign((size_t)ord_words(n), 0), olist[q].assign((size_t)n, 0), octl[q].assign(166, 0);
    heads[q].assign((size_t)n, 0xFFFFFFFFu), nexts[q].assign((size_t)n, 0xFFFFFFFFu);
  }
  for (int64_t j = 0; j < n; ++j) suid[(size_t)j] = uid[(size_t)j] = j;
  SrnnArgs ia{};
  ia.n = n, ia.seed = 19, ia.W = seqW.data(), ia.uid = suid.data();
  run(OP_INIT, c, ia);
  buf[0] = seqW;
  auto base = [&]() {
    SrnnArgs a{};
    a.n = a.n_total = n, a.seed = 19, a.lr = 0.01f, a.eps = 1e-4f;
    a.attacking_rate = 0.3f, a.learn_from_rate = 0.3f, a.epochs = 2, a.severity = 2;
    a.flags = SRNN_F_SHUFFLE | SRNN_F_REMOVE_DIVERGENT | SRNN_F_REMOVE_ZERO | SRNN_F_FUSED_CENSUS;
    return a;
  };
  SrnnArgs sa = base();
  sa.W = seqW.data(), sa.gen_ptr = sgen.data(), sa.uid_base = snext.data(), sa.uid_out = suid.data();
  sa.action = sact.data(), sa.counterpart = scp.data(), sa.loss = sloss.data(), sa.respawn = srs.data();
  sa.steps = gens;
  run(OP_SOUP_SEQ, c, sa);
  auto plan_args = [&](int q, bool nxt, int p) {
    SrnnArgs a = base();
    a.gen_ptr = ring.data() + p;
    a.o_src = osrc[q].data(), a.o_list = olist[q].data(), a.o_ctl = octl[q].data();
    a.heads = heads[q].data(), a.nexts = nexts[q].data();
    if (nxt) a.flags |= SRNN_F_ORD_NEXT;
    return a;
  };
  int p = 0;
  if (pipe) {
    run(OP_ORD_PLAN, c, plan_args(0, false, 0));
  } else {
    SrnnArgs d = base();
    d.gen_ptr = ring.data(), d.heads = heads[0].data(), d.nexts = nexts[0].data();
    run(OP_SOUP_DECIDE, c, d);
  }
  for (int g = 0; g < gens; ++g) {
    const int q = pipe ? p : 0;
    if (pipe == 1) run(OP_ORD_PLAN, c, plan_args(1 - p, true, p));
    SrnnArgs a = base();
    a.W2 = buf[p].data(), a.W = buf[1 - p].data(), a.W3 = W3.data();
    a.gen_ptr = ring.data() + p, a.gen_out = ring.data() + (1 - p);
    a.o_src = osrc[q].data(), a.o_list = olist[q].data(), a.o_ctl = octl[q].data(), a.o_levels = 4;
    a.heads = heads[p].data(), a.nexts = nexts[p].data();
    a.heads_next = heads[1 - p].data(), a.nexts_next = nexts[1 - p].data();
    a.uid_base = next.data(), a.uid_out = uid.data(), a.counts = counts.data();
    a.action = act.data(), a.counterpart = cp.data(), a.loss = loss.data(), a.respawn = rs.data();
    if (pipe) a.flags |= SRNN_F_ORD_PLANNED;
    if (pipe == 2) {
      a.flags |= SRNN_F_ORD_INPLAN;
      a.o_src_next = osrc[1 - p].data(), a.o_list_next = olist[1 - p].data(), a.o_ctl_next = octl[1 - p].data();
      a.o_plan_groups = 1;
    }
    run(OP_SOUP_ORDERED, c, a);
    CHECK(octl[q][18] == 0);  // error bits
    p = 1 - p;
  }
  CHECK(std::memcmp(buf[p].data(), seqW.data(), R * 4) == 0);
  CHECK(uid == suid && next == snext && act == sact && rs == srs && cp == scp);
  CHECK(std::memcmp(loss.data(), sloss.data(), (size_t)n * 4) == 0);
  CHECK(ring[(size_t)p] == sgen[0]);
}

int main() {
  CHECK(srnn_abi_version() == 31);
  ordered_soup(ww22(), 257, 4, 0);
  ordered_soup(ww22(), 257, 4, 1);
  ordered_soup(ww22(), 257, 4, 2);
  ordered_soup(agg422(), 129, 3, 2);
  seq_soup(ww22(), 257, 4);
  seq_soup(agg422(), 129, 3);
  ops_smoke(ww22(), 1000);
  ops_smoke(agg422(), 777);
  ops_smoke(cfg(2, 2, 2, 0, 17), 300);              // Recurrent(2,2): templated BPTT
  ops_smoke(cfg(3, 2, 2, 4, 20), 300);              // FFT(4,2,2)
  ops_smoke(cfg(0, 2, 2, 0, 14, 0, 1), 300);        // bf16 table (srnn_lowp.hip)
  ops_smoke(cfg(1, 2, 2, 4, 20, 1, 2), 300);        // fp16 + shuffle_random
  // runtime-shape engine (srnn_generic.hip): shapes with no template, and the GPU-only
  // wave-per-particle shapes on the host
  ops_smoke(cfg(0, 3, 3, 0, 33), 200);              // Weightwise(3,3)
  ops_smoke(cfg(2, 3, 2, 0, 34), 100);              // Recurrent(3,2)
  ops_smoke(cfg(1, 10, 3, 4, 280), 64);             // Aggregating(4,10,3): the north-star net
  ops_smoke(cfg(1, 3, 2, 4, 33, 1, 1), 64);         // Aggregating(4,3,2), shuffle_random, bf16
  ops_smoke(cfg(0, 16, 2, 0, 336), 32);             // Weightwise(16,2) (MFMA path on the GPU)
  CHECK(srnn_comm_available("/nonexistent/librccl.so") == 0 || srnn_comm_available("/nonexistent/librccl.so") == 1);
  std::vector<int64_t> u1, u2, u3;
  int64_t n1 = 0, n2 = 0, n3 = 0;
  const int64_t N = 301;
  std::vector<float> w1 = soup(1, N, 5, &u1, &n1);
  std::vector<float> w2 = soup(2, N, 5, &u2, &n2);
  std::vector<float> w3 = soup(3, N, 5, &u3, &n3);
  CHECK(w1.size() == w2.size() && std::memcmp(w1.data(), w2.data(), w1.size() * 4) == 0);
  CHECK(w1.size() == w3.size() && std::memcmp(w1.data(), w3.data(), w1.size() * 4) == 0);
  CHECK(u1 == u2 && u1 == u3);
  CHECK(n1 == n2 && n1 == n3);
  std::printf("host_selftest: %s (next_uid %lld)\n", g_fail ? "FAILED" : "ok", (long long)n1);
  return g_fail ? 1 : 0;
}
