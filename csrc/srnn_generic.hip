// srnn_generic.hip — runtime-shape engine: every (kind, width, depth, aggregates) the
// reference constructors accept (code/network.py:222-230 Weightwise, :324-333
// Aggregating, :465-474 FFT, :526-535 Recurrent), on the host and on the GPU.
//
// The templated kernels (srnn_kernels.h, srnn_bignet.hip, srnn_wide.hip) keep a
// particle's weights in VGPRs and are instantiated for a list of shapes; every other shape
// -- and every operator a specialised path does not provide (e.g. soups of the P = 280
// north-star net, shuffle_random on it, host execution of the GPU-only paths) -- runs
// here.  The per-particle arithmetic is the same, in the same order (x[0]*k then fmaf over
// the inputs, Keras SGD with the folded step, chunk means as double sums, BPTT of the
// linear SimpleRNN stack), with the same Philox streams, so on the same device a generic
// run is bitwise equal to the templated one (tests/test_generic.py).
//
// Execution: lane per particle with a grid-stride loop over rows.  The layer tables live
// in the kernel argument (GShape), the weight-point coordinate table in LDS, and every
// per-particle vector (weights, targets, activations, samples, BPTT states) in a scratch
// buffer laid out element-major -- element e of lane L at scratch[e * lanes + L] -- so the
// 64 lanes of a wave touch 64 consecutive floats (coalesced) on every access.
#include "srnn_kernels.h"

#include <cstdlib>
#include <cstring>
#include <vector>

namespace srnn {

constexpr int GMAXL = 33;  // dense layers (depth <= 32) / SimpleRNN layers
constexpr int GTB = 64;    // threads per block: one wave, the respawn ballot is per 64 rows

struct GShape {
  int kind, W, D, A, P, PP, NL;
  int aggregator, shuffler, dtype;
  int rows[GMAXL], cols[GMAXL], off[GMAXL];  // dense layers (Weightwise / Aggregating / FFT)
  int in_[GMAXL], un[GMAXL], koff[GMAXL], roff[GMAXL];  // SimpleRNN layers
  int IN, OUT, NACT, HS, MAXV, CS;
  // scratch layout (float offsets of every per-item region)
  int o_w, o_t, o_o, o_f, o_acts, o_v1, o_v2, o_v3, o_v4, o_samp, o_perm, o_hs, o_gw, o_orth, sfloats;
  int orthd;  // doubles of lane-private orthogonal-init scratch (recurrent: W*W)
};

static inline int gmax(int a, int b) { return a > b ? a : b; }
SRNN_HD int64_t g_lane_bytes(const struct GShape& s);

// host: layer tables + scratch layout of a configuration; false if it is not a valid shape
static bool make_gshape(const SrnnCfg& c, GShape& s, const char** why) {
  std::memset(&s, 0, sizeof(s));
  s.kind = c.kind, s.W = c.width, s.D = c.depth, s.A = c.aggregates;
  s.aggregator = c.aggregator, s.shuffler = c.shuffler, s.dtype = c.dtype;
  if (s.W < 1 || s.D < 1 || s.D + 1 > GMAXL) {
    *why = "generic engine: width >= 1 and 1 <= depth <= 32 required";
    return false;
  }
  int P = 0;
  if (s.kind == 2) {  // recurrent: (1,w)+(w,w), (w,w)+(w,w) x (d-1), (w,1)+(1,1)
    s.NL = s.D + 1;
    for (int l = 0; l < s.NL; ++l) {
      s.in_[l] = l == 0 ? 1 : s.W;
      s.un[l] = l == s.D ? 1 : s.W;
      s.koff[l] = P;
      s.roff[l] = P + s.in_[l] * s.un[l];
      P += s.in_[l] * s.un[l] + s.un[l] * s.un[l];
    }
    s.HS = s.D * s.W + 1;
    s.IN = 1, s.OUT = 1;
  } else if (s.kind == 0 || s.kind == 1 || s.kind == 3) {
    s.IN = s.kind == 0 ? 4 : s.A;
    s.OUT = s.kind == 0 ? 1 : s.A;
    if (s.kind != 0 && s.A < 1) {
      *why = "generic engine: aggregating / fft nets need aggregates >= 1";
      return false;
    }
    s.NL = s.D + 1;
    for (int l = 0; l < s.NL; ++l) {
      s.rows[l] = l == 0 ? s.IN : s.W;
      s.cols[l] = l == s.D ? s.OUT : s.W;
      s.off[l] = P;
      P += s.rows[l] * s.cols[l];
    }
  } else {
    *why = "unknown network kind";
    return false;
  }
  s.P = P;
  s.PP = (P + 3) & ~3;
  if (c.p != s.P || c.pp != s.PP) {
    *why = "layout mismatch (p/pp) for the generic engine";
    return false;
  }
  if (s.kind == 1) {
    s.CS = P / s.A;
    if (s.CS < 1 || P / s.CS != s.A) {
      *why = "aggregating net cannot be cut into `aggregates` chunks (SURVEY S4)";
      return false;
    }
  }
  if (s.kind == 3 && s.A > P) {
    *why = "fft aggregates must not exceed the number of weights";
    return false;
  }
  s.NACT = s.IN + s.D * s.W;
  s.MAXV = gmax(gmax(s.IN, s.OUT), gmax(s.W, s.HS)) + 1;
  int o = 0;
  auto take = [&](int n) { int r = o; o += n; return r; };
  s.o_w = take(s.PP), s.o_t = take(s.PP), s.o_o = take(s.PP), s.o_f = take(s.PP);
  s.o_acts = take(s.NACT + 1);
  s.o_v1 = take(s.MAXV), s.o_v2 = take(s.MAXV), s.o_v3 = take(s.MAXV), s.o_v4 = take(s.MAXV);
  s.o_samp = take(s.kind == 0 ? s.P : 0);            // sample values (coordinates from the table)
  s.o_perm = take(s.P);                              // permutation (one index per float slot)
  s.o_hs = take(s.kind == 2 ? s.P * s.HS + 3 * s.HS : 0);  // BPTT states + h / carry / zeros
  s.o_gw = take(s.kind == 2 ? s.P : 0);
  s.o_orth = 0;
  s.sfloats = o;
  s.orthd = s.kind == 2 ? s.W * s.W : 0;  // after the strided region: lane L at [L * orthd]
  return true;
}

SRNN_HD int64_t g_lane_bytes(const GShape& s) { return (int64_t)s.sfloats * 4 + (int64_t)s.orthd * 8; }
// lane-private doubles of lane L after the strided float region of `lanes` lanes
SRNN_HD double* g_orth(const GShape& s, void* scratch, int64_t lanes, int64_t L) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(scratch) + lanes * (int64_t)s.sfloats * 4) + L * s.orthd;
}

// ---------------------------------------------------------------------------------
// Strided scratch vectors: element k at p[k * st] (st = lanes on the device, 1 on host)
// ---------------------------------------------------------------------------------
struct SV {
  float* p;
  int64_t st;
  SRNN_HD float& operator[](int64_t k) const { return p[k * st]; }
  SRNN_HD SV at(int64_t k) const { return SV{p + k * st, st}; }
};

struct GCtx {  // one item's view of the shape, its scratch and the coordinate table
  const GShape* s;
  float* base;
  int64_t st;
  const float* coords;  // [P][3] (Weightwise)
  double* orth;         // recurrent init: un*un doubles, lane-private (contiguous)
  SRNN_HD SV v(int off) const { return SV{base + (int64_t)off * st, st}; }
};

// ---------------------------------------------------------------- storage formats
SRNN_HD float g_dec(const char* row, int k, int dtype) {
  if (dtype == 0) return reinterpret_cast<const float*>(row)[k];
  const uint16_t h = reinterpret_cast<const uint16_t*>(row)[k];
  return dtype == 1 ? StBF16::dec(h) : StF16::dec(h);
}
SRNN_HD float g_q(float x, int dtype) { return dtype == 0 ? x : dtype == 1 ? StBF16::q(x) : StF16::q(x); }
SRNN_HD void g_load(const GShape& s, const char* row, SV w) {
  for (int k = 0; k < s.P; ++k) w[k] = g_dec(row, k, s.dtype);
}
SRNN_HD void g_store(const GShape& s, char* row, SV w) {
  for (int k = 0; k < s.PP; ++k) {
    const float v = k < s.P ? w[k] : 0.f;
    if (s.dtype == 0) reinterpret_cast<float*>(row)[k] = v;
    else reinterpret_cast<uint16_t*>(row)[k] = s.dtype == 1 ? StBF16::enc(v) : StF16::enc(v);
  }
}
SRNN_HD void g_quant(const GShape& s, SV w) {
  if (s.dtype != 0)
    for (int k = 0; k < s.P; ++k) w[k] = g_q(w[k], s.dtype);
}
SRNN_HD int64_t g_rb(const GShape& s) { return (int64_t)s.PP * (s.dtype == 0 ? 4 : 2); }
SRNN_HD void g_copy(const GShape& s, SV d, SV src) {
  for (int k = 0; k < s.P; ++k) d[k] = src[k];
}

// ---------------------------------------------------------------- dense layers
// y = x . K (row-major (I, O) kernel at k): acc = x[0]*k[j], then fma over the inputs
SRNN_HD void g_dense(const SV& k, int I, int O, const SV& x, SV y) {
  for (int j = 0; j < O; ++j) {
    float acc = x[0] * k[j];
    for (int i = 1; i < I; ++i) acc = fmaf(x[i], k[(int64_t)i * O + j], acc);
    y[j] = acc;
  }
}
// si = K . so (pre-update K); K += x (x) so  (MLP::step_layer)
SRNN_HD void g_step_layer(SV k, int I, int O, const SV& x, const SV& so, SV si, bool want_in) {
  if (want_in) {
    for (int i = 0; i < I; ++i) {
      float acc = k[(int64_t)i * O] * so[0];
      for (int j = 1; j < O; ++j) acc = fmaf(k[(int64_t)i * O + j], so[j], acc);
      si[i] = acc;
    }
  }
  for (int i = 0; i < I; ++i)
    for (int j = 0; j < O; ++j) k[(int64_t)i * O + j] = fmaf(x[i], so[j], k[(int64_t)i * O + j]);
}
// MLP forward keeping every layer's input in acts = [x][h1]...[hD]
SRNN_HD void g_forward(const GShape& s, const SV& w, const SV& x, SV acts, SV y) {
  for (int i = 0; i < s.IN; ++i) acts[i] = x[i];
  g_dense(w.at(s.off[0]), s.IN, s.cols[0], acts, acts.at(s.IN));
  for (int l = 1; l < s.D; ++l) g_dense(w.at(s.off[l]), s.W, s.W, acts.at(s.IN + (l - 1) * s.W), acts.at(s.IN + l * s.W));
  g_dense(w.at(s.off[s.D]), s.W, s.OUT, acts.at(s.IN + (s.D - 1) * s.W), y);
}
// forward through the MLP with ping-pong vectors h, g (MLP::forward_only)
SRNN_HD void g_forward_only(const GShape& s, const SV& w, const SV& x, SV h, SV g, SV y) {
  g_dense(w.at(s.off[0]), s.IN, s.W, x, h);
  for (int l = 1; l < s.D; ++l) {
    g_dense(w.at(s.off[l]), s.W, s.W, h, g);
    for (int j = 0; j < s.W; ++j) h[j] = g[j];
  }
  g_dense(w.at(s.off[s.D]), s.W, s.OUT, h, y);
}
// one SGD step given dL/dy (MLP::backward_update); so / si are MAXV vectors
SRNN_HD void g_backward(const GShape& s, SV w, const SV& acts, const SV& gy, float lr, SV so, SV si) {
  for (int j = 0; j < s.OUT; ++j) so[j] = -lr * gy[j];
  g_step_layer(w.at(s.off[s.D]), s.W, s.OUT, acts.at(s.IN + (s.D - 1) * s.W), so, si, true);
  for (int l = s.D - 1; l >= 1; --l) {
    for (int j = 0; j < s.W; ++j) so[j] = si[j];
    g_step_layer(w.at(s.off[l]), s.W, s.W, acts.at(s.IN + (l - 1) * s.W), so, si, true);
  }
  for (int j = 0; j < s.W; ++j) so[j] = si[j];
  g_step_layer(w, s.IN, s.W, acts, so, si, false);
}

// ---------------------------------------------------------------- coordinates
// (layer, cell, position) of every Weightwise weight (reference code/network.py:240-255)
static void make_coords_host(const GShape& s, float* c) {
  int k = 0;
  for (int l = 0; l < s.NL; ++l)
    for (int i = 0; i < s.rows[l]; ++i)
      for (int j = 0; j < s.cols[l]; ++j) {
        c[3 * k + 0] = norm_id(l, s.NL - 1);
        c[3 * k + 1] = norm_id(i, s.rows[l] - 1);
        c[3 * k + 2] = norm_id(j, s.cols[l] - 1);
        ++k;
      }
}
__device__ void make_coords_dev(const GShape& s, float* c) {  // whole block, then a barrier
  for (int k = threadIdx.x; k < s.P; k += blockDim.x) {
    int l = 0;
    while (l + 1 < s.NL && s.off[l + 1] <= k) ++l;
    const int q = k - s.off[l], i = q / s.cols[l], j = q - i * s.cols[l];
    c[3 * k + 0] = norm_id(l, s.NL - 1);
    c[3 * k + 1] = norm_id(i, s.rows[l] - 1);
    c[3 * k + 2] = norm_id(j, s.cols[l] - 1);
  }
  __syncthreads();
}

// ---------------------------------------------------------------- permutations
// nibble permutation of [0, n), n <= 16 (srnn_core.h)
SRNN_HD uint64_t g_perm_nibbles(int n, uint64_t u) { return perm_from_bits_n(n, u); }
// Fisher-Yates into a strided vector (fisher_yates of srnn_core.h, same draws)
SRNN_HD void g_fisher_yates(SV perm, int n, const Rng& rng, uint64_t id, uint32_t step, uint32_t purpose) {
  for (int i = 0; i < n; ++i) perm[i] = (float)i;
  U4 r{0, 0, 0, 0};
  int used = 4;
  uint32_t blk = 0;
  for (int i = n - 1; i > 0; --i) {
    if (used == 4) {
      r = rng.draw(id, step, purpose + (blk << 8));  // (fisher_yates of srnn_core.h)
      ++blk;
      used = 0;
    }
    uint32_t x = used == 0 ? r.x : used == 1 ? r.y : used == 2 ? r.z : r.w;
    ++used;
    int j = (int)(u01(x) * (float)(i + 1));
    if (j > i) j = i;
    const float t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
}

// ---------------------------------------------------------------- init
SRNN_HD void g_glorot(SV w, int off, int r, int c, const Rng& rng, uint64_t uid) {
  const float lim = sqrtf(6.0f / (float)(r + c));
  const int n = r * c;
  for (int b = 0; b < (n + 3) / 4; ++b) {
    U4 u = rng.draw(uid, (uint32_t)off * 1024u + (uint32_t)b, P_INIT);
    uint32_t xs[4] = {u.x, u.y, u.z, u.w};
    for (int q = 0; q < 4; ++q) {
      int k = b * 4 + q;
      if (k < n) w[off + k] = -lim + 2.0f * lim * u01(xs[q]);
    }
  }
}
SRNN_HD void g_orthogonal(SV w, int off, int N, double* a, const Rng& rng, uint64_t uid) {
  // orthogonal_fill of srnn_core.h with a runtime N; `a` is N*N doubles of scratch
  int cnt = 0;
  U4 u{0, 0, 0, 0};
  float nrm[4] = {0, 0, 0, 0};
  uint32_t blk = 0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      if ((cnt & 3) == 0) {
        u = rng.draw(uid, (uint32_t)off * 1024u + blk, P_NORMAL);
        ++blk;
        float r1 = sqrtf(-2.0f * logf(u01_open0(u.x)));
        float t1 = 6.283185307179586f * u01(u.y);
        float r2 = sqrtf(-2.0f * logf(u01_open0(u.z)));
        float t2 = 6.283185307179586f * u01(u.w);
        nrm[0] = r1 * cosf(t1);
        nrm[1] = r1 * sinf(t1);
        nrm[2] = r2 * cosf(t2);
        nrm[3] = r2 * sinf(t2);
      }
      a[i * N + j] = (double)nrm[cnt & 3];
      ++cnt;
    }
  if (N == 2) {  // Keras / LAPACK convention (lapack_u2 of srnn_core.h)
    double m[2][2] = {{a[0], a[1]}, {a[2], a[3]}};
    lapack_u2(m);
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) w[off + i * 2 + j] = (float)m[i][j];
    return;
  }
  for (int j = 0; j < N; ++j) {
    for (int p = 0; p < j; ++p) {
      double d = 0.0;
      for (int i = 0; i < N; ++i) d = fma(a[i * N + p], a[i * N + j], d);
      for (int i = 0; i < N; ++i) a[i * N + j] = fma(-d, a[i * N + p], a[i * N + j]);
    }
    double sq = 0.0;
    for (int i = 0; i < N; ++i) sq = fma(a[i * N + j], a[i * N + j], sq);
    const double inv = 1.0 / sqrt(sq);
    for (int i = 0; i < N; ++i) a[i * N + j] *= inv;
  }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) w[off + i * N + j] = (float)a[i * N + j];
}
SRNN_HD void g_init(const GCtx& x, SV w, const Rng& rng, uint64_t uid) {
  const GShape& s = *x.s;
  if (s.kind == 2) {
    for (int l = 0; l < s.NL; ++l) {
      g_glorot(w, s.koff[l], s.in_[l], s.un[l], rng, uid);
      g_orthogonal(w, s.roff[l], s.un[l], x.orth, rng, uid);
    }
  } else {
    for (int l = 0; l < s.NL; ++l) g_glorot(w, s.off[l], s.rows[l], s.cols[l], rng, uid);
  }
}

// ---------------------------------------------------------------- aggregation / fft
SRNN_HD int g_clen(const GShape& s, int k) { return k == s.A - 1 ? s.P - s.CS * (s.A - 1) : s.CS; }
SRNN_HD void g_aggregate(const GShape& s, const SV& t, SV g, int aggregator) {
  for (int k = 0; k < s.A; ++k) {
    const int b = k * s.CS, len = g_clen(s, k);
    if (aggregator == 0) {
      double acc = 0.0;
      for (int i = 0; i < len; ++i) acc += (double)t[b + i];
      g[k] = (float)(acc / (double)len);
    } else {
      float m = t[b];
      for (int i = 0; i < len; ++i) {
        const float v = t[b + i];
        if (aggregator == 1) m = (v > m) ? v : m;
        else m = (v > m && v != 0.0f) ? v : m;
      }
      g[k] = m;
    }
  }
}
SRNN_HD void g_fft_reduce(const GShape& s, const SV& t, SV g) {
  for (int k = 0; k < s.A; ++k) {
    float acc = 0.f;
    for (int n = 0; n < s.A; ++n)
      acc = fmaf(t[n], cosf(6.283185307179586f * (float)((k * n) % s.A) / (float)s.A), acc);
    g[k] = acc;
  }
}
// shuffle_random (reference code/network.py:319-322): out[k] = out[perm[k]]
SRNN_HD void g_shuffle_out(const GCtx& x, SV out, const ApplyCtx& c) {
  const GShape& s = *x.s;
  if (c.shuffler != 1) return;
  SV perm = x.v(s.o_perm), tmp = x.v(s.o_f);
  g_fisher_yates(perm, s.P, c.rng, c.uid, c.ctr, P_AGGSHUF);
  for (int k = 0; k < s.P; ++k) tmp[k] = out[k];
  for (int k = 0; k < s.P; ++k) out[k] = tmp[(int)perm[k]];
}

// ---------------------------------------------------------------- recurrent
// one time step of every layer; h holds the hidden state of layer l at offset l*W
SRNN_HD void g_rnn_step(const GShape& s, const SV& w, float x0, SV h, SV xk, SV hr) {
  for (int L = 0; L < s.NL; ++L) {
    const int I = s.in_[L], U = s.un[L];
    // cell: hn = x . K + h_prev . R, x = the scalar input (L = 0) or layer L-1's new state
    if (L == 0) {
      for (int j = 0; j < U; ++j) xk[j] = x0 * w[s.koff[0] + j];
    } else {
      g_dense(w.at(s.koff[L]), I, U, h.at((L - 1) * s.W), xk);
    }
    g_dense(w.at(s.roff[L]), U, U, h.at(L * s.W), hr);
    for (int j = 0; j < U; ++j) h[L * s.W + j] = xk[j] + hr[j];
  }
}

// ---------------------------------------------------------------- apply (f_a(t))
SRNN_HD void g_apply(const GCtx& x, const SV& a, const SV& t, SV out, const ApplyCtx& ac) {
  const GShape& s = *x.s;
  SV v1 = x.v(s.o_v1), v2 = x.v(s.o_v2), v3 = x.v(s.o_v3), v4 = x.v(s.o_v4);
  if (s.kind == 0) {
    for (int k = 0; k < s.P; ++k) {
      v1[0] = t[k];
      v1[1] = x.coords[3 * k + 0];
      v1[2] = x.coords[3 * k + 1];
      v1[3] = x.coords[3 * k + 2];
      g_forward_only(s, a, v1, v2, v3, v4);
      out[k] = v4[0];
    }
  } else if (s.kind == 1 || s.kind == 3) {
    if (s.kind == 1) g_aggregate(s, t, v1, ac.aggregator);
    else g_fft_reduce(s, t, v1);
    SV h = x.v(s.o_acts);  // forward_only's output (A floats)
    g_forward_only(s, a, v1, v2, v3, h);
    if (s.kind == 1) {
      for (int k = 0; k < s.A; ++k)
        for (int i = 0; i < g_clen(s, k); ++i) out[k * s.CS + i] = h[k];
    } else {
      for (int m = 0; m < s.P; ++m) {
        float acc = 0.f;
        for (int k = 0; k < s.A; ++k)
          acc = fmaf(h[k], cosf(6.283185307179586f * (float)((k * m) % s.P) / (float)s.P), acc);
        out[m] = acc / (float)s.P;
      }
    }
    g_shuffle_out(x, out, ac);
  } else {
    SV h = x.v(s.o_hs);
    for (int q = 0; q < s.HS; ++q) h[q] = 0.f;
    for (int st = 0; st < s.P; ++st) {
      g_rnn_step(s, a, t[st], h, v1, v2);
      out[st] = h[s.D * s.W];
    }
  }
}

// ---------------------------------------------------------------- one training epoch
// Keras fit(batch_size=1) epoch on the samples of `smp` (frozen), in place on w.
SRNN_HD float g_train_epoch(const GCtx& x, SV w, const SV& smp, TrainCtx& c) {
  const GShape& s = *x.s;
  SV v1 = x.v(s.o_v1), v2 = x.v(s.o_v2), v3 = x.v(s.o_v3), v4 = x.v(s.o_v4), acts = x.v(s.o_acts);
  if (s.kind == 0) {
    SV sv = x.v(s.o_samp), perm = x.v(s.o_perm);
    for (int k = 0; k < s.P; ++k) sv[k] = smp[k];
    uint64_t pn = 0;
    if (s.P <= 16) {
      if (c.shuffle) pn = g_perm_nibbles(s.P, perm_bits(perm_draw(c.rng, c.uid, c.ctr, P_SHUFFLE), c.ctr));
      else
        for (int k = 0; k < s.P; ++k) pn |= (uint64_t)k << (4 * k);
    } else if (c.shuffle) {
      g_fisher_yates(perm, s.P, c.rng, c.uid, c.ctr, P_SHUFFLE);
    }
    float loss = 0.f;
    for (int q = 0; q < s.P; ++q) {
      int idx;
      if (s.P <= 16) idx = (int)((pn >> (4 * q)) & 15u);
      else idx = c.shuffle ? (int)perm[q] : q;
      v1[0] = sv[idx];
      v1[1] = x.coords[3 * idx + 0];
      v1[2] = x.coords[3 * idx + 1];
      v1[3] = x.coords[3 * idx + 2];
      g_forward(s, w, v1, acts, v2);
      float e = v2[0] - v1[0];
      loss += e * e;
      v2[0] = e;  // the folded step -(2 lr) * e (Weightwise::train_epoch)
      g_backward(s, w, acts, v2, 2.0f * c.lr, v3, v4);
    }
    c.ctr += 1;
    return loss / (float)s.P;
  }
  if (s.kind == 1 || s.kind == 3) {
    SV g = x.v(s.o_v1), h = x.v(s.o_v2), gy = x.v(s.o_v2);
    if (s.kind == 1) g_aggregate(s, smp, g, c.aggregator);
    else g_fft_reduce(s, smp, g);
    g_forward(s, w, g, acts, h);
    float loss = 0.f;
    for (int k = 0; k < s.A; ++k) {
      float e = h[k] - g[k];
      loss += e * e;
      gy[k] = 2.0f * e / (float)s.A;  // h[k] is dead after this line: gy aliases h
    }
    g_backward(s, w, acts, gy, c.lr, v3, v4);
    c.ctr += 1;
    return loss / (float)s.A;
  }
  // recurrent: one (1, P, 1) sequence, BPTT, one SGD step
  SV hs = x.v(s.o_hs), h = x.v(s.o_hs + s.P * s.HS), carry = x.v(s.o_hs + s.P * s.HS + s.HS),
     zeros = x.v(s.o_hs + s.P * s.HS + 2 * s.HS), gw = x.v(s.o_gw);
  for (int q = 0; q < s.HS; ++q) h[q] = 0.f, carry[q] = 0.f, zeros[q] = 0.f;
  for (int t = 0; t < s.P; ++t) {
    g_rnn_step(s, w, smp[t], h, v1, v2);
    for (int q = 0; q < s.HS; ++q) hs[(int64_t)t * s.HS + q] = h[q];
  }
  for (int k = 0; k < s.P; ++k) gw[k] = 0.f;
  float loss = 0.f;
  SV dtop = v1, dh = v2, dx = v3, cr = v4;
  for (int t = s.P - 1; t >= 0; --t) {
    const SV hst = hs.at((int64_t)t * s.HS), hsp = t > 0 ? hs.at((int64_t)(t - 1) * s.HS) : zeros;
    float e = hst[s.D * s.W] - smp[t];
    loss += e * e;
    dtop[0] = 2.0f * e / (float)s.P;
    for (int L = s.D; L >= 0; --L) {
      const int U = s.un[L], I = s.in_[L];
      for (int j = 0; j < U; ++j) dh[j] = dtop[j] + carry[L * s.W + j];
      // cell_bwd: kernel / recurrent-kernel grads, input grad (L > 0), carry
      for (int i = 0; i < I; ++i) {
        const float xi = L == 0 ? smp[t] : hst[(L - 1) * s.W + i];
        for (int j = 0; j < U; ++j) gw[s.koff[L] + i * U + j] = fmaf(xi, dh[j], gw[s.koff[L] + i * U + j]);
      }
      for (int i = 0; i < U; ++i)
        for (int j = 0; j < U; ++j) gw[s.roff[L] + i * U + j] = fmaf(hsp[L * s.W + i], dh[j], gw[s.roff[L] + i * U + j]);
      if (L > 0) {
        for (int i = 0; i < I; ++i) {
          float acc = 0.f;
          for (int j = 0; j < U; ++j) acc = fmaf(w[s.koff[L] + i * U + j], dh[j], acc);
          dx[i] = acc;
        }
      }
      for (int i = 0; i < U; ++i) {
        float acc = 0.f;
        for (int j = 0; j < U; ++j) acc = fmaf(w[s.roff[L] + i * U + j], dh[j], acc);
        cr[i] = acc;
      }
      for (int j = 0; j < U; ++j) carry[L * s.W + j] = cr[j];
      for (int i = 0; i < I && L > 0; ++i) dtop[i] = dx[i];
    }
  }
  for (int k = 0; k < s.P; ++k) w[k] = fmaf(gw[k], -c.lr, w[k]);
  c.ctr += 1;
  return loss / (float)s.P;
}

// E epochs; SELF: the samples are the weights at each epoch start, else the fixed teacher t
SRNN_HD float g_train_epochs(const GCtx& x, SV w, const SV& t, int E, bool self, TrainCtx& c) {
  const GShape& s = *x.s;
  SV smp = x.v(s.o_t);
  if (!self && smp.p != t.p) g_copy(s, smp, t);
  float loss = 0.f;
  for (int e = 0; e < E; ++e) {
    if (self) g_copy(s, smp, w);
    loss = g_train_epoch(x, w, smp, c);
  }
  return loss;
}

// ---------------------------------------------------------------- predicates
SRNN_HD bool g_diverged(const GShape& s, const SV& w) {
  bool bad = false;
  for (int k = 0; k < s.P; ++k) bad |= !finitef(w[k]);
  return bad;
}
SRNN_HD bool g_zero(const GShape& s, const SV& w, float eps) {
  bool ok = true;
  for (int k = 0; k < s.P; ++k) ok &= (-eps <= w[k]) && (w[k] <= eps);
  return ok;
}
SRNN_HD bool g_within(const GShape& s, const SV& a, const SV& b, float eps) {
  bool ok = true;
  for (int k = 0; k < s.P; ++k) ok &= !(fabsf(a[k] - b[k]) >= eps);
  return ok;
}
// classification of w (reference code/experiment.py:79-91); uses o and f as scratch
SRNN_HD int8_t g_classify_w(const GCtx& x, const SV& w, float eps, bool with_sec, const ApplyCtx& ac) {
  const GShape& s = *x.s;
  if (g_diverged(s, w)) return C_DIVERGENT;
  SV f1 = x.v(s.o_o);
  g_apply(x, w, w, f1, ac);
  g_quant(s, f1);
  if (!g_diverged(s, f1) && g_within(s, f1, w, eps)) return g_zero(s, w, eps) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    SV f2 = x.v(s.o_f);  // g_apply's shuffle uses o_f as its own scratch: stage f2 in o_t
    SV f2b = x.v(s.o_t);
    g_apply(x, w, f1, f2b, ac);
    (void)f2;
    g_quant(s, f2b);
    if (!g_diverged(s, f2b) && g_within(s, f2b, w, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}

// ==================================================================================
// Per-item operators (mirror Item<Net, S> of srnn_kernels.h)
// ==================================================================================
struct GItem {
  SRNN_HD static Rng rng(const SrnnArgs& a) { return Rng{(uint32_t)a.seed, (uint32_t)(a.seed >> 32)}; }
  SRNN_HD static uint64_t uid_of(const SrnnArgs& a, int64_t i) { return a.uid ? (uint64_t)a.uid[i] : (uint64_t)(a.lo + i); }
  SRNN_HD static char* rowp(const GShape& s, float* b, int64_t i) { return reinterpret_cast<char*>(b) + i * g_rb(s); }
  SRNN_HD static const char* rowp(const GShape& s, const float* b, int64_t i) {
    return reinterpret_cast<const char*>(b) + i * g_rb(s);
  }
  SRNN_HD static ApplyCtx actx(const SrnnArgs& a, const GShape& s, uint64_t uid, uint32_t ctr) {
    ApplyCtx x;
    x.rng = rng(a);
    x.uid = uid;
    x.ctr = ctr;
    x.aggregator = s.aggregator;
    x.shuffler = s.shuffler;
    x.perm = nullptr;
    return x;
  }
  SRNN_HD static TrainCtx tctx(const SrnnArgs& a, const GShape& s, uint64_t uid, uint32_t ctr) {
    TrainCtx tc;
    tc.lr = a.lr;
    tc.rng = rng(a);
    tc.uid = uid;
    tc.ctr = ctr;
    tc.samp = nullptr;
    tc.perm = nullptr;
    tc.shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
    tc.stride = 1;
    tc.aggregator = s.aggregator;
    return tc;
  }
  SRNN_HD static void init(const GCtx& x, const SrnnArgs& a, int64_t i) {
    SV w = x.v(x.s->o_w);
    g_init(x, w, rng(a), uid_of(a, i));
    g_store(*x.s, rowp(*x.s, a.W, i), w);
  }
  SRNN_HD static void apply(const GCtx& x, const SrnnArgs& a, int64_t i) {
    const GShape& s = *x.s;
    const int64_t fi = a.idx_f ? a.idx_f[i] : i, ti = a.idx_t ? a.idx_t[i] : i, oi = a.idx_o ? a.idx_o[i] : i;
    SV f = x.v(s.o_w), t = x.v(s.o_t), o = x.v(s.o_o);
    g_load(s, rowp(s, a.W, fi), f);
    g_load(s, rowp(s, a.W, ti), t);
    const uint64_t ouid = a.uid ? (uint64_t)a.uid[ti] : (uint64_t)ti;
    g_apply(x, f, t, o, actx(a, s, ouid, a.ctr));
    g_quant(s, o);
    g_store(s, rowp(s, a.W2, oi), o);
  }
  SRNN_HD static void run_fixpoint(const GCtx& x, const SrnnArgs& a, int64_t i) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w), nw = x.v(s.o_t);
    g_load(s, rowp(s, a.W, i), w);
    ApplyCtx ac = actx(a, s, uid_of(a, i), a.ctr);
    if (a.traj) g_store(s, rowp(s, a.traj, i), w);
    int st = 0;
    for (; st < a.steps; ++st) {
      if (a.early_exit) {
        if (g_diverged(s, w)) break;
        g_apply(x, w, w, nw, ac);
        g_quant(s, nw);
        if (!g_diverged(s, nw) && g_within(s, nw, w, a.eps)) break;
      } else {
        g_apply(x, w, w, nw, ac);
        g_quant(s, nw);
      }
      g_copy(s, w, nw);
      ac.ctr += 1;
      if (a.traj) g_store(s, rowp(s, a.traj, (int64_t)(st + 1) * a.n + i), w);
    }
    g_store(s, rowp(s, a.W, i), w);
    if (a.nsteps) a.nsteps[i] = st;
    if (a.cls) a.cls[i] = g_classify_w(x, w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, ac);
  }
  SRNN_HD static void vary_run(const GCtx& x, const SrnnArgs& a, int64_t i) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w), nw = x.v(s.o_t);
    g_load(s, rowp(s, a.W, i), w);
    ApplyCtx ac = actx(a, s, uid_of(a, i), a.ctr);
    int tts = 0, taf = 0;
    bool still = true;
    for (int st = 0; st < a.steps; ++st) {
      g_apply(x, w, w, nw, ac);
      g_quant(s, nw);
      g_copy(s, w, nw);
      if (g_zero(s, w, a.eps) || g_diverged(s, w)) break;
      g_apply(x, w, w, nw, ac);
      g_quant(s, nw);
      const bool fix = !g_diverged(s, nw) && g_within(s, nw, w, a.eps);
      if (fix) {
        if (still) ++taf;
        else still = true;
      } else {
        still = false;
      }
      ++tts;
    }
    g_store(s, rowp(s, a.W, i), w);
    a.nsteps[i] = tts;
    a.loss[i] = (float)taf;
  }
  SRNN_HD static void perturb(const GCtx& x, const SrnnArgs& a, int64_t i) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w);
    g_load(s, rowp(s, a.W, i), w);
    const Rng r = rng(a);
    const uint64_t uid = uid_of(a, i);
    for (int k = 0; k < s.P; ++k) {
      U4 u = r.draw(uid, a.ctr * 1024u + (uint32_t)k, P_PERTURB);
      double mag = (double)u01(u.y) * (double)a.eps;
      w[k] = u01(u.x) < 0.5f ? (float)((double)w[k] + mag) : (float)((double)w[k] - mag);
    }
    g_store(s, rowp(s, a.W, i), w);
  }
  SRNN_HD static void train(const GCtx& x, const SrnnArgs& a, int64_t i, bool learn) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w), t = x.v(s.o_t);
    g_load(s, rowp(s, a.W, i), w);
    if (learn) g_load(s, rowp(s, a.W2, a.idx_t ? a.idx_t[i] : i), t);
    TrainCtx tc = tctx(a, s, uid_of(a, i), a.ctr);
    const float loss = g_train_epochs(x, w, t, a.epochs, !learn, tc);
    g_store(s, rowp(s, a.W, i), w);
    if (a.loss) a.loss[i] = loss;
  }
  SRNN_HD static int8_t classify(const GCtx& x, const SrnnArgs& a, int64_t i) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w);
    g_load(s, rowp(s, a.W, i), w);
    const int8_t k = g_classify_w(x, w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, actx(a, s, uid_of(a, i), a.ctr));
    if (a.cls) a.cls[i] = k;
    return k;
  }

  // ---------------------------------------------------------------- soup
  // synchronous generation of local row j (Item::soup_evolve): attacks received in
  // ascending attacker-slot order, learn_from, self-train, respawn; tk: the received row of
  // a remote teacher (SRNN_F_X2).  Returns the respawn code.
  SRNN_HD static int8_t soup_evolve(const GCtx& x, const SrnnArgs& a, int64_t j, uint32_t tk = SRNN_NIL) {
    const GShape& s = *x.s;
    const int64_t g = a.lo + j;
    const int64_t rb = g_rb(s);
    SV w = x.v(s.o_w), f = x.v(s.o_t), o = x.v(s.o_o);
    g_load(s, rowp(s, a.W2, j), w);
    const uint64_t uid = (uint64_t)g;  // stream key of this slot (Item::soup_evolve)
    const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
    const bool x2 = (a.flags & SRNN_F_X2) != 0;
    ApplyCtx ac = actx(a, s, uid, (uint32_t)gen * 1024u);
    for_each_attacker<false>(a, j, [&](uint32_t e, int64_t slot) {
      const char* r = ent_row(a, e, rb);
      if (x2 && (int64_t)e >= a.n) x2_check(a, r, rb, slot, gen);
      g_load(s, r, f);
      g_apply(x, f, w, o, ac);
      g_quant(s, o);
      ac.ctr += 1;
      g_copy(s, w, o);
    });
    int64_t my_at, te;
    Item<Weightwise<1, 1>, StF32>::decision(a, g, gen, my_at, te);
    int8_t act = A_NONE;
    int64_t cp = -1;
    if (my_at >= 0) act = A_ATTACKING, cp = my_at;
    TrainCtx tc = tctx(a, s, uid, (uint32_t)gen * 1024u + 512u);
    float loss = 0.f;
    if (te >= 0) {
      const char* r = teacher_row(a, te, tk, rb);
      if (x2 && tk != SRNN_NIL) x2_check(a, r, rb, te, gen);
      g_load(s, r, f);
      if (a.severity > 0) loss = g_train_epochs(x, w, f, a.severity, false, tc);
      act = A_LEARN_FROM;
      cp = te;
    }
    if (a.epochs > 0) {
      loss = g_train_epochs(x, w, f, a.epochs, true, tc);
      act = A_TRAIN_SELF;
      cp = -1;
    }
    g_quant(s, w);
    int8_t rs = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && g_diverged(s, w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && g_zero(s, w, a.eps)) rs = 2;
    if (rs && (a.flags & SRNN_F_RESPAWN_INLINE)) g_init(x, w, rng(a), respawn_key(gen, g));
    g_store(s, rowp(s, a.W, j), w);
    if (a.action) a.action[j] = act;
    if (a.counterpart) a.counterpart[j] = cp;
    if (a.loss) a.loss[j] = loss;
    if (a.respawn) a.respawn[j] = rs;
    return rs;
  }
  // census class of the stored row j (the fused census key: slot, counter 0x7FFFFFF0)
  SRNN_HD static int8_t census_class(const GCtx& x, const SrnnArgs& a, int64_t j) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w);
    g_load(s, rowp(s, a.W, j), w);
    return g_classify_w(x, w, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0, actx(a, s, (uint64_t)(a.lo + j), 0x7FFFFFF0u));
  }
  // sequential (Gauss-Seidel) step of particle j in generation gen (Item::soup_seq_one)
  SRNN_HD static void soup_seq_one(const GCtx& x, const SrnnArgs& a, int64_t j, int32_t gen) {
    const GShape& s = *x.s;
    SV w = x.v(s.o_w), f = x.v(s.o_t), o = x.v(s.o_o);
    int64_t at, te;
    Item<Weightwise<1, 1>, StF32>::decision(a, j, gen, at, te);
    int8_t act = A_NONE;
    int64_t cp = -1;
    if (at >= 0) {  // the victim's weights become f_j(victim)
      g_load(s, rowp(s, a.W, j), w);
      g_load(s, rowp(s, a.W, at), f);
      g_apply(x, w, f, o, actx(a, s, (uint64_t)j, (uint32_t)gen * 1024u + 1u));
      g_quant(s, o);
      g_store(s, rowp(s, a.W, at), o);
      act = A_ATTACKING;
      cp = at;
    }
    g_load(s, rowp(s, a.W, j), w);
    TrainCtx tc = tctx(a, s, (uint64_t)j, (uint32_t)gen * 1024u + 512u);
    float loss = 0.f;
    if (te >= 0) {
      g_load(s, rowp(s, a.W, te), f);
      if (a.severity > 0) loss = g_train_epochs(x, w, f, a.severity, false, tc);
      act = A_LEARN_FROM;
      cp = te;
    }
    if (a.epochs > 0) {
      loss = g_train_epochs(x, w, f, a.epochs, true, tc);
      act = A_TRAIN_SELF;
      cp = -1;
    }
    g_quant(s, w);
    int8_t rs = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && g_diverged(s, w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && g_zero(s, w, a.eps)) rs = 2;
    if (a.W2) g_store(s, rowp(s, a.W2, j), w);  // recording: the state before any respawn
    if (rs) g_init(x, w, rng(a), respawn_key(gen, j));
    g_store(s, rowp(s, a.W, j), w);
    if (a.action) a.action[j] = act;
    if (a.counterpart) a.counterpart[j] = (a.W2 && cp >= 0) ? a.uid_out[cp] : cp;
    if (a.loss) a.loss[j] = loss;
    if (a.respawn) a.respawn[j] = rs;
  }
  SRNN_HD static void respawn(const GCtx& x, const SrnnArgs& a, int64_t j) {
    if (a.respawn[j] == 0) return;
    SV w = x.v(x.s->o_w);
    const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
    g_init(x, w, rng(a), respawn_key(gen, a.lo + j));
    g_store(*x.s, rowp(*x.s, a.W, j), w);
  }
};

// ==================================================================================
// Device kernels (grid-stride, lane per row; scratch element-major over all lanes)
// ==================================================================================
constexpr int GOP_CLASSIFY_COUNT = 100, GOP_EVOLVE = 101, GOP_X2_REMOTE = 102;

template <int OP>
__global__ __launch_bounds__(GTB) void k_generic(GShape s, SrnnArgs a, int64_t lanes) {
  extern __shared__ float s_coords[];
  __shared__ uint32_t s_cnt[6];
  if (s.kind == 0) make_coords_dev(s, s_coords);
  if (threadIdx.x < 6) s_cnt[threadIdx.x] = 0;
  const int64_t lane_id = (int64_t)blockIdx.x * GTB + threadIdx.x;
  GCtx x{&s, reinterpret_cast<float*>(a.scratch) + lane_id, lanes, s_coords, g_orth(s, a.scratch, lanes, lane_id)};
  const int64_t stride = (int64_t)gridDim.x * GTB;
  const int64_t items = OP == GOP_X2_REMOTE ? (int64_t)*(volatile const int32_t*)a.x_rcount : a.n;
  for (int64_t base = (int64_t)blockIdx.x * GTB; base < items; base += stride) {
    const int64_t i = base + threadIdx.x;
    const bool on = i < items;
    if constexpr (OP == OP_INIT) {
      if (on) GItem::init(x, a, i);
    } else if constexpr (OP == OP_APPLY) {
      if (on) GItem::apply(x, a, i);
    } else if constexpr (OP == OP_RUN_FIXPOINT) {
      if (on) GItem::run_fixpoint(x, a, i);
    } else if constexpr (OP == OP_TRAIN || OP == OP_LEARN) {
      if (on) GItem::train(x, a, i, OP == OP_LEARN);
    } else if constexpr (OP == OP_PERTURB) {
      if (on) GItem::perturb(x, a, i);
    } else if constexpr (OP == OP_VARY_RUN) {
      if (on) GItem::vary_run(x, a, i);
    } else if constexpr (OP == OP_RESPAWN) {
      if (on) GItem::respawn(x, a, i);
    } else if constexpr (OP == OP_CLASSIFY || OP == GOP_CLASSIFY_COUNT) {
      int8_t k = on ? GItem::classify(x, a, i) : (int8_t)-1;
      if constexpr (OP == GOP_CLASSIFY_COUNT) {
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          const unsigned long long m = __ballot(k == q);
          if (threadIdx.x == 0 && m) s_cnt[q] += (uint32_t)__popcll(m);
        }
        if (a.flags & SRNN_F_COUNT_RESPAWNS) {
          const unsigned long long m = __ballot(on && a.respawn[i] != 0);
          if (threadIdx.x == 0) s_cnt[5] += (uint32_t)__popcll(m);
        }
      }
    } else if constexpr (OP == GOP_EVOLVE) {
      // single rank / all-gather: 64-row ballots (or per-row flags); X2 local: the rows that
      // need no remote row (x_dep), block stats by atomics (srnn_kernels.h bs_publish_*)
      const bool x2 = (a.flags & SRNN_F_X2) != 0;
      const bool act = on && !(x2 && x2_dep(a, i));
      bool rs = false;
      int8_t k = -1;
      if (act) {
        rs = GItem::soup_evolve(x, a, i) != 0;
        if (x2 && (a.flags & SRNN_F_FUSED_CENSUS)) k = GItem::census_class(x, a, i);
      }
      if (x2) {
        const int64_t wd = (base / GTB) * 2 + threadIdx.x;
        if (threadIdx.x < 2 && wd * 32 < a.n) a.x_dep[wd] = 0u;
        bs_publish_wave(reinterpret_cast<unsigned long long*>(a.temp), base / GTB, rs, k);
      } else if (a.flags & SRNN_F_ROW_FLAGS) {
        if (on && a.rowflags) a.rowflags[i] = rs ? 1 : 0;
      } else if (a.ballots) {
        const unsigned long long m = __ballot(rs);  // the 64 rows of this block: one ballot word
        if (threadIdx.x == 0) a.ballots[base / GTB] = m;
      }
    } else if constexpr (OP == GOP_X2_REMOTE) {
      // items = the remote-dependent list (x_rlist, length x_rcount on the device)
      if (on) {
        const int64_t j = a.x_rlist[2 * i];
        const bool rs = GItem::soup_evolve(x, a, j, a.x_rlist[2 * i + 1]) != 0;
        const int8_t k = (a.flags & SRNN_F_FUSED_CENSUS) ? GItem::census_class(x, a, j) : (int8_t)-1;
        bs_publish_lane(reinterpret_cast<unsigned long long*>(a.temp), j, rs, k);
      }
    }
  }
  if constexpr (OP == GOP_X2_REMOTE) {
    int32_t prev = 0;
    if (threadIdx.x == 0) prev = atomicAdd(a.x_ctl + 3, 1);
    prev = __shfl(prev, 0);
    if (prev == (int32_t)gridDim.x - 1 && threadIdx.x == 0) {
      *a.x_rcount = 0;
      a.x_ctl[3] = 0;
    }
  }
  if constexpr (OP == GOP_CLASSIFY_COUNT) {
    if (threadIdx.x < 6 && s_cnt[threadIdx.x] && (threadIdx.x < 5 || (a.flags & SRNN_F_COUNT_RESPAWNS)))
      atomicAdd(a.counts + threadIdx.x, (uint64_t)s_cnt[threadIdx.x]);
    if ((a.flags & SRNN_F_GEN_ADVANCE) && blockIdx.x == 0 && threadIdx.x == 0) {
      if (a.gen_out) a.gen_out[0] = a.gen_ptr[0] + 1;
      else ((int32_t*)a.gen_ptr)[0] = a.gen_ptr[0] + 1;
    }
  }
}

// Single-rank respawn (k_respawn_seq with runtime shapes): one workgroup scans the 64-row
// respawn ballots in slot order, assigns the uids, re-initialises the rows, advances
// next_uid and the generation counter.
constexpr int GTBR = 1024;
__global__ __launch_bounds__(GTBR) void k_g_respawn_seq(GShape s, SrnnArgs a) {
  __shared__ int32_t s_wave[GTBR / 64];
  const unsigned long long* masks = a.ballots;
  const int64_t nb = (a.n + GTB - 1) / GTB, ch = (nb + GTBR - 1) / GTBR;
  const int64_t b0 = (int64_t)threadIdx.x * ch, b1 = b0 + ch < nb ? b0 + ch : nb;
  int32_t cnt = 0;
  for (int64_t b = b0; b < b1; ++b) cnt += __popcll(masks[b]);
  int32_t total;
  const int32_t incl = block_incl_scan<GTBR>(cnt, s_wave, &total);
  const int64_t base = *(volatile const int64_t*)a.uid_base;
  GCtx x{&s, reinterpret_cast<float*>(a.scratch) + threadIdx.x, GTBR, nullptr, g_orth(s, a.scratch, GTBR, threadIdx.x)};
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  int64_t k = base + incl - cnt;
  for (int64_t b = b0; b < b1 && cnt; ++b) {
    unsigned long long m = masks[b];
    while (m) {
      const int bit = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int64_t r = b * GTB + bit;
      a.uid_out[r] = k++;
      if (a.flags & SRNN_F_RESPAWN_INLINE) continue;  // re-initialised inline by the evolve kernel
      SV w = x.v(s.o_w);
      g_init(x, w, GItem::rng(a), respawn_key(gen, a.lo + r));
      g_store(s, GItem::rowp(s, a.W, r), w);
    }
  }
  // the ballots are consumed (the lanes-per-particle soup kernel ORs its respawns into them)
  for (int64_t b = b0; b < b1; ++b) a.ballots[b] = 0ull;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.uid_base[0] = base + total;
    if (a.gen_out) a.gen_out[0] = gen + 1;
    else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = gen + 1;
  }
  if (a.counts && threadIdx.x < 5) a.counts[threadIdx.x] = 0;
}

// ==================================================================================
// Host execution (thread pool; per-thread scratch) and dispatch
// ==================================================================================
static void host_generic(int op, const GShape& s, const SrnnArgs& a) {
  std::vector<float> coords((size_t)(3 * s.P + 3));
  if (s.kind == 0) make_coords_host(s, coords.data());
  auto with_ctx = [&](auto&& f) {
    return [&, f](int64_t i) {
      thread_local std::vector<float> buf;
      thread_local std::vector<double> orth;
      if (buf.size() < (size_t)s.sfloats) buf.resize((size_t)s.sfloats);
      if (orth.size() < (size_t)s.orthd + 1) orth.resize((size_t)s.orthd + 1);
      GCtx x{&s, buf.data(), 1, coords.data(), orth.data()};
      f(x, i);
    };
  };
  switch (op) {
    case OP_INIT: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::init(x, a, i); })); break;
    case OP_APPLY: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::apply(x, a, i); })); break;
    case OP_RUN_FIXPOINT:
      host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::run_fixpoint(x, a, i); }));
      break;
    case OP_TRAIN: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::train(x, a, i, false); })); break;
    case OP_LEARN: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::train(x, a, i, true); })); break;
    case OP_PERTURB: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::perturb(x, a, i); })); break;
    case OP_VARY_RUN: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::vary_run(x, a, i); })); break;
    case OP_RESPAWN: host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::respawn(x, a, i); })); break;
    case OP_SOUP_EVOLVE: {
      if (a.flags & SRNN_F_X2) {
        const bool census = (a.flags & SRNN_F_FUSED_CENSUS) != 0;
        unsigned long long* bs = reinterpret_cast<unsigned long long*>(a.temp);
        if (a.flags & SRNN_F_X2_REMOTE) {
          host_parallel(*a.x_rcount, with_ctx([&](const GCtx& x, int64_t q) {
            const int64_t j = a.x_rlist[2 * q];
            const bool rs = GItem::soup_evolve(x, a, j, a.x_rlist[2 * q + 1]) != 0;
            bs_publish_host(bs, j, rs, census ? GItem::census_class(x, a, j) : (int8_t)-1);
          }));
          *a.x_rcount = 0;
        } else {
          host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) {
            if (x2_dep(a, i)) return;
            const bool rs = GItem::soup_evolve(x, a, i) != 0;
            bs_publish_host(bs, i, rs, census ? GItem::census_class(x, a, i) : (int8_t)-1);
          }));
          for (int64_t w = 0; w < (a.n + 31) / 32; ++w) a.x_dep[w] = 0u;
        }
        break;
      }
      host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { GItem::soup_evolve(x, a, i); }));
      if ((a.flags & SRNN_F_ROW_FLAGS) && a.rowflags) {
        for (int64_t i = 0; i < a.n; ++i) a.rowflags[i] = a.respawn[i] != 0 ? 1 : 0;
      } else if (a.ballots) {
        for (int64_t b = 0; b < (a.n + GTB - 1) / GTB; ++b) {
          unsigned long long m = 0;
          for (int64_t i = b * GTB; i < a.n && i < (b + 1) * GTB; ++i)
            if (a.respawn[i]) m |= 1ull << (i - b * GTB);
          a.ballots[b] = m;
        }
      }
      break;
    }
    case OP_SOUP_SEQ: {
      // sequential soups of runtime shapes (Item soup_seq): serial by definition, host only
      std::vector<float> buf((size_t)s.sfloats);
      std::vector<double> orth((size_t)s.orthd + 1);
      GCtx x{&s, buf.data(), 1, coords.data(), orth.data()};
      const int32_t gen0 = a.gen_ptr ? a.gen_ptr[0] : a.gen;
      int64_t next = a.uid_base[0];
      for (int32_t st = 0; st < a.steps; ++st)
        for (int64_t j = 0; j < a.n; ++j) {
          GItem::soup_seq_one(x, a, j, gen0 + st);
          if (a.respawn && a.respawn[j]) a.uid_out[j] = next++;
        }
      a.uid_base[0] = next;
      if (a.gen_out) a.gen_out[0] = gen0 + a.steps;
      else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = gen0 + a.steps;
      break;
    }
    case OP_CLASSIFY: {
      std::vector<int8_t> ks((size_t)a.n);
      host_parallel(a.n, with_ctx([&](const GCtx& x, int64_t i) { ks[(size_t)i] = GItem::classify(x, a, i); }));
      if (a.counts) {
        uint64_t local[5] = {0, 0, 0, 0, 0};
        for (int64_t i = 0; i < a.n; ++i) local[ks[(size_t)i]]++;
        for (int q = 0; q < 5; ++q) a.counts[q] += local[q];
        if (a.flags & SRNN_F_COUNT_RESPAWNS)
          for (int64_t i = 0; i < a.n; ++i) a.counts[5] += a.respawn[i] != 0;
        if (a.flags & SRNN_F_GEN_ADVANCE) {
          if (a.gen_out) a.gen_out[0] = a.gen_ptr[0] + 1;
          else ((int32_t*)a.gen_ptr)[0] = a.gen_ptr[0] + 1;
        }
      }
      break;
    }
    case OP_RESPAWN_SEQ: {
      std::vector<float> buf((size_t)s.sfloats);
      std::vector<double> orth((size_t)s.orthd + 1);
      GCtx x{&s, buf.data(), 1, coords.data(), orth.data()};
      int64_t k = a.uid_base[0];
      const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
      for (int64_t i = 0; i < a.n; ++i) {
        if (a.respawn[i] == 0) continue;
        a.uid_out[i] = k++;
        if (a.flags & SRNN_F_RESPAWN_INLINE) continue;  // re-initialised inline by the evolve
        SV w = x.v(s.o_w);
        g_init(x, w, GItem::rng(a), respawn_key(gen, a.lo + i));
        g_store(s, GItem::rowp(s, a.W, i), w);
      }
      a.uid_base[0] = k;
      if (a.gen_out) a.gen_out[0] = gen + 1;
      else if (a.gen_ptr) ((int32_t*)a.gen_ptr)[0] = gen + 1;
      if (a.counts)
        for (int q = 0; q < 5; ++q) a.counts[q] = 0;
      break;
    }
    default: break;
  }
}

// ==================================================================================
// Long recurrent nets, wave per particle (the analogue of long context is the
// sequence length P of a Recurrent net -- its own weight vector).  The lane-per-particle
// path above streams every weight and state of a wide net through its element-major
// scratch on every multiply (RecurrentNeuralNetwork(16, 2), P = 801: 30M BPTT timesteps/s).
// Here one 64-lane wave owns a particle: the weights, the gradient accumulators and the
// input sequence live in LDS (3P floats), lane j computes unit j of a layer, the hidden
// state is double-buffered in LDS (one wave barrier per layer and timestep), and the
// per-timestep states needed by BPTT go to a per-wave region of device scratch (written
// forward, read backward, coalesced).  Every dot product keeps the lane path's order (x[0]*k
// then fma over the inputs; BPTT sums over j from 0), so results equal the lane path's.
// ==================================================================================
constexpr int RW_MIN_WIDTH = 8;  // narrower nets stay lane per particle (64 particles per wave)

struct RWave {
  float* w;      // [P] the net's weights
  float* aux;    // [P] gradient accumulators / application output
  float* seq;    // [P] input sequence (samples / target weights)
  float* h0;     // [HS] hidden state, double-buffered
  float* h1;
  float* carry;  // [HS]
  float* dtop;   // [64]
  float* dh;     // [64]
  float* hst;    // [HS] staged states of timestep t and t - 1 (BPTT)
  float* hsp;
};
__device__ __forceinline__ RWave rw_layout(const GShape& s, float* sm) {
  RWave r;
  r.w = sm;
  r.aux = r.w + s.P;
  r.seq = r.aux + s.P;
  r.h0 = r.seq + s.P;
  r.h1 = r.h0 + s.HS;
  r.carry = r.h1 + s.HS;
  r.hst = r.carry + s.HS;
  r.hsp = r.hst + s.HS;
  r.dtop = r.hsp + s.HS;
  r.dh = r.dtop + 64;
  return r;
}
static inline size_t rw_lds_bytes(const GShape& s) { return ((size_t)3 * s.P + 6 * s.HS + 128) * sizeof(float); }
__device__ __forceinline__ void rw_sync() { __syncthreads(); }  // one-wave workgroup: orders LDS

// acc = x[0]*k[0] then fma over i (mul_first), or fma over i from acc; k strided by ks.  The
// LDS loads of 8 terms are issued together before their (ordered) fma chain: the same
// rounding as the plain loop, without one LDS round trip per multiply-add
__device__ __forceinline__ float rw_dot(const float* x, const float* k, int ks, int n, bool mul_first, float acc) {
  int i = 0;
  if (mul_first && n > 0) {
    acc = x[0] * k[0];
    i = 1;
  }
  for (; i < n; i += 8) {
    float xv[8], kv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i + u < n) xv[u] = x[i + u], kv[u] = k[(i + u) * ks];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i + u < n) acc = fmaf(xv[u], kv[u], acc);
  }
  return acc;
}

// Layer geometry of a SimpleRNN stack from (width, depth) alone (make_gshape's kind-2 tables
// in closed form): compile-time when the kernel is instantiated for one width / depth, so the
// layer and dot-product loops unroll and the ~420 SALU instructions per timestep of table
// lookups and loop control of the runtime-shape form (profiles/r2h_long_recurrent_wave.md)
// go away; WT = DT = 0 is the runtime-shape instantiation (same formulas, runtime W / D).
template <int WT, int DT>
struct RD {
  int w_, d_;
  __device__ explicit RD(const GShape& s) : w_(WT ? WT : s.W), d_(DT ? DT : s.D) {}
  __device__ __forceinline__ int W() const { return WT ? WT : w_; }
  __device__ __forceinline__ int D() const { return DT ? DT : d_; }
  __device__ __forceinline__ int NL() const { return D() + 1; }
  __device__ __forceinline__ int in_(int L) const { return L == 0 ? 1 : W(); }
  __device__ __forceinline__ int un(int L) const { return L == D() ? 1 : W(); }
  __device__ __forceinline__ int koff(int L) const { return L == 0 ? 0 : W() + W() * W() + (L - 1) * 2 * W() * W(); }
  __device__ __forceinline__ int roff(int L) const { return koff(L) + in_(L) * un(L); }
  __device__ __forceinline__ int P() const { return koff(D()) + W() + 1; }
  __device__ __forceinline__ int HS() const { return D() * W() + 1; }
};

// forward over the sequence: y_t = h_D[t][0]; states to hs (global, [P][HS]) and/or the
// outputs to out (LDS, [P]) when given
template <int WT, int DT>
__device__ void rw_forward(const GShape& s, const RWave& r, const float* wts, const float* seq, float* hs,
                           float* out) {
  const RD<WT, DT> d(s);
  const int lane = threadIdx.x;
  float* hc = r.h0;  // time t
  float* hp = r.h1;  // time t - 1
  for (int q = lane; q < d.HS(); q += 64) hc[q] = 0.f, hp[q] = 0.f;
  rw_sync();
  for (int t = 0; t < d.P(); ++t) {
    const float x0 = seq[t];
#pragma unroll
    for (int L = 0; L < (DT ? DT + 1 : d.NL()); ++L) {
      const int I = d.in_(L), U = d.un(L);
      float hn = 0.f;
      if (lane < U) {
        const float* K = wts + d.koff(L);
        const float* R = wts + d.roff(L);
        // layer L-1 at time t (this timestep), or the scalar input
        const float xk = L == 0 ? x0 * K[lane] : rw_dot(hc + (L - 1) * d.W(), K + lane, U, I, true, 0.f);
        const float hr = rw_dot(hp + L * d.W(), R + lane, U, U, true, 0.f);
        hn = xk + hr;
      }
      if (lane < U) hc[L * d.W() + lane] = hn;
      rw_sync();
    }
    if (hs)
      for (int q = lane; q < d.HS(); q += 64) hs[(int64_t)t * d.HS() + q] = hc[q];
    if (out && lane == 0) out[t] = hc[d.D() * d.W()];
    float* tmp = hc;  // h(t) becomes h(t - 1); the old buffer is overwritten layer by layer
    hc = hp;
    hp = tmp;
    rw_sync();
  }
}

// one self-train / learn epoch (g_train_epoch, recurrent branch): forward with states, BPTT,
// one SGD step; returns the loss (mean over timesteps)
template <int WT, int DT>
__device__ float rw_train_epoch(const GShape& s, const RWave& r, float* hs, float lr) {
  const RD<WT, DT> d(s);
  const int lane = threadIdx.x;
  rw_forward<WT, DT>(s, r, r.w, r.seq, hs, nullptr);
  // the states are read back by other lanes of this wave: the stores are at L2 after the
  // wait, and the reads below are memory-side (L2) loads -- never a stale L1 line left by the
  // previous particle's pass over the same region
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* gw = r.aux;
  const int P = d.P(), HS = d.HS(), Wd = d.W();
  // specialised widths up to 16: lane j's gradient column of every layer in registers (<= 98
  // floats at RNN(16, 3)) instead of an LDS read-modify-write per multiply-add; the same fma
  // sequence per element, so the result is the LDS form's
  constexpr bool REG = WT > 0 && (WT <= 16 || DT == 2);
  constexpr int RL = REG ? DT + 1 : 1, RW = REG ? WT : 1;
  float ak[RL][RW], ar[RL][RW];
  if constexpr (REG) {
#pragma unroll
    for (int L = 0; L < RL; ++L)
#pragma unroll
      for (int i = 0; i < RW; ++i) ak[L][i] = 0.f, ar[L][i] = 0.f;
  }
  for (int k = lane; k < P; k += 64) gw[k] = 0.f;
  for (int q = lane; q < HS; q += 64) r.carry[q] = 0.f;
  rw_sync();
  float loss = 0.f;
  for (int t = P - 1; t >= 0; --t) {
    for (int q = lane; q < HS; q += 64) {
      r.hst[q] = __hip_atomic_load(hs + (int64_t)t * HS + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.hsp[q] = t > 0 ? __hip_atomic_load(hs + (int64_t)(t - 1) * HS + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0.f;
    }
    rw_sync();
    const float e = r.hst[d.D() * Wd] - r.seq[t];
    loss += e * e;
    if (lane == 0) r.dtop[0] = 2.0f * e / (float)P;
    rw_sync();
#pragma unroll
    for (int L = (DT ? DT : d.D()); L >= 0; --L) {
      const int U = d.un(L), I = d.in_(L);
      float dhj = 0.f;
      if (lane < U) dhj = r.dtop[lane] + r.carry[L * Wd + lane];
      if (lane < U) r.dh[lane] = dhj;
      rw_sync();
      if (lane < U) {  // kernel / recurrent-kernel gradients of column j = lane
        if constexpr (REG) {
#pragma unroll
          for (int i = 0; i < I; ++i) ak[L][i] = fmaf(L == 0 ? r.seq[t] : r.hst[(L - 1) * Wd + i], dhj, ak[L][i]);
#pragma unroll
          for (int i = 0; i < U; ++i) ar[L][i] = fmaf(r.hsp[L * Wd + i], dhj, ar[L][i]);
        } else {
          for (int i = 0; i < I; ++i) {
            const float xi = L == 0 ? r.seq[t] : r.hst[(L - 1) * Wd + i];
            float* gk = gw + d.koff(L) + i * U + lane;
            *gk = fmaf(xi, dhj, *gk);
          }
          for (int i = 0; i < U; ++i) {
            float* gr = gw + d.roff(L) + i * U + lane;
            *gr = fmaf(r.hsp[L * Wd + i], dhj, *gr);
          }
        }
      }
      float dxi = 0.f, cri = 0.f;
      if (L > 0 && lane < I) dxi = rw_dot(r.dh, r.w + d.koff(L) + lane * U, 1, U, false, 0.f);
      if (lane < U) cri = rw_dot(r.dh, r.w + d.roff(L) + lane * U, 1, U, false, 0.f);
      rw_sync();
      if (lane < U) r.carry[L * Wd + lane] = cri;
      if (L > 0 && lane < I) r.dtop[lane] = dxi;
      rw_sync();
    }
  }
  if constexpr (REG) {
#pragma unroll
    for (int L = 0; L < RL; ++L) {
      const int U = d.un(L), I = d.in_(L);
      if (lane < U) {
#pragma unroll
        for (int i = 0; i < I; ++i) gw[d.koff(L) + i * U + lane] = ak[L][i];
#pragma unroll
        for (int i = 0; i < U; ++i) gw[d.roff(L) + i * U + lane] = ar[L][i];
      }
    }
    rw_sync();
  }
  for (int k = lane; k < P; k += 64) r.w[k] = fmaf(gw[k], -lr, r.w[k]);
  rw_sync();
  return loss / (float)P;
}

__device__ __forceinline__ bool rw_all(bool b) { return __ballot(!b) == 0ull; }
__device__ bool rw_diverged(const GShape& s, const float* v) {
  bool bad = false;
  for (int k = threadIdx.x; k < s.P; k += 64) bad |= !finitef(v[k]);
  return !rw_all(!bad);
}
__device__ bool rw_within(const GShape& s, const float* a, const float* b, float eps) {
  bool ok = true;
  for (int k = threadIdx.x; k < s.P; k += 64) ok &= !(fabsf(a[k] - b[k]) >= eps);
  return rw_all(ok);
}
__device__ bool rw_zero(const GShape& s, const float* v, float eps) {
  bool ok = true;
  for (int k = threadIdx.x; k < s.P; k += 64) ok &= (-eps <= v[k]) && (v[k] <= eps);
  return rw_all(ok);
}
__device__ void rw_load(const GShape& s, const char* row, float* dst) {
  for (int k = threadIdx.x; k < s.P; k += 64) dst[k] = g_dec(row, k, s.dtype);
}
__device__ void rw_store(const GShape& s, char* row, const float* src) {
  for (int k = threadIdx.x; k < s.PP; k += 64) {
    const float v = k < s.P ? src[k] : 0.f;
    if (s.dtype == 0) reinterpret_cast<float*>(row)[k] = v;
    else reinterpret_cast<uint16_t*>(row)[k] = s.dtype == 1 ? StBF16::enc(v) : StF16::enc(v);
  }
}
__device__ void rw_quant(const GShape& s, float* v) {
  if (s.dtype != 0)
    for (int k = threadIdx.x; k < s.P; k += 64) v[k] = g_q(v[k], s.dtype);
}

// classification (g_classify_w): f1 = apply(w, w), f2 = apply(w, f1); uses aux and seq
template <int WT, int DT>
__device__ int8_t rw_classify(const GShape& s, const RWave& r, float eps, bool with_sec) {
  if (rw_diverged(s, r.w)) return C_DIVERGENT;
  float* f1 = r.aux;
  rw_forward<WT, DT>(s, r, r.w, r.w, nullptr, f1);
  rw_quant(s, f1);
  rw_sync();
  if (!rw_diverged(s, f1) && rw_within(s, f1, r.w, eps)) return rw_zero(s, r.w, eps) ? C_FIX_ZERO : C_FIX_OTHER;
  if (with_sec) {
    float* f2 = r.seq;
    rw_forward<WT, DT>(s, r, r.w, f1, nullptr, f2);
    rw_quant(s, f2);
    rw_sync();
    if (!rw_diverged(s, f2) && rw_within(s, f2, r.w, eps)) return C_FIX_SEC;
  }
  return C_OTHER;
}

template <int OP, int WT, int DT>
__global__ __launch_bounds__(64) void k_rnn_wave(GShape s, SrnnArgs a) {
  extern __shared__ float sm[];
  const RWave r = rw_layout(s, sm);
  const int lane = threadIdx.x;
  float* hs = reinterpret_cast<float*>(a.scratch) + (int64_t)blockIdx.x * s.P * s.HS;
  for (int64_t i = blockIdx.x; i < a.n; i += gridDim.x) {
    if constexpr (OP == OP_APPLY) {
      const int64_t fi = a.idx_f ? a.idx_f[i] : i, ti = a.idx_t ? a.idx_t[i] : i, oi = a.idx_o ? a.idx_o[i] : i;
      rw_load(s, GItem::rowp(s, a.W, fi), r.w);
      rw_load(s, GItem::rowp(s, a.W, ti), r.seq);
      rw_sync();
      rw_forward<WT, DT>(s, r, r.w, r.seq, nullptr, r.aux);
      rw_quant(s, r.aux);
      rw_sync();
      rw_store(s, GItem::rowp(s, a.W2, oi), r.aux);
    } else if constexpr (OP == OP_TRAIN || OP == OP_LEARN) {
      rw_load(s, GItem::rowp(s, a.W, i), r.w);
      if (OP == OP_LEARN) rw_load(s, GItem::rowp(s, a.W2, a.idx_t ? a.idx_t[i] : i), r.seq);
      rw_sync();
      float loss = 0.f;
      for (int e = 0; e < a.epochs; ++e) {
        if (OP == OP_TRAIN) {  // samples = the weights at the epoch start
          for (int k = lane; k < s.P; k += 64) r.seq[k] = r.w[k];
          rw_sync();
        }
        loss = rw_train_epoch<WT, DT>(s, r, hs, a.lr);
      }
      rw_store(s, GItem::rowp(s, a.W, i), r.w);
      if (a.loss && lane == 0) a.loss[i] = loss;
    } else if constexpr (OP == OP_RUN_FIXPOINT) {
      rw_load(s, GItem::rowp(s, a.W, i), r.w);
      rw_sync();
      int st = 0;
      for (; st < a.steps; ++st) {
        if (a.early_exit && rw_diverged(s, r.w)) break;
        rw_forward<WT, DT>(s, r, r.w, r.w, nullptr, r.aux);
        rw_quant(s, r.aux);
        rw_sync();
        if (a.early_exit && !rw_diverged(s, r.aux) && rw_within(s, r.aux, r.w, a.eps)) break;
        for (int k = lane; k < s.P; k += 64) r.w[k] = r.aux[k];
        rw_sync();
      }
      rw_store(s, GItem::rowp(s, a.W, i), r.w);
      if (a.nsteps && lane == 0) a.nsteps[i] = st;
      if (a.cls) {
        const int8_t k = rw_classify<WT, DT>(s, r, a.eps, (a.flags & SRNN_F_FIX_SEC) != 0);
        if (lane == 0) a.cls[i] = k;
      }
    }
    rw_sync();
  }
}

// per-workgroup device scratch of the wave soup: BPTT states (P x HS floats, padded to a
// double) + the orthogonal-init matrix of an inline respawn (W x W doubles)
SRNN_HD int64_t rw_soup_scratch_bytes(const GShape& s) {
  const int64_t hsf = ((int64_t)s.P * s.HS + 1) & ~(int64_t)1;
  return hsf * 4 + (int64_t)s.W * s.W * 8;
}

// Soup generation of the single-rank runtime-shape engine for wide Recurrent nets, one wave per
// particle, in GItem::soup_evolve's order: attacks received in ascending attacker-slot order
// (attacker net over the victim's weight sequence, quantised), decision, learn_from the
// teacher's generation-start row, self-train, respawn (inline re-init on lane 0 with the lane
// path's g_init); respawn flags per row (SRNN_F_ROW_FLAGS) or OR-ed into the 64-row ballots
// (zeroed by their consumer, k_g_respawn_seq)
template <int WT, int DT>
__global__ __launch_bounds__(64) void k_rnn_wave_soup(GShape s, SrnnArgs a) {
  extern __shared__ float sm[];
  const RWave r = rw_layout(s, sm);
  const int lane = threadIdx.x;
  char* scr = reinterpret_cast<char*>(a.scratch) + (int64_t)blockIdx.x * rw_soup_scratch_bytes(s);
  float* hs = reinterpret_cast<float*>(scr);
  double* orth = reinterpret_cast<double*>(scr + (((int64_t)s.P * s.HS + 1) & ~(int64_t)1) * 4);
  const int64_t rb = g_rb(s);
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  __shared__ uint32_t s_be;
  for (int64_t j = blockIdx.x; j < a.n; j += gridDim.x) {
    const int64_t gs = a.lo + j;
    rw_load(s, GItem::rowp(s, a.W2, j), r.w);
    const uint32_t head = a.heads[j];
    uint64_t last = 0;
    bool first = true;
    for (;;) {  // 1. attacks
      if (lane == 0) {
        uint32_t be = SRNN_NIL;
        if (head != SRNN_NIL) {
          uint64_t best = ~0ull;
          for (uint32_t e = head; e != SRNN_NIL; e = a.nexts[e]) {
            const uint64_t sl = ent_slot(a, e);
            if ((first || sl > last) && sl < best) best = sl, be = e;
          }
          if (be != SRNN_NIL) last = best, first = false;
        }
        s_be = be;
      }
      rw_sync();
      const uint32_t be = s_be;
      if (be == SRNN_NIL) break;
      rw_load(s, ent_row(a, be, rb), r.seq);  // the attacker's weights
      rw_sync();
      rw_forward<WT, DT>(s, r, r.seq, r.w, nullptr, r.aux);
      rw_quant(s, r.aux);
      rw_sync();
      for (int k = lane; k < s.P; k += 64) r.w[k] = r.aux[k];
      rw_sync();
    }
    if (lane == 0 && head != SRNN_NIL) a.heads[j] = SRNN_NIL;  // consumed
    // 2. decision, learn_from, self-train
    int64_t my_at = -1, te = -1;
    Item<Weightwise<1, 1>, StF32>::decision(a, gs, gen, my_at, te);
    int8_t act = my_at >= 0 ? A_ATTACKING : A_NONE;
    int64_t cp = my_at >= 0 ? my_at : -1;
    float loss = 0.f;
    if (te >= 0) {
      rw_load(s, teacher_row(a, te, SRNN_NIL, rb), r.seq);
      rw_sync();
      for (int e = 0; e < a.severity; ++e) loss = rw_train_epoch<WT, DT>(s, r, hs, a.lr);
      act = A_LEARN_FROM;
      cp = te;
    }
    if (a.epochs > 0) {
      for (int e = 0; e < a.epochs; ++e) {
        for (int k = lane; k < s.P; k += 64) r.seq[k] = r.w[k];
        rw_sync();
        loss = rw_train_epoch<WT, DT>(s, r, hs, a.lr);
      }
      act = A_TRAIN_SELF;
      cp = -1;
    }
    // 3. respawn
    rw_quant(s, r.w);
    rw_sync();
    int8_t rs = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && rw_diverged(s, r.w)) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && rw_zero(s, r.w, a.eps)) rs = 2;
    if (rs && (a.flags & SRNN_F_RESPAWN_INLINE)) {
      if (lane == 0) {
        const GCtx x{&s, nullptr, 1, nullptr, orth};
        g_init(x, SV{r.w, 1}, GItem::rng(a), respawn_key(gen, gs));
      }
      rw_sync();
    }
    rw_store(s, GItem::rowp(s, a.W, j), r.w);
    if (lane == 0) {
      if (a.action) a.action[j] = act;
      if (a.counterpart) a.counterpart[j] = cp;
      if (a.loss) a.loss[j] = loss;
      if (a.respawn) a.respawn[j] = rs;
      if (a.flags & SRNN_F_ROW_FLAGS) {
        if (a.rowflags) a.rowflags[j] = rs ? 1 : 0;
      } else if (a.ballots && rs) {
        atomicOr(a.ballots + (j >> 6), 1ull << (j & 63));
      }
    }
    rw_sync();
  }
}

// recurrent nets at least RW_MIN_WIDTH wide whose three P-vectors fit a workgroup's LDS run
// apply / train / learn / run_fixpoint (no trajectory) wave per particle
// knob SRNN_KNOB_RNN_WAVE = 0: lane path for every width (A/B tests)
extern "C" void srnn_set_rnn_wave(int on) { srnn_set_knob(SRNN_KNOB_RNN_WAVE, on ? 1 : 0); }
// width / depth-specialised instantiations (RNN(8|16|32, 2), RNN(8|16, 3); RNN(32, 3) fully
// unrolled spills past 256 VGPRs and stays runtime-shape); 0: the runtime-shape kernel
// for every shape (A/B tests, SRNN_RNN_SPEC=0)
extern "C" void srnn_set_rnn_spec(int on) { srnn_set_knob(SRNN_KNOB_RNN_SPEC, on ? 1 : 0); }
// wave-per-particle soup generations of wide Recurrent nets (knob SRNN_KNOB_RNN_SOUP = 0: the lane path)
extern "C" void srnn_set_rnn_soup(int on) { srnn_set_knob(SRNN_KNOB_RNN_SOUP, on ? 1 : 0); }
template <int WT, int DT>
static void rw_launch_shape(int op, dim3 grid, size_t lds, hipStream_t st, const GShape& s, const SrnnArgs& a) {
  switch (op) {
    case OP_APPLY: hipLaunchKernelGGL((k_rnn_wave<OP_APPLY, WT, DT>), grid, dim3(64), lds, st, s, a); break;
    case OP_TRAIN: hipLaunchKernelGGL((k_rnn_wave<OP_TRAIN, WT, DT>), grid, dim3(64), lds, st, s, a); break;
    case OP_LEARN: hipLaunchKernelGGL((k_rnn_wave<OP_LEARN, WT, DT>), grid, dim3(64), lds, st, s, a); break;
    case OP_SOUP_EVOLVE: hipLaunchKernelGGL((k_rnn_wave_soup<WT, DT>), grid, dim3(64), lds, st, s, a); break;
    default: hipLaunchKernelGGL((k_rnn_wave<OP_RUN_FIXPOINT, WT, DT>), grid, dim3(64), lds, st, s, a); break;
  }
}
static bool rw_serves(int op, const GShape& s, const SrnnArgs& a) {
  if (knob(SRNN_KNOB_RNN_WAVE, 1) == 0) return false;
  if (s.kind != 2 || s.W < RW_MIN_WIDTH || s.W > 64 || rw_lds_bytes(s) > 60 * 1024 || !a.dev) return false;
  // RD's closed form of the layer tables must be make_gshape's
  for (int l = 0; l < s.NL; ++l) {
    const int kl = l == 0 ? 0 : s.W + s.W * s.W + (l - 1) * 2 * s.W * s.W;
    if (s.koff[l] != kl || s.roff[l] != kl + s.in_[l] * s.un[l] || s.un[l] != (l == s.D ? 1 : s.W) ||
        s.in_[l] != (l == 0 ? 1 : s.W))
      return false;
  }
  if (s.P != s.koff[s.D] + s.W + 1 || s.HS != s.D * s.W + 1) return false;
  if (op == OP_SOUP_EVOLVE)  // single-rank generations (sharded exchanges: the lane path)
    return knob(SRNN_KNOB_RNN_SOUP, 1) != 0 && !(a.flags & (SRNN_F_X2 | SRNN_F_FULL_TABLE)) && a.heads && a.nexts;
  if (op == OP_RUN_FIXPOINT) return a.traj == nullptr;
  return op == OP_APPLY || op == OP_TRAIN || op == OP_LEARN;
}
static int rw_launch(int op, const GShape& s, const SrnnArgs& a) {
  if (a.n <= 0) return 0;
  const int64_t per = op == OP_SOUP_EVOLVE ? rw_soup_scratch_bytes(s) : (int64_t)s.P * s.HS * (int64_t)sizeof(float);
  int64_t blocks = a.scratch ? a.scratch_bytes / per : 0;
  if (op != OP_TRAIN && op != OP_LEARN && op != OP_SOUP_EVOLVE) blocks = 4096;  // no BPTT states
  blocks = blocks < a.n ? blocks : a.n;
  blocks = blocks < 8192 ? blocks : 8192;
  if (blocks <= 0) {
    set_error("generic engine: scratch buffer missing or too small for the recurrent wave path");
    return -5;
  }
  const size_t lds = rw_lds_bytes(s);
  hipStream_t st = (hipStream_t)a.stream;
  if (op != OP_APPLY && op != OP_TRAIN && op != OP_LEARN && op != OP_RUN_FIXPOINT && op != OP_SOUP_EVOLVE) {
    set_error("recurrent wave path: op");
    return -1;
  }
  const bool spec = knob(SRNN_KNOB_RNN_SPEC, 1) != 0;
  const int w = spec ? s.W : 0, d = spec ? s.D : 0;
  const dim3 grid((unsigned)blocks);
  if (w == 8 && d == 2) rw_launch_shape<8, 2>(op, grid, lds, st, s, a);
  else if (w == 16 && d == 2) rw_launch_shape<16, 2>(op, grid, lds, st, s, a);
  else if (w == 32 && d == 2) rw_launch_shape<32, 2>(op, grid, lds, st, s, a);
  else if (w == 8 && d == 3) rw_launch_shape<8, 3>(op, grid, lds, st, s, a);
  else if (w == 16 && d == 3) rw_launch_shape<16, 3>(op, grid, lds, st, s, a);
  else rw_launch_shape<0, 0>(op, grid, lds, st, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

static bool generic_op_supported(int op) {
  switch (op) {
    case OP_INIT: case OP_APPLY: case OP_RUN_FIXPOINT: case OP_TRAIN: case OP_LEARN: case OP_CLASSIFY:
    case OP_PERTURB: case OP_SOUP_DECIDE: case OP_RESPAWN_SEQ: case OP_SOUP_EVOLVE: case OP_RESPAWN:
    case OP_VARY_RUN:
      return true;
    default: return false;
  }
}

extern "C" int srnn_generic_op_supported(int op, int dev) {
  return generic_op_supported(op) || (op == OP_SOUP_SEQ && !dev) ? 1 : 0;  // sequential: host loop
}

// ==================================================================================
// Wide Weightwise nets, U lanes per particle (SGD: train / learn_from).  The lane-per-particle
// path streams every weight, activation and sample through element-major scratch in HBM
// (WW(16, 2): 0.27 TFLOP/s, profiles/r3d).  Here a wave holds G = 64 / U particles, U = the
// next power of two >= width: lane u of a particle computes unit u of every layer, the weights
// (hidden W x W layers with a padded row stride: the backward pass reads rows), the frozen
// samples, the permutation and the activations live in LDS, and the coordinate table is shared
// by the block.  Every dot product keeps the lane path's order (x[0]*k then fma over the inputs;
// the output unit's chain on one lane), every weight gets the same single fma, so results are
// bitwise those of g_train_epochs (tests/test_generic_gpu.py).
// ==================================================================================
struct WWave {
  int U, G, PW, GS;         // lanes per particle, particles per wave, padded weights, floats per particle
  int poff[GMAXL], pst[GMAXL];  // padded layer offsets and row strides
  int o_sv, o_perm, o_acts, o_sa, o_sb, o_misc;
};
static bool ww_wave_geom(const GShape& s, WWave& g, bool soup = false) {
  if (s.kind != 0 || s.P <= 16 || s.W < 3 || s.W > 64) return false;
  g.U = 4;
  while (g.U < s.W) g.U *= 2;
  g.G = 64 / g.U;
  int o = 0;
  for (int l = 0; l < s.NL; ++l) {
    g.pst[l] = s.cols[l] + ((l > 0 && l < s.D) ? 1 : 0);  // hidden layers: odd row stride
    g.poff[l] = o;
    o += s.rows[l] * g.pst[l];
  }
  g.PW = o;
  g.o_sv = o;
  g.o_perm = g.o_sv + s.P;
  g.o_acts = g.o_perm + s.P;
  g.o_sa = g.o_acts + s.IN + s.D * s.W;
  g.o_sb = g.o_sa + s.W;
  g.o_misc = g.o_sb + s.W;
  g.GS = g.o_misc + 4 + (soup ? s.P + 2 * g.U * s.W : 0);  // soups: apply output + per-lane vectors
  return true;
}
static size_t ww_wave_lds(const GShape& s, const WWave& g) { return ((size_t)3 * s.P + (size_t)g.G * g.GS) * 4; }

// padded LDS index of flat weight k
__device__ __forceinline__ int ww_pidx(const GShape& s, const WWave& g, int k) {
  int l = 0;
  while (l + 1 < s.NL && s.off[l + 1] <= k) ++l;
  const int q = k - s.off[l], i = q / s.cols[l], j = q - i * s.cols[l];
  return g.poff[l] + i * g.pst[l] + j;
}

// per-particle LDS regions of a WWave group
struct WWGroup {
  float* w;      // padded weights
  float* sv;     // frozen samples / teacher or attacker row (flat)
  int* perm;
  float* acts;   // [x (4)][h_1 (W)] ... [h_D (W)]
  float* sa;
  float* sb;
  float* misc;   // [0] the step so, [1..3] per-particle scalars
  float* ob;     // (soups) apply output, flat
  float* hb;     // (soups) per-lane forward vectors, 2 W per lane of the group
};
__device__ __forceinline__ WWGroup ww_group(const GShape& s, const WWave& g, float* sm, int grp) {
  float* pw = sm + 3 * s.P + grp * g.GS;
  WWGroup r;
  r.w = pw;
  r.sv = pw + g.o_sv;
  r.perm = reinterpret_cast<int*>(pw + g.o_perm);
  r.acts = pw + g.o_acts;
  r.sa = pw + g.o_sa;
  r.sb = pw + g.o_sb;
  r.misc = pw + g.o_misc;
  r.ob = pw + g.o_misc + 4;
  r.hb = r.ob + s.P;
  return r;
}

// E SGD epochs of one particle per group (g_train_epochs): SELF -- the samples are the weights
// at each epoch start, else the row already in sv.  Every lane of the wave calls it (barriers);
// only `live` groups draw shuffles and update their weights (a soup's non-learners sit out the
// learn_from epochs of the wave).  Returns the last epoch's mean loss (lane u == 0).
__device__ float ww_epochs(const GShape& s, const WWave& g, const WWGroup& R, const float* coords, int u, bool live,
                           int E, bool self, uint64_t uid, uint32_t& ctr, float lr, bool shuffle, const Rng& rng) {
  const int W = s.W, D = s.D;
  const float lr2 = 2.0f * lr;  // the folded step -(2 lr) * e (Weightwise::train_epoch)
  float loss = 0.f;
  for (int e = 0; e < E; ++e) {
    if (self)  // samples = the weights at the epoch start
      for (int k = u; k < s.P; k += g.U) R.sv[k] = R.w[ww_pidx(s, g, k)];
    __syncthreads();
    if (shuffle) {
      // g_fisher_yates (same draws: one Philox block per 4 swaps, stream (uid, ctr, purpose +
      // block << 8)); the swap chain on lane 0 of the particle
      for (int k = u; k < s.P; k += g.U) R.perm[k] = k;
      __syncthreads();
      if (u == 0 && live) {
        U4 r{0, 0, 0, 0};
        int used = 4;
        uint32_t blk = 0;
        for (int t = s.P - 1; t > 0; --t) {
          if (used == 4) {
            r = rng.draw(uid, ctr, P_SHUFFLE + (blk << 8));
            ++blk;
            used = 0;
          }
          const uint32_t x = used == 0 ? r.x : used == 1 ? r.y : used == 2 ? r.z : r.w;
          ++used;
          int j = (int)(u01(x) * (float)(t + 1));
          if (j > t) j = t;
          const int pt = R.perm[t];
          R.perm[t] = R.perm[j];
          R.perm[j] = pt;
        }
      }
      __syncthreads();
    }
    float acc = 0.f;
    for (int q = 0; q < s.P; ++q) {
      const int idx = shuffle ? R.perm[q] : q;
      const float x0 = R.sv[idx];
      const float x1 = coords[3 * idx], x2 = coords[3 * idx + 1], x3 = coords[3 * idx + 2];
      // layer 0: h1[u] = x0*K0[0][u] then fma over the 3 coordinates
      if (u < W) {
        const float* K = R.w + g.poff[0];
        float h = x0 * K[u];
        h = fmaf(x1, K[g.pst[0] + u], h);
        h = fmaf(x2, K[2 * g.pst[0] + u], h);
        h = fmaf(x3, K[3 * g.pst[0] + u], h);
        R.acts[4 + u] = h;
      }
      __syncthreads();
      for (int l = 1; l < D; ++l) {  // hidden layers: column u
        if (u < W) {
          const float* K = R.w + g.poff[l];
          const float* x = R.acts + 4 + (l - 1) * W;
          float h = x[0] * K[u];
          for (int r = 1; r < W; ++r) h = fmaf(x[r], K[r * g.pst[l] + u], h);
          R.acts[4 + l * W + u] = h;
        }
        __syncthreads();
      }
      // output unit (one chain, lane 0) -> error, loss, the step so = -(2 lr) * e
      if (u == 0) {
        const float* K = R.w + g.poff[D];
        const float* x = R.acts + 4 + (D - 1) * W;
        float y = x[0] * K[0];
        for (int r = 1; r < W; ++r) y = fmaf(x[r], K[r], y);
        const float err = y - x0;
        acc += err * err;
        R.misc[0] = -lr2 * err;
      }
      __syncthreads();
      // last layer (W x 1): si[u] = K[u] * so (pre-update), K[u] += h_D[u] * so
      float* si = R.sa;
      float* sn = R.sb;
      if (u < W) {
        float* K = R.w + g.poff[D];
        const float so = R.misc[0];
        si[u] = K[u] * so;
        if (live) K[u] = fmaf(R.acts[4 + (D - 1) * W + u], so, K[u]);
      }
      __syncthreads();
      for (int l = D - 1; l >= 1; --l) {  // hidden layers: row u (si from the pre-update row)
        if (u < W) {
          float* K = R.w + g.poff[l] + u * g.pst[l];
          float sacc = K[0] * si[0];
          for (int c = 1; c < W; ++c) sacc = fmaf(K[c], si[c], sacc);
          const float xr = R.acts[4 + (l - 1) * W + u];
          if (live)
            for (int c = 0; c < W; ++c) K[c] = fmaf(xr, si[c], K[c]);
          sn[u] = sacc;
        }
        __syncthreads();
        float* t = si;
        si = sn;
        sn = t;
      }
      // layer 0 (4 x W): column u, no input gradient
      if (u < W && live) {
        float* K = R.w + g.poff[0];
        const float so = si[u];
        K[u] = fmaf(x0, so, K[u]);
        K[g.pst[0] + u] = fmaf(x1, so, K[g.pst[0] + u]);
        K[2 * g.pst[0] + u] = fmaf(x2, so, K[2 * g.pst[0] + u]);
        K[3 * g.pst[0] + u] = fmaf(x3, so, K[3 * g.pst[0] + u]);
      }
      __syncthreads();
    }
    loss = acc / (float)s.P;
    ctr += 1;
  }
  return loss;
}


// ---------------------------------------------------------------------------------------------
// ww_epochs with the particle's weights in VGPRs (compile-time width W, depth D; U = 4 lanes per
// particle for W <= 4, 16 for W <= 16).  Lane u keeps column u of the input layer, column u AND
// row u of every hidden layer (the diagonal twice, both copies updated by the same fma), and the
// whole output layer (replicated; its own entry also as kd_own): the forward dot products read
// the other units' values through DPP broadcasts within the group (quad_perm for U = 4,
// row_newbcast for U = 16), the backward pass the other units' steps the same way.  Same fma
// sequence per value as ww_epochs / g_train_epochs (bitwise, tests/test_ww_wave_gpu.py); no LDS
// traffic and no barriers inside the SGD step (the LDS form waited on LDS 4.6x its issue time,
// profiles/r3d).  Samples, the permutation and the coordinates stay in LDS.  live = false: the
// epochs run but the weights in LDS are left as they were (a soup's non-learners).
template <int U, int R_>
__device__ __forceinline__ float wr_bcast(float v) {
  if constexpr (U == 4) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), R_ * 0x55, 0xF, 0xF, true));
  else return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + R_, 0xF, 0xF, true));
}
template <int U, int W, int R_ = 0>
__device__ __forceinline__ void wr_bcast_all(float v, float* out) {
  if constexpr (R_ < W) {
    out[R_] = wr_bcast<U, R_>(v);
    wr_bcast_all<U, W, R_ + 1>(v, out);
  }
}
template <int W, int D>
__device__ float ww_epochs_reg(const GShape& s, const WWave& g, const WWGroup& R, const float* coords, int u, bool live,
                               int E, bool self, uint64_t uid, uint32_t& ctr, float lr, bool shuffle, const Rng& rng) {
  constexpr int U = W <= 4 ? 4 : 16;
  constexpr int H = D - 1 > 0 ? D - 1 : 1;  // hidden layers (at least one array slot)
  const bool on = u < W;
  const int uu = on ? u : 0;
  float k0[4], kc[H][W], kr[H][W], kd[W], kd_own;
#pragma unroll
  for (int i = 0; i < 4; ++i) k0[i] = R.w[g.poff[0] + i * g.pst[0] + uu];
#pragma unroll
  for (int l = 1; l < D; ++l)
#pragma unroll
    for (int r = 0; r < W; ++r) {
      kc[l - 1][r] = R.w[g.poff[l] + r * g.pst[l] + uu];
      kr[l - 1][r] = R.w[g.poff[l] + uu * g.pst[l] + r];
    }
#pragma unroll
  for (int r = 0; r < W; ++r) kd[r] = R.w[g.poff[D] + r * g.pst[D]];
  kd_own = R.w[g.poff[D] + uu * g.pst[D]];
  const float lr2 = 2.0f * lr;
  float loss = 0.f;
  for (int e = 0; e < E; ++e) {
    if (self && on) {  // samples = the weights at the epoch start (flat, row-major)
#pragma unroll
      for (int i = 0; i < 4; ++i) R.sv[s.off[0] + i * W + u] = k0[i];
#pragma unroll
      for (int l = 1; l < D; ++l)
#pragma unroll
        for (int r = 0; r < W; ++r) R.sv[s.off[l] + r * W + u] = kc[l - 1][r];
      R.sv[s.off[D] + u] = kd_own;
    }
    __syncthreads();
    if (shuffle) {  // the permutation: exactly ww_epochs' (lane 0 of the particle)
      for (int k = u; k < s.P; k += g.U) R.perm[k] = k;
      __syncthreads();
      if (u == 0 && live) {
        U4 r{0, 0, 0, 0};
        int used = 4;
        uint32_t blk = 0;
        for (int t = s.P - 1; t > 0; --t) {
          if (used == 4) {
            r = rng.draw(uid, ctr, P_SHUFFLE + (blk << 8));
            ++blk;
            used = 0;
          }
          const uint32_t x = used == 0 ? r.x : used == 1 ? r.y : used == 2 ? r.z : r.w;
          ++used;
          int j = (int)(u01(x) * (float)(t + 1));
          if (j > t) j = t;
          const int pt = R.perm[t];
          R.perm[t] = R.perm[j];
          R.perm[j] = pt;
        }
      }
      __syncthreads();
    }
    float acc = 0.f;
    for (int q = 0; q < s.P; ++q) {
      const int idx = shuffle ? R.perm[q] : q;
      const float x0 = R.sv[idx];
      const float x1 = coords[3 * idx], x2 = coords[3 * idx + 1], x3 = coords[3 * idx + 2];
      float hin[D][W], hown[D];
      float h = x0 * k0[0];
      h = fmaf(x1, k0[1], h);
      h = fmaf(x2, k0[2], h);
      h = fmaf(x3, k0[3], h);
      hown[0] = h;
      wr_bcast_all<U, W>(h, hin[0]);
#pragma unroll
      for (int l = 1; l < D; ++l) {  // hidden layer l: column u
        float z = hin[l - 1][0] * kc[l - 1][0];
#pragma unroll
        for (int r = 1; r < W; ++r) z = fmaf(hin[l - 1][r], kc[l - 1][r], z);
        hown[l] = z;
        wr_bcast_all<U, W>(z, hin[l]);
      }
      float y = hin[D - 1][0] * kd[0];  // the output unit's chain (every lane, same order)
#pragma unroll
      for (int r = 1; r < W; ++r) y = fmaf(hin[D - 1][r], kd[r], y);
      const float err = y - x0;
      acc += err * err;
      const float so = -lr2 * err;
      float si = kd_own * so;  // pre-update K_D[u]
      kd_own = fmaf(hown[D - 1], so, kd_own);
#pragma unroll
      for (int r = 0; r < W; ++r) kd[r] = fmaf(hin[D - 1][r], so, kd[r]);
#pragma unroll
      for (int l = D - 1; l >= 1; --l) {  // hidden layers: row u with the pre-update row
        float sall[W];
        wr_bcast_all<U, W>(si, sall);
        float sacc = kr[l - 1][0] * sall[0];
#pragma unroll
        for (int c = 1; c < W; ++c) sacc = fmaf(kr[l - 1][c], sall[c], sacc);
#pragma unroll
        for (int r = 0; r < W; ++r) kc[l - 1][r] = fmaf(hin[l - 1][r], si, kc[l - 1][r]);
#pragma unroll
        for (int c = 0; c < W; ++c) kr[l - 1][c] = fmaf(hown[l - 1], sall[c], kr[l - 1][c]);
        si = sacc;
      }
      k0[0] = fmaf(x0, si, k0[0]);
      k0[1] = fmaf(x1, si, k0[1]);
      k0[2] = fmaf(x2, si, k0[2]);
      k0[3] = fmaf(x3, si, k0[3]);
    }
    loss = acc / (float)s.P;
    ctr += 1;
  }
  __syncthreads();  // every lane read the LDS weights before any write-back
  if (live && on) {
#pragma unroll
    for (int i = 0; i < 4; ++i) R.w[g.poff[0] + i * g.pst[0] + u] = k0[i];
#pragma unroll
    for (int l = 1; l < D; ++l)
#pragma unroll
      for (int r = 0; r < W; ++r) R.w[g.poff[l] + r * g.pst[l] + u] = kc[l - 1][r];
    R.w[g.poff[D] + u * g.pst[D]] = kd_own;
  }
  __syncthreads();
  return loss;
}
// E epochs on the register form for the instantiated shapes (WT > 0), else the LDS form
template <int WT, int DT>
__device__ __forceinline__ float ww_epochs_any(const GShape& s, const WWave& g, const WWGroup& R, const float* coords,
                                               int u, bool live, int E, bool self, uint64_t uid, uint32_t& ctr,
                                               float lr, bool shuffle, const Rng& rng) {
  if constexpr (WT > 0) return ww_epochs_reg<WT, DT>(s, g, R, coords, u, live, E, self, uid, ctr, lr, shuffle, rng);
  else return ww_epochs(s, g, R, coords, u, live, E, self, uid, ctr, lr, shuffle, rng);
}

__device__ void ww_load(const GShape& s, const WWave& g, float* pw, const char* row, int u) {
  for (int k = u; k < s.P; k += g.U) pw[ww_pidx(s, g, k)] = g_dec(row, k, s.dtype);
}
__device__ void ww_store(const GShape& s, const WWave& g, const float* pw, char* row, int u) {
  for (int k = u; k < s.PP; k += g.U) {
    const float v = k < s.P ? pw[ww_pidx(s, g, k)] : 0.f;
    if (s.dtype == 0) reinterpret_cast<float*>(row)[k] = v;
    else reinterpret_cast<uint16_t*>(row)[k] = s.dtype == 1 ? StBF16::enc(v) : StF16::enc(v);
  }
}

template <int OP, int WT = 0, int DT = 0>
__global__ __launch_bounds__(64) void k_ww_wave(GShape s, WWave g, SrnnArgs a) {
  extern __shared__ float sm[];
  float* coords = sm;  // [P][3], whole block
  make_coords_dev(s, coords);
  const int lane = threadIdx.x, u = lane % g.U, grp = lane / g.U;
  const WWGroup R = ww_group(s, g, sm, grp);
  const bool shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
  const Rng rng = GItem::rng(a);
  for (int64_t base = (int64_t)blockIdx.x * g.G; base < a.n; base += (int64_t)gridDim.x * g.G) {
    const int64_t i = base + grp;
    const bool active = i < a.n;
    if (active) {
      ww_load(s, g, R.w, GItem::rowp(s, a.W, i), u);
      if (OP == OP_LEARN) {
        const char* t = GItem::rowp(s, a.W2, a.idx_t ? a.idx_t[i] : i);
        for (int k = u; k < s.P; k += g.U) R.sv[k] = g_dec(t, k, s.dtype);
      }
    }
    __syncthreads();
    uint32_t ctr = a.ctr;
    const float loss = ww_epochs_any<WT, DT>(s, g, R, coords, u, active, a.epochs, OP == OP_TRAIN,
                                 active ? GItem::uid_of(a, i) : 0, ctr, a.lr, shuffle, rng);
    if (active) {
      ww_store(s, g, R.w, GItem::rowp(s, a.W, i), u);
      if (a.loss && u == 0) a.loss[i] = loss;
    }
    __syncthreads();
  }
}

// Soup generation of the single-rank runtime-shape engine (GItem::soup_evolve):
// attacks received in ascending attacker-slot order (the attacker net evaluated at the
// victim's P weight points, lanes over the points), learn_from, self-train, respawn with
// inline re-init; respawn flags per row (SRNN_F_ROW_FLAGS) or OR-ed into the 64-row ballots
// (zeroed by their consumer, k_g_respawn_seq).
template <int WT = 0, int DT = 0>
__global__ __launch_bounds__(64) void k_ww_wave_soup(GShape s, WWave g, SrnnArgs a) {
  extern __shared__ float sm[];
  float* coords = sm;
  make_coords_dev(s, coords);
  const int lane = threadIdx.x, u = lane % g.U, grp = lane / g.U;
  const WWGroup R = ww_group(s, g, sm, grp);
  const bool shuffle = (a.flags & SRNN_F_SHUFFLE) != 0;
  const Rng rng = GItem::rng(a);
  const int64_t rb = g_rb(s);
  const int32_t gen = a.gen_ptr ? a.gen_ptr[0] : a.gen;
  const int W = s.W, D = s.D;
  int* ictl = reinterpret_cast<int*>(R.misc);  // [1] attacker entry, [2] its state
  for (int64_t base = (int64_t)blockIdx.x * g.G; base < a.n; base += (int64_t)gridDim.x * g.G) {
    const int64_t j = base + grp;
    const bool active = j < a.n;
    const int64_t gs = a.lo + j;
    if (active) ww_load(s, g, R.w, GItem::rowp(s, a.W2, j), u);
    // 1. attacks: lane 0 of the group walks the list for the next attacker (ascending slot)
    uint32_t head = SRNN_NIL;
    if (active) head = a.heads[j];
    uint64_t last = 0;
    bool first = true;
    for (;;) {
      if (u == 0) {
        uint32_t be = SRNN_NIL;
        if (active && head != SRNN_NIL) {
          uint64_t best = ~0ull;
          for (uint32_t e = head; e != SRNN_NIL; e = a.nexts[e]) {
            const uint64_t sl = ent_slot(a, e);
            if ((first || sl > last) && sl < best) best = sl, be = e;
          }
          if (be != SRNN_NIL) last = best, first = false;
        }
        ictl[1] = (int)be;
      }
      __syncthreads();
      const uint32_t be = (uint32_t)ictl[1];
      const bool more = be != SRNN_NIL;
      if (__ballot(more) == 0ull) break;  // every group of the wave is done
      if (more) {
        const char* r = ent_row(a, be, rb);
        for (int k = u; k < s.P; k += g.U) R.sv[k] = g_dec(r, k, s.dtype);  // the attacker's weights
      }
      __syncthreads();
      if (more) {  // out[k] = f_attacker(w[k], coords k) for the points of this lane
        float* h = R.hb + u * 2 * W;
        float* h2 = h + W;
        for (int k = u; k < s.P; k += g.U) {
          const float x0 = R.w[ww_pidx(s, g, k)], x1 = coords[3 * k], x2 = coords[3 * k + 1], x3 = coords[3 * k + 2];
          const float* K = R.sv;  // flat: layer l at s.off[l], row-major (rows x cols)
          for (int c = 0; c < W; ++c) {
            float acc = x0 * K[c];
            acc = fmaf(x1, K[W + c], acc);
            acc = fmaf(x2, K[2 * W + c], acc);
            acc = fmaf(x3, K[3 * W + c], acc);
            h[c] = acc;
          }
          for (int l = 1; l < D; ++l) {
            const float* Kl = R.sv + s.off[l];
            for (int c = 0; c < W; ++c) {
              float acc = h[0] * Kl[c];
              for (int r = 1; r < W; ++r) acc = fmaf(h[r], Kl[r * W + c], acc);
              h2[c] = acc;
            }
            for (int c = 0; c < W; ++c) h[c] = h2[c];
          }
          const float* KD = R.sv + s.off[D];
          float y = h[0] * KD[0];
          for (int r = 1; r < W; ++r) y = fmaf(h[r], KD[r], y);
          R.ob[k] = g_q(y, s.dtype);
        }
      }
      __syncthreads();
      if (more)
        for (int k = u; k < s.P; k += g.U) R.w[ww_pidx(s, g, k)] = R.ob[k];
      __syncthreads();
    }
    if (active && u == 0 && head != SRNN_NIL) a.heads[j] = SRNN_NIL;  // consumed
    // 2. decisions of this slot, learn_from the teacher's generation-start row
    int64_t my_at = -1, te = -1;
    if (active) Item<Weightwise<1, 1>, StF32>::decision(a, gs, gen, my_at, te);
    int8_t act = my_at >= 0 ? A_ATTACKING : A_NONE;
    int64_t cp = my_at >= 0 ? my_at : -1;
    const bool learn = active && te >= 0;
    if (learn) {
      const char* r = teacher_row(a, te, SRNN_NIL, rb);
      for (int k = u; k < s.P; k += g.U) R.sv[k] = g_dec(r, k, s.dtype);
    }
    __syncthreads();
    uint32_t ctr = (uint32_t)gen * 1024u + 512u;
    float loss = 0.f;
    // the groups of a wave learn together (a group without a teacher runs the epochs on its own
    // samples with its lanes masked out of every write: live = false keeps its state)
    if (__ballot(learn) != 0ull && a.severity > 0) {
      const float l2 =
          ww_epochs_any<WT, DT>(s, g, R, coords, u, learn, a.severity, false, (uint64_t)gs, ctr, a.lr, shuffle, rng);
      if (learn) loss = l2;
    }
    if (learn) act = A_LEARN_FROM, cp = te;
    if (a.epochs > 0) {
      uint32_t c2 = (uint32_t)gen * 1024u + 512u + (learn ? (uint32_t)a.severity : 0u);
      loss = ww_epochs_any<WT, DT>(s, g, R, coords, u, active, a.epochs, true, (uint64_t)gs, c2, a.lr, shuffle, rng);
      act = A_TRAIN_SELF;
      cp = -1;
    }
    // 3. respawn (the zero test on the old particle; at most one of the two)
    bool bad = false, nz = false;
    for (int k = u; k < s.P; k += g.U) {
      float& v = R.w[ww_pidx(s, g, k)];
      v = g_q(v, s.dtype);
      bad |= !finitef(v);
      nz |= !((-a.eps <= v) && (v <= a.eps));
    }
    const unsigned long long gm = (g.U == 64 ? ~0ull : ((1ull << g.U) - 1ull)) << (grp * g.U);
    const bool div = (__ballot(bad) & gm) != 0ull, zero = (__ballot(nz) & gm) == 0ull;
    int8_t rs = 0;
    if ((a.flags & SRNN_F_REMOVE_DIVERGENT) && div) rs = 1;
    else if ((a.flags & SRNN_F_REMOVE_ZERO) && zero) rs = 2;
    __syncthreads();
    if (active && rs && (a.flags & SRNN_F_RESPAWN_INLINE)) {  // g_init: glorot per layer
      const uint64_t key = respawn_key(gen, gs);
      for (int l = 0; l < s.NL; ++l) {
        const int n = s.rows[l] * s.cols[l];
        const float lim = sqrtf(6.0f / (float)(s.rows[l] + s.cols[l]));
        for (int b = u; b < (n + 3) / 4; b += g.U) {
          const U4 q4 = rng.draw(key, (uint32_t)s.off[l] * 1024u + (uint32_t)b, P_INIT);
          const uint32_t xs[4] = {q4.x, q4.y, q4.z, q4.w};
          for (int q = 0; q < 4; ++q) {
            const int k = b * 4 + q;
            if (k < n) R.w[ww_pidx(s, g, s.off[l] + k)] = -lim + 2.0f * lim * u01(xs[q]);
          }
        }
      }
    }
    __syncthreads();
    if (active) {
      ww_store(s, g, R.w, GItem::rowp(s, a.W, j), u);
      if (u == 0) {
        if (a.action) a.action[j] = act;
        if (a.counterpart) a.counterpart[j] = cp;
        if (a.loss) a.loss[j] = loss;
        if (a.respawn) a.respawn[j] = rs;
        if (a.flags & SRNN_F_ROW_FLAGS) {
          if (a.rowflags) a.rowflags[j] = rs ? 1 : 0;
        } else if (a.ballots && rs) {
          atomicOr(a.ballots + (j >> 6), 1ull << (j & 63));
        }
      }
    }
    __syncthreads();
  }
}

// knob SRNN_KNOB_WW_WAVE = 0: lane path for every width (A/B tests)
extern "C" void srnn_set_ww_wave(int on) { srnn_set_knob(SRNN_KNOB_WW_WAVE, on ? 1 : 0); }
static bool ww_serves(int op, const GShape& s, const SrnnArgs& a, WWave& g) {
  if (knob(SRNN_KNOB_WW_WAVE, 1) == 0 || !a.dev) return false;
  if (op == OP_SOUP_EVOLVE) {  // single-rank generations (sharded exchanges: the lane path)
    if (a.flags & (SRNN_F_X2 | SRNN_F_FULL_TABLE)) return false;
    return ww_wave_geom(s, g, true) && ww_wave_lds(s, g) <= 64 * 1024;
  }
  if (op != OP_TRAIN && op != OP_LEARN) return false;
  return ww_wave_geom(s, g) && ww_wave_lds(s, g) <= 64 * 1024;
}
template <int WT, int DT>
static void ww_launch_shape(int op, dim3 grid, size_t lds, hipStream_t st, const GShape& s, const WWave& g,
                            const SrnnArgs& a) {
  if (op == OP_TRAIN) hipLaunchKernelGGL((k_ww_wave<OP_TRAIN, WT, DT>), grid, dim3(64), lds, st, s, g, a);
  else if (op == OP_LEARN) hipLaunchKernelGGL((k_ww_wave<OP_LEARN, WT, DT>), grid, dim3(64), lds, st, s, g, a);
  else hipLaunchKernelGGL((k_ww_wave_soup<WT, DT>), grid, dim3(64), lds, st, s, g, a);
}
static int ww_launch(int op, const GShape& s, const WWave& g, const SrnnArgs& a) {
  if (a.n <= 0) return 0;
  int64_t blocks = (a.n + g.G - 1) / g.G;
  blocks = blocks < 65536 ? blocks : 65536;
  const size_t lds = ww_wave_lds(s, g);
  hipStream_t st = (hipStream_t)a.stream;
  const dim3 grid((unsigned)blocks);
  // register-resident SGD for the instantiated shapes (knob SRNN_KNOB_WW_WAVE = 2: the LDS form)
  const bool reg = knob(SRNN_KNOB_WW_WAVE, 1) != 2;
  const int w = reg ? s.W : 0, d = reg ? s.D : 0;
  if (w == 3 && d == 3 && g.U == 4) ww_launch_shape<3, 3>(op, grid, lds, st, s, g, a);
  else if (w == 3 && d == 4 && g.U == 4) ww_launch_shape<3, 4>(op, grid, lds, st, s, g, a);
  else if (w == 10 && d == 2 && g.U == 16) ww_launch_shape<10, 2>(op, grid, lds, st, s, g, a);
  else if (w == 10 && d == 3 && g.U == 16) ww_launch_shape<10, 3>(op, grid, lds, st, s, g, a);
  else if (w == 16 && d == 2 && g.U == 16) ww_launch_shape<16, 2>(op, grid, lds, st, s, g, a);
  else if (w == 16 && d == 3 && g.U == 16) ww_launch_shape<16, 3>(op, grid, lds, st, s, g, a);
  else ww_launch_shape<0, 0>(op, grid, lds, st, s, g, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

// lanes of a device launch and the scratch bytes they need
static int64_t generic_lanes(const GShape& s, const SrnnArgs& a, int64_t items) {
  const int64_t per = g_lane_bytes(s);
  int64_t cap = per > 0 ? a.scratch_bytes / per : 0;
  cap = (cap / GTB) * GTB;
  int64_t want = ((items + GTB - 1) / GTB) * GTB;
  return want < cap ? want : cap;
}

static int generic_launch(int op, const GShape& s, const SrnnArgs& a) {
  hipStream_t st = (hipStream_t)a.stream;
  if (op == OP_SOUP_DECIDE) {
    // shape-independent: the decisions / attack lists of srnn_kernels.h
    SrnnCfg dummy{};
    return launch<Weightwise<1, 1>, OP_SOUP_DECIDE, StF32>(dummy, a);
  }
  if (op == OP_RESPAWN_SEQ) {
    if (!a.scratch || a.scratch_bytes < (int64_t)GTBR * g_lane_bytes(s)) {
      set_error("generic respawn_seq needs scratch >= 1024 lanes (srnn_generic_scratch_bytes)");
      return -5;
    }
    hipLaunchKernelGGL(k_g_respawn_seq, dim3(1), dim3(GTBR), 0, st, s, a);
  } else if (rw_serves(op, s, a)) {
    return rw_launch(op, s, a);
  } else if (WWave g; ww_serves(op, s, a, g)) {
    return ww_launch(op, s, g, a);
  } else {
    if (a.n <= 0) return 0;
    const int64_t lanes = generic_lanes(s, a, a.n);
    if (lanes <= 0) {
      set_error("generic engine: scratch buffer missing or too small (srnn_generic_scratch_bytes)");
      return -5;
    }
    const size_t lds = s.kind == 0 ? (size_t)s.P * 3 * sizeof(float) : 0;
    if (lds > 150 * 1024) {
      set_error("generic engine: weightwise coordinate table exceeds LDS (P > 12800)");
      return -5;
    }
    const dim3 grid((unsigned)(lanes / GTB)), block(GTB);
    switch (op) {
#define SRNN_GK(OPC) hipLaunchKernelGGL((k_generic<OPC>), grid, block, lds, st, s, a, lanes); break;
      case OP_INIT: SRNN_GK(OP_INIT)
      case OP_APPLY: SRNN_GK(OP_APPLY)
      case OP_RUN_FIXPOINT: SRNN_GK(OP_RUN_FIXPOINT)
      case OP_TRAIN: SRNN_GK(OP_TRAIN)
      case OP_LEARN: SRNN_GK(OP_LEARN)
      case OP_PERTURB: SRNN_GK(OP_PERTURB)
      case OP_VARY_RUN: SRNN_GK(OP_VARY_RUN)
      case OP_RESPAWN: SRNN_GK(OP_RESPAWN)
      case OP_SOUP_EVOLVE:
        if ((a.flags & SRNN_F_X2) && (a.flags & SRNN_F_X2_REMOTE)) {
          // the list length is on the device: a bounded grid-stride launch over the list
          int64_t rl = ((x2_remote_bound(a) + GTB - 1) / GTB) * GTB;
          rl = rl < lanes ? rl : lanes;
          rl = rl < X2_REMOTE_WAVES * GTB ? rl : X2_REMOTE_WAVES * GTB;
          hipLaunchKernelGGL((k_generic<GOP_X2_REMOTE>), dim3((unsigned)(rl / GTB)), block, lds, st, s, a, rl);
          break;
        }
        SRNN_GK(GOP_EVOLVE)
      case OP_CLASSIFY:
        if (a.counts) {
          SRNN_GK(GOP_CLASSIFY_COUNT)
        } else {
          SRNN_GK(OP_CLASSIFY)
        }
#undef SRNN_GK
      default: set_error("op not supported by the generic engine"); return -1;
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(hipGetErrorString(e));
    return -3;
  }
  return 0;
}

}  // namespace srnn

// 0 ok / negative error; 1 = not a valid shape for the generic engine, 2 = op not supported
extern "C" int srnn_dispatch_generic(int op, const SrnnCfg* c, const SrnnArgs* a) {
  srnn::GShape s;
  const char* why = "";
  if (!srnn::make_gshape(*c, s, &why)) {
    srnn::set_error(why);
    return 1;
  }
  if (op < 0) return 0;
  if (op == OP_SOUP_SEQ && !a->dev) {  // sequential soups: host only (a serial chain)
    srnn::host_generic(op, s, *a);
    return 0;
  }
  if (!srnn::generic_op_supported(op)) return 2;
  if (!a->dev) {
    if (op == OP_SOUP_DECIDE) {
      SrnnCfg dummy{};
      return srnn::host_run<srnn::Weightwise<1, 1>, OP_SOUP_DECIDE, srnn::StF32>(dummy, *a);
    }
    srnn::host_generic(op, s, *a);
    return 0;
  }
  return srnn::generic_launch(op, s, *a);
}

// Scratch bytes a device launch of the generic engine wants for n rows (lanes = n rounded
// up to a wave, at most `max_lanes`; the respawn workgroup needs 1024 lanes); 0 = no scratch
extern "C" int64_t srnn_generic_scratch_bytes(const SrnnCfg* c, int64_t n, int64_t max_lanes) {
  srnn::GShape s;
  const char* why = "";
  if (!srnn::make_gshape(*c, s, &why)) return -1;
  int64_t lanes = ((n + srnn::GTB - 1) / srnn::GTB) * srnn::GTB;
  if (max_lanes > 0 && lanes > max_lanes) lanes = (max_lanes / srnn::GTB) * srnn::GTB;
  if (lanes < srnn::GTBR) lanes = srnn::GTBR;
  return lanes * srnn::g_lane_bytes(s);
}
