// srnn_core.h — per-particle math of the self-replicating-network engine.
//
// Every function here is `SRNN_HD` (host + device): the same code runs inside the
// lane-per-particle HIP kernels (srnn_kernels.hip) and inside the host thread-pool
// loops used on CPU tensors.  One particle = one flat fp32 weight vector laid out in
// Keras `get_weights()` order (layer by layer, each kernel row-major (in, out); a
// SimpleRNN layer contributes [kernel, recurrent_kernel]) — reference
// code/network.py:100-104.  Networks are linear and bias-free.
//
// Architectures are compile-time templates so that every loop over weights is fully
// unrolled and the weights of a particle live in VGPRs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define SRNN_HD __host__ __device__ __forceinline__

namespace srnn {

// ----------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG.  ctr = (c0,c1,c2,c3), key = (k0,k1).
// Streams: key = seed, ctr = (id_lo, id_hi, step, purpose).
// ----------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

SRNN_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

SRNN_HD U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c.x, hi0, lo0);
    mulhilo(0xCD9E8D57u, c.z, hi1, lo1);
    U4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

enum Purpose : uint32_t {
  P_INIT = 1,        // glorot uniform init         ctr=(uid, blk)
  P_NORMAL = 2,      // normals for orthogonal init ctr=(uid, blk)
  P_SHUFFLE = 3,     // per-epoch sample permutation ctr=(uid, op_ctr)
  P_AGGSHUF = 4,     // aggregating shuffle_random   ctr=(uid, op_ctr)
  P_SOUP = 5,        // soup decisions               ctr=(slot, generation)
  P_PERTURB = 6,     // known-fixpoint variation     ctr=(uid, op_ctr)
  P_SOUP_WIDE = 7,   // soup partners of populations > 2^32 slots (64-bit draws) ctr=(slot, generation)
};

struct Rng {
  uint32_t k0, k1;
  SRNN_HD U4 draw(uint64_t id, uint32_t step, uint32_t purpose) const {
    U4 c{(uint32_t)id, (uint32_t)(id >> 32), step, purpose};
    return philox(c, k0, k1);
  }
};

// uniform in [0,1) with 24 random bits
SRNN_HD float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
// uniform in (0,1]
SRNN_HD float u01_open0(uint32_t x) { return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f); }

SRNN_HD bool finitef(float v) { return (__builtin_isfinite(v)) != 0; }

// Permutation of [0, n) (n <= 16) packed as nibbles of a 64-bit register.  Fisher-Yates
// whose swap indices j_i in [0, i] are the mixed-radix digits of ONE uniform 64-bit value
// u (radices n, n-1, ..., 2): j = hi64(u * (i+1)), u = lo64(u * (i+1)).  log2(16!) = 44.3
// bits are consumed, so every permutation's probability is off by < 16!/2^64 (~1e-6
// relative): uniform for all practical purposes.  One Philox draw (128 bits) serves two
// consecutive epochs (steps 2k and 2k+1).  No memory traffic.
SRNN_HD uint64_t perm_bits(const U4& r, uint32_t step) {
  return (step & 1u) ? (((uint64_t)r.w << 32) | r.z) : (((uint64_t)r.y << 32) | r.x);
}
SRNN_HD U4 perm_draw(const Rng& rng, uint64_t id, uint32_t step, uint32_t purpose) {
  return rng.draw(id, (step >> 1) * 64u, purpose);
}
template <int N>
SRNN_HD uint64_t perm_from_bits(uint64_t u) {
  static_assert(N <= 16, "nibble permutation holds at most 16 entries");
  // nibbles 0-7 in plo, 8-15 in phi.  j <= i, so for i < 8 (i is a compile-time constant
  // after unrolling) both nibbles live in plo and the swap is 32-bit (v_bfe_u32 + shifts)
  // instead of variable 64-bit shifts; identical permutation.
  uint32_t plo = 0, phi = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (k < 8) plo |= (uint32_t)k << (4 * k);
    else phi |= (uint32_t)k << (4 * (k - 8));
  }
  uint32_t ul = (uint32_t)u, uh = (uint32_t)(u >> 32);
#pragma unroll
  for (int i = N - 1; i > 0; --i) {
    const uint64_t lo = (uint64_t)ul * (uint32_t)(i + 1);
    const uint64_t hi = (uint64_t)uh * (uint32_t)(i + 1) + (lo >> 32);
    const uint32_t j = (uint32_t)(hi >> 32);
    ul = (uint32_t)lo;
    uh = (uint32_t)hi;
    if (i < 8) {
      const uint32_t ni = (plo >> (4 * i)) & 15u;
      const uint32_t nj = (plo >> (4 * j)) & 15u;
      const uint32_t x = ni ^ nj;
      plo ^= (x << (4 * i)) | (x << (4 * j));
    } else {
      uint64_t p = ((uint64_t)phi << 32) | plo;
      const uint64_t ni = (p >> (4 * i)) & 15u;
      const uint64_t nj = (p >> (4 * j)) & 15u;
      const uint64_t x = ni ^ nj;
      p ^= (x << (4 * i)) | (x << (4 * j));
      plo = (uint32_t)p;
      phi = (uint32_t)(p >> 32);
    }
  }
  return ((uint64_t)phi << 32) | plo;
}
// runtime-n form of perm_from_bits<N> (same permutation; tables built outside a templated kernel)
SRNN_HD uint64_t perm_from_bits_n(int n, uint64_t u) {
  uint64_t p = 0;
  for (int k = 0; k < n; ++k) p |= (uint64_t)k << (4 * k);
  uint32_t ul = (uint32_t)u, uh = (uint32_t)(u >> 32);
  for (int i = n - 1; i > 0; --i) {
    const uint64_t lo = (uint64_t)ul * (uint32_t)(i + 1);
    const uint64_t hi = (uint64_t)uh * (uint32_t)(i + 1) + (lo >> 32);
    const uint32_t j = (uint32_t)(hi >> 32);
    ul = (uint32_t)lo;
    uh = (uint32_t)hi;
    const uint64_t ni = (p >> (4 * i)) & 15u, nj = (p >> (4 * j)) & 15u, x = ni ^ nj;
    p ^= (x << (4 * i)) | (x << (4 * j));
  }
  return p;
}
template <int N>
SRNN_HD uint64_t shuffle16(const Rng& rng, uint64_t id, uint32_t step, uint32_t purpose) {
  return perm_from_bits<N>(perm_bits(perm_draw(rng, id, step, purpose), step));
}

// ----------------------------------------------------------------------------------
// The permutation-table SGD paths load epoch e+1's permutation word at the top of epoch e and
// consume it at the next epoch.  The first word is loaded right before the epoch loop; left
// pending into the loop header, it makes the compiler's wait insertion put an
// `s_waitcnt vmcnt(0)` at the top of EVERY epoch, right behind the next word's load -- a
// whole global-memory latency per epoch on a latency-bound chain (30 % of a lone wave's
// cycles).  Draining it before the loop leaves each word in flight for a whole epoch.
SRNN_HD void perm_prologue_wait() {
#if defined(__HIP_DEVICE_COMPILE__)
  // the builtin (not inline asm): the wait-insertion pass must SEE this wait to know the
  // word is no longer pending at the loop header.  gfx9 encoding: vmcnt(0) expcnt(7) lgkmcnt(15)
  __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
}

// ----------------------------------------------------------------------------------
// Dense layer helpers (row-major (IN, OUT) kernel, y = x . K, fma chain over i).
// ----------------------------------------------------------------------------------
template <int IN, int OUT>
SRNN_HD void dense_fwd(const float* __restrict__ k, const float* __restrict__ x, float* __restrict__ y) {
#pragma unroll
  for (int j = 0; j < OUT; ++j) {
    float acc = x[0] * k[j];
#pragma unroll
    for (int i = 1; i < IN; ++i) acc = fmaf(x[i], k[i * OUT + j], acc);
    y[j] = acc;
  }
}

// gx = K . gy  (gradient wrt the input), then K += x^T (-lr gy)  (in place; one fma per
// weight: the step -lr*gy is formed once per output unit).
template <int IN, int OUT>
SRNN_HD void dense_bwd_update(float* __restrict__ k, const float* __restrict__ x, const float* __restrict__ gy,
                              float* __restrict__ gx, float lr, bool want_gx) {
  if (want_gx) {
#pragma unroll
    for (int i = 0; i < IN; ++i) {
      float acc = k[i * OUT] * gy[0];
#pragma unroll
      for (int j = 1; j < OUT; ++j) acc = fmaf(k[i * OUT + j], gy[j], acc);
      gx[i] = acc;
    }
  }
  float step[OUT];
#pragma unroll
  for (int j = 0; j < OUT; ++j) step[j] = -lr * gy[j];
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < OUT; ++j) k[i * OUT + j] = fmaf(x[i], step[j], k[i * OUT + j]);
}

// ----------------------------------------------------------------------------------
// A plain MLP  IN -> W (x D-1 hidden W->W) -> OUT, linear, no bias.
// Kernels flat: [IN*W][ (D-1) * W*W ][ W*OUT ].
// ----------------------------------------------------------------------------------
template <int IN, int W, int D, int OUT>
struct MLP {
  static constexpr int P = IN * W + (D - 1) * W * W + W * OUT;
  static constexpr int off(int l) { return l == 0 ? 0 : IN * W + (l - 1) * W * W; }
  static constexpr int NACT = IN + D * W;  // activations kept for backprop (inputs of every layer)

  // forward; acts receives the input of every layer: [x (IN)][h1 (W)]...[hD (W)]
  SRNN_HD static void forward(const float* __restrict__ w, const float* __restrict__ x, float* __restrict__ acts,
                              float* __restrict__ y) {
#pragma unroll
    for (int i = 0; i < IN; ++i) acts[i] = x[i];
    dense_fwd<IN, W>(w, acts, acts + IN);
#pragma unroll
    for (int l = 1; l < D; ++l) dense_fwd<W, W>(w + off(l), acts + IN + (l - 1) * W, acts + IN + l * W);
    dense_fwd<W, OUT>(w + off(D), acts + IN + (D - 1) * W, y);
  }

  SRNN_HD static void forward_only(const float* __restrict__ w, const float* __restrict__ x, float* __restrict__ y) {
    float h[W], g[W];
    dense_fwd<IN, W>(w, x, h);
#pragma unroll
    for (int l = 1; l < D; ++l) {
      dense_fwd<W, W>(w + off(l), h, g);
#pragma unroll
      for (int j = 0; j < W; ++j) h[j] = g[j];
    }
    dense_fwd<W, OUT>(w + off(D), h, y);
  }

  // one SGD step given dL/dy (gy), activations from forward(); updates w in place.
  // Folded form: the step st = -lr * dL/d(out) is propagated instead of the gradient
  // (st_in = K . st_out with the pre-update K), so every weight costs one fma and no
  // layer needs a separate -lr scaling.
  SRNN_HD static void backward_update(float* __restrict__ w, const float* __restrict__ acts,
                                      const float* __restrict__ gy, float lr) {
    float so[OUT > W ? OUT : W], si[IN > W ? IN : W];
#pragma unroll
    for (int j = 0; j < OUT; ++j) so[j] = -lr * gy[j];
    step_layer<W, OUT>(w + off(D), acts + IN + (D - 1) * W, so, si, true);
#pragma unroll
    for (int l = D - 1; l >= 1; --l) {
#pragma unroll
      for (int j = 0; j < W; ++j) so[j] = si[j];
      step_layer<W, W>(w + off(l), acts + IN + (l - 1) * W, so, si, true);
    }
#pragma unroll
    for (int j = 0; j < W; ++j) so[j] = si[j];
    step_layer<IN, W>(w, acts, so, si, false);
  }

  // si = K . so (pre-update K) ; K += x (x) so
  template <int I, int O>
  SRNN_HD static void step_layer(float* __restrict__ k, const float* __restrict__ x, const float* __restrict__ so,
                                 float* __restrict__ si, bool want_in) {
    if (want_in) {
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float acc = k[i * O] * so[0];
#pragma unroll
        for (int j = 1; j < O; ++j) acc = fmaf(k[i * O + j], so[j], acc);
        si[i] = acc;
      }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < O; ++j) k[i * O + j] = fmaf(x[i], so[j], k[i * O + j]);
  }
};

// ----------------------------------------------------------------------------------
// Layer shape tables (used for coordinates and init) as constexpr data.
// ----------------------------------------------------------------------------------
struct Shape { int r, c, off; int ortho; };

template <int NL>
struct ShapeTable { Shape s[NL]; };

// normalize_id (reference code/network.py:216-220): v/m if m > 1 else v
constexpr float norm_id(int v, int m) { return m > 1 ? (float)v / (float)m : (float)v; }

template <int P>
struct CoordTable { float c[P][3]; };

template <int P, int NL>
constexpr CoordTable<P> make_coords(const ShapeTable<NL> t) {
  CoordTable<P> ct{};
  int k = 0;
  for (int l = 0; l < NL; ++l)
    for (int i = 0; i < t.s[l].r; ++i)
      for (int j = 0; j < t.s[l].c; ++j) {
        ct.c[k][0] = norm_id(l, NL - 1);
        ct.c[k][1] = norm_id(i, t.s[l].r - 1);
        ct.c[k][2] = norm_id(j, t.s[l].c - 1);
        ++k;
      }
  return ct;
}

// ----------------------------------------------------------------------------------
// Common per-particle predicates (reference code/network.py:44-62, 133-157)
// ----------------------------------------------------------------------------------
template <int P>
SRNN_HD bool is_diverged(const float* w) {
  bool bad = false;
#pragma unroll
  for (int k = 0; k < P; ++k) bad |= !finitef(w[k]);
  return bad;
}
template <int P>
SRNN_HD bool is_zero(const float* w, float eps) {  // inclusive bounds
  bool ok = true;
#pragma unroll
  for (int k = 0; k < P; ++k) ok &= (-eps <= w[k]) && (w[k] <= eps);
  return ok;
}
template <int P>
SRNN_HD bool within_eps(const float* a, const float* b, float eps) {  // strict |a-b| < eps, NaN -> handled by caller
  bool ok = true;
#pragma unroll
  for (int k = 0; k < P; ++k) ok &= !(fabsf(a[k] - b[k]) >= eps);
  return ok;
}

enum Cls : int8_t { C_DIVERGENT = 0, C_FIX_ZERO = 1, C_FIX_OTHER = 2, C_FIX_SEC = 3, C_OTHER = 4 };

// Fisher-Yates permutation of [0,n) driven by one philox stream; perm in byte scratch.
SRNN_HD void fisher_yates(uint8_t* perm, int n, const Rng& rng, uint64_t id, uint32_t step, uint32_t purpose) {
  for (int i = 0; i < n; ++i) perm[i] = (uint8_t)i;
  U4 r{0, 0, 0, 0};
  int used = 4;
  uint32_t blk = 0;
  for (int i = n - 1; i > 0; --i) {
    if (used == 4) {
      // every 4-draw block its own counter: the block index in the purpose word's high bits
      // (step * 64 + blk would run into the next step's blocks for n > 257)
      r = rng.draw(id, step, purpose + (blk << 8));
      ++blk;
      used = 0;
    }
    uint32_t x = used == 0 ? r.x : used == 1 ? r.y : used == 2 ? r.z : r.w;
    ++used;
    int j = (int)(u01(x) * (float)(i + 1));
    if (j > i) j = i;
    uint8_t t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
}

// glorot uniform for a (r, c) kernel at flat offset `off` of particle `uid`
SRNN_HD void glorot_fill(float* w, int off, int r, int c, const Rng& rng, uint64_t uid) {
  const float lim = sqrtf(6.0f / (float)(r + c));
  const int n = r * c;
  for (int b = 0; b < (n + 3) / 4; ++b) {
    U4 u = rng.draw(uid, (uint32_t)off * 1024u + (uint32_t)b, P_INIT);  // blocks unique per (layer offset, block)
    uint32_t xs[4] = {u.x, u.y, u.z, u.w};
    for (int q = 0; q < 4; ++q) {
      int k = b * 4 + q;
      if (k < n) w[off + k] = -lim + 2.0f * lim * u01(xs[q]);
    }
  }
}

// Keras 2.2.4's Orthogonal initializer is the left singular matrix U of a gaussian matrix,
// taken from numpy.linalg.svd -- LAPACK dgesdd, whose sign conventions make U far from Haar:
// for 2x2 it is ALWAYS a reflection (det -1) with a biased angle, for 1x1 it is sign(a).
// That changes the dynamics of linear SimpleRNN stacks: RecurrentNeuralNetwork(2, 2)
// self-training diverges for 76 % of the nets with LAPACK's U (the published 38/50) and for
// ~48 % with a Haar-distributed orthogonal kernel (bench/rnn_divergence_bisect.py).
// lapack_u2 reproduces dgesdd's U for a 2x2 matrix step by step (dgebrd: one Householder
// reflector dlarfg on the first column; dbdsqr on the 2x2 upper bidiagonal: dlasv2's left
// rotation; singular values made positive by flipping rows of V^T, already sorted), which
// tests/test_native_cpu.py checks against numpy.linalg.svd to ~1e-14.
SRNN_HD double f_sign(double a, double b) { return b >= 0.0 ? fabs(a) : -fabs(a); }  // Fortran SIGN
SRNN_HD void dlasv2_left(double f, double g, double h, double* csl, double* snl) {
  double ft = f, fa = fabs(f), ht = h, ha = fabs(h);
  int pmax = 1;
  const bool swap = ha > fa;
  if (swap) {
    pmax = 3;
    double t = ft; ft = ht; ht = t;
    t = fa; fa = ha; ha = t;
  }
  const double gt = g, ga = fabs(g);
  double clt, crt, slt, srt;
  if (ga == 0.0) {
    clt = 1.0, crt = 1.0, slt = 0.0, srt = 0.0;
  } else {
    bool gasmal = true;
    if (ga > fa) {
      pmax = 2;
      if (fa / ga < 2.220446049250313e-16) {
        gasmal = false;
        clt = 1.0, slt = ht / gt, srt = 1.0, crt = ft / gt;
      }
    }
    if (gasmal) {
      const double d = fa - ha;
      double l = (d == fa) ? 1.0 : d / fa;
      const double m = gt / ft;
      double t = 2.0 - l;
      const double mm = m * m, tt = t * t;
      const double s = sqrt(tt + mm);
      const double r = (l == 0.0) ? fabs(m) : sqrt(l * l + mm);
      const double a = 0.5 * (s + r);
      if (mm == 0.0) t = (l == 0.0) ? f_sign(2.0, ft) * f_sign(1.0, gt) : gt / f_sign(d, ft) + m / t;
      else t = (m / (s + t) + m / (r + l)) * (1.0 + a);
      l = sqrt(t * t + 4.0);
      crt = 2.0 / l, srt = t / l;
      clt = (crt + srt * m) / a;
      slt = (ht / ft) * srt / a;
    }
  }
  (void)pmax;
  if (swap) *csl = srt, *snl = crt;
  else *csl = clt, *snl = slt;
}
// U of numpy.linalg.svd(a) for a 2x2 a (row-major), in place
SRNN_HD void lapack_u2(double (&a)[2][2]) {
  const double a11 = a[0][0], a12 = a[0][1], a21 = a[1][0], a22 = a[1][1];
  double tau = 0.0, v = 0.0, beta = a11;
  if (a21 != 0.0) {  // dlarfg(2, a11, a21)
    beta = -f_sign(hypot(a11, a21), a11);
    tau = (beta - a11) / beta;
    v = a21 / (a11 - beta);
  }
  const double w = a12 + v * a22;
  double csl, snl;
  dlasv2_left(beta, a12 - tau * w, a22 - tau * v * w, &csl, &snl);
  // U = (I - tau [1 v]^T [1 v]) * [[csl, -snl], [snl, csl]]
  const double q00 = 1.0 - tau, q01 = -tau * v, q11 = 1.0 - tau * v * v;
  a[0][0] = q00 * csl + q01 * snl;
  a[0][1] = -q00 * snl + q01 * csl;
  a[1][0] = q01 * csl + q11 * snl;
  a[1][1] = -q01 * snl + q11 * csl;
}

// orthogonal (n, n) kernel by modified Gram-Schmidt of a gaussian matrix with
// sign(diag R) correction == QR with positive diagonal (Haar distributed).  The
// orthogonalisation runs in double (Keras' initializer is a float64 numpy QR): in float32
// a single MGS pass loses orthogonality ~ eps32 * cond(A), 1e-4 for unlucky draws.
template <int N>
SRNN_HD void orthogonal_fill(float* w, int off, const Rng& rng, uint64_t uid) {
  double a[N][N];  // a[row][col]
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
      a[i][j] = (double)nrm[cnt & 3];
      ++cnt;
    }
  if constexpr (N == 2) {  // Keras / LAPACK convention (see lapack_u2)
    lapack_u2(a);
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) w[off + i * N + j] = (float)a[i][j];
    return;
  }
  // Gram-Schmidt on columns (N = 1: sign(a), LAPACK's U too; N >= 3: Haar, an approximation
  // of LAPACK's sign conventions -- parity is pinned for the reference's width-2 nets)
  for (int j = 0; j < N; ++j) {
    for (int p = 0; p < j; ++p) {
      double d = 0.0;
      for (int i = 0; i < N; ++i) d = fma(a[i][p], a[i][j], d);
      for (int i = 0; i < N; ++i) a[i][j] = fma(-d, a[i][p], a[i][j]);
    }
    double s = 0.0;
    for (int i = 0; i < N; ++i) s = fma(a[i][j], a[i][j], s);
    const double inv = 1.0 / sqrt(s);
    for (int i = 0; i < N; ++i) a[i][j] *= inv;
  }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) w[off + i * N + j] = (float)a[i][j];
}

// ----------------------------------------------------------------------------------
// Training context: scratch memory for frozen samples / permutation.
// On device it points into LDS (lane-private slices), on host into a stack array.
// ----------------------------------------------------------------------------------
struct TrainCtx {
  float lr;
  Rng rng;
  uint64_t uid;      // particle uid (keys shuffles)
  uint32_t ctr;      // op counter (one per epoch consumed)
  float4* samp;      // >= P float4 slots, slot k at samp[k * stride]
  uint8_t* perm;     // >= P bytes (only for P > 16)
  bool shuffle;
  int stride;        // device: threads per block (slot-major, lane fastest: conflict-free b128)
  int aggregator;    // aggregating nets: samples come from the configured aggregator
  // precomputed epoch permutations (nibble nets, shuffle on): epoch with counter ctr uses
  // ptab[(ctr - pbase) * pstride] (ptab already points at this particle's column), so the
  // SGD chain carries no Philox / Fisher-Yates work (k_perm_table computes them beforehand)
  const uint64_t* ptab = nullptr;
  int64_t pstride = 0;
  uint32_t pbase = 0;
#if defined(SRNN_ORD_TRACE_FINE)
  uint64_t* etrace = nullptr;  // diagnostic build: s_memrealtime at each table epoch's start
#endif
};

struct ApplyCtx {
  Rng rng;
  uint64_t uid;      // uid of the particle whose weights are written (keys shuffle_random)
  uint32_t ctr;
  int aggregator;    // 0 mean, 1 max, 2 max (reference and/or quirk)
  int shuffler;      // 0 none, 1 random
  uint8_t* perm;     // >= P bytes when shuffler == 1
};

// ==================================================================================
// Weightwise(W, D): MLP 4 -> W ... -> 1 evaluated at every (weight, layer, cell, pos)
// point of the target (reference code/network.py:213-289).
// ==================================================================================
template <int W_, int D_>
struct Weightwise {
  static constexpr int KIND = 0;
  static constexpr int W = W_, D = D_, A = 0;
  using Net = MLP<4, W, D, 1>;
  static constexpr int P = Net::P;
  static constexpr int PP = (P + 3) & ~3;
  static constexpr int NL = D + 1;
  static constexpr ShapeTable<NL> shapes() {
    ShapeTable<NL> t{};
    for (int l = 0; l < NL; ++l) {
      t.s[l].r = l == 0 ? 4 : W;
      t.s[l].c = l == D ? 1 : W;
      t.s[l].off = Net::off(l);
      t.s[l].ortho = 0;
    }
    return t;
  }
  static constexpr CoordTable<P> coords = make_coords<P, NL>(shapes());

  // out = f_a(t): every target weight replaced by the net's output at its point.
  SRNN_HD static void apply(const float* __restrict__ a, const float* __restrict__ t, float* __restrict__ out,
                            const ApplyCtx&) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      float x[4] = {t[k], coords.c[k][0], coords.c[k][1], coords.c[k][2]};
      float y[1];
      Net::forward_only(a, x, y);
      out[k] = y[0];
    }
  }

  // Frozen SGD samples in the lane's scratch (LDS on the device, slot-major, lane fastest):
  // P <= 16 keeps (value, coordinates) as float4 per sample (one b128 read per step);
  // larger nets keep only the value per sample (4 B instead of 16 B of LDS per sample and
  // lane: WW(4,3) drops from 53 KB to 13 KB per wave) and read the coordinates of the
  // permuted sample from the constant table.
  static constexpr int SAMP_F4 = P <= 16 ? P : (P + 3) / 4;  // float4 slots per lane

  // One Keras epoch of fit(x, y, batch_size=1, shuffle=True) on the samples of `s`
  // (x_k = point k of s, y_k = s[k]); samples frozen at epoch start. Returns mean loss.
  SRNN_HD static float train_epoch(float* __restrict__ w, const float* __restrict__ s, TrainCtx& c) {
    float* sv = reinterpret_cast<float*>(c.samp);  // P > 16: values only
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if constexpr (P <= 16) c.samp[k * c.stride] = make_float4(s[k], coords.c[k][0], coords.c[k][1], coords.c[k][2]);
      else sv[k * c.stride] = s[k];
    }
    uint64_t pn = 0;
    if constexpr (P <= 16) {
      if (c.shuffle) pn = shuffle16<P>(c.rng, c.uid, c.ctr, P_SHUFFLE);
      else
#pragma unroll
        for (int k = 0; k < P; ++k) pn |= (uint64_t)k << (4 * k);
    } else {
      if (c.shuffle) fisher_yates(c.perm, P, c.rng, c.uid, c.ctr, P_SHUFFLE);
    }
    float loss = 0.f;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      int idx;
      if constexpr (P <= 16) idx = (int)((pn >> (4 * q)) & 15u);
      else idx = c.shuffle ? (int)c.perm[q] : q;
      float4 smp;
      if constexpr (P <= 16) smp = c.samp[idx * c.stride];
      else smp = make_float4(sv[idx * c.stride], coords.c[idx][0], coords.c[idx][1], coords.c[idx][2]);
      float x[4] = {smp.x, smp.y, smp.z, smp.w};
      float acts[Net::NACT], y[1];
      Net::forward(w, x, acts, y);
      float e = y[0] - smp.x;
      loss += e * e;
      // dL/dy = 2e; the folded step -lr * 2e is formed as -(2 lr) * e: the same real product,
      // rounded once, with one multiply less on the per-sample chain
      float gy[1] = {e};
      Net::backward_update(w, acts, gy, 2.0f * c.lr);
    }
    c.ctr += 1;
    return loss / (float)P;
  }

  // E epochs (samples = the weights at each epoch start when SELF, else the fixed
  // teacher row `t`), arithmetic identical to E calls of train_epoch.  Latency-hiding
  // schedule for the nibble-permutation nets (P <= 16, lane per particle, 1-2 waves per
  // SIMD at the 100k-particle soup): the coordinates go to LDS once, each epoch writes
  // only the sample values, all P samples of an epoch are read ahead of its SGD chain in
  // permuted order, and the next epoch's permutation (Philox + Fisher-Yates, independent
  // of the weights) is computed inside the current epoch's block for the scheduler to
  // interleave with the dependent SGD chain.
  // train_epochs with the epoch permutations read from a precomputed table (TrainCtx::ptab):
  // the same permutations, samples and SGD chain -- the next epoch's permutation is a load
  // issued a whole epoch ahead instead of a Philox draw + Fisher-Yates on the chain's SIMD --
  // and the loss accumulated in the last epoch only (earlier epochs' losses are discarded)
  template <bool SELF>
  SRNN_HD static float train_epochs_tab(float* __restrict__ w, const float* __restrict__ t, int E, TrainCtx& c) {
    static_assert(P <= 16, "nibble permutations");
#pragma unroll
    for (int k = 0; k < P; ++k)
      c.samp[k * c.stride] = make_float4(SELF ? w[k] : t[k], coords.c[k][0], coords.c[k][1], coords.c[k][2]);
    const uint64_t* pt = c.ptab + (int64_t)(c.ctr - c.pbase) * c.pstride;
    uint64_t pn = pt[0];
    perm_prologue_wait();
    const float lr2 = 2.0f * c.lr;  // folded step -(2 lr) * err (train_epoch)
    float loss = 0.f;
    for (int e = 0; e < E; ++e) {
#if defined(SRNN_ORD_TRACE_FINE) && defined(__HIP_DEVICE_COMPILE__)
      if (SELF && c.etrace && e < 24) c.etrace[e] = __builtin_amdgcn_s_memrealtime();
#endif
      if (SELF && e > 0)
#pragma unroll
        for (int k = 0; k < P; ++k) reinterpret_cast<float*>(&c.samp[k * c.stride])[0] = w[k];
      const bool last = e + 1 == E;
      const uint64_t pn_next = last ? 0ull : pt[(int64_t)(e + 1) * c.pstride];
      float4 smp[P];
#pragma unroll
      for (int q = 0; q < P; ++q) smp[q] = c.samp[(int)((pn >> (4 * q)) & 15u) * c.stride];
      if (!last) {
#pragma unroll
        for (int q = 0; q < P; ++q) {
          float x[4] = {smp[q].x, smp[q].y, smp[q].z, smp[q].w};
          float acts[Net::NACT], y[1];
          Net::forward(w, x, acts, y);
          float gy[1] = {y[0] - smp[q].x};
          Net::backward_update(w, acts, gy, lr2);
        }
      } else {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          float x[4] = {smp[q].x, smp[q].y, smp[q].z, smp[q].w};
          float acts[Net::NACT], y[1];
          Net::forward(w, x, acts, y);
          float err = y[0] - smp[q].x;
          acc += err * err;
          float gy[1] = {err};
          Net::backward_update(w, acts, gy, lr2);
        }
        loss = acc / (float)P;
      }
      c.ctr += 1;
      pn = pn_next;
    }
    return loss;
  }

  template <bool SELF>
  SRNN_HD static float train_epochs(float* __restrict__ w, const float* __restrict__ t, int E, TrainCtx& c) {
    if constexpr (P <= 16) {
      if (c.ptab && c.shuffle && E > 0) return train_epochs_tab<SELF>(w, t, E, c);
    }
    if constexpr (P > 16) {
      float s[P], loss = 0.f;
#pragma unroll
      for (int k = 0; k < P; ++k) s[k] = SELF ? w[k] : t[k];
      for (int e = 0; e < E; ++e) {
        if (SELF && e > 0)
#pragma unroll
          for (int k = 0; k < P; ++k) s[k] = w[k];
        loss = train_epoch(w, s, c);
      }
      return loss;
    } else {
      if (E <= 0) return 0.f;
#pragma unroll
      for (int k = 0; k < P; ++k)
        c.samp[k * c.stride] = make_float4(SELF ? w[k] : t[k], coords.c[k][0], coords.c[k][1], coords.c[k][2]);
      uint64_t ident = 0;
#pragma unroll
      for (int k = 0; k < P; ++k) ident |= (uint64_t)k << (4 * k);
      float loss = 0.f;
      // one Philox draw per pair of epochs (c.ctr is the same for every lane: uniform branch)
      U4 rr = perm_draw(c.rng, c.uid, c.ctr, P_SHUFFLE);
      uint32_t pair = c.ctr >> 1;
      uint64_t pn = c.shuffle ? perm_from_bits<P>(perm_bits(rr, c.ctr)) : ident;
      const float lr2 = 2.0f * c.lr;  // folded step -(2 lr) * err (train_epoch)
      for (int e = 0; e < E; ++e) {
        if (SELF && e > 0)
#pragma unroll
          for (int k = 0; k < P; ++k) reinterpret_cast<float*>(&c.samp[k * c.stride])[0] = w[k];
        uint64_t pn_next = ident;
        if (c.shuffle) {
          const uint32_t nx = c.ctr + 1u;
          if ((nx >> 1) != pair) {
            pair = nx >> 1;
            rr = perm_draw(c.rng, c.uid, nx, P_SHUFFLE);
          }
          pn_next = perm_from_bits<P>(perm_bits(rr, nx));
        }
        float4 smp[P];
#pragma unroll
        for (int q = 0; q < P; ++q) smp[q] = c.samp[(int)((pn >> (4 * q)) & 15u) * c.stride];
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          float x[4] = {smp[q].x, smp[q].y, smp[q].z, smp[q].w};
          float acts[Net::NACT], y[1];
          Net::forward(w, x, acts, y);
          float err = y[0] - smp[q].x;
          acc += err * err;
          float gy[1] = {err};
          Net::backward_update(w, acts, gy, lr2);
        }
        loss = acc / (float)P;
        c.ctr += 1;
        pn = pn_next;
      }
      return loss;
    }
  }

  SRNN_HD static void init(float* w, const Rng& rng, uint64_t uid) {
    constexpr ShapeTable<NL> t = shapes();
#pragma unroll
    for (int l = 0; l < NL; ++l) glorot_fill(w, t.s[l].off, t.s[l].r, t.s[l].c, rng, uid);
  }
};

// chunk layout of aggregating / fft nets (reference code/network.py:389-403)
template <int P, int A>
struct Chunks {
  static constexpr int CS = P / A;
  static constexpr int LEFT = P - CS * A;
  static_assert(CS >= 1, "aggregates > weights");
  static_assert(P / CS == A, "collect_weights would not produce `aggregates` chunks (SURVEY S4)");
  static constexpr int start(int k) { return k * CS; }
  static constexpr int len(int k) { return k == A - 1 ? CS + LEFT : CS; }
};

template <int P, int A>
SRNN_HD void aggregate(const float* __restrict__ t, float* __restrict__ g, int aggregator) {
  using C = Chunks<P, A>;
#pragma unroll
  for (int k = 0; k < A; ++k) {
    if (aggregator == 0) {
      double acc = 0.0;  // reference sums python floats (double)
#pragma unroll
      for (int i = 0; i < C::len(k); ++i) acc += (double)t[C::start(k) + i];
      g[k] = (float)(acc / (double)C::len(k));
    } else {
      float m = t[C::start(k)];
#pragma unroll
      for (int i = 0; i < C::len(k); ++i) {
        float v = t[C::start(k) + i];
        if (aggregator == 1) m = (v > m) ? v : m;
        else m = (v > m && v != 0.0f) ? v : m;  // `weight > max and weight or max` quirk
      }
      g[k] = m;
    }
  }
}

template <int P>
SRNN_HD void shuffle_out(float* __restrict__ out, const ApplyCtx& c) {
  if (c.shuffler != 1) return;
  fisher_yates(c.perm, P, c.rng, c.uid, c.ctr, P_AGGSHUF);
  float tmp[P];
#pragma unroll
  for (int k = 0; k < P; ++k) tmp[k] = out[k];
  // out[k] = tmp[perm[k]]  (dynamic index into the copy; P is small)
  for (int k = 0; k < P; ++k) {
    int src = c.perm[k];
    float v = tmp[0];
#pragma unroll
    for (int q = 1; q < P; ++q) v = (src == q) ? tmp[q] : v;
    out[k] = v;
  }
}

// ==================================================================================
// Aggregating(A, W, D): chunk-mean -> MLP A->...->A -> broadcast back
// (reference code/network.py:292-439).
// ==================================================================================
template <int A_, int W_, int D_>
struct Aggregating {
  static constexpr int KIND = 1;
  static constexpr int W = W_, D = D_, A = A_;
  using Net = MLP<A, W, D, A>;
  static constexpr int P = Net::P;
  static constexpr int PP = (P + 3) & ~3;
  static constexpr int NL = D + 1;
  using C = Chunks<P, A>;

  SRNN_HD static void apply(const float* __restrict__ a, const float* __restrict__ t, float* __restrict__ out,
                            const ApplyCtx& c) {
    float g[A], h[A];
    aggregate<P, A>(t, g, c.aggregator);
    Net::forward_only(a, g, h);
#pragma unroll
    for (int k = 0; k < A; ++k)
#pragma unroll
      for (int i = 0; i < C::len(k); ++i) out[C::start(k) + i] = h[k];
    shuffle_out<P>(out, c);
  }

  // one sample x = y = aggregated weights (reference :414-417); loss mean over A outputs
  SRNN_HD static float train_epoch(float* __restrict__ w, const float* __restrict__ s, TrainCtx& c) {
    float g[A], acts[Net::NACT], h[A], gy[A];
    aggregate<P, A>(s, g, c.aggregator);  // compute_samples -> get_aggregated_weights (network.py:414)
    Net::forward(w, g, acts, h);
    float loss = 0.f;
#pragma unroll
    for (int k = 0; k < A; ++k) {
      float e = h[k] - g[k];
      loss += e * e;
      gy[k] = 2.0f * e / (float)A;
    }
    Net::backward_update(w, acts, gy, c.lr);
    c.ctr += 1;
    return loss / (float)A;
  }

  SRNN_HD static void init(float* w, const Rng& rng, uint64_t uid) {
    glorot_fill(w, 0, A, W, rng, uid);
    for (int l = 1; l < D; ++l) glorot_fill(w, Net::off(l), W, W, rng, uid);
    glorot_fill(w, Net::off(D), W, A, rng, uid);
  }
};

// ==================================================================================
// FFT(A, W, D): defined real-valued semantics of the reference's broken FFT net
// (code/network.py:442-521):
//   g_k   = Re(FFT_A(t[0:A]))_k              (np.fft.fftn(flat, (A,)) truncates to A)
//   h     = MLP(g)
//   out_m = Re(IFFT_P(pad(h, P)))_m          (np.fft.ifftn(h, (P,)) zero-pads to P)
// The target's weights are used (the reference FFT'd the applying net's own weights).
// ==================================================================================
template <int A_, int W_, int D_>
struct FFTNet {
  static constexpr int KIND = 3;
  static constexpr int W = W_, D = D_, A = A_;
  using Net = MLP<A, W, D, A>;
  static constexpr int P = Net::P;
  static constexpr int PP = (P + 3) & ~3;
  static_assert(A <= P, "fft aggregates must be <= weights");

  SRNN_HD static void reduce(const float* __restrict__ t, float* __restrict__ g) {
#pragma unroll
    for (int k = 0; k < A; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int n = 0; n < A; ++n) acc = fmaf(t[n], cosf(6.283185307179586f * (float)((k * n) % A) / (float)A), acc);
      g[k] = acc;
    }
  }
  SRNN_HD static void apply(const float* __restrict__ a, const float* __restrict__ t, float* __restrict__ out,
                            const ApplyCtx& c) {
    float g[A], h[A];
    reduce(t, g);
    Net::forward_only(a, g, h);
#pragma unroll
    for (int m = 0; m < P; ++m) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < A; ++k) acc = fmaf(h[k], cosf(6.283185307179586f * (float)((k * m) % P) / (float)P), acc);
      out[m] = acc / (float)P;
    }
    shuffle_out<P>(out, c);
  }
  SRNN_HD static float train_epoch(float* __restrict__ w, const float* __restrict__ s, TrainCtx& c) {
    float g[A], acts[Net::NACT], h[A], gy[A];
    reduce(s, g);
    Net::forward(w, g, acts, h);
    float loss = 0.f;
#pragma unroll
    for (int k = 0; k < A; ++k) {
      float e = h[k] - g[k];
      loss += e * e;
      gy[k] = 2.0f * e / (float)A;
    }
    Net::backward_update(w, acts, gy, c.lr);
    c.ctr += 1;
    return loss / (float)A;
  }
  SRNN_HD static void init(float* w, const Rng& rng, uint64_t uid) {
    glorot_fill(w, 0, A, W, rng, uid);
    for (int l = 1; l < D; ++l) glorot_fill(w, Net::off(l), W, W, rng, uid);
    glorot_fill(w, Net::off(D), W, A, rng, uid);
  }
};

// ==================================================================================
// Recurrent(W, D): stacked linear SimpleRNN (1 -> W, W -> W x (D-1), W -> 1) run over
// the flat weight sequence; per-step output replaces the weight
// (reference code/network.py:524-574).  Weights: [K0 R0 K1 R1 ... KD RD].
// ==================================================================================
template <int W_, int D_>
struct Recurrent {
  static constexpr int KIND = 2;
  static constexpr int W = W_, D = D_, A = 0;
  static constexpr int NL = D + 1;  // rnn layers
  static constexpr int in_(int l) { return l == 0 ? 1 : W; }
  static constexpr int un_(int l) { return l == D ? 1 : W; }
  static constexpr int koff(int l) {
    int o = 0;
    for (int q = 0; q < l; ++q) o += in_(q) * un_(q) + un_(q) * un_(q);
    return o;
  }
  static constexpr int roff(int l) { return koff(l) + in_(l) * un_(l); }
  static constexpr int P = koff(NL);
  static constexpr int PP = (P + 3) & ~3;
  static constexpr int HS = D * W + 1;  // hidden units summed over layers

  // one time step of layer l: hn = x.K + hp.R
  template <int L>
  SRNN_HD static void cell(const float* __restrict__ w, const float* __restrict__ x, const float* __restrict__ hp,
                           float* __restrict__ hn) {
    constexpr int I = in_(L), U = un_(L);
    float xk[U], hr[U];
    dense_fwd<I, U>(w + koff(L), x, xk);
    dense_fwd<U, U>(w + roff(L), hp, hr);
#pragma unroll
    for (int j = 0; j < U; ++j) hn[j] = xk[j] + hr[j];
  }

  template <int L>
  SRNN_HD static void step_layers(const float* __restrict__ w, const float* __restrict__ x, float* __restrict__ h) {
    // h holds the hidden state of all layers: layer l at offset l*W
    constexpr int U = un_(L);
    float hn[U];
    cell<L>(w, x, h + L * W, hn);
#pragma unroll
    for (int j = 0; j < U; ++j) h[L * W + j] = hn[j];
    if constexpr (L < D) step_layers<L + 1>(w, h + L * W, h);
  }

  SRNN_HD static void apply(const float* __restrict__ a, const float* __restrict__ t, float* __restrict__ out,
                            const ApplyCtx&) {
    float h[HS];
#pragma unroll
    for (int q = 0; q < HS; ++q) h[q] = 0.f;
#pragma unroll
    for (int s = 0; s < P; ++s) {
      float x[1] = {t[s]};
      step_layers<0>(a, x, h);
      out[s] = h[D * W];
    }
  }

  // backward through one layer at one time step. dh: gradient wrt this layer's output
  // at time s (already includes the carry from s+1). Writes dx (grad wrt layer input)
  // and the new carry (dh . R^T); accumulates kernel grads into gw.
  template <int L>
  SRNN_HD static void cell_bwd(const float* __restrict__ w, float* __restrict__ gw, const float* __restrict__ x,
                               const float* __restrict__ hp, const float* __restrict__ dh, float* __restrict__ dx,
                               float* __restrict__ carry) {
    constexpr int I = in_(L), U = un_(L);
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < U; ++j) gw[koff(L) + i * U + j] = fmaf(x[i], dh[j], gw[koff(L) + i * U + j]);
#pragma unroll
    for (int i = 0; i < U; ++i)
#pragma unroll
      for (int j = 0; j < U; ++j) gw[roff(L) + i * U + j] = fmaf(hp[i], dh[j], gw[roff(L) + i * U + j]);
    if (L > 0) {
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < U; ++j) acc = fmaf(w[koff(L) + i * U + j], dh[j], acc);
        dx[i] = acc;
      }
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < U; ++j) acc = fmaf(w[roff(L) + i * U + j], dh[j], acc);
      carry[i] = acc;
    }
  }

  template <int L>
  SRNN_HD static void bwd_layers(const float* __restrict__ w, float* __restrict__ gw, const float* __restrict__ hs_t,
                                 const float* __restrict__ hs_p, float x0, float* __restrict__ dtop,
                                 float* __restrict__ carry) {
    // dtop: gradient wrt layer L's output coming from layer L+1 (or the loss)
    constexpr int U = un_(L), I = in_(L);
    float dh[U], dx[I > 0 ? I : 1], cr[U];
#pragma unroll
    for (int j = 0; j < U; ++j) dh[j] = dtop[j] + carry[L * W + j];
    float xin[I];
    if constexpr (L == 0) xin[0] = x0;
    else {
#pragma unroll
      for (int i = 0; i < I; ++i) xin[i] = hs_t[(L - 1) * W + i];
    }
    cell_bwd<L>(w, gw, xin, hs_p + L * W, dh, dx, cr);
#pragma unroll
    for (int j = 0; j < U; ++j) carry[L * W + j] = cr[j];
    if constexpr (L > 0) bwd_layers<L - 1>(w, gw, hs_t, hs_p, x0, dx, carry);
  }

  // one sample x = y = s (1, P, 1), loss mean over P; one SGD step (BPTT)
  SRNN_HD static float train_epoch(float* __restrict__ w, const float* __restrict__ s, TrainCtx& c) {
    float hs[P][HS];  // hidden states of every layer at every step
    float h[HS];
#pragma unroll
    for (int q = 0; q < HS; ++q) h[q] = 0.f;
#pragma unroll
    for (int t = 0; t < P; ++t) {
      float x[1] = {s[t]};
      step_layers<0>(w, x, h);
#pragma unroll
      for (int q = 0; q < HS; ++q) hs[t][q] = h[q];
    }
    float gw[P];
#pragma unroll
    for (int k = 0; k < P; ++k) gw[k] = 0.f;
    float carry[HS];
#pragma unroll
    for (int q = 0; q < HS; ++q) carry[q] = 0.f;
    float loss = 0.f;
    float zeros[HS];
#pragma unroll
    for (int q = 0; q < HS; ++q) zeros[q] = 0.f;
#pragma unroll
    for (int t = P - 1; t >= 0; --t) {
      float e = hs[t][D * W] - s[t];
      loss += e * e;
      float dtop[1] = {2.0f * e / (float)P};
      bwd_layers<D>(w, gw, hs[t], t > 0 ? hs[t - 1] : zeros, s[t], dtop, carry);
    }
#pragma unroll
    for (int k = 0; k < P; ++k) w[k] = fmaf(gw[k], -c.lr, w[k]);
    c.ctr += 1;
    return loss / (float)P;
  }

  template <int L>
  SRNN_HD static void init_layers(float* w, const Rng& rng, uint64_t uid) {
    glorot_fill(w, koff(L), in_(L), un_(L), rng, uid);
    orthogonal_fill<un_(L)>(w, roff(L), rng, uid);
    if constexpr (L < D) init_layers<L + 1>(w, rng, uid);
  }
  SRNN_HD static void init(float* w, const Rng& rng, uint64_t uid) { init_layers<0>(w, rng, uid); }
};

}  // namespace srnn
