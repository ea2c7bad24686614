/*
 * oracle/lcd_oracle.c — CPU restatement of Kimera-Multi-LCD's loop-closure
 * verification. TEST INFRASTRUCTURE
 * ONLY (parity checker + cpu_baseline of bench.py); never linked into the
 * product (kimera-multi_amd/kmx).
 *
 * PARITY STATUS: Kimera-Multi-LCD, opengv, OpenCV and DBoW2 are not vendored
 *  => "parity unpinned" against upstream. Pinned here by:
 *   - the sampler against the real libstdc++ std::mt19937 /
 *     std::uniform_int_distribution<int>(0, INT_MAX) of this container (GCC 11
 *     variant, tests/golden/mt19937_gcc11.json) and the GCC-9 rejection path
 *     restated from uniform_int_dist.h:318-325 (SURVEY.md §0 finding 5);
 *   - analytic known answers: noise-free planted relative poses must be
 *     recovered and planted inlier sets found (tests/test_oracle_lcd.py).
 *
 * Restated behaviour (citations are the in-tree evidence for each rule):
 *   knn2 + Lowe ........ computeMatchedIndices (drawio:2583-2586), matcher
 *                        "BruteForce-L1" (docker/copy/kimera_multi_lcd.patch:33-35)
 *                        or Hamming, lowe_ratio 0.7 (params/D455/LcdParams.yaml:16);
 *                        OpenCV batchDistance insertion order: the two smallest
 *                        (distance, train index) pairs, strict '<' keeps ties in
 *                        index order.
 *   2D-2D RANSAC ........ geometricVerificationNister (drawio:2589-2592):
 *                        opengv sac::Ransac loop (k = log(1-p)/log(1-w^5),
 *                        max_skip = 10 * max_iterations), CentralRelativePose
 *                        problem with the 5-point solver selected by
 *                        ransac_2d2d_algorithm (LcdParams.yaml:73): 0
 *                        Stewenius (the reference config; graded 10x20
 *                        Gauss-Jordan -> 10x10 action matrix -> eigen-
 *                        decomposition, orc_fivept_stewenius) or 1 Nister
 *                        (10x20 Gauss-Jordan -> 3x3 polynomial matrix ->
 *                        degree-10 polynomial, real roots by Sturm bisection), models
 *                        = the 4 (R, t) decompositions of every essential
 *                        matrix, the one with the smallest error on the sample
 *                        kept; error = (1 - f1.r1) + (1 - f2.r2) after mid-point
 *                        triangulation; threshold 1e-6, 500 iterations, p 0.995,
 *                        fixed seed 12345 (LcdParams.yaml:55, 64-66).
 *   3D-3D .............. recoverPose (drawio:2595-2598) with
 *                        ransac_use_1point_3d3d = 1 (LcdParams.yaml:58): the
 *                        2D-2D rotation is kept, every stereo correspondence
 *                        votes for t_j = p_q - R p_m, the largest consistent set
 *                        (|t_j - t_i| < 0.3 m, LcdParams.yaml:56) wins; = 0:
 *                        Arun 3-point RANSAC (ransac_arun).
 *   accept ............. mono >= 10, stereo >= 5 (LcdParams.yaml:51-52).
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/kmx_abi.h"

/* ------------------------------------------------------------- sampler -- */
typedef struct {
  uint32_t mt[624];
  int idx;
} orc_mt19937;

static void mt_seed(orc_mt19937* m, uint32_t s) {
  m->mt[0] = s;
  for (int i = 1; i < 624; ++i) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
  m->idx = 624;
}

static uint32_t mt_next(orc_mt19937* m) {
  if (m->idx >= 624) {
    for (int i = 0; i < 624; ++i) {
      const uint32_t y = (m->mt[i] & 0x80000000u) | (m->mt[(i + 1) % 624] & 0x7fffffffu);
      m->mt[i] = m->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->idx = 0;
  }
  uint32_t y = m->mt[m->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* std::uniform_int_distribution<int>(0, INT_MAX)(mt19937): urange 2^31 - 1 from a
 * 32-bit engine. GCC 9: downscaling by 2 divisions, scaling = 1, reject x >= 2^31.
 * GCC 11: Lemire with range 2^31, threshold 0 -> (x * 2^31) >> 32 = x >> 1. */
static int uid_draw(orc_mt19937* m, int variant) {
  if (variant == KMX_RNG_GCC11) return (int)(mt_next(m) >> 1);
  uint32_t x;
  do x = mt_next(m);
  while (x >= 0x80000000u);
  return (int)x;
}

/* The engine a RANSAC problem draws from (LC5, README.md:35-36). rng_stream 0:
 * every SampleConsensusProblem seeds its own engine with ransac_seed (opengv's
 * constructor: rng_alg_.seed(12345u), and std::bind copies the engine into the
 * problem's generator, so a problem never advances anyone else's engine);
 * rng_stream 1: the fork's thread_local engine read as ONE engine per
 * verification thread that every problem continues, seeded once when the
 * thread starts (the caller passes it as `stream`). */
static orc_mt19937* problem_rng(const kmx_lcd_params* P, orc_mt19937* local, orc_mt19937* stream) {
  if (stream) return stream;
  mt_seed(local, P->ransac_seed);
  return local;
}

int orc_mt19937_stream(uint32_t seed, int variant, int32_t n, int32_t* out) {
  orc_mt19937 m;
  mt_seed(&m, seed);
  for (int i = 0; i < n; ++i) out[i] = (variant < 0) ? (int32_t)mt_next(&m) : uid_draw(&m, variant);
  return 0;
}

/* opengv SampleConsensusProblem::drawIndexSample over the persistent shuffled
 * index vector; one call per RANSAC pass. Writes the sample sequence of
 * `passes` passes for K correspondences (test hook + GPU table check). */
int orc_ransac_samples(uint32_t seed, int variant, int32_t K, int32_t passes, int32_t* out /* passes*5 */) {
  if (K < 5) return KMX_EINVAL;
  orc_mt19937 m;
  mt_seed(&m, seed);
  int32_t* sh = (int32_t*)malloc(sizeof(int32_t) * K);
  for (int i = 0; i < K; ++i) sh[i] = i;
  for (int p = 0; p < passes; ++p) {
    for (int i = 0; i < 5; ++i) {
      const int r = uid_draw(&m, variant);
      const int j = i + (int)((size_t)r % (size_t)(K - i));
      const int32_t t = sh[i];
      sh[i] = sh[j];
      sh[j] = t;
    }
    for (int i = 0; i < 5; ++i) out[p * 5 + i] = sh[i];
  }
  free(sh);
  return 0;
}

/* ---------------------------------------------------------------- knn2 -- */
static int desc_dist(int norm, const uint8_t* a, const uint8_t* b) {
  int s = 0;
  if (norm == KMX_NORM_HAMMING) {
    for (int k = 0; k < 32; ++k) s += __builtin_popcount((unsigned)(a[k] ^ b[k]));
  } else {
    for (int k = 0; k < 32; ++k) s += abs((int)a[k] - (int)b[k]);
  }
  return s;
}

int orc_lcd_knn2(int norm, double lowe, const uint8_t* q, int32_t nq, const uint8_t* m, int32_t nm,
                 int32_t* pairs, int32_t* k) {
  int cnt = 0;
  if (nm >= 2) {
    for (int i = 0; i < nq; ++i) {
      int d0 = INT_MAX, d1 = INT_MAX, j0 = -1, j1 = -1;
      for (int j = 0; j < nm; ++j) {
        const int d = desc_dist(norm, q + 32 * i, m + 32 * j);
        if (d < d1) { /* batchDistance insertion, strict '<' */
          if (d < d0) { d1 = d0; j1 = j0; d0 = d; j0 = j; }
          else { d1 = d; j1 = j; }
        }
      }
      (void)j1;
      if ((double)(float)d0 < lowe * (double)(float)d1) {
        pairs[2 * cnt] = i;
        pairs[2 * cnt + 1] = j0;
        ++cnt;
      }
    }
  }
  *k = cnt;
  return 0;
}

/* ------------------------------------------------- small linear algebra -- */
static void cross3(const double a[3], const double b[3], double c[3]) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double det3(const double M[9]) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* symmetric 3x3 Jacobi eigen-decomposition (same rotation sequence as the GPU) */
static void sym_eig3(double A[9], double V[9]) {
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    if (A[1] == 0.0 && A[2] == 0.0 && A[5] == 0.0) break; /* every rotation would be skipped */
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        const double apq = A[p * 3 + q];
        if (apq == 0.0) continue;
        const double app = A[p * 3 + p], aqq = A[q * 3 + q];
        /* negligible next to both diagonal entries: zero it (Rutishauser's threshold rule, Handbook for Automatic Computation II/1, 1971) */
        const double g = 100.0 * fabs(apq);
        if (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq)) {
          A[p * 3 + q] = 0.0;
          A[q * 3 + p] = 0.0;
          continue;
        }
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cs = 1.0 / sqrt(t * t + 1.0), sn = t * cs;
        for (int k = 0; k < 3; ++k) {
          const double akp = A[k * 3 + p], akq = A[k * 3 + q];
          A[k * 3 + p] = cs * akp - sn * akq;
          A[k * 3 + q] = sn * akp + cs * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = A[p * 3 + k], aqk = A[q * 3 + k];
          A[p * 3 + k] = cs * apk - sn * aqk;
          A[q * 3 + k] = sn * apk + cs * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
          V[k * 3 + p] = cs * vkp - sn * vkq;
          V[k * 3 + q] = sn * vkp + cs * vkq;
        }
      }
  }
}

/* SVD of a 3x3 matrix: E = U diag(s) V^T, s descending, U = [E v1/s1, E v2/s2, u1 x u2]. */
static void svd3(const double E[9], double U[9], double s[3], double V[9]) {
  double A[9], W[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 3; ++k) acc += E[k * 3 + i] * E[k * 3 + j];
      A[i * 3 + j] = acc;
    }
  sym_eig3(A, W);
  int ord[3] = {0, 1, 2};
  for (int a = 0; a < 3; ++a) /* sort eigenvalues descending (stable) */
    for (int b = 0; b < 2 - a; ++b)
      if (A[ord[b] * 4] < A[ord[b + 1] * 4]) { const int t = ord[b]; ord[b] = ord[b + 1]; ord[b + 1] = t; }
  for (int c = 0; c < 3; ++c) {
    s[c] = sqrt(fmax(A[ord[c] * 4], 0.0));
    for (int r = 0; r < 3; ++r) V[r * 3 + c] = W[r * 3 + ord[c]];
  }
  double u[3][3];
  for (int c = 0; c < 2; ++c) {
    for (int r = 0; r < 3; ++r) u[c][r] = (E[r * 3 + 0] * V[0 * 3 + c] + E[r * 3 + 1] * V[1 * 3 + c] + E[r * 3 + 2] * V[2 * 3 + c]);
    const double n = sqrt(dot3(u[c], u[c]));
    for (int r = 0; r < 3; ++r) u[c][r] = (n > 0.0) ? u[c][r] / n : 0.0;
  }
  cross3(u[0], u[1], u[2]);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) U[r * 3 + c] = u[c][r];
}

/* ------------------------------------------------ 5-point (Nister 2004) -- */
/* Polynomials in (x, y, z): degree-1 terms [x, y, z, 1]; degree-2 terms in
 * the order D2 below; degree-3 terms in the column order MONO of the 10x20
 * system (Nister 2004). Products accumulate term by term in (i, j) order. */
static const int D1[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
static const int D2[10][3] = {{2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {0, 2, 0}, {0, 1, 1},
                              {0, 0, 2}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
static const int MONO[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                                {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                                {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
static int idx2(int a, int b, int c) {
  for (int i = 0; i < 10; ++i)
    if (D2[i][0] == a && D2[i][1] == b && D2[i][2] == c) return i;
  return -1;
}
static int idx3(int a, int b, int c) {
  for (int i = 0; i < 20; ++i)
    if (MONO[i][0] == a && MONO[i][1] == b && MONO[i][2] == c) return i;
  return -1;
}
/* out2 = a1 * b1 ; out3 = a2 * b1 (out arrays zeroed by the callee) */
static void mul11(const double* a, const double* b, double* out) {
  for (int k = 0; k < 10; ++k) out[k] = 0.0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      out[idx2(D1[i][0] + D1[j][0], D1[i][1] + D1[j][1], D1[i][2] + D1[j][2])] += a[i] * b[j];
}
static void mul21(const double* a, const double* b, double* out) {
  for (int k = 0; k < 20; ++k) out[k] = 0.0;
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 4; ++j)
      out[idx3(D2[i][0] + D1[j][0], D2[i][1] + D1[j][1], D2[i][2] + D1[j][2])] += a[i] * b[j];
}

/* 4-dim null space of the 5x9 epipolar system via Householder QR of its transpose */
static void nullspace_5x9(const double Q[5][9], double N[4][9]) {
  double A[9][5];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 5; ++j) A[i][j] = Q[j][i];
  double vs[5][9];
  for (int k = 0; k < 5; ++k) {
    double nx = 0.0;
    for (int i = k; i < 9; ++i) nx += A[i][k] * A[i][k];
    nx = sqrt(nx);
    const double alpha = (A[k][k] >= 0.0) ? -nx : nx;
    double v[9] = {0};
    for (int i = k; i < 9; ++i) v[i] = A[i][k];
    v[k] -= alpha;
    double nv = 0.0;
    for (int i = k; i < 9; ++i) nv += v[i] * v[i];
    nv = sqrt(nv);
    for (int i = 0; i < 9; ++i) vs[k][i] = (nv > 0.0 && i >= k) ? v[i] / nv : 0.0;
    for (int j = k; j < 5; ++j) {
      double d = 0.0;
      for (int i = k; i < 9; ++i) d += vs[k][i] * A[i][j];
      for (int i = k; i < 9; ++i) A[i][j] -= 2.0 * vs[k][i] * d;
    }
  }
  for (int c = 0; c < 4; ++c) { /* N_c = H0 H1 H2 H3 H4 e_{5+c} */
    double x[9] = {0};
    x[5 + c] = 1.0;
    for (int k = 4; k >= 0; --k) {
      double d = 0.0;
      for (int i = k; i < 9; ++i) d += vs[k][i] * x[i];
      for (int i = k; i < 9; ++i) x[i] -= 2.0 * vs[k][i] * d;
    }
    for (int i = 0; i < 9; ++i) N[c][i] = x[i];
  }
}

static double poly_eval(const double* c, int deg, double z) {
  double v = c[deg];
  for (int i = deg - 1; i >= 0; --i) v = v * z + c[i];
  return v;
}

/* Safeguarded Newton on an isolating interval [a, b]: Newton steps that
 * leave the bracket fall back to bisection; the bracket follows the sign at
 * its left end; stops when a step moves less than 1e-15 relative. */
static double refine_root(const double* c, int deg, double a, double b) {
  double dc[10];
  for (int i = 0; i < deg; ++i) dc[i] = (double)(i + 1) * c[i + 1];
  double fa = poly_eval(c, deg, a);
  double x = 0.5 * (a + b);
  for (int it = 0; it < 60; ++it) {
    const double fx = poly_eval(c, deg, x);
    if (fx == 0.0) return x;
    if ((fx < 0.0) == (fa < 0.0)) { a = x; fa = fx; }
    else b = x;
    const double dfx = poly_eval(dc, deg - 1, x);
    double xn = (dfx != 0.0) ? x - fx / dfx : 0.5 * (a + b);
    if (fabs(xn - x) <= 1e-15 * fmax(1.0, fabs(x))) return xn;  /* converged (before the safeguard) */
    if (!(xn > a && xn < b)) {
      xn = 0.5 * (a + b);
      if (fabs(xn - x) <= 1e-15 * fmax(1.0, fabs(x))) return xn;
    }
    x = xn;
  }
  return x;
}

/* Root bound of the monic a (degree deg), Fujiwara's
 *   |z| <= 2 max_i |a_i|^(1/(deg-i))
 * with every term rounded up to a power of two by exponent arithmetic only
 * (ilogb / ldexp are exact, so host and device agree bit for bit):
 * |a_i| < 2^(e+1), e = ilogb(a_i) => term <= 2^ceil((e+1)/(deg-i)). Non-finite
 * coefficients fall back to Cauchy's 1 + max |a_i|; p = z^deg gives 1. */
static double root_bound(const double* a, int deg) {
  int kmax = INT_MIN, fin = 1;
  double cauchy = 0.0;
  for (int i = 0; i < deg; ++i) {
    cauchy = fmax(cauchy, fabs(a[i]));
    if (!isfinite(a[i])) {
      fin = 0;
    } else if (a[i] != 0.0) {
      const int x = ilogb(a[i]) + 1, m = deg - i;
      const int k = x >= 0 ? (x + m - 1) / m : -((-x) / m);
      if (k > kmax) kmax = k;
    }
  }
  if (!fin) return cauchy + 1.0;
  if (kmax == INT_MIN) return 1.0;
  return ldexp(1.0, kmax + 1);
}

/* real roots of a polynomial (ascending coefficients) by Sturm-sequence
 * bisection; deterministic fixed-depth refinement. */
static int real_roots(const double* coef, int deg_in, double* roots) {
  int deg = deg_in;
  while (deg > 0 && coef[deg] == 0.0) --deg;
  if (deg <= 0) return 0;
  double S[11][11];
  int sd[11];
  int ns = 0;
  for (int i = 0; i <= deg; ++i) S[0][i] = coef[i] / coef[deg];
  sd[0] = deg;
  for (int i = 0; i < deg; ++i) S[1][i] = (double)(i + 1) * S[0][i + 1];
  sd[1] = deg - 1;
  ns = 2;
  while (sd[ns - 1] > 0 && ns < 11) {
    double r[11];
    const int da = sd[ns - 2], db = sd[ns - 1];
    for (int i = 0; i <= da; ++i) r[i] = S[ns - 2][i];
    for (int k = da - db; k >= 0; --k) { /* long division remainder */
      const double f = r[k + db] / S[ns - 1][db];
      for (int i = 0; i <= db; ++i) r[k + i] -= f * S[ns - 1][i];
    }
    int dr = db - 1;
    double mx = 0.0;
    for (int i = 0; i <= da; ++i) mx = fmax(mx, fabs(S[ns - 2][i]));
    while (dr >= 0 && fabs(r[dr]) <= 1e-14 * mx) --dr;
    if (dr < 0) break; /* repeated roots: stop the sequence here */
    for (int i = 0; i <= dr; ++i) S[ns][i] = -r[i];
    sd[ns] = dr;
    ++ns;
  }
  const double bound = root_bound(S[0], deg);
#define SIGNCH(zv, out)                                        \
  do {                                                         \
    int ch_ = 0;                                               \
    double prev_ = 0.0;                                        \
    for (int s_ = 0; s_ < ns; ++s_) {                          \
      const double v_ = poly_eval(S[s_], sd[s_], (zv));        \
      if (v_ != 0.0) {                                         \
        if (prev_ != 0.0 && ((v_ < 0.0) != (prev_ < 0.0))) ++ch_; \
        prev_ = v_;                                            \
      }                                                        \
    }                                                          \
    (out) = ch_;                                               \
  } while (0)
  /* 64-ary Sturm isolation: an interval is cut at the 63 points
   * lo + i * ((hi - lo) / 64); the root counts of the 64 pieces come from the
   * sign-change counts at those points (pieces with count 1 are refined by
   * refine_root, count > 1 recurse, up to RR_DEPTH levels). The GPU evaluates
   * the 63 points of a level in one wavefront, so both sides use exactly
   * these points, and refines all isolated roots in parallel lanes. */
#define RR_SPLIT 64
#define RR_DEPTH 12
  double st_lo[RR_SPLIT * RR_DEPTH + 1], st_hi[RR_SPLIT * RR_DEPTH + 1];
  int st_vl[RR_SPLIT * RR_DEPTH + 1], st_vh[RR_SPLIT * RR_DEPTH + 1], st_d[RR_SPLIT * RR_DEPTH + 1];
  int sp = 0, nr = 0;
  int vlo, vhi;
  SIGNCH(-bound, vlo);
  SIGNCH(bound, vhi);
  st_lo[sp] = -bound; st_hi[sp] = bound; st_vl[sp] = vlo; st_vh[sp] = vhi; st_d[sp] = 0; ++sp;
  while (sp > 0) {
    --sp;
    const double lo = st_lo[sp], hi = st_hi[sp];
    const int vl = st_vl[sp], vh = st_vh[sp], dep = st_d[sp];
    const int cnt = vl - vh;
    if (cnt <= 0) continue;
    if (cnt == 1 || dep >= RR_DEPTH) {
      if (nr < 10) roots[nr++] = refine_root(S[0], deg, lo, hi);
      continue;
    }
    const double w = (hi - lo) / RR_SPLIT;
    int v[RR_SPLIT + 1];
    double x[RR_SPLIT + 1];
    x[0] = lo; v[0] = vl;
    x[RR_SPLIT] = hi; v[RR_SPLIT] = vh;
    for (int i = 1; i < RR_SPLIT; ++i) {
      x[i] = lo + (double)i * w;
      SIGNCH(x[i], v[i]);
    }
    for (int j = RR_SPLIT - 1; j >= 0; --j) /* pushed right to left: popped in increasing x */
      if (v[j] - v[j + 1] > 0) {
        st_lo[sp] = x[j]; st_hi[sp] = x[j + 1]; st_vl[sp] = v[j]; st_vh[sp] = v[j + 1]; st_d[sp] = dep + 1; ++sp;
      }
  }
#undef SIGNCH
  /* ascending order */
  for (int a = 0; a < nr; ++a)
    for (int b = 0; b + 1 < nr - a; ++b)
      if (roots[b] > roots[b + 1]) { const double t = roots[b]; roots[b] = roots[b + 1]; roots[b + 1] = t; }
  return nr;
}

/* The 5-point constraint system shared by both minimal solvers: the null
 * space N of the 5x9 epipolar rows (E = x N0 + y N1 + z N2 + N3) and the 10
 * cubic constraints (rows 0..8: 2 E E^T E - tr(E E^T) E = 0, row 9: det E = 0)
 * in the 20 monomials of MONO. */
static void fivept_system(const double* f1, const double* f2, double N[4][9], double A[10][20]) {
  double Q[5][9];
  for (int i = 0; i < 5; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) Q[i][a * 3 + b] = f1[3 * i + a] * f2[3 * i + b];
  nullspace_5x9(Q, N);
  double E[9][4]; /* E_e(x, y, z) = N0_e x + N1_e y + N2_e z + N3_e */
  for (int e = 0; e < 9; ++e)
    for (int c = 0; c < 4; ++c) E[e][c] = N[c][e];
  /* row 9: det(E) by cofactors of the first row */
  {
    double t1[10], t2[10], c2[10], m[20];
    for (int k = 0; k < 20; ++k) A[9][k] = 0.0;
    mul11(E[4], E[8], t1); mul11(E[5], E[7], t2);
    for (int k = 0; k < 10; ++k) c2[k] = t1[k] - t2[k];
    mul21(c2, E[0], m);
    for (int k = 0; k < 20; ++k) A[9][k] += m[k];
    mul11(E[3], E[8], t1); mul11(E[5], E[6], t2);
    for (int k = 0; k < 10; ++k) c2[k] = t1[k] - t2[k];
    mul21(c2, E[1], m);
    for (int k = 0; k < 20; ++k) A[9][k] -= m[k];
    mul11(E[3], E[7], t1); mul11(E[4], E[6], t2);
    for (int k = 0; k < 10; ++k) c2[k] = t1[k] - t2[k];
    mul21(c2, E[2], m);
    for (int k = 0; k < 20; ++k) A[9][k] += m[k];
  }
  /* rows 0..8: 2 E E^T E - tr(E E^T) E */
  {
    double EEt[9][10], tr[10], t[10], m[20];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        for (int k = 0; k < 10; ++k) EEt[i * 3 + j][k] = 0.0;
        for (int l = 0; l < 3; ++l) {
          mul11(E[i * 3 + l], E[j * 3 + l], t);
          for (int k = 0; k < 10; ++k) EEt[i * 3 + j][k] += t[k];
        }
      }
    for (int k = 0; k < 10; ++k) tr[k] = EEt[0][k] + EEt[4][k] + EEt[8][k];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double* r = A[i * 3 + j];
        for (int k = 0; k < 20; ++k) r[k] = 0.0;
        for (int l = 0; l < 3; ++l) {
          mul21(EEt[i * 3 + l], E[l * 3 + j], m);
          for (int k = 0; k < 20; ++k) r[k] += 2.0 * m[k];
        }
        mul21(tr, E[i * 3 + j], m);
        for (int k = 0; k < 20; ++k) r[k] -= m[k];
      }
  }
}

/* Gauss-Jordan with partial pivoting on the first 10 columns of the 10x20
 * system: A = [I | C] on success, 0 on a zero pivot. */
static int gj_10x20(double A[10][20]) {
  for (int k = 0; k < 10; ++k) {
    int p = k;
    for (int i = k + 1; i < 10; ++i)
      if (fabs(A[i][k]) > fabs(A[p][k])) p = i;
    if (A[p][k] == 0.0) return 0;
    if (p != k)
      for (int c = 0; c < 20; ++c) { const double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
    const double inv = 1.0 / A[k][k];
    for (int c = 0; c < 20; ++c) A[k][c] *= inv;
    for (int i = 0; i < 10; ++i) {
      if (i == k) continue;
      const double f = A[i][k];
      if (f == 0.0) continue;
      for (int c = 0; c < 20; ++c) A[i][c] -= f * A[k][c];
    }
  }
  return 1;
}

/* Essential matrices E (row-major, unit Frobenius norm) with f1^T E f2 = 0 for
 * the five bearing pairs; returns their number (<= 10). */
int orc_fivept_nister(const double* f1 /*5x3*/, const double* f2 /*5x3*/, double* Es /*10x9*/) {
  double N[4][9], A[10][20];
  fivept_system(f1, f2, N, A);
  if (!gj_10x20(A)) return 0;
  /* <k> = e - z f, <l> = g - z h, <m> = i - z j (rows 4..9); B(z) = [x-coef, y-coef, 1-coef] */
  double Bp[3][3][5];
  for (int q = 0; q < 3; ++q) {
    const double* e = &A[4 + 2 * q][10];
    const double* f = &A[5 + 2 * q][10];
    /* right monomials: 0 xz2, 1 xz, 2 x, 3 yz2, 4 yz, 5 y, 6 z3, 7 z2, 8 z, 9 1 */
    double* px = Bp[q][0];
    double* py = Bp[q][1];
    double* pc = Bp[q][2];
    px[0] = e[2]; px[1] = e[1] - f[2]; px[2] = e[0] - f[1]; px[3] = -f[0]; px[4] = 0.0;
    py[0] = e[5]; py[1] = e[4] - f[5]; py[2] = e[3] - f[4]; py[3] = -f[3]; py[4] = 0.0;
    pc[0] = e[9]; pc[1] = e[8] - f[9]; pc[2] = e[7] - f[8]; pc[3] = e[6] - f[7]; pc[4] = -f[6];
  }
  /* n(z) = det B(z), degree <= 10 */
  double n[11] = {0};
  {
    double c1[8], c2[8], c3[8];
#define PMUL(a, da, b, db, out)                                        \
  do {                                                                 \
    for (int i_ = 0; i_ <= (da) + (db); ++i_) (out)[i_] = 0.0;         \
    for (int i_ = 0; i_ <= (da); ++i_)                                 \
      for (int j_ = 0; j_ <= (db); ++j_) (out)[i_ + j_] += (a)[i_] * (b)[j_]; \
  } while (0)
    double t1[8], t2[8];
    /* q_l r_m - r_l q_m (deg 7) */
    PMUL(Bp[1][1], 3, Bp[2][2], 4, t1); PMUL(Bp[1][2], 4, Bp[2][1], 3, t2);
    for (int i = 0; i < 8; ++i) c1[i] = t1[i] - t2[i];
    /* p_l r_m - r_l p_m */
    PMUL(Bp[1][0], 3, Bp[2][2], 4, t1); PMUL(Bp[1][2], 4, Bp[2][0], 3, t2);
    for (int i = 0; i < 8; ++i) c2[i] = t1[i] - t2[i];
    /* p_l q_m - q_l p_m (deg 6) */
    PMUL(Bp[1][0], 3, Bp[2][1], 3, t1); PMUL(Bp[1][1], 3, Bp[2][0], 3, t2);
    for (int i = 0; i < 7; ++i) c3[i] = t1[i] - t2[i];
    c3[7] = 0.0;
    double u1[11], u2[11], u3[11];
    PMUL(Bp[0][0], 3, c1, 7, u1);
    PMUL(Bp[0][1], 3, c2, 7, u2);
    PMUL(Bp[0][2], 4, c3, 6, u3);
    for (int i = 0; i < 11; ++i) n[i] = u1[i] - u2[i] + u3[i];
#undef PMUL
  }
  double roots[10];
  const int nr = real_roots(n, 10, roots);
  int ns = 0;
  for (int ri = 0; ri < nr; ++ri) {
    const double z = roots[ri];
    double row[3][3];
    for (int q = 0; q < 3; ++q)
      for (int c = 0; c < 3; ++c) row[q][c] = poly_eval(Bp[q][c], c == 2 ? 4 : 3, z);
    double v[3];
    cross3(row[0], row[1], v);
    if (v[2] == 0.0) continue;
    const double x = v[0] / v[2], y = v[1] / v[2];
    double* Eo = Es + 9 * ns;
    double nn = 0.0;
    for (int e = 0; e < 9; ++e) {
      Eo[e] = x * N[0][e] + y * N[1][e] + z * N[2][e] + N[3][e];
      nn += Eo[e] * Eo[e];
    }
    nn = sqrt(nn);
    if (!(nn > 0.0)) continue;
    for (int e = 0; e < 9; ++e) Eo[e] /= nn;
    ++ns;
  }
  return ns;
}

/* ---------------------------------------- 5-point (Stewenius 2006) -- */
/* opengv fivept_stewenius (Stewenius, Engels, Nister, "Recent developments on
 * direct relative orientation", ISPRS J. 2006), the solver the reference
 * config selects (ransac_2d2d_algorithm: 0, LcdParams.yaml:73). Restated
 * procedure:
 *   - the same 10 cubic constraints in the null-space coordinates (x, y, z)
 *     as Nister (fivept_system), with the monomials in graded order: the 10
 *     cubics GORD[0..9] first, then the basis
 *       b = [x^2, xy, xz, y^2, yz, z^2, x, y, z, 1];
 *   - Gauss-Jordan on the cubic columns: cubic_i = -sum_j C[i][j] b_j;
 *   - the action matrix of multiplication by x on b (10x10):
 *       x*b_i for i < 6 is cubic i -> row -C[i]; x*x = b_0, x*y = b_1,
 *       x*z = b_2, x*1 = b_6;
 *   - its eigen-decomposition: each eigenvector is b evaluated at a solution,
 *     (x, y, z) = (v6, v7, v8) / v9; E = x N0 + y N1 + z N2 + N3;
 *   - as opengv's CentralRelativePoseSacProblem does with the complex
 *     essentials of fivept_stewenius, every solution enters RANSAC through the
 *     real part of its E (a complex-conjugate pair gives one real part; it is
 *     taken once, from the member with positive imaginary part).
 * Eigenvalues: Hessenberg reduction by stabilised elimination and the
 * Francis double-shift QR iteration (EISPACK elmhes / hqr, restated from the
 * public-domain EISPACK Fortran below) on the action matrix; eigenvectors: complex
 * LU with partial pivoting of (M - lambda I), v9 = 1, back substitution.
 * Eigen's EigenSolver (opengv) reaches the same eigenpairs by a different QR
 * variant: solution ORDER can differ from opengv [U]; E per solution agrees
 * to rounding. */
static const int GORD[20] = {0, 2, 4, 3, 8, 10, 1, 6, 13, 16, 5, 9, 11, 7, 14, 17, 12, 15, 18, 19};

typedef struct {
  double re, im;
} cplx;
static cplx c_mul(cplx a, cplx b) {
  cplx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
  return r;
}
static cplx c_sub(cplx a, cplx b) {
  cplx r = {a.re - b.re, a.im - b.im};
  return r;
}
static cplx c_div(cplx a, cplx d) { /* Smith's algorithm */
  cplx r;
  if (fabs(d.re) >= fabs(d.im)) {
    const double q = d.im / d.re, den = d.re + d.im * q;
    r.re = (a.re + a.im * q) / den;
    r.im = (a.im - a.re * q) / den;
  } else {
    const double q = d.re / d.im, den = d.re * q + d.im;
    r.re = (a.re * q + a.im) / den;
    r.im = (a.im * q - a.re) / den;
  }
  return r;
}
static double c_abs1(cplx a) { return fabs(a.re) + fabs(a.im); }

/* Reduction to upper Hessenberg form by stabilised elementary similarity
 * transformations: EISPACK ELMHES (B. T. Smith et al., "Matrix Eigensystem
 * Routines - EISPACK Guide", Springer LNCS 6, 1976; public domain, netlib
 * eispack/elmhes.f) with low = 1, igh = n, 0-based. For each column mm1 = m-1
 * the pivot is the first largest |a(j,mm1)|, j >= m; rows and columns m and the
 * pivot are interchanged; the multipliers y = a(i,mm1)/x are applied to row i
 * (columns m..n) and column m (rows 1..igh). The multipliers EISPACK leaves
 * below the subdiagonal are cleared here (hqr never reads them). */
static void hessenberg10(double a[10][10]) {
  const int n = 10, la = n - 2;
  for (int m = 1; m <= la; ++m) {
    const int mm1 = m - 1;
    double x = 0.0;
    int piv = m;
    for (int j = m; j < n; ++j) {
      if (fabs(a[j][mm1]) <= fabs(x)) continue;
      x = a[j][mm1];
      piv = j;
    }
    if (piv != m) {  /* interchange rows and columns piv, m */
      for (int j = mm1; j < n; ++j) { const double y = a[piv][j]; a[piv][j] = a[m][j]; a[m][j] = y; }
      for (int j = 0; j < n; ++j) { const double y = a[j][piv]; a[j][piv] = a[j][m]; a[j][m] = y; }
    }
    if (x == 0.0) continue;
    for (int i = m + 1; i < n; ++i) {
      double y = a[i][mm1];
      if (y == 0.0) continue;
      y = y / x;
      a[i][mm1] = y;
      for (int j = m; j < n; ++j) a[i][j] = a[i][j] - y * a[m][j];
      for (int j = 0; j < n; ++j) a[j][m] = a[j][m] + y * a[j][i];
    }
  }
  for (int i = 2; i < n; ++i)
    for (int j = 0; j < i - 1; ++j) a[i][j] = 0.0;
}

/* Eigenvalues of an upper Hessenberg matrix by the double-shift QR method:
 * EISPACK HQR (same source as elmhes above; netlib eispack/hqr.f) with
 * low = 1, igh = n, 0-based, its GOTO structure as loops: en is the last row
 * of the active block, na = en - 1, enm2 = na - 1; l is found by the backward
 * search for a negligible subdiagonal h(l,l-1) (tst2 == tst1); one root
 * (l = en) or two (l = na) deflate; otherwise a double-shift QR sweep with
 * the ad hoc shifts at its = 10 and 20, starting at the row m found by the
 * two-small-subdiagonals test. A complex pair is stored as EISPACK does,
 * wi(na) = +zz, wi(en) = -zz. At most 30 n sweeps in all (itn); returns 0 when
 * they run out (EISPACK ierr = en). */
static int hqr10(double h[10][10], double wr[10], double wi[10]) {
  const int n = 10;
  double norm = 0.0;
  for (int i = 0, k = 0; i < n; k = i, ++i)  /* the norm of the Hessenberg part, row by row */
    for (int j = k; j < n; ++j) norm += fabs(h[i][j]);
  int en = n - 1, itn = 30 * n;
  double t = 0.0;
  while (en >= 0) {  /* label 60: search for the next eigenvalues */
    int its = 0;
    const int na = en - 1, enm2 = na - 1;
    for (;;) {
      int l;
      for (l = en; l > 0; --l) {  /* label 70: single small subdiagonal element */
        double s = fabs(h[l - 1][l - 1]) + fabs(h[l][l]);
        if (s == 0.0) s = norm;
        const double tst1 = s, tst2 = tst1 + fabs(h[l][l - 1]);
        if (tst2 == tst1) break;
      }
      double x = h[en][en];  /* label 100: form shift */
      if (l == en) {  /* label 270: one root */
        wr[en] = x + t;
        wi[en] = 0.0;
        en = na;
        break;
      }
      double y = h[na][na], w = h[en][na] * h[na][en];
      if (l == na) {  /* label 280: two roots */
        const double p = (y - x) / 2.0, q = p * p + w;
        double zz = sqrt(fabs(q));
        x = x + t;
        if (q >= 0.0) {  /* real pair */
          zz = p + (p >= 0.0 ? fabs(zz) : -fabs(zz));
          wr[na] = x + zz;
          wr[en] = wr[na];
          if (zz != 0.0) wr[en] = x - w / zz;
          wi[na] = 0.0;
          wi[en] = 0.0;
        } else {  /* complex pair */
          wr[na] = x + p;
          wr[en] = x + p;
          wi[na] = zz;
          wi[en] = -zz;
        }
        en = enm2;
        break;
      }
      if (itn == 0) return 0;  /* label 1000 */
      if (its == 10 || its == 20) {  /* form exceptional shift */
        t = t + x;
        for (int i = 0; i <= en; ++i) h[i][i] = h[i][i] - x;
        const double s = fabs(h[en][na]) + fabs(h[na][enm2]);
        x = 0.75 * s;
        y = x;
        w = -0.4375 * s * s;
      }
      ++its;  /* label 130 */
      --itn;
      double p = 0.0, q = 0.0, r = 0.0, zz;
      int m;
      for (m = enm2; m >= l; --m) {  /* label 140: two consecutive small subdiagonal elements */
        zz = h[m][m];
        r = x - zz;
        double s = y - zz;
        p = (r * s - w) / h[m + 1][m] + h[m][m + 1];
        q = h[m + 1][m + 1] - zz - r - s;
        r = h[m + 2][m + 1];
        s = fabs(p) + fabs(q) + fabs(r);
        p = p / s;
        q = q / s;
        r = r / s;
        if (m == l) break;
        const double tst1 = fabs(p) * (fabs(h[m - 1][m - 1]) + fabs(zz) + fabs(h[m + 1][m + 1]));
        const double tst2 = tst1 + fabs(h[m][m - 1]) * (fabs(q) + fabs(r));
        if (tst2 == tst1) break;
      }
      for (int i = m + 2; i <= en; ++i) {  /* label 150 */
        h[i][i - 2] = 0.0;
        if (i != m + 2) h[i][i - 3] = 0.0;
      }
      for (int k = m; k <= na; ++k) {  /* double QR step on rows l..en, columns m..en */
        const int notlas = k != na;
        if (k != m) {
          p = h[k][k - 1];
          q = h[k + 1][k - 1];
          r = 0.0;
          if (notlas) r = h[k + 2][k - 1];
          x = fabs(p) + fabs(q) + fabs(r);
          if (x == 0.0) continue;
          p = p / x;
          q = q / x;
          r = r / x;
        }
        const double sq = sqrt(p * p + q * q + r * r), s = p >= 0.0 ? sq : -sq;  /* label 170: dsign */
        if (k == m) {
          if (l != m) h[k][k - 1] = -h[k][k - 1];  /* label 180 */
        } else {
          h[k][k - 1] = -s * x;
        }
        p = p + s;  /* label 190 */
        x = p / s;
        y = q / s;
        zz = r / s;
        q = q / p;
        r = r / p;
        if (notlas) {  /* label 225 */
          for (int j = k; j <= en; ++j) {  /* row modification */
            p = h[k][j] + q * h[k + 1][j] + r * h[k + 2][j];
            h[k][j] = h[k][j] - p * x;
            h[k + 1][j] = h[k + 1][j] - p * y;
            h[k + 2][j] = h[k + 2][j] - p * zz;
          }
          const int jmax = en < k + 3 ? en : k + 3;
          for (int i = l; i <= jmax; ++i) {  /* column modification */
            p = x * h[i][k] + y * h[i][k + 1] + zz * h[i][k + 2];
            h[i][k] = h[i][k] - p;
            h[i][k + 1] = h[i][k + 1] - p * q;
            h[i][k + 2] = h[i][k + 2] - p * r;
          }
        } else {
          for (int j = k; j <= en; ++j) {
            p = h[k][j] + q * h[k + 1][j];
            h[k][j] = h[k][j] - p * x;
            h[k + 1][j] = h[k + 1][j] - p * y;
          }
          const int jmax = en < k + 3 ? en : k + 3;
          for (int i = l; i <= jmax; ++i) {
            p = x * h[i][k] + y * h[i][k + 1];
            h[i][k] = h[i][k] - p;
            h[i][k + 1] = h[i][k + 1] - p * q;
          }
        }
      }
    }
  }
  return 1;
}

/* Eigenvector of M for the eigenvalue lam normalised to v9 = 1: LU with
 * partial pivoting (|re| + |im|) of M - lam I over columns 0..8, then back
 * substitution. Returns 0 on a zero pivot. */
static int eigvec10(const double M[10][10], cplx lam, cplx v[10]) {
  cplx B[10][10];
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 10; ++j) {
      B[i][j].re = M[i][j];
      B[i][j].im = 0.0;
    }
  for (int i = 0; i < 10; ++i) B[i][i] = c_sub(B[i][i], lam);
  for (int k = 0; k < 9; ++k) {
    int p = k;
    for (int i = k + 1; i < 10; ++i)
      if (c_abs1(B[i][k]) > c_abs1(B[p][k])) p = i;
    if (c_abs1(B[p][k]) == 0.0) return 0;
    if (p != k)
      for (int j = 0; j < 10; ++j) { const cplx t = B[k][j]; B[k][j] = B[p][j]; B[p][j] = t; }
    for (int i = k + 1; i < 10; ++i) {
      const cplx f = c_div(B[i][k], B[k][k]);
      for (int j = k + 1; j < 10; ++j) B[i][j] = c_sub(B[i][j], c_mul(f, B[k][j]));
    }
  }
  v[9].re = 1.0;
  v[9].im = 0.0;
  for (int i = 8; i >= 0; --i) {
    cplx s = {0.0, 0.0};
    for (int j = i + 1; j < 10; ++j) s = c_sub(s, c_mul(B[i][j], v[j]));
    v[i] = c_div(s, B[i][i]);
  }
  return 1;
}

int orc_fivept_stewenius(const double* f1 /*5x3*/, const double* f2 /*5x3*/, double* Es /*10x9*/) {
  double N[4][9], A0[10][20], A[10][20];
  fivept_system(f1, f2, N, A0);
  for (int i = 0; i < 10; ++i)
    for (int c = 0; c < 20; ++c) A[i][c] = A0[i][GORD[c]];
  if (!gj_10x20(A)) return 0;
  double M[10][10];
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 10; ++j) M[i][j] = (i < 6) ? -A[i][10 + j] : 0.0;
  M[6][0] = 1.0;
  M[7][1] = 1.0;
  M[8][2] = 1.0;
  M[9][6] = 1.0;
  double H[10][10], wr[10], wi[10];
  memcpy(H, M, sizeof(H));
  hessenberg10(H);
  if (!hqr10(H, wr, wi)) return 0;
  int ns = 0;
  for (int s = 0; s < 10; ++s) {
    if (wi[s] < 0.0) continue; /* the conjugate of s + 1 */
    cplx lam = {wr[s], wi[s]}, v[10];
    if (!eigvec10(M, lam, v)) continue;
    const double x = v[6].re, y = v[7].re, z = v[8].re;
    double* Eo = Es + 9 * ns;
    double nn = 0.0;
    for (int e = 0; e < 9; ++e) {
      Eo[e] = x * N[0][e] + y * N[1][e] + z * N[2][e] + N[3][e];
      nn += Eo[e] * Eo[e];
    }
    nn = sqrt(nn);
    if (!(nn > 0.0) || !isfinite(nn)) continue;
    for (int e = 0; e < 9; ++e) Eo[e] /= nn;
    ++ns;
  }
  return ns;
}

/* ----------------------------------------------- opengv-style scoring -- */
/* error of correspondence (f1, f2) under model (R = R12, t = t12):
 * mid-point triangulation (opengv triangulate2) + bearing errors 1 - cos. */
static double model_error(const double R[9], const double t[3], const double f1[3], const double f2[3]) {
  double f2u[3];
  for (int i = 0; i < 3; ++i) f2u[i] = R[i * 3 + 0] * f2[0] + R[i * 3 + 1] * f2[1] + R[i * 3 + 2] * f2[2];
  const double b0 = dot3(t, f1), b1 = dot3(t, f2u);
  const double a00 = dot3(f1, f1), a10 = dot3(f1, f2u), a01 = -a10, a11 = -dot3(f2u, f2u);
  const double det = a00 * a11 - a01 * a10;
  const double l0 = (a11 * b0 - a01 * b1) / det;
  const double l1 = (-a10 * b0 + a00 * b1) / det;
  double p[3];
  for (int i = 0; i < 3; ++i) p[i] = 0.5 * (l0 * f1[i] + (t[i] + l1 * f2u[i]));
  double q[3], d[3];
  for (int i = 0; i < 3; ++i) d[i] = p[i] - t[i];
  for (int i = 0; i < 3; ++i) q[i] = R[0 * 3 + i] * d[0] + R[1 * 3 + i] * d[1] + R[2 * 3 + i] * d[2];
  const double np = sqrt(dot3(p, p)), nq = sqrt(dot3(q, q));
  const double e1 = 1.0 - (f1[0] * p[0] + f1[1] * p[1] + f1[2] * p[2]) / np;
  const double e2 = 1.0 - (f2[0] * q[0] + f2[1] * q[1] + f2[2] * q[2]) / nq;
  return e1 + e2;
}

/* computeModelCoefficients: 5-point essentials, 4 decompositions each, keep
 * the (R, t) with the smallest summed error over the sample. */
static int model_from_sample(int algo, const double* F1, const double* F2, const int32_t* smp, double R[9],
                             double t[3]) {
  double f1[15], f2[15];
  for (int i = 0; i < 5; ++i)
    for (int c = 0; c < 3; ++c) {
      f1[3 * i + c] = F1[3 * smp[i] + c];
      f2[3 * i + c] = F2[3 * smp[i] + c];
    }
  double Es[90];
  const int ne = (algo == KMX_ALGO_NISTER) ? orc_fivept_nister(f1, f2, Es) : orc_fivept_stewenius(f1, f2, Es);
  if (ne == 0) return 0;
  double best = DBL_MAX;
  int found = 0;
  for (int e = 0; e < ne; ++e) {
    double U[9], s[3], V[9];
    svd3(Es + 9 * e, U, s, V);
    /* R = U W V^T, U W^T V^T with W = [0 -1 0; 1 0 0; 0 0 1] */
    double Ra[9], Rb[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        /* (U W)_ik: col0 = u1*0 + u2*1 -> u2 ; col1 = -u1 ; col2 = u3 */
        const double uw0 = U[i * 3 + 1], uw1 = -U[i * 3 + 0], uw2 = U[i * 3 + 2];
        Ra[i * 3 + j] = uw0 * V[j * 3 + 0] + uw1 * V[j * 3 + 1] + uw2 * V[j * 3 + 2];
        const double uv0 = -U[i * 3 + 1], uv1 = U[i * 3 + 0], uv2 = U[i * 3 + 2];
        Rb[i * 3 + j] = uv0 * V[j * 3 + 0] + uv1 * V[j * 3 + 1] + uv2 * V[j * 3 + 2];
      }
    if (det3(Ra) < 0.0)
      for (int i = 0; i < 9; ++i) Ra[i] = -Ra[i];
    if (det3(Rb) < 0.0)
      for (int i = 0; i < 9; ++i) Rb[i] = -Rb[i];
    const double tu[3] = {U[0 * 3 + 2], U[1 * 3 + 2], U[2 * 3 + 2]};
    for (int cand = 0; cand < 4; ++cand) {
      const double* Rc = (cand < 2) ? Ra : Rb;
      const double sg = (cand & 1) ? -1.0 : 1.0;
      const double tc[3] = {sg * tu[0], sg * tu[1], sg * tu[2]};
      double err = 0.0;
      for (int i = 0; i < 5; ++i) err += model_error(Rc, tc, f1 + 3 * i, f2 + 3 * i);
      if (err < best) {
        best = err;
        memcpy(R, Rc, sizeof(double) * 9);
        memcpy(t, tc, sizeof(double) * 3);
        found = 1;
      }
    }
  }
  return found;
}

/* opengv sac::Ransac::computeModel over the pair list; returns 1 on success. */
static int ransac_2d2d(const kmx_lcd_params* P, const double* F1, const double* F2, int K, double R[9], double t[3],
                       uint8_t* inl, int* n_inl, int* iters_out, orc_mt19937* stream) {
  *n_inl = 0;
  *iters_out = 0;
  if (K < 5) return 0;
  orc_mt19937 m0;
  orc_mt19937* m = problem_rng(P, &m0, stream);
  int32_t* sh = (int32_t*)malloc(sizeof(int32_t) * K);
  for (int i = 0; i < K; ++i) sh[i] = i;
  int iterations = 0, skipped = 0, best_cnt = -INT_MAX, have = 0;
  const int max_skip = P->ransac_max_iterations * 10;
  double k = 1.0;
  double bR[9], bt[3];
  while (iterations < k && skipped < max_skip) {
    int32_t smp[5];
    for (int i = 0; i < 5; ++i) {
      const int r = uid_draw(m, P->rng_variant);
      const int j = i + (int)((size_t)r % (size_t)(K - i));
      const int32_t tt = sh[i];
      sh[i] = sh[j];
      sh[j] = tt;
    }
    for (int i = 0; i < 5; ++i) smp[i] = sh[i];
    double Rm[9], tm[3];
    if (!model_from_sample(P->algorithm_2d2d, F1, F2, smp, Rm, tm)) {
      ++skipped;
      continue;
    }
    int cnt = 0;
    for (int j = 0; j < K; ++j)
      if (model_error(Rm, tm, F1 + 3 * j, F2 + 3 * j) < P->ransac_threshold_2d2d) ++cnt;
    if (cnt > best_cnt) {
      best_cnt = cnt;
      memcpy(bR, Rm, sizeof(bR));
      memcpy(bt, tm, sizeof(bt));
      have = 1;
      const double w = (double)cnt / (double)K;
      double p_no = 1.0 - pow(w, 5.0);
      p_no = fmax(DBL_EPSILON, p_no);
      p_no = fmin(1.0 - DBL_EPSILON, p_no);
      k = log(1.0 - P->ransac_probability) / log(p_no);
    }
    ++iterations;
    if (iterations > P->ransac_max_iterations) break;
  }
  free(sh);
  *iters_out = iterations;
  if (!have) return 0;
  int c = 0;
  for (int j = 0; j < K; ++j) {
    const int in = model_error(bR, bt, F1 + 3 * j, F2 + 3 * j) < P->ransac_threshold_2d2d;
    inl[j] = (uint8_t)in;
    c += in;
  }
  *n_inl = c;
  memcpy(R, bR, sizeof(bR));
  memcpy(t, bt, sizeof(bt));
  return 1;
}

/* ------------------------------------------- EPnP (Lepetit et al. 2009) -- */
/* opengv absolute_pose::epnp as used by AbsolutePoseSacProblem(EPNP) for the
 * PnP pose recovery (LcdParams.yaml:53,57,63,74). Bearings f (camera) and
 * points p (world = match frame); image coordinates u = f0/f2, v = f1/f2
 * (unit focal, zero principal point). Restated algorithm:
 *   control points: centroid + principal axes scaled by sqrt(eig / n);
 *   barycentric alphas; M (2n x 12); MtM eigen (cyclic Jacobi) -> the 4
 *   eigenvectors of the smallest eigenvalues; L_6x10 and rho; betas from the
 *   three linearisations (L_6x4, L_6x3, L_6x5 least squares by Householder
 *   QR) each refined by 5 Gauss-Newton steps; R, t by Horn/Umeyama (SVD of
 *   the 3x3 cross-covariance); the solution with the smallest mean
 *   reprojection error wins. Returns (R_wc, t_wc) = camera orientation and
 *   position in the world frame (opengv convention). [U: opengv solves the
 *   linear systems with SVD; parity unpinned.] */
static void jacobi_sym(int n, double* A, double* V) {
  for (int i = 0; i < n * n; ++i) V[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) off += A[p * n + q] * A[p * n + q];
    if (off == 0.0) break;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (apq == 0.0) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cs = 1.0 / sqrt(t * t + 1.0), sn = t * cs;
        for (int k = 0; k < n; ++k) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = cs * akp - sn * akq;
          A[k * n + q] = sn * akp + cs * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = cs * apk - sn * aqk;
          A[q * n + k] = sn * apk + cs * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = cs * vkp - sn * vkq;
          V[k * n + q] = sn * vkp + cs * vkq;
        }
      }
  }
}

/* least squares min |A x - b| for A (m x n, row-major, m >= n) by Householder
 * QR; A and b are overwritten. Returns 0 when rank deficient. */
static int qr_lsq(int m, int n, double* A, double* b, double* x) {
  for (int k = 0; k < n; ++k) {
    double nrm = 0.0;
    for (int i = k; i < m; ++i) nrm += A[i * n + k] * A[i * n + k];
    nrm = sqrt(nrm);
    if (nrm == 0.0) return 0;
    const double alpha = (A[k * n + k] > 0.0) ? -nrm : nrm;
    double vk = A[k * n + k] - alpha;
    double vnorm2 = vk * vk;
    for (int i = k + 1; i < m; ++i) vnorm2 += A[i * n + k] * A[i * n + k];
    if (vnorm2 == 0.0) return 0;
    /* v = (vk, A[k+1..m-1][k]); H = I - 2 v v^T / (v^T v) */
    for (int j = k + 1; j < n; ++j) {
      double sdot = vk * A[k * n + j];
      for (int i = k + 1; i < m; ++i) sdot += A[i * n + k] * A[i * n + j];
      const double f = 2.0 * sdot / vnorm2;
      A[k * n + j] -= f * vk;
      for (int i = k + 1; i < m; ++i) A[i * n + j] -= f * A[i * n + k];
    }
    {
      double sdot = vk * b[k];
      for (int i = k + 1; i < m; ++i) sdot += A[i * n + k] * b[i];
      const double f = 2.0 * sdot / vnorm2;
      b[k] -= f * vk;
      for (int i = k + 1; i < m; ++i) b[i] -= f * A[i * n + k];
    }
    A[k * n + k] = alpha;
  }
  for (int k = n - 1; k >= 0; --k) {
    double sacc = b[k];
    for (int j = k + 1; j < n; ++j) sacc -= A[k * n + j] * x[j];
    x[k] = sacc / A[k * n + k];
  }
  return 1;
}

static const int PAIR_A[6] = {0, 0, 0, 1, 1, 2}, PAIR_B[6] = {1, 2, 3, 2, 3, 3};

static void epnp_gauss_newton(const double L[60], const double rho[6], double bt[4]) {
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6], x[4];
    for (int i = 0; i < 6; ++i) {
      const double* l = L + 10 * i;
      A[4 * i + 0] = 2 * l[0] * bt[0] + l[1] * bt[1] + l[3] * bt[2] + l[6] * bt[3];
      A[4 * i + 1] = l[1] * bt[0] + 2 * l[2] * bt[1] + l[4] * bt[2] + l[7] * bt[3];
      A[4 * i + 2] = l[3] * bt[0] + l[4] * bt[1] + 2 * l[5] * bt[2] + l[8] * bt[3];
      A[4 * i + 3] = l[6] * bt[0] + l[7] * bt[1] + l[8] * bt[2] + 2 * l[9] * bt[3];
      b[i] = rho[i] - (l[0] * bt[0] * bt[0] + l[1] * bt[0] * bt[1] + l[2] * bt[1] * bt[1] + l[3] * bt[0] * bt[2] +
                       l[4] * bt[1] * bt[2] + l[5] * bt[2] * bt[2] + l[6] * bt[0] * bt[3] + l[7] * bt[1] * bt[3] +
                       l[8] * bt[2] * bt[3] + l[9] * bt[3] * bt[3]);
    }
    if (!qr_lsq(6, 4, A, b, x)) return;
    for (int k = 0; k < 4; ++k) bt[k] += x[k];
  }
}

/* camera-frame control points from betas, then R, t (world -> camera) by
 * Horn; returns the mean reprojection error. */
static double epnp_R_t(int n, const double* pw, const double* uv, const double* alphas, const double V4[4][12],
                       const double bt[4], double R[9], double t[3]) {
  double ccs[12];
  for (int j = 0; j < 12; ++j) ccs[j] = bt[0] * V4[0][j] + bt[1] * V4[1][j] + bt[2] * V4[2][j] + bt[3] * V4[3][j];
  double* pc = (double*)malloc(sizeof(double) * 3 * (size_t)n);
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c)
      pc[3 * i + c] = alphas[4 * i + 0] * ccs[c] + alphas[4 * i + 1] * ccs[3 + c] + alphas[4 * i + 2] * ccs[6 + c] +
                      alphas[4 * i + 3] * ccs[9 + c];
  if (pc[2] < 0.0) /* solve_for_sign: the first point in front of the camera */
    for (int i = 0; i < 3 * n; ++i) pc[i] = -pc[i];
  double c0[3] = {0, 0, 0}, w0[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      c0[c] += pc[3 * i + c];
      w0[c] += pw[3 * i + c];
    }
  for (int c = 0; c < 3; ++c) {
    c0[c] /= n;
    w0[c] /= n;
  }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) H[a * 3 + b] += (pc[3 * i + a] - c0[a]) * (pw[3 * i + b] - w0[b]);
  double U[9], sv[3], Vm[9];
  svd3(H, U, sv, Vm);
  /* svd3's U is right-handed (u3 = u1 x u2): for a proper rotation the third
   * left vector carries det(V) (Umeyama: R = U diag(1, 1, det U det V) V^T) */
  if (det3(Vm) < 0.0)
    for (int a = 0; a < 3; ++a) U[a * 3 + 2] = -U[a * 3 + 2];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R[a * 3 + b] = U[a * 3 + 0] * Vm[b * 3 + 0] + U[a * 3 + 1] * Vm[b * 3 + 1] + U[a * 3 + 2] * Vm[b * 3 + 2];
  if (det3(R) < 0.0)
    for (int b = 0; b < 3; ++b) R[2 * 3 + b] = -R[2 * 3 + b];
  for (int a = 0; a < 3; ++a) t[a] = c0[a] - (R[a * 3 + 0] * w0[0] + R[a * 3 + 1] * w0[1] + R[a * 3 + 2] * w0[2]);
  double err = 0.0;
  for (int i = 0; i < n; ++i) {
    double x[3];
    for (int a = 0; a < 3; ++a)
      x[a] = R[a * 3 + 0] * pw[3 * i + 0] + R[a * 3 + 1] * pw[3 * i + 1] + R[a * 3 + 2] * pw[3 * i + 2] + t[a];
    const double du = uv[2 * i] - x[0] / x[2], dv = uv[2 * i + 1] - x[1] / x[2];
    err += sqrt(du * du + dv * dv);
  }
  free(pc);
  return err / n;
}

int orc_epnp(int n, const double* pw, const double* f, double R_out[9], double t_out[3]) {
  if (n < 4) return 0;
  double* uv = (double*)malloc(sizeof(double) * 2 * (size_t)n);
  double* alphas = (double*)malloc(sizeof(double) * 4 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    uv[2 * i] = f[3 * i] / f[3 * i + 2];
    uv[2 * i + 1] = f[3 * i + 1] / f[3 * i + 2];
  }
  /* control points */
  double cw[12];
  for (int c = 0; c < 3; ++c) cw[c] = 0.0;
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) cw[c] += pw[3 * i + c];
  for (int c = 0; c < 3; ++c) cw[c] /= n;
  double C3[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, E3[9];
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) C3[a * 3 + b] += (pw[3 * i + a] - cw[a]) * (pw[3 * i + b] - cw[b]);
  sym_eig3(C3, E3);
  for (int k = 0; k < 3; ++k) {
    const double sc = sqrt(fmax(C3[k * 4], 0.0) / n);
    for (int c = 0; c < 3; ++c) cw[3 * (k + 1) + c] = cw[c] + sc * E3[c * 3 + k];
  }
  /* barycentric coordinates */
  double CC[9], CI[9];
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) CC[r * 3 + k] = cw[3 * (k + 1) + r] - cw[r];
  const double dC = det3(CC);
  int ok = (dC != 0.0);
  if (ok) {
    CI[0] = (CC[4] * CC[8] - CC[5] * CC[7]) / dC;
    CI[1] = (CC[2] * CC[7] - CC[1] * CC[8]) / dC;
    CI[2] = (CC[1] * CC[5] - CC[2] * CC[4]) / dC;
    CI[3] = (CC[5] * CC[6] - CC[3] * CC[8]) / dC;
    CI[4] = (CC[0] * CC[8] - CC[2] * CC[6]) / dC;
    CI[5] = (CC[2] * CC[3] - CC[0] * CC[5]) / dC;
    CI[6] = (CC[3] * CC[7] - CC[4] * CC[6]) / dC;
    CI[7] = (CC[1] * CC[6] - CC[0] * CC[7]) / dC;
    CI[8] = (CC[0] * CC[4] - CC[1] * CC[3]) / dC;
    for (int i = 0; i < n; ++i) {
      const double d[3] = {pw[3 * i] - cw[0], pw[3 * i + 1] - cw[1], pw[3 * i + 2] - cw[2]};
      double s1 = 0.0;
      for (int k = 0; k < 3; ++k) {
        const double a = CI[k * 3 + 0] * d[0] + CI[k * 3 + 1] * d[1] + CI[k * 3 + 2] * d[2];
        alphas[4 * i + 1 + k] = a;
        s1 += a;
      }
      alphas[4 * i] = 1.0 - s1;
    }
  }
  double V4[4][12];
  double L[60], rho[6];
  if (ok) {
    /* MtM accumulated row pair by row pair */
    double MtM[144], W[144];
    for (int i = 0; i < 144; ++i) MtM[i] = 0.0;
    for (int i = 0; i < n; ++i) {
      double m1[12], m2[12];
      for (int j = 0; j < 4; ++j) {
        const double a = alphas[4 * i + j];
        m1[3 * j] = a; m1[3 * j + 1] = 0.0; m1[3 * j + 2] = -a * uv[2 * i];
        m2[3 * j] = 0.0; m2[3 * j + 1] = a; m2[3 * j + 2] = -a * uv[2 * i + 1];
      }
      for (int r = 0; r < 12; ++r)
        for (int c = 0; c < 12; ++c) MtM[r * 12 + c] += m1[r] * m1[c] + m2[r] * m2[c];
    }
    jacobi_sym(12, MtM, W);
    /* the 4 smallest eigenvalues, ascending (stable on ties) */
    int ord[12];
    for (int i = 0; i < 12; ++i) ord[i] = i;
    for (int a = 0; a < 12; ++a)
      for (int b = 0; b < 11 - a; ++b)
        if (MtM[ord[b + 1] * 13] < MtM[ord[b] * 13]) { const int tt = ord[b]; ord[b] = ord[b + 1]; ord[b + 1] = tt; }
    for (int k = 0; k < 4; ++k)
      for (int j = 0; j < 12; ++j) V4[k][j] = W[j * 12 + ord[k]];
    for (int pi = 0; pi < 6; ++pi) {
      const int a = PAIR_A[pi], b = PAIR_B[pi];
      double dv[4][3];
      for (int k = 0; k < 4; ++k)
        for (int c = 0; c < 3; ++c) dv[k][c] = V4[k][3 * a + c] - V4[k][3 * b + c];
      double* l = L + 10 * pi;
      l[0] = dot3(dv[0], dv[0]);
      l[1] = 2.0 * dot3(dv[0], dv[1]);
      l[2] = dot3(dv[1], dv[1]);
      l[3] = 2.0 * dot3(dv[0], dv[2]);
      l[4] = 2.0 * dot3(dv[1], dv[2]);
      l[5] = dot3(dv[2], dv[2]);
      l[6] = 2.0 * dot3(dv[0], dv[3]);
      l[7] = 2.0 * dot3(dv[1], dv[3]);
      l[8] = 2.0 * dot3(dv[2], dv[3]);
      l[9] = dot3(dv[3], dv[3]);
      double d[3];
      for (int c = 0; c < 3; ++c) d[c] = cw[3 * a + c] - cw[3 * b + c];
      rho[pi] = dot3(d, d);
    }
  }
  double best_err = DBL_MAX, Rb[9], tb[3];
  int found = 0;
  for (int approx = 1; ok && approx <= 3; ++approx) {
    static const int COLS1[4] = {0, 1, 3, 6}, COLS2[3] = {0, 1, 2}, COLS3[5] = {0, 1, 2, 3, 4};
    const int nc = approx == 1 ? 4 : approx == 2 ? 3 : 5;
    const int* cols = approx == 1 ? COLS1 : approx == 2 ? COLS2 : COLS3;
    double A[30], b[6], x[5], bt[4] = {0, 0, 0, 0};
    for (int i = 0; i < 6; ++i) {
      for (int k = 0; k < nc; ++k) A[i * nc + k] = L[10 * i + cols[k]];
      b[i] = rho[i];
    }
    if (!qr_lsq(6, nc, A, b, x)) continue;
    if (approx == 1) {
      if (x[0] < 0.0) {
        bt[0] = sqrt(-x[0]);
        bt[1] = -x[1] / bt[0]; bt[2] = -x[2] / bt[0]; bt[3] = -x[3] / bt[0];
      } else {
        bt[0] = sqrt(x[0]);
        bt[1] = x[1] / bt[0]; bt[2] = x[2] / bt[0]; bt[3] = x[3] / bt[0];
      }
    } else {
      if (x[0] < 0.0) {
        bt[0] = sqrt(-x[0]);
        bt[1] = (x[2] < 0.0) ? sqrt(-x[2]) : 0.0;
      } else {
        bt[0] = sqrt(x[0]);
        bt[1] = (x[2] > 0.0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0.0) bt[0] = -bt[0];
      if (approx == 3) bt[2] = x[3] / bt[0];
    }
    epnp_gauss_newton(L, rho, bt);
    double R[9], t[3];
    const double err = epnp_R_t(n, pw, uv, alphas, V4, bt, R, t);
    if (err < best_err) {
      best_err = err;
      memcpy(Rb, R, sizeof(Rb));
      memcpy(tb, t, sizeof(tb));
      found = 1;
    }
  }
  free(uv);
  free(alphas);
  if (!found) return 0;
  /* opengv returns the camera pose in the world: R_wc = R^T, t_wc = -R^T t */
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R_out[a * 3 + b] = Rb[b * 3 + a];
  for (int a = 0; a < 3; ++a) t_out[a] = -(Rb[0 * 3 + a] * tb[0] + Rb[1 * 3 + a] * tb[1] + Rb[2 * 3 + a] * tb[2]);
  return 1;
}

/* AbsolutePoseSacProblem error: 1 - f . normalize(R^T (p - t)) */
static double pnp_error(const double R[9], const double t[3], const double p[3], const double f[3]) {
  const double d[3] = {p[0] - t[0], p[1] - t[1], p[2] - t[2]};
  double q[3];
  for (int i = 0; i < 3; ++i) q[i] = R[0 * 3 + i] * d[0] + R[1 * 3 + i] * d[1] + R[2 * 3 + i] * d[2];
  const double nq = sqrt(dot3(q, q));
  return 1.0 - (q[0] * f[0] + q[1] * f[1] + q[2] * f[2]) / nq;
}

/* opengv sac::Ransac over the AbsolutePoseSacProblem (sample size 6, EPnP). */
static int ransac_pnp(const kmx_lcd_params* P, const double* Fq, const double* Pm, int K, double R[9], double t[3],
                      uint8_t* inl, int* n_inl, orc_mt19937* stream) {
  *n_inl = 0;
  const int S = 6;
  if (K < S) return 0;
  orc_mt19937 m0;
  orc_mt19937* m = problem_rng(P, &m0, stream);
  int32_t* sh = (int32_t*)malloc(sizeof(int32_t) * K);
  for (int i = 0; i < K; ++i) sh[i] = i;
  int iterations = 0, skipped = 0, best_cnt = -INT_MAX, have = 0;
  const int max_skip = P->ransac_max_iterations * 10;
  double k = 1.0;
  double bR[9], bt[3];
  while (iterations < k && skipped < max_skip) {
    double sp[18], sf[18];
    for (int i = 0; i < S; ++i) {
      const int r = uid_draw(m, P->rng_variant);
      const int j = i + (int)((size_t)r % (size_t)(K - i));
      const int32_t tt = sh[i];
      sh[i] = sh[j];
      sh[j] = tt;
    }
    for (int i = 0; i < S; ++i)
      for (int c = 0; c < 3; ++c) {
        sp[3 * i + c] = Pm[3 * sh[i] + c];
        sf[3 * i + c] = Fq[3 * sh[i] + c];
      }
    double Rm[9], tm[3];
    if (!orc_epnp(S, sp, sf, Rm, tm)) {
      ++skipped;
      continue;
    }
    int cnt = 0;
    for (int j = 0; j < K; ++j)
      if (pnp_error(Rm, tm, Pm + 3 * j, Fq + 3 * j) < P->ransac_threshold_2d3d) ++cnt;
    if (cnt > best_cnt) {
      best_cnt = cnt;
      memcpy(bR, Rm, sizeof(bR));
      memcpy(bt, tm, sizeof(bt));
      have = 1;
      const double w = (double)cnt / (double)K;
      double p_no = 1.0 - pow(w, (double)S);
      p_no = fmax(DBL_EPSILON, p_no);
      p_no = fmin(1.0 - DBL_EPSILON, p_no);
      k = log(1.0 - P->ransac_probability) / log(p_no);
    }
    ++iterations;
    if (iterations > P->ransac_max_iterations) break;
  }
  free(sh);
  if (!have) return 0;
  int c = 0;
  for (int j = 0; j < K; ++j) {
    const int in = pnp_error(bR, bt, Pm + 3 * j, Fq + 3 * j) < P->ransac_threshold_2d3d;
    inl[j] = (uint8_t)in;
    c += in;
  }
  *n_inl = c;
  memcpy(R, bR, sizeof(bR));
  memcpy(t, bt, sizeof(bt));
  return 1;
}

/* 1-point 3D-3D given the 2D-2D rotation (ransac_use_1point_3d3d = 1). */
static int given_rotation_3d3d(const kmx_lcd_params* P, const double R[9], const double* Pq, const double* Pm,
                               const uint8_t* valid, int K, double t_out[3], uint8_t* inl) {
  double* T = (double*)malloc(sizeof(double) * 3 * (K + 1));
  for (int j = 0; j < K; ++j)
    for (int i = 0; i < 3; ++i)
      T[3 * j + i] = Pq[3 * j + i] - (R[i * 3 + 0] * Pm[3 * j + 0] + R[i * 3 + 1] * Pm[3 * j + 1] + R[i * 3 + 2] * Pm[3 * j + 2]);
  const double thr2 = P->ransac_threshold_3d3d * P->ransac_threshold_3d3d;
  int best = -1, best_cnt = 0;
  for (int i = 0; i < K; ++i) {
    if (!valid[i]) continue;
    int c = 0;
    for (int j = 0; j < K; ++j) {
      if (!valid[j]) continue;
      const double dx = T[3 * j] - T[3 * i], dy = T[3 * j + 1] - T[3 * i + 1], dz = T[3 * j + 2] - T[3 * i + 2];
      if (dx * dx + dy * dy + dz * dz < thr2) ++c;
    }
    if (c > best_cnt) { best_cnt = c; best = i; }
  }
  t_out[0] = t_out[1] = t_out[2] = 0.0;
  if (best < 0) { free(T); return 0; }
  int c = 0;
  double s[3] = {0, 0, 0};
  for (int j = 0; j < K; ++j) {
    int in = 0;
    if (valid[j]) {
      const double dx = T[3 * j] - T[3 * best], dy = T[3 * j + 1] - T[3 * best + 1], dz = T[3 * j + 2] - T[3 * best + 2];
      in = dx * dx + dy * dy + dz * dz < thr2;
    }
    inl[j] = (uint8_t)in;
    if (in) {
      for (int i = 0; i < 3; ++i) s[i] += T[3 * j + i];
      ++c;
    }
  }
  for (int i = 0; i < 3; ++i) t_out[i] = s[i] / (double)c;
  free(T);
  return c;
}

/* Arun 3-point 3D-3D (ransac_use_1point_3d3d = 0, LcdParams.yaml:58): opengv
 * sac::Ransac over the PointCloudSacProblem with point_cloud::threept_arun
 * (Arun, Huang, Blostein 1987), restated: centroids of the 3 sampled pairs,
 * H = sum (p_m - c_m)(p_q - c_q)^T, H = U S V^T, R = V U^T with V's third
 * column negated when det R < 0 (Kabsch), t = c_q - R c_m; the model maps
 * match-frame points to the query frame (p_q = R p_m + t). Error of a pair:
 * |p_q - (R p_m + t)| (Euclidean, metres) against ransac_threshold_3d3d.
 * Sampler and stopping rule as the 2D-2D RANSAC with sample size 3, on the
 * stereo-valid 2D-2D inliers in pair-list order [U: opengv's exact point
 * cloud error definition; optimize_3d3d_pose_from_inliers = 0, no refit]. */
static void arun_model(const double* Pq, const double* Pm, const int32_t* smp, double R[9], double t[3]) {
  double cq[3] = {0.0, 0.0, 0.0}, cm[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < 3; ++i)
    for (int c = 0; c < 3; ++c) {
      cq[c] += Pq[3 * smp[i] + c];
      cm[c] += Pm[3 * smp[i] + c];
    }
  for (int c = 0; c < 3; ++c) {
    cq[c] /= 3.0;
    cm[c] /= 3.0;
  }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    double dq[3], dm[3];
    for (int c = 0; c < 3; ++c) {
      dq[c] = Pq[3 * smp[i] + c] - cq[c];
      dm[c] = Pm[3 * smp[i] + c] - cm[c];
    }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) H[a * 3 + b] += dm[a] * dq[b];
  }
  double U[9], sv[3], V[9];
  svd3(H, U, sv, V);
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
  if (det3(R) < 0.0) {
    for (int a = 0; a < 3; ++a) V[a * 3 + 2] = -V[a * 3 + 2];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        R[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
  }
  for (int a = 0; a < 3; ++a) t[a] = cq[a] - (R[a * 3 + 0] * cm[0] + R[a * 3 + 1] * cm[1] + R[a * 3 + 2] * cm[2]);
}

/* refine_pose: 1 (LcdParams.yaml:14). Kimera-VIO's LoopClosureDetector
 * refinePoses re-estimates T_query_match after an accepted recovery by a small
 * GTSAM optimisation over the stereo landmarks of the inlier matches, with the
 * match pose fixed by a prior [U: Kimera-VIO is not vendored; restated from
 * its published description]. In this pool's data model a stereo observation
 * is the 3D point itself; with isotropic unit noise on both frames'
 * observations the optimal landmark is the midpoint, and the problem reduces
 * to least squares over the inlier pairs, min_{R,t} sum |p_q - (R p_m + t)|^2:
 * closed form (centroids over ALL inliers, H = sum (p_m - c_m)(p_q - c_q)^T,
 * Kabsch R with the reflection fix, t = c_q - R c_m), i.e. arun_model over
 * the whole inlier set. in[j] selects the inlier pairs of Pq / Pm (j < n). */
static void refit_3d3d(int n, const double* Pq, const double* Pm, const uint8_t* in, double R[9], double t[3]) {
  double cq[3] = {0.0, 0.0, 0.0}, cm[3] = {0.0, 0.0, 0.0};
  int c = 0;
  for (int j = 0; j < n; ++j) {
    if (!in[j]) continue;
    for (int k = 0; k < 3; ++k) {
      cq[k] += Pq[3 * j + k];
      cm[k] += Pm[3 * j + k];
    }
    ++c;
  }
  for (int k = 0; k < 3; ++k) {
    cq[k] /= (double)c;
    cm[k] /= (double)c;
  }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < n; ++j) {
    if (!in[j]) continue;
    double dq[3], dm[3];
    for (int k = 0; k < 3; ++k) {
      dq[k] = Pq[3 * j + k] - cq[k];
      dm[k] = Pm[3 * j + k] - cm[k];
    }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) H[a * 3 + b] += dm[a] * dq[b];
  }
  double U[9], sv[3], V[9];
  svd3(H, U, sv, V);
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
  if (det3(R) < 0.0) {
    for (int a = 0; a < 3; ++a) V[a * 3 + 2] = -V[a * 3 + 2];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        R[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
  }
  for (int a = 0; a < 3; ++a) t[a] = cq[a] - (R[a * 3 + 0] * cm[0] + R[a * 3 + 1] * cm[1] + R[a * 3 + 2] * cm[2]);
}

static double arun_error(const double R[9], const double t[3], const double pq[3], const double pm[3]) {
  double d[3];
  for (int a = 0; a < 3; ++a) d[a] = pq[a] - (R[a * 3 + 0] * pm[0] + R[a * 3 + 1] * pm[1] + R[a * 3 + 2] * pm[2] + t[a]);
  return sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
}

static int ransac_arun(const kmx_lcd_params* P, const double* Pq, const double* Pm, int K, double R[9], double t[3],
                       uint8_t* inl, int* n_inl, orc_mt19937* stream) {
  *n_inl = 0;
  const int S = 3;
  if (K < S) return 0;
  orc_mt19937 m0;
  orc_mt19937* m = problem_rng(P, &m0, stream);
  int32_t* sh = (int32_t*)malloc(sizeof(int32_t) * K);
  for (int i = 0; i < K; ++i) sh[i] = i;
  int iterations = 0, best_cnt = -INT_MAX, have = 0;
  double k = 1.0;
  double bR[9], bt[3];
  while (iterations < k) {
    for (int i = 0; i < S; ++i) {
      const int r = uid_draw(m, P->rng_variant);
      const int j = i + (int)((size_t)r % (size_t)(K - i));
      const int32_t tt = sh[i];
      sh[i] = sh[j];
      sh[j] = tt;
    }
    double Rm[9], tm[3];
    arun_model(Pq, Pm, sh, Rm, tm);
    int cnt = 0;
    for (int j = 0; j < K; ++j)
      if (arun_error(Rm, tm, Pq + 3 * j, Pm + 3 * j) < P->ransac_threshold_3d3d) ++cnt;
    if (cnt > best_cnt) {
      best_cnt = cnt;
      memcpy(bR, Rm, sizeof(bR));
      memcpy(bt, tm, sizeof(bt));
      have = 1;
      const double w = (double)cnt / (double)K;
      double p_no = 1.0 - pow(w, (double)S);
      p_no = fmax(DBL_EPSILON, p_no);
      p_no = fmin(1.0 - DBL_EPSILON, p_no);
      k = log(1.0 - P->ransac_probability) / log(p_no);
    }
    ++iterations;
    if (iterations > P->ransac_max_iterations) break;
  }
  free(sh);
  if (!have) return 0;
  int c = 0;
  for (int j = 0; j < K; ++j) {
    const int in = arun_error(bR, bt, Pq + 3 * j, Pm + 3 * j) < P->ransac_threshold_3d3d;
    inl[j] = (uint8_t)in;
    c += in;
  }
  *n_inl = c;
  memcpy(R, bR, sizeof(bR));
  memcpy(t, bt, sizeof(bt));
  return 1;
}

/* Verification of one candidate on a given correspondence list (pairs[2j] =
 * query feature, pairs[2j+1] = match feature, j < K): geometricVerificationNister
 * (KMX_LCD_STAGE_2D2D, drawio:2589-2592) then recoverPose (KMX_LCD_STAGE_RECOVER,
 * drawio:2595-2598), the two calls Kimera-Distributed's verifyLoopSpin makes on
 * computeMatchedIndices' output (drawio:2638-2657).
 *   - without the 2D-2D stage every pair counts as a 2D-2D inlier (the caller
 *     passes geometricVerificationNister's inliers to recoverPose) and the
 *     rotation of the 1-point 3D-3D recovery is T_prior's (the caller's
 *     2D-2D pose); recovery then runs whatever K is;
 *   - without the recovery stage, accepted = the 2D-2D model exists and has
 *     >= min_2d2d_inliers (geometricVerificationNister's bool), T = its pose.
 * masks (optional): [max_feats] bytes, bit0 2D-2D inlier, bit1 3D-3D / 2D-3D
 * inlier, indexed by position in the pair list. */
static void verify_pairs(const kmx_lcd_params* P, const kmx_lcd_batch_desc* pool, int32_t q, int32_t mfr, int K,
                         const int32_t* pairs, int stages, const double* T_prior, orc_mt19937* stream,
                         kmx_lcd_result* res, uint8_t* mask) {
  memset(res, 0, sizeof(*res));
  const int F = pool->max_feats;
  res->n_matches = K;
  if (mask) memset(mask, 0, (size_t)F);
  double* F1 = (double*)malloc(sizeof(double) * 3 * (K + 1));
  double* F2 = (double*)malloc(sizeof(double) * 3 * (K + 1));
  for (int j = 0; j < K; ++j)
    for (int c = 0; c < 3; ++c) {
      F1[3 * j + c] = pool->bearings[((size_t)q * F + pairs[2 * j]) * 3 + c];
      F2[3 * j + c] = pool->bearings[((size_t)mfr * F + pairs[2 * j + 1]) * 3 + c];
    }
  uint8_t* inl = (uint8_t*)calloc((size_t)K + 1, 1);
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
  int n_inl = 0, iters = 0, ok = 0, gate = 0;
  if (stages & KMX_LCD_STAGE_2D2D) {
    ok = ransac_2d2d(P, F1, F2, K, R, t, inl, &n_inl, &iters, stream);
    res->iterations_2d2d = iters;
    res->mono_inliers = ok ? n_inl : 0;
    gate = ok && n_inl >= P->min_2d2d_inliers;
  } else {
    for (int j = 0; j < K; ++j) inl[j] = 1;
    n_inl = K;
    ok = 1;
    gate = 1;
    res->mono_inliers = K;
    if (T_prior) {
      memcpy(R, T_prior, sizeof(R));
      memcpy(t, T_prior + 9, sizeof(t));
    }
  }
  if (ok && mask)
    for (int j = 0; j < K; ++j) mask[j] = inl[j];
  if (gate && (stages & KMX_LCD_STAGE_RECOVER)) {
    /* stereo points of the 2D-2D inliers, in pair-list order */
    double* Pq = (double*)malloc(sizeof(double) * 3 * (K + 1));
    double* Pm = (double*)malloc(sizeof(double) * 3 * (K + 1));
    uint8_t* valid = (uint8_t*)calloc((size_t)K + 1, 1);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (K + 1));
    int n3 = 0;
    for (int j = 0; j < K; ++j) {
      if (!inl[j]) continue;
      const double* a = pool->points + ((size_t)q * F + pairs[2 * j]) * 3;
      const double* b = pool->points + ((size_t)mfr * F + pairs[2 * j + 1]) * 3;
      for (int c = 0; c < 3; ++c) { Pq[3 * n3 + c] = a[c]; Pm[3 * n3 + c] = b[c]; }
      valid[n3] = !(isnan(a[0]) || isnan(a[1]) || isnan(a[2]) || isnan(b[0]) || isnan(b[1]) || isnan(b[2]));
      idx[n3] = j;
      ++n3;
    }
    uint8_t* in3 = (uint8_t*)calloc((size_t)n3 + 1, 1);
    if (P->pose_recovery_type == 1) {
      /* PnP: query bearings vs match-frame points of the 2D-2D inliers with
       * a valid stereo point, in pair-list order */
      double* Fq = (double*)malloc(sizeof(double) * 3 * (n3 + 1));
      double* Pw = (double*)malloc(sizeof(double) * 3 * (n3 + 1));
      int32_t* id2 = (int32_t*)malloc(sizeof(int32_t) * (n3 + 1));
      int n2 = 0;
      for (int j = 0; j < n3; ++j) {
        if (!valid[j]) continue;
        const int pj = idx[j];
        for (int c = 0; c < 3; ++c) {
          Fq[3 * n2 + c] = F1[3 * pj + c];
          Pw[3 * n2 + c] = Pm[3 * j + c];
        }
        id2[n2++] = pj;
      }
      double Ro[9], to[3];
      int np = 0;
      const int okp = ransac_pnp(P, Fq, Pw, n2, Ro, to, in3, &np, stream);
      res->pnp_inliers = okp ? np : 0;
      if (okp) {
        if (mask)
          for (int j = 0; j < n2; ++j)
            if (in3[j]) mask[id2[j]] |= 2;
        /* camera pose (R_o, t_o) in the match frame -> T_query_match: p_q = R p_m + t */
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) res->T_query_match[a * 3 + b] = Ro[b * 3 + a];
        for (int a = 0; a < 3; ++a)
          res->T_query_match[9 + a] = -(Ro[0 * 3 + a] * to[0] + Ro[1 * 3 + a] * to[1] + Ro[2 * 3 + a] * to[2]);
      }
      res->accepted = (okp && np >= P->min_2d3d_inliers) ? 1 : 0;
      free(Fq); free(Pw); free(id2);
    } else if (!P->use_1point_3d3d) {
      /* Arun RANSAC over the stereo-valid inliers, in pair-list order */
      double* Aq = (double*)malloc(sizeof(double) * 3 * (n3 + 1));
      double* Am = (double*)malloc(sizeof(double) * 3 * (n3 + 1));
      int32_t* id2 = (int32_t*)malloc(sizeof(int32_t) * (n3 + 1));
      int n2 = 0;
      for (int j = 0; j < n3; ++j) {
        if (!valid[j]) continue;
        for (int c = 0; c < 3; ++c) {
          Aq[3 * n2 + c] = Pq[3 * j + c];
          Am[3 * n2 + c] = Pm[3 * j + c];
        }
        id2[n2++] = idx[j];
      }
      double Ra[9], ta[3];
      int na = 0;
      const int oka = ransac_arun(P, Aq, Am, n2, Ra, ta, in3, &na, stream);
      res->stereo_inliers = oka ? na : 0;
      if (oka) {
        if (mask)
          for (int j = 0; j < n2; ++j)
            if (in3[j]) mask[id2[j]] |= 2;
        for (int i = 0; i < 9; ++i) res->T_query_match[i] = Ra[i];
        for (int i = 0; i < 3; ++i) res->T_query_match[9 + i] = ta[i];
      }
      res->accepted = (oka && na >= P->min_3d3d_inliers) ? 1 : 0;
      if (res->accepted && P->refine_pose) refit_3d3d(n2, Aq, Am, in3, res->T_query_match, res->T_query_match + 9);
      free(Aq); free(Am); free(id2);
    } else {
      double t3[3];
      const int c3 = given_rotation_3d3d(P, R, Pq, Pm, valid, n3, t3, in3);
      res->stereo_inliers = c3;
      if (mask)
        for (int j = 0; j < n3; ++j)
          if (in3[j]) mask[idx[j]] |= 2;
      for (int i = 0; i < 9; ++i) res->T_query_match[i] = R[i];
      for (int i = 0; i < 3; ++i) res->T_query_match[9 + i] = t3[i];
      res->accepted = (c3 >= P->min_3d3d_inliers) ? 1 : 0;
      if (res->accepted && P->refine_pose) refit_3d3d(n3, Pq, Pm, in3, res->T_query_match, res->T_query_match + 9);
    }
    free(Pq); free(Pm); free(valid); free(idx); free(in3);
  } else if (ok && (stages & KMX_LCD_STAGE_2D2D)) {
    for (int i = 0; i < 9; ++i) res->T_query_match[i] = R[i];
    for (int i = 0; i < 3; ++i) res->T_query_match[9 + i] = t[i];
    if (!(stages & KMX_LCD_STAGE_RECOVER)) res->accepted = gate;
  }
  free(F1); free(F2); free(inl);
}

/* Full verification of one candidate from a frame pool (same layout as
 * kmx_lcd_batch_desc): computeMatchedIndices (knn2 + Lowe), then both stages.
 * `stream`: the verification thread's engine when rng_stream = 1 (NULL:
 * every problem seeds its own). */
static void verify_one(const kmx_lcd_params* P, const kmx_lcd_batch_desc* pool, int32_t q, int32_t mfr,
                       orc_mt19937* stream, kmx_lcd_result* res, uint8_t* mask) {
  const int F = pool->max_feats;
  const int nq = pool->n_feats[q], nm = pool->n_feats[mfr];
  int32_t* pairs = (int32_t*)malloc(sizeof(int32_t) * 2 * (nq + 1));
  int32_t K = 0;
  orc_lcd_knn2(P->norm, (double)P->lowe_ratio, pool->desc + (size_t)q * F * 32, nq,
               pool->desc + (size_t)mfr * F * 32, nm, pairs, &K);
  verify_pairs(P, pool, q, mfr, K, pairs, KMX_LCD_STAGE_2D2D | KMX_LCD_STAGE_RECOVER, NULL, stream, res, mask);
  free(pairs);
}

int orc_lcd_verify(const kmx_lcd_params* P, const kmx_lcd_batch_desc* pool, int32_t q, int32_t mfr,
                   kmx_lcd_result* res, uint8_t* mask) {
  orc_mt19937 s;
  if (P->rng_stream) mt_seed(&s, P->ransac_seed);
  verify_one(P, pool, q, mfr, P->rng_stream ? &s : NULL, res, mask);
  return 0;
}

/* Candidates in order, as Kimera-Distributed's single verification thread
 * takes them off its queue (drawio:246, 405); with rng_stream = 1 the thread's
 * engine is seeded once at the start of the batch and continues from problem
 * to problem (2D-2D, then the Arun / EPnP recovery). */
int orc_lcd_verify_batch(const kmx_lcd_params* P, const kmx_lcd_batch_desc* pool, int32_t n,
                         const int32_t* cq, const int32_t* cm, kmx_lcd_result* res, uint8_t* masks) {
  orc_mt19937 s;
  if (P->rng_stream) mt_seed(&s, P->ransac_seed);
  for (int i = 0; i < n; ++i)
    verify_one(P, pool, cq[i], cm[i], P->rng_stream ? &s : NULL, res + i,
               masks ? masks + (size_t)i * pool->max_feats : NULL);
  return 0;
}

/* geometricVerificationNister / recoverPose on caller-supplied correspondences
 * (kmx_lcd_verify_matches): candidate i's pairs are
 * (i_query[k], i_match[k]) for k in [mptr[i], mptr[i+1]); T_prior [n][12]
 * (R row-major, t) is read only without the 2D-2D stage. */
int orc_lcd_verify_pairs_batch(const kmx_lcd_params* P, const kmx_lcd_batch_desc* pool, int32_t n,
                               const int32_t* cq, const int32_t* cm, const int64_t* mptr, const int32_t* i_query,
                               const int32_t* i_match, int stages, const double* T_prior, kmx_lcd_result* res,
                               uint8_t* masks) {
  orc_mt19937 s;
  if (P->rng_stream) mt_seed(&s, P->ransac_seed);
  for (int i = 0; i < n; ++i) {
    const int K = (int)(mptr[i + 1] - mptr[i]);
    int32_t* pairs = (int32_t*)malloc(sizeof(int32_t) * 2 * (K + 1));
    for (int k = 0; k < K; ++k) {
      pairs[2 * k] = i_query[mptr[i] + k];
      pairs[2 * k + 1] = i_match[mptr[i] + k];
    }
    verify_pairs(P, pool, cq[i], cm[i], K, pairs, stages, T_prior ? T_prior + 12 * (size_t)i : NULL,
                 P->rng_stream ? &s : NULL, res + i, masks ? masks + (size_t)i * pool->max_feats : NULL);
    free(pairs);
  }
  return 0;
}
