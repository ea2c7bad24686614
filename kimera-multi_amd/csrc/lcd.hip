// lcd.hip — Kimera-Multi-LCD loop-closure verification on MI355X (gfx950).
//
// Replaces LoopClosureDetector::computeMatchedIndices / geometricVerification-
// Nister / recoverPose (drawio:2583-2598) behind kmx_lcd_* (include/kmx_abi.h).
// Design (DESIGN.md "LCD"):
//   * k_knn2: one workgroup per candidate. The match frame's descriptors sit in
//     LDS (32 B each, read as broadcast); each lane owns a contiguous run of
//     query descriptors (two per LDS read), computes L1 (v_sad_u8 on 4-byte
//     words) or Hamming (xor + popcount) to every match descriptor, keeps the
//     two nearest as ordered keys (distance << 10 | index: OpenCV's strict-'<'
//     insertion), applies Lowe, and the workgroup compacts the pairs in query
//     order with a prefix sum.
//   * k_ransac_coop: a work queue of one-wave workgroups (one per resident
//     slot), each taking the next candidate from a counter; per candidate the
//     opengv RANSAC loop in its serial order with all 64 lanes cooperating on
//     each 5-point solve (Stewenius: six hypotheses' eigenvalue stages at once,
//     groups of 10 lanes), then the 1-point 3D-3D voting on the 2D-2D inliers.
//     Samples come from a host-built table of the opengv sampler (std::mt19937,
//     seed 12345, GCC-9 or GCC-11 uniform_int_distribution) indexed by K.
//   * k_recover: EPnP or Arun 3-point RANSAC on the 2D-2D inliers (lane per
//     hypothesis, lane 0 replays the serial control).
// The solver code is a line-by-line port of oracle/lcd_oracle.c and this file
// is compiled with -ffp-contract=off, so the inlier sets are bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <functional>
#include <random>
#include <thread>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"

namespace {

constexpr int KNN_BLOCK = 256;
constexpr int RS_BLOCK = 64;          // one wavefront per candidate
constexpr int RS_MAX_SLOTS = 8192;    // k_ransac_coop waves per launch at most (256 CUs x 32 waves)
constexpr int MAX_FEATS = 1024;
constexpr int LCD_SLOTS = 4;          // candidate slots: calls in flight at once (kmx_lcd_verify_async)

// ------------------------------------------------------------------ knn2 --
// The two-nearest update of ordered keys k0 <= k1 with a new key: k1' is the
// median of (k0, key, k1) (one v_med3_u32 in place of a max and a min), k0'
// the minimum. Same keys, same result as the min / max form.
__device__ __forceinline__ void two_nearest(uint32_t& k0, uint32_t& k1, uint32_t key) {
  uint32_t m;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m) : "v"(k0), "v"(key), "v"(k1));
  k1 = m;
  k0 = min(k0, key);
}

// The norm is a template parameter so the inner loop carries no branch on it
// (the runtime form evaluated the test twice per match descriptor).
template <bool HAMMING>
__device__ __forceinline__ void knn2_body(const uint32_t* desc, const int* nfeat, int N, const int* cq, const int* cm,
                                          double lowe, int2* pairs, int* Kout, uint32_t* sm_u32) {
  uint32_t* sdesc = sm_u32;                    // [nm][8]
  int* scnt = reinterpret_cast<int*>(sm_u32 + (size_t)N * 8);  // [KNN_BLOCK + 1]
  const int c = blockIdx.x;
  const int q = cq[c], m = cm[c];
  const int nq = nfeat[q], nm = nfeat[m];
  const uint32_t* dq = desc + (size_t)q * N * 8;
  const uint32_t* dm = desc + (size_t)m * N * 8;
  for (int i = threadIdx.x; i < nm * 8; i += KNN_BLOCK) sdesc[i] = dm[i];
  __syncthreads();
  const int per = (nq + KNN_BLOCK - 1) / KNN_BLOCK;
  const int i0 = threadIdx.x * per, i1 = min(nq, i0 + per);
  int found = 0;
  int bestj[4];  // per <= 4 for N <= MAX_FEATS
  bool pass[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) { bestj[u] = -1; pass[u] = false; }
  // The two nearest neighbours as ordered keys (distance << 10 | match index;
  // distance <= 32 x 255 < 2^13, index < 1024): the smallest key is the first
  // match at the smallest distance and the second smallest carries the second
  // distance (a repeat of the first included) — the serial scan's d0 / j0 / d1
  // with its strict tests — in two operations per pair (two_nearest). Each
  // match descriptor read from LDS serves two of the thread's queries.
  auto dist = [&](const uint32_t a[8], const uint32_t b[8]) -> uint32_t {
    uint32_t d = 0;
    if constexpr (HAMMING) {
#pragma unroll
      for (int w = 0; w < 8; ++w) d += __popc(a[w] ^ b[w]);
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) d = __builtin_amdgcn_sad_u8(a[w], b[w], d);
    }
    return d;
  };
  if (nm >= 2) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {  // per <= 4: at most two pairs, unrolled (static register indices)
      const int i = i0 + 2 * pp, u = 2 * pp;
      if (i >= i1) break;
      const bool two = i + 1 < i1;
      uint32_t a0[8], a1[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        a0[w] = dq[(size_t)i * 8 + w];
        a1[w] = two ? dq[(size_t)(i + 1) * 8 + w] : a0[w];
      }
      uint32_t k00 = 0xffffffffu, k01 = 0xffffffffu, k10 = 0xffffffffu, k11 = 0xffffffffu;
      for (int j = 0; j < nm; ++j) {
        const uint4* b4 = reinterpret_cast<const uint4*>(sdesc + j * 8);
        const uint4 x = b4[0], y = b4[1];
        const uint32_t b[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        two_nearest(k00, k01, (dist(a0, b) << 10) | (uint32_t)j);
        two_nearest(k10, k11, (dist(a1, b) << 10) | (uint32_t)j);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const uint32_t k0 = h ? k10 : k00, k1 = h ? k11 : k01;
        const int d0 = (int)(k0 >> 10), d1 = (int)(k1 >> 10);
        bestj[u + h] = (int)(k0 & 1023u);
        pass[u + h] = (double)(float)d0 < lowe * (double)(float)d1;
        found += pass[u + h] ? 1 : 0;
      }
    }
  }
  // exclusive prefix sum of per-thread counts (query order = thread order)
  scnt[threadIdx.x] = found;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int t = 0; t < KNN_BLOCK; ++t) {
      const int v = scnt[t];
      scnt[t] = s;
      s += v;
    }
    scnt[KNN_BLOCK] = s;
  }
  __syncthreads();
  int pos = scnt[threadIdx.x];
  int2* out = pairs + (size_t)c * N;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i0 + u < i1 && pass[u]) out[pos++] = make_int2(i0 + u, bestj[u]);
  if (threadIdx.x == 0) Kout[c] = scnt[KNN_BLOCK];
}

__global__ __launch_bounds__(KNN_BLOCK) void k_knn2(const uint32_t* desc, const int* nfeat, int N,
                                                    const int* cq, const int* cm, int norm, double lowe,
                                                    int2* pairs, int* Kout) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm_u32[];
  if (norm == KMX_NORM_HAMMING) knn2_body<true>(desc, nfeat, N, cq, cm, lowe, pairs, Kout, sm_u32);
  else knn2_body<false>(desc, nfeat, N, cq, cm, lowe, pairs, Kout, sm_u32);
}

// k_knn2 with four queries per thread (N <= 512; used for Hamming, see
// kmx_lcd::knn_q): each match descriptor read
// from LDS serves four queries instead of two, which halves the LDS-to-VGPR
// traffic per descriptor pair (2 x 16-B broadcast reads per match and wave);
// two waves per candidate. Query i lives on thread i / 4, so the compaction in
// thread order is query order: the same rows and K as k_knn2.
constexpr int KQ_BLOCK = 128, KQ_Q = 4;
template <bool HAMMING>
__global__ __launch_bounds__(KQ_BLOCK) void k_knn2q(const uint32_t* desc, const int* nfeat, int N, const int* cq,
                                                    const int* cm, double lowe, int2* pairs, int* Kout) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm_u32[];
  uint4* sdesc = reinterpret_cast<uint4*>(sm_u32);  // [nm][2]
  __shared__ int wtot[KQ_BLOCK / 64];
  const int c = blockIdx.x;
  const int q = cq[c], m = cm[c];
  const int nq = nfeat[q], nm = nfeat[m];
  const int tid = threadIdx.x;
  const uint4* dm = reinterpret_cast<const uint4*>(desc + (size_t)m * N * 8);
  for (int i = tid; i < nm * 2; i += KQ_BLOCK) sdesc[i] = dm[i];
  const int i0 = tid * KQ_Q;
  uint32_t a[KQ_Q][8];
#pragma unroll
  for (int u = 0; u < KQ_Q; ++u) {
    const uint4* d4 = reinterpret_cast<const uint4*>(desc + ((size_t)q * N + min(i0 + u, max(nq - 1, 0))) * 8);
    const uint4 x = d4[0], y = d4[1];
    a[u][0] = x.x; a[u][1] = x.y; a[u][2] = x.z; a[u][3] = x.w;
    a[u][4] = y.x; a[u][5] = y.y; a[u][6] = y.z; a[u][7] = y.w;
  }
  __syncthreads();
  uint32_t k0[KQ_Q], k1[KQ_Q];
#pragma unroll
  for (int u = 0; u < KQ_Q; ++u) k0[u] = k1[u] = 0xffffffffu;
  if (nm >= 2 && i0 < nq) {
    for (int j = 0; j < nm; ++j) {
      const uint4 x = sdesc[2 * j], y = sdesc[2 * j + 1];
      const uint32_t b[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
      for (int u = 0; u < KQ_Q; ++u) {
        uint32_t d = 0;
        if constexpr (HAMMING) {
#pragma unroll
          for (int w = 0; w < 8; ++w) d += __popc(a[u][w] ^ b[w]);
        } else {
#pragma unroll
          for (int w = 0; w < 8; ++w) d = __builtin_amdgcn_sad_u8(a[u][w], b[w], d);
        }
        two_nearest(k0[u], k1[u], (d << 10) | (uint32_t)j);
      }
    }
  }
  int found = 0;
  bool pass[KQ_Q];
#pragma unroll
  for (int u = 0; u < KQ_Q; ++u) {
    const int d0 = (int)(k0[u] >> 10), d1 = (int)(k1[u] >> 10);
    pass[u] = nm >= 2 && i0 + u < nq && (double)(float)d0 < lowe * (double)(float)d1;
    found += pass[u] ? 1 : 0;
  }
  // exclusive prefix of the per-thread counts in thread (= query) order
  const int lane = tid & 63, wv = tid >> 6;
  int incl = found;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wtot[wv] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wv; ++w) base += wtot[w];
  int pos = base + incl - found;
  int2* out = pairs + (size_t)c * N;
#pragma unroll
  for (int u = 0; u < KQ_Q; ++u)
    if (pass[u]) out[pos++] = make_int2(i0 + u, (int)(k0[u] & 1023u));
  if (tid == KQ_BLOCK - 1) Kout[c] = base + incl;
}

// kNN2 of a small synchronous call (the reference's verification thread
// matches ONE candidate per call: computeMatchedIndices, drawio:2583-2586).
// k_knn2 gives a candidate one workgroup, whose 4 waves scan every match
// descriptor for their queries (~65 us on one CU at N = 500). Here a
// candidate's queries are split over S = ceil(N / 64) workgroups of 64
// queries, and each query's match set over the workgroup's 4 waves: wave w
// keeps the two nearest keys of its quarter, and the four pairs are merged.
// A key is (distance << 10 | match index), unique per match, so the two
// smallest keys of the union are the serial scan's (d0, j0, d1) whatever
// the quarter boundaries. The last workgroup of a candidate to finish (an
// agent-scope counter; its writers fence first) compacts the per-query
// results in query order into k_knn2's pair rows: the same rows, the same K.
constexpr int KS_Q = 64;  // queries per workgroup of k_knn2s
template <bool HAMMING>
__global__ __launch_bounds__(KNN_BLOCK) void k_knn2s(const uint32_t* desc, const int* nfeat, int N, const int* cq,
                                                     const int* cm, double lowe, int2* pairs, int* Kout, int* qbest,
                                                     unsigned* cnt, int S, unsigned* done, unsigned seq) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm_u32[];
  uint32_t* sdesc = sm_u32;                                        // [nm][8]
  uint32_t* mk = sm_u32 + (size_t)N * 8;                           // [4][KS_Q][2] the quarters' keys
  int* scnt = reinterpret_cast<int*>(mk + 4 * KS_Q * 2);           // [KNN_BLOCK + 1]
  __shared__ int last;
  const int c = blockIdx.x / S, s = blockIdx.x - c * S;
  const int q = cq[c], m = cm[c];
  const int nq = nfeat[q], nm = nfeat[m];
  const int tid = threadIdx.x, ql = tid & (KS_Q - 1), part = tid >> 6;
  const int qi = s * KS_Q + ql;
  int* qb = qbest + (size_t)c * N;
  if (s * KS_Q < nq && nm >= 2) {
    const uint32_t* dm = desc + (size_t)m * N * 8;
    for (int i = tid; i < nm * 8; i += KNN_BLOCK) sdesc[i] = dm[i];
    __syncthreads();
    uint32_t k0 = 0xffffffffu, k1 = 0xffffffffu;
    if (qi < nq) {
      uint32_t a[8];
      const uint32_t* dq = desc + ((size_t)q * N + qi) * 8;
#pragma unroll
      for (int w = 0; w < 8; ++w) a[w] = dq[w];
      const int j0 = part * nm / 4, j1 = (part + 1) * nm / 4;
      for (int j = j0; j < j1; ++j) {
        const uint4* b4 = reinterpret_cast<const uint4*>(sdesc + j * 8);
        const uint4 x = b4[0], y = b4[1];
        const uint32_t b[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        uint32_t d = 0;
        if constexpr (HAMMING) {
#pragma unroll
          for (int w = 0; w < 8; ++w) d += __popc(a[w] ^ b[w]);
        } else {
#pragma unroll
          for (int w = 0; w < 8; ++w) d = __builtin_amdgcn_sad_u8(a[w], b[w], d);
        }
        two_nearest(k0, k1, (d << 10) | (uint32_t)j);
      }
    }
    mk[(part * KS_Q + ql) * 2] = k0;
    mk[(part * KS_Q + ql) * 2 + 1] = k1;
    __syncthreads();
    if (part == 0 && qi < nq) {
#pragma unroll
      for (int p = 1; p < 4; ++p) {
        two_nearest(k0, k1, mk[(p * KS_Q + ql) * 2]);
        two_nearest(k0, k1, mk[(p * KS_Q + ql) * 2 + 1]);
      }
      const int d0 = (int)(k0 >> 10), d1 = (int)(k1 >> 10);
      const bool pass = (double)(float)d0 < lowe * (double)(float)d1;
      qb[qi] = pass ? (int)(k0 & 1023u) : -1;
    }
  } else if (part == 0 && qi < nq) {
    qb[qi] = -1;  // fewer than two match features: no pair (k_knn2's nm >= 2 test)
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(cnt + c, 1u) == (unsigned)(S - 1);
  __syncthreads();
  if (!last) return;
  __threadfence();
  // compaction in query order (k_knn2's per-thread ranges and prefix sum)
  const int per = (nq + KNN_BLOCK - 1) / KNN_BLOCK;
  const int i0 = tid * per, i1 = min(nq, i0 + per);
  int found = 0;
  for (int i = i0; i < i1; ++i) found += __hip_atomic_load(qb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0;
  scnt[tid] = found;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int t = 0; t < KNN_BLOCK; ++t) {
      const int v = scnt[t];
      scnt[t] = acc;
      acc += v;
    }
    scnt[KNN_BLOCK] = acc;
    cnt[c] = 0u;  // the next call's count starts at zero
  }
  __syncthreads();
  int pos = scnt[tid];
  int2* out = pairs + (size_t)c * N;
  for (int i = i0; i < i1; ++i) {
    const int j = __hip_atomic_load(qb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j >= 0) out[pos++] = make_int2(i, j);
  }
  if (tid == 0) Kout[c] = scnt[KNN_BLOCK];
  if (done) {  // a one-candidate call's completion word (wait_done), after every row
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// --------------------------------------------------- small linear algebra --
__device__ void cross3(const double a[3], const double b[3], double c[3]) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ double det3(const double M[9]) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

__device__ void sym_eig3(double A[9], double V[9]) {
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    if (A[1] == 0.0 && A[2] == 0.0 && A[5] == 0.0) break;  // every rotation would be skipped
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        const double apq = A[p * 3 + q];
        if (apq == 0.0) continue;
        const double app = A[p * 3 + p], aqq = A[q * 3 + q];
        // negligible next to both diagonal entries: zero it (Rutishauser's threshold rule, Handbook for Automatic Computation II/1, 1971)
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

__device__ void svd3(const double E[9], double U[9], double s[3], double V[9]) {
  double A[9], W[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 3; ++k) acc += E[k * 3 + i] * E[k * 3 + j];
      A[i * 3 + j] = acc;
    }
  sym_eig3(A, W);
  // descending bubble sort of the eigenvalues (register selects, no indexing)
  auto ev = [&](int o) { return o == 0 ? A[0] : (o == 1 ? A[4] : A[8]); };
  int o0 = 0, o1 = 1, o2 = 2, tt;
  if (ev(o0) < ev(o1)) { tt = o0; o0 = o1; o1 = tt; }
  if (ev(o1) < ev(o2)) { tt = o1; o1 = o2; o2 = tt; }
  if (ev(o0) < ev(o1)) { tt = o0; o0 = o1; o1 = tt; }
  const int ord[3] = {o0, o1, o2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int o = ord[c];
    s[c] = sqrt(fmax(ev(o), 0.0));
#pragma unroll
    for (int r = 0; r < 3; ++r) V[r * 3 + c] = (o == 0) ? W[r * 3] : (o == 1 ? W[r * 3 + 1] : W[r * 3 + 2]);
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

__device__ double poly_eval(const double* c, int deg, double z) {
  double v = c[deg];
  for (int i = deg - 1; i >= 0; --i) v = v * z + c[i];
  return v;
}

constexpr int RR_SPLIT = 64, RR_DEPTH = 12;

// Fujiwara root bound with power-of-two terms (oracle/lcd_oracle.c root_bound)
__device__ __forceinline__ int root_bound_term(double ai, int m) {  // INT_MIN: none
  if (!(ai != 0.0) || !isfinite(ai)) return INT_MIN;
  const int x = ilogb(ai) + 1;
  return x >= 0 ? (x + m - 1) / m : -((-x) / m);
}

// 2D-2D sample error of a model (oracle/lcd_oracle.c model_error): the point
// triangulated from both bearings, 1 - cos to it in each frame, summed.
__device__ double model_error(const double R[9], const double t[3], const double f1[3], const double f2[3]) {
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

// ------------------------------------------------------------- EPnP ------
// Port of oracle/lcd_oracle.c orc_epnp for the RANSAC minimal sample (n = 6):
// same operations in the same order, so models are bit-identical.
constexpr int PNP_S = 6;

__device__ void jacobi_sym12(double* A, double* V) {
  constexpr int n = 12;
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

__device__ int qr_lsq(int m, int n, double* A, double* b, double* x) {
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

__constant__ int PAIR_A[6] = {0, 0, 0, 1, 1, 2};
__constant__ int PAIR_B[6] = {1, 2, 3, 2, 3, 3};
__constant__ int BCOLS[3][5] = {{0, 1, 3, 6, 0}, {0, 1, 2, 0, 0}, {0, 1, 2, 3, 4}};

__device__ void epnp_gauss_newton(const double L[60], const double rho[6], double bt[4]) {
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

__device__ double epnp_R_t(const double* pw, const double* uv, const double* alphas, const double V4[4][12],
                           const double bt[4], double R[9], double t[3]) {
  constexpr int n = PNP_S;
  double ccs[12];
  for (int j = 0; j < 12; ++j) ccs[j] = bt[0] * V4[0][j] + bt[1] * V4[1][j] + bt[2] * V4[2][j] + bt[3] * V4[3][j];
  double pc[3 * n];
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c)
      pc[3 * i + c] = alphas[4 * i + 0] * ccs[c] + alphas[4 * i + 1] * ccs[3 + c] + alphas[4 * i + 2] * ccs[6 + c] +
                      alphas[4 * i + 3] * ccs[9 + c];
  if (pc[2] < 0.0)
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
  return err / n;
}

// EPnP on a 6-point sample: camera pose (R_wc, t_wc) in the points' frame.
__device__ int epnp6(const double* pw, const double* f, double R_out[9], double t_out[3]) {
  constexpr int n = PNP_S;
  double uv[2 * n], alphas[4 * n];
  for (int i = 0; i < n; ++i) {
    uv[2 * i] = f[3 * i] / f[3 * i + 2];
    uv[2 * i + 1] = f[3 * i + 1] / f[3 * i + 2];
  }
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
  double CC[9], CI[9];
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) CC[r * 3 + k] = cw[3 * (k + 1) + r] - cw[r];
  const double dC = det3(CC);
  if (!(dC != 0.0)) return 0;
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
  double V4[4][12], L[60], rho[6];
  {
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
    jacobi_sym12(MtM, W);
    int ord[12];
    for (int i = 0; i < 12; ++i) ord[i] = i;
    for (int a = 0; a < 12; ++a)
      for (int b = 0; b < 11 - a; ++b)
        if (MtM[ord[b + 1] * 13] < MtM[ord[b] * 13]) { const int tt = ord[b]; ord[b] = ord[b + 1]; ord[b + 1] = tt; }
    for (int k = 0; k < 4; ++k)
      for (int j = 0; j < 12; ++j) V4[k][j] = W[j * 12 + ord[k]];
  }
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
  double best_err = DBL_MAX, Rb[9], tb[3];
  int found = 0;
  for (int approx = 1; approx <= 3; ++approx) {
    const int nc = approx == 1 ? 4 : approx == 2 ? 3 : 5;
    double A[30], b[6], x[5], bt[4] = {0, 0, 0, 0};
    for (int i = 0; i < 6; ++i) {
      for (int k = 0; k < nc; ++k) A[i * nc + k] = L[10 * i + BCOLS[approx - 1][k]];
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
    const double err = epnp_R_t(pw, uv, alphas, V4, bt, R, t);
    if (err < best_err) {
      best_err = err;
      for (int i = 0; i < 9; ++i) Rb[i] = R[i];
      for (int i = 0; i < 3; ++i) tb[i] = t[i];
      found = 1;
    }
  }
  if (!found) return 0;
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R_out[a * 3 + b] = Rb[b * 3 + a];
  for (int a = 0; a < 3; ++a) t_out[a] = -(Rb[0 * 3 + a] * tb[0] + Rb[1 * 3 + a] * tb[1] + Rb[2 * 3 + a] * tb[2]);
  return 1;
}

__device__ double pnp_error(const double R[9], const double t[3], const double p[3], const double f[3]) {
  const double d[3] = {p[0] - t[0], p[1] - t[1], p[2] - t[2]};
  double q[3];
  for (int i = 0; i < 3; ++i) q[i] = R[0 * 3 + i] * d[0] + R[1 * 3 + i] * d[1] + R[2 * 3 + i] * d[2];
  const double nq = sqrt(dot3(q, q));
  return 1.0 - (q[0] * f[0] + q[1] * f[1] + q[2] * f[2]) / nq;
}

struct RsParams {
  double thr2d, thr3d, prob;
  int max_iter, min2d, min3d, pmax;
  int refine;  // refine_pose: least-squares T over the 3D-3D inliers of an accepted recovery (refit_3d3d)
  int pnp;  // PnP or Arun recovery: k_ransac stops after 2D-2D, k_recover recovers the pose
  int prof; // diagnostic phase timers (k_ransac_coop)
  int algo; // KMX_ALGO_*: 5-point minimal solver (k_ransac_coop; k_ransac is Nister only)
  int stages;       // KMX_LCD_STAGE_* (kmx_lcd_verify: both)
  int tab_fixed;    // ordered sampler (rng_stream 1): `table` is this candidate's own row
  const double* prior;  // [n][12] 2D-2D pose of the 1-point recovery without the 2D-2D stage
  int* hyps;        // ordered sampler: passes the serial loop drew (iterations + skipped) per candidate
  int* nrec;        // ordered sampler: size of the recovery problem (stereo-valid 2D-2D inliers)
};
struct PnpParams {
  double thr, prob;
  int max_iter, min2d, min_pnp, pmax;
  int refine;     // Arun recovery only (refit_3d3d)
  int tab_fixed;  // as RsParams
  int* hyps;      // as RsParams
};

// refine_pose (oracle/lcd_oracle.c refit_3d3d, the same operations in the same
// order): least-squares T over the inlier pairs — centroids of all inliers,
// H = sum (p_m - c_m)(p_q - c_q)^T, Kabsch R with the reflection fix,
// t = c_q - R c_m. Serial (one lane); fetch(j, pq, pm) returns whether pair j
// is an inlier and, if so, its two points. Two passes (centroids, then H).
template <typename Fetch>
__device__ void refit_3d3d(int n, Fetch&& fetch, double R[9], double t[3]) {
  double cq[3] = {0.0, 0.0, 0.0}, cm[3] = {0.0, 0.0, 0.0};
  int c = 0;
  for (int j = 0; j < n; ++j) {
    double pq[3], pm[3];
    if (!fetch(j, pq, pm)) continue;
    for (int k = 0; k < 3; ++k) {
      cq[k] += pq[k];
      cm[k] += pm[k];
    }
    ++c;
  }
  for (int k = 0; k < 3; ++k) {
    cq[k] /= (double)c;
    cm[k] /= (double)c;
  }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < n; ++j) {
    double pq[3], pm[3];
    if (!fetch(j, pq, pm)) continue;
    double dq[3], dm[3];
    for (int k = 0; k < 3; ++k) {
      dq[k] = pq[k] - cq[k];
      dm[k] = pm[k] - cm[k];
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

// Diagnostic phase timers (kmx_lcd_debug_phase_times): cycles per phase summed
// over the first 64 candidates' hypotheses.
__device__ unsigned long long g_phase[16];
// KMX_RS_PROF=2 (diagnostic): each candidate's wave start / end (wall clock,
// 100 MHz) for the first STAMPS candidates of a launch: loaded latency and
// resident waves over time (scripts/lcd_stamps.py)
constexpr int STAMPS = 1 << 16;
__device__ unsigned long long g_stamp[2 * STAMPS];
struct WaveStamp {
  int c;
  bool on;
  __device__ WaveStamp(int c_, bool on_) : c(c_), on(on_ && c_ < STAMPS) {
    if (on && threadIdx.x == 0) g_stamp[2 * c] = wall_clock64();
  }
  __device__ ~WaveStamp() {
    if (on && threadIdx.x == 0) g_stamp[2 * c + 1] = wall_clock64();
  }
};
#define KMX_PT(i)                                                              \
  do {                                                                         \
    if (prof && lane == 0) {                                                   \
      const unsigned long long t_ = wall_clock64();                            \
      atomicAdd(&g_phase[i], t_ - t_prev);                                     \
      t_prev = t_;                                                             \
    }                                                                          \
  } while (0)

// ---------------------------------------------- cooperative 2D-2D RANSAC --
// k_ransac_coop: one wavefront per candidate, one hypothesis at a time with
// all 64 lanes cooperating on the 5-point solve (LDS workspace, ~6 KB), so
// no lane holds the 10x20 system or the Sturm sequence in registers (the
// lane-per-hypothesis k_ransac spills 4.9 KB/lane to scratch at 1 wave/SIMD).
// Every element is computed with the same operations in the same order as
// the serial code (oracle/lcd_oracle.c), so models, inlier sets and iteration
// counts stay bit-identical; hypotheses run in the serial loop's order, so no
// work is spent past the adaptive iteration count.
struct CoopWS {
  double f1[15], f2[15];
  double N[4][9];             // null space (until the essentials are formed)
  union {
    struct {                  // nullspace + system construction
      double vs[5][9];
      double c2[3][10];
      double EEt[9][10];
      double tr[10];
    };
    struct {                  // roots
      double S[12][11];       // Sturm sequence, zero padded (row 11: always zero)
      double cc[3][8];        // c1, c2, c3 of the degree-10 polynomial
      double st_lo[16], st_hi[16];
      int st_vl[16], st_vh[16], st_d[16];
    };
  };
  union {
    struct {                  // system + elimination
      double A[10][20];
    };
    struct {                  // models (A is dead once Bp is extracted)
      double Rab[10][2][9];   // per E: the two rotations (det fixed)
      double tu[10][3];       // per E: U's third column
    };
  };
  double Bp[3][3][5];
  double roots[10];
  double mR[9], mt[3];       // model of the current hypothesis
  double bestm[12];          // best model so far
  int nr, ok;
  signed char t11[10][2][2], t21[20][3][2];  // LDS copies of T11 / T21
};
// The Stewenius kernels' workspace: what the null space, the system and the
// recovery tail use (coop_system writes the 10 x 20 system straight into the
// wave's global stash, where the batched Gauss-Jordan reads it, and the
// Sturm / model areas are Nister's), 2.2 KB against CoopWS's 4.7 KB, so that
// with the batch (StewBatch) a wave stays below 10 KB of LDS: four waves per
// SIMD fit in the CU's 160 KB.
struct CoopWSS {
  double f1[15], f2[15];
  double N[4][9];
  double vs[5][9];
  double c2[3][10];
  double EEt[9][10];
  double tr[10];
  double bestm[12];
  int ok;
  signed char t11[10][2][2], t21[20][3][2];
};

// The block is one wavefront and a wave's LDS operations complete in issue
// order, so lane-to-lane hand-offs through LDS need only a compiler barrier
// (the pattern of pgo.hip's group_symYtG), not a workgroup barrier with its
// memory-count waits.
__device__ __forceinline__ void wsync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// The lane index as an opaque value at the start of each phase: the phases'
// lane-derived indices and LDS addresses are then formed where they are used
// instead of being hoisted out of the hypothesis loop by the compiler, where
// dozens of them stayed live across every phase (168 VGPRs + 596 B of scratch
// per lane, and the scratch-backed waves capped the resident waves).
__device__ __forceinline__ int fresh_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

// Candidate of workgroup b: blocks b and b + 8 run on the same XCD (the XCDs
// take workgroups round robin, statically), so XCD x is given one contiguous
// range of the candidates instead of every eighth one — a list whose costly
// candidates fall on a stride (the synthetic pools alternate true / false
// pairs: every true one went to the even XCDs) no longer leaves XCDs idle.
__device__ __forceinline__ int xcd_candidate(int b, int nwg) {
  const int q = nwg >> 3, rr = nwg & 7, x = b & 7;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
}

__device__ __forceinline__ double rdlane(double v, int src) {  // src wave-uniform
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_fmax(double v) {  // exact in any order
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// nullspace_5x9: Householder QR of Q^T with lane 9j+i holding A[i][j]
// (column j in 9 consecutive lanes); the column norms and the reflector are
// formed from readlane broadcasts in the serial order, each d_j from a
// 9-term gather of column j. Then the 4 back-substitutions (lanes 0-3).
template <typename WS>
__device__ void coop_nullspace(WS& w, int lane) {
  lane = fresh_lane(lane);
  const int li = lane % 9, lj = lane / 9;  // lanes >= 45 carry a dummy column
  double a = (lane < 45) ? w.f1[3 * lj + li / 3] * w.f2[3 * lj + li % 3] : 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    double v[9];
    double nx = 0.0;
#pragma unroll
    for (int i = k; i < 9; ++i) {
      v[i] = rdlane(a, 9 * k + i);
      nx += v[i] * v[i];
    }
    nx = sqrt(nx);
    const double alpha = (v[k] >= 0.0) ? -nx : nx;
    v[k] -= alpha;
    double nv = 0.0;
#pragma unroll
    for (int i = k; i < 9; ++i) nv += v[i] * v[i];
    nv = sqrt(nv);
    // the reflector's entries: lane i < 9 divides entry i (one quotient per
    // lane instead of nine per lane), then every lane reads them back
    double mine = 0.0;
#pragma unroll
    for (int i = k; i < 9; ++i) mine = (lane == i) ? v[i] : mine;
    mine = (nv > 0.0 && lane >= k && lane < 9) ? mine / nv : 0.0;
    double vs[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) vs[i] = i >= k ? rdlane(mine, i) : 0.0;
    if (lane < 9) w.vs[k][lane] = mine;
    // d_j = sum_{i >= k} vs[i] A[i][j] over this lane's column j
    double d = 0.0;
#pragma unroll
    for (int i = k; i < 9; ++i) d += vs[i] * __shfl(a, 9 * lj + i, 64);
    double my_vs = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) my_vs = (li == i) ? vs[i] : my_vs;
    if (lane < 45 && li >= k && lj >= k) a -= 2.0 * my_vs * d;
  }
  wsync();
  if (lane < 4) {
    double x[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = (i == 5 + lane) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 4; k >= 0; --k) {
      double d = 0.0;
#pragma unroll
      for (int i = k; i < 9; ++i) d += w.vs[k][i] * x[i];
#pragma unroll
      for (int i = k; i < 9; ++i) x[i] -= 2.0 * w.vs[k][i] * d;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) w.N[lane][i] = x[i];
  }
  wsync();
}

// E[e][c] = N[c][e]. Coefficient k of mul11(a, b) / mul21(a, b): its terms in
// the serial loop's (i, j) order (T11 / T21 list them), summed from 0.0.
__constant__ signed char T11[10][2][2] = {{{0, 0}, {-1, -1}}, {{0, 1}, {1, 0}}, {{0, 2}, {2, 0}}, {{1, 1}, {-1, -1}},
                                          {{1, 2}, {2, 1}}, {{2, 2}, {-1, -1}}, {{0, 3}, {3, 0}}, {{1, 3}, {3, 1}},
                                          {{2, 3}, {3, 2}}, {{3, 3}, {-1, -1}}};
__constant__ signed char T21[20][3][2] = {
    {{0, 0}, {-1, -1}, {-1, -1}}, {{3, 1}, {-1, -1}, {-1, -1}}, {{0, 1}, {1, 0}, {-1, -1}},
    {{1, 1}, {3, 0}, {-1, -1}},   {{0, 2}, {2, 0}, {-1, -1}},   {{0, 3}, {6, 0}, {-1, -1}},
    {{3, 2}, {4, 1}, {-1, -1}},   {{3, 3}, {7, 1}, {-1, -1}},   {{1, 2}, {2, 1}, {4, 0}},
    {{1, 3}, {6, 1}, {7, 0}},     {{2, 2}, {5, 0}, {-1, -1}},   {{2, 3}, {6, 2}, {8, 0}},
    {{6, 3}, {9, 0}, {-1, -1}},   {{4, 2}, {5, 1}, {-1, -1}},   {{4, 3}, {7, 2}, {8, 1}},
    {{7, 3}, {9, 1}, {-1, -1}},   {{5, 2}, {-1, -1}, {-1, -1}}, {{5, 3}, {8, 2}, {-1, -1}},
    {{8, 3}, {9, 2}, {-1, -1}},   {{9, 3}, {-1, -1}, {-1, -1}}};
// Coefficient k of mul11(E_ea, E_eb) / mul21(a, E_eb), E_e[c] = N[c][e]:
// the terms of the serial loop in its (i, j) order (LDS copies of T11 / T21).
template <typename WS>
__device__ __forceinline__ double mul11_e(const WS& w, int ea, int eb, int k) {
  double s = 0.0;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int i = w.t11[k][t][0];
    if (i >= 0) s += w.N[i][ea] * w.N[w.t11[k][t][1]][eb];
  }
  return s;
}
template <typename WS>
__device__ __forceinline__ double mul21_e(const double* a, const WS& w, int eb, int k) {
  double s = 0.0;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int i = w.t21[k][t][0];
    if (i >= 0) s += a[i] * w.N[w.t21[k][t][1]][eb];
  }
  return s;
}

// The system goes to A (row-major 10 x 20): w.A for Nister, the wave's global
// stash for the batched Stewenius Gauss-Jordan.
template <typename WS>
__device__ void coop_system(WS& w, int lane, double* A) {
  lane = fresh_lane(lane);
  // EEt[ij][k] = sum_l mul11(E[i*3+l], E[j*3+l])[k] (l = 0, 1, 2 in order); c2 for row 9:
  // c2_q = mul11(E_a, E_b) - mul11(E_c, E_d), (a, b, c, d) = (4,8,5,7), (3,8,5,6), (3,7,4,6)
  for (int t = lane; t < 90 + 30; t += RS_BLOCK) {
    if (t < 90) {
      const int ij = t / 10, k = t % 10, i = ij / 3, j = ij % 3;
      double acc = 0.0;
      for (int l = 0; l < 3; ++l) acc += mul11_e(w, i * 3 + l, j * 3 + l, k);
      w.EEt[ij][k] = acc;
    } else {
      const int q = (t - 90) / 10, k = (t - 90) % 10;
      const int ea = q == 0 ? 4 : 3, eb = q == 2 ? 7 : 8, ec = q == 2 ? 4 : 5, ed = q == 0 ? 7 : 6;
      w.c2[q][k] = mul11_e(w, ea, eb, k) - mul11_e(w, ec, ed, k);
    }
  }
  wsync();
  if (lane < 10) w.tr[lane] = w.EEt[0][lane] + w.EEt[4][lane] + w.EEt[8][lane];
  wsync();
  // rows 0..8: r[k] = sum_l 2 mul21(EEt[i*3+l], E[l*3+j])[k] - mul21(tr, E[ij])[k]; row 9
  for (int t = lane; t < 200; t += RS_BLOCK) {
    const int row = t / 20, k = t % 20;
    double r = 0.0;
    if (row < 9) {
      const int i = row / 3, j = row % 3;
      for (int l = 0; l < 3; ++l) r += 2.0 * mul21_e(w.EEt[i * 3 + l], w, l * 3 + j, k);
      r -= mul21_e(w.tr, w, row, k);
    } else {
      r += mul21_e(w.c2[0], w, 0, k);
      r -= mul21_e(w.c2[1], w, 1, k);
      r += mul21_e(w.c2[2], w, 2, k);
    }
    A[row * 20 + k] = r;
  }
  wsync();
}

// Gauss-Jordan with partial pivoting on the 10x20 system (serial order per
// element; lanes own columns). Returns 0 on a zero pivot.
// Lanes own columns (lane c < 20 holds A[0..9][c] in registers); column k
// is broadcast with readlane, so a pivot step touches no LDS. Same
// operations per element as the serial elimination (fivept_nister).
// graded: the columns are first permuted to Stewenius' graded order GORD.
__constant__ signed char GORD_D[20] = {0, 2, 4, 3, 8, 10, 1, 6, 13, 16, 5, 9, 11, 7, 14, 17, 12, 15, 18, 19};
__device__ int coop_gj(CoopWS& w, int lane, bool graded) {
  lane = fresh_lane(lane);
  const int cl = lane < 20 ? lane : 19;  // lanes >= 20 shadow column 19, never store
  const int src = graded ? GORD_D[cl] : cl;
  double a[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) a[i] = w.A[i][src];
  for (int k = 0; k < 10; ++k) {
    double col[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) col[i] = rdlane(a[i], k);
    int p = k;
    double pv = 0.0, pa = -1.0, ck = 0.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (i == k) { ck = col[i]; pv = ck; pa = fabs(ck); }
      else if (i > k && fabs(col[i]) > pa) { p = i; pv = col[i]; pa = fabs(col[i]); }
    }
    if (pv == 0.0) return 0;  // uniform
    const double inv = 1.0 / pv;
    double ak = 0.0, ap = 0.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      ak = (i == k) ? a[i] : ak;
      ap = (i == p) ? a[i] : ap;
    }
    const double rk = ap * inv;  // swapped (p == k: ap == ak), scaled pivot row
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (i == k) {
        a[i] = rk;
      } else {
        double ai = (i == p) ? ak : a[i];         // row p now holds the old row k
        const double f = (i == p) ? ck : col[i];  // column k after the swap
        if (f != 0.0) ai -= f * rk;
        a[i] = ai;
      }
    }
  }
  if (lane < 20) {
#pragma unroll
    for (int i = 0; i < 10; ++i) w.A[i][lane] = a[i];
  }
  wsync();
  return 1;
}

// Sign changes of the (zero-padded) Sturm sequence at z. Horner over the 11
// padded coefficients of each row gives the same value as
// poly_eval over sd[s] (leading zeros contribute exact signed zeros that the
// first non-zero coefficient absorbs), rows >= ns are all zero and skipped.
__device__ int coop_sign_changes(const CoopWS& w, double z) {
  int ch = 0;
  double prev = 0.0;
  auto step = [&](double v) {
    if (v != 0.0) {
      if (prev != 0.0 && ((v < 0.0) != (prev < 0.0))) ++ch;
      prev = v;
    }
  };
#pragma unroll 1
  for (int s = 0; s < 12; s += 2) {  // two independent Horner chains (row 11 is zero)
    double c0[11], c1[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) {
      c0[i] = w.S[s][i];
      c1[i] = w.S[s + 1][i];
    }
    double v0 = c0[10], v1 = c1[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) {
      v0 = v0 * z + c0[i];
      v1 = v1 * z + c1[i];
    }
    step(v0);
    step(v1);
  }
  return ch;
}

// pmul coefficient k (terms in increasing i from 0.0, as pmul accumulates)
__device__ __forceinline__ double pmul_k(const double* a, int da, const double* b, int db, int k) {
  double s = 0.0;
  for (int i = 0; i <= da; ++i) {
    const int j = k - i;
    if (j >= 0 && j <= db) s += a[i] * b[j];
  }
  return s;
}

// Newton refinement (refine_root) with the polynomial in registers; the
// derivative coefficients (i + 1) * c[i + 1] are formed on the fly.
__device__ double refine_root_reg(const double c[11], double a, double b) {
  auto ev = [&](double z) {
    double v = c[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) v = v * z + c[i];
    return v;
  };
  double fa = ev(a);
  double x = 0.5 * (a + b);
  for (int it = 0; it < 60; ++it) {
    double fx = c[10], dfx = 10.0 * c[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) {
      fx = fx * x + c[i];
      if (i >= 1) dfx = dfx * x + (double)i * c[i];
    }
    if (fx == 0.0) return x;
    if ((fx < 0.0) == (fa < 0.0)) { a = x; fa = fx; }
    else b = x;
    double xn = (dfx != 0.0) ? x - fx / dfx : 0.5 * (a + b);
    if (fabs(xn - x) <= 1e-15 * fmax(1.0, fabs(x))) return xn;  // converged (before the safeguard)
    if (!(xn > a && xn < b)) {
      xn = 0.5 * (a + b);
      if (fabs(xn - x) <= 1e-15 * fmax(1.0, fabs(x))) return xn;
    }
    x = xn;
  }
  return x;
}

// Bp, the degree-10 polynomial and its Sturm sequence with lanes owning
// coefficients (same operations per element as fivept_nister / real_roots),
// then the 64-ary isolation with one point per lane and one lane per root.
// Leaves w.nr roots in ascending order in w.roots.
__device__ void coop_roots(CoopWS& w, int lane, bool prof) {
  lane = fresh_lane(lane);
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  if (lane < 45) {  // Bp[q][c][i]
    const int q = lane / 15, c = (lane / 5) % 3, i = lane % 5;
    const double* e = &w.A[4 + 2 * q][10];
    const double* f = &w.A[5 + 2 * q][10];
    const int base = (c == 2) ? 9 : 3 * c + 2, imax = (c == 2) ? 3 : 2;
    double v;
    if (i == 0) v = e[base];
    else if (i <= imax) v = e[base - i] - f[base - i + 1];
    else if (i == imax + 1) v = -f[base - imax];
    else v = 0.0;
    w.Bp[q][c][i] = v;
  }
  for (int t = lane; t < 132; t += RS_BLOCK) (&w.S[0][0])[t] = 0.0;
  wsync();
  if (lane < 24) {  // c1 (8), c2 (8), c3 (7 + the zero c3[7])
    const int g = lane / 8, k = lane % 8;
    double v;
    if (g == 0) v = pmul_k(w.Bp[1][1], 3, w.Bp[2][2], 4, k) - pmul_k(w.Bp[1][2], 4, w.Bp[2][1], 3, k);
    else if (g == 1) v = pmul_k(w.Bp[1][0], 3, w.Bp[2][2], 4, k) - pmul_k(w.Bp[1][2], 4, w.Bp[2][0], 3, k);
    else v = (k < 7) ? pmul_k(w.Bp[1][0], 3, w.Bp[2][1], 3, k) - pmul_k(w.Bp[1][1], 3, w.Bp[2][0], 3, k) : 0.0;
    w.cc[g][k] = v;
  }
  wsync();
  double nco = 0.0;
  if (lane < 11)
    nco = pmul_k(w.Bp[0][0], 3, w.cc[0], 7, lane) - pmul_k(w.Bp[0][1], 3, w.cc[1], 7, lane) +
          pmul_k(w.Bp[0][2], 4, w.cc[2], 6, lane);
  KMX_PT(7);
  // degree: highest non-zero coefficient (0 when none)
  const unsigned long long nzm = __ballot(lane >= 1 && lane <= 10 && !(nco == 0.0)) ;
  const int deg = nzm ? 63 - __clzll(nzm) : 0;
  int nr = 0;
  double my_lo = 0.0, my_hi = 0.0;  // lane r: isolating interval of root r
  double c0 = 0.0;                  // lane i: S[0][i]
  if (deg > 0) {
    const double lead = rdlane(nco, deg);
    double a = (lane <= deg) ? nco / lead : 0.0;
    c0 = a;
    const double a_up = __shfl(a, (lane + 1) & 63, 64);
    double b = (lane < deg) ? (double)(lane + 1) * a_up : 0.0;
    if (lane <= deg) w.S[0][lane] = a;
    if (lane < deg) w.S[1][lane] = b;
    int ns = 2, da = deg, db = deg - 1;
    while (db > 0 && ns < 11) {
      double r = a;
      const double bd = rdlane(b, db);
      for (int k = da - db; k >= 0; --k) {
        const double fk = rdlane(r, k + db) / bd;
        const double bs = __shfl(b, (lane - k) & 63, 64);
        if (lane >= k && lane <= k + db) r -= fk * bs;
      }
      double mx = 0.0;  // max |S[ns-2][i]|, i <= da (lanes above da hold 0)
#pragma unroll
      for (int i = 0; i < 11; ++i) mx = fmax(mx, fabs(rdlane(a, i)));
      const unsigned long long keep = __ballot(lane < db && !(fabs(r) <= 1e-14 * mx));
      if (!keep) break;
      const int dr = 63 - __clzll(keep);
      const double nb = (lane <= dr) ? -r : 0.0;
      if (lane <= dr) w.S[ns][lane] = nb;
      a = b;
      b = nb;
      da = db;
      db = dr;
      ++ns;
    }
    // root_bound, lane-parallel (max over exact integer terms)
    const bool nonfin = lane < deg && !isfinite(c0);
    double bound;
    if (__ballot(nonfin)) {
      bound = wave_fmax((lane < deg) ? fabs(c0) : 0.0) + 1.0;
    } else {
      int km = (lane < deg) ? root_bound_term(c0, deg - lane) : INT_MIN;
      for (int off = 32; off > 0; off >>= 1) km = max(km, __shfl_xor(km, off, 64));
      bound = (km == INT_MIN) ? 1.0 : ldexp(1.0, km + 1);
    }
    wsync();
    KMX_PT(8);
    // 64-ary isolation; the stack (LDS) is popped uniformly, pieces are
    // pushed right to left so the leftmost is popped first (real_roots)
    if (lane == 0) {
      w.st_lo[0] = -bound; w.st_hi[0] = bound; w.st_d[0] = 0;
    }
    const int v_lo = coop_sign_changes(w, -bound);
    const int v_hi = coop_sign_changes(w, bound);
    if (lane == 0) { w.st_vl[0] = v_lo; w.st_vh[0] = v_hi; }
    int sp = 1;
    wsync();
    while (sp > 0) {
      --sp;
      const double lo = w.st_lo[sp], hi = w.st_hi[sp];
      const int vl = w.st_vl[sp], vh = w.st_vh[sp], dep = w.st_d[sp];
      const int cnt = vl - vh;
      if (cnt <= 0) continue;
      if (cnt == 1 || dep >= RR_DEPTH) {
        if (nr < 10) {
          if (lane == nr) { my_lo = lo; my_hi = hi; }
          ++nr;
        }
        continue;
      }
      const double wd = (hi - lo) / RR_SPLIT;
      const double x = (lane == 0) ? lo : lo + (double)lane * wd;
      const int v = (lane == 0) ? vl : coop_sign_changes(w, x);
      double xn = __shfl(x, (lane + 1) & 63, 64);
      int vn = __shfl(v, (lane + 1) & 63, 64);
      if (lane == RS_BLOCK - 1) { xn = hi; vn = vh; }
      const bool has = v - vn > 0;
      const unsigned long long hm = __ballot(has);
      const int above = (lane == RS_BLOCK - 1) ? 0 : __popcll(hm >> (lane + 1));
      const int slot = sp + above;
      wsync();  // the popped entry has been read by every lane
      if (has && slot < 16) {
        w.st_lo[slot] = x; w.st_hi[slot] = xn; w.st_vl[slot] = v; w.st_vh[slot] = vn; w.st_d[slot] = dep + 1;
      }
      sp = min(sp + __popcll(hm), 16);
      wsync();
    }
  }
  KMX_PT(9);
  double root = 0.0;
  if (lane < nr) {
    double c[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) c[i] = w.S[0][i];
    root = refine_root_reg(c, my_lo, my_hi);
  }
  // ascending order (stable rank = the bubble sort's order)
  int rank = 0;
  for (int j = 0; j < nr; ++j) {
    const double rj = rdlane(root, j);
    if (rj < root || (rj == root && j < lane)) ++rank;
  }
  if (lane < nr) w.roots[rank] = root;
  if (lane == 0) w.nr = nr;
  wsync();
  KMX_PT(10);
}

__device__ void coop_decompose(CoopWS& w, int lane, bool ok_root, const double Eo[9]);

// Essential matrices from the roots (lane per root), then coop_decompose.
__device__ void coop_models(CoopWS& w, int lane) {
  lane = fresh_lane(lane);
  const int nr = w.nr;
  int ok_root = 0;
  double Eo[9];
  if (lane < nr) {
    const double z = w.roots[lane];
    double row[3][3];
    for (int q = 0; q < 3; ++q)
      for (int c = 0; c < 3; ++c) row[q][c] = poly_eval(w.Bp[q][c], c == 2 ? 4 : 3, z);
    double v[3];
    cross3(row[0], row[1], v);
    if (v[2] != 0.0) {
      const double x = v[0] / v[2], y = v[1] / v[2];
      double nn = 0.0;
      for (int e = 0; e < 9; ++e) {
        Eo[e] = x * w.N[0][e] + y * w.N[1][e] + z * w.N[2][e] + w.N[3][e];
        nn += Eo[e] * Eo[e];
      }
      nn = sqrt(nn);
      if (nn > 0.0) {
        for (int e = 0; e < 9; ++e) Eo[e] /= nn;
        ok_root = 1;
      }
    }
  }
  coop_decompose(w, lane, ok_root != 0, Eo);
}

// Per E (lane per E, compacted in the solver's order: fivept_*'s ns counter)
// the 4 decompositions scored on the sample; the first minimum in (E, cand)
// order wins, as in model_from_sample. Result in w.mR / w.mt, w.ok.
__device__ void coop_decompose(CoopWS& w, int lane, bool ok_root, const double Eo[9]) {
  lane = fresh_lane(lane);
  const unsigned long long m = __ballot(ok_root);
  const int slot = __popcll(m & ((1ull << lane) - 1ull));
  const int ne = __popcll(m);
  if (ok_root) {
    // the two rotations and the translation direction of E (lane per E)
    double U[9], s[3], V[9];
    svd3(Eo, U, s, V);
    double Ra[9], Rb[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const double uw0 = U[i * 3 + 1], uw1 = -U[i * 3 + 0], uw2 = U[i * 3 + 2];
        Ra[i * 3 + j] = uw0 * V[j * 3 + 0] + uw1 * V[j * 3 + 1] + uw2 * V[j * 3 + 2];
        const double uv0 = -U[i * 3 + 1], uv1 = U[i * 3 + 0], uv2 = U[i * 3 + 2];
        Rb[i * 3 + j] = uv0 * V[j * 3 + 0] + uv1 * V[j * 3 + 1] + uv2 * V[j * 3 + 2];
      }
    const bool na = det3(Ra) < 0.0, nb = det3(Rb) < 0.0;
    for (int i = 0; i < 9; ++i) {
      w.Rab[slot][0][i] = na ? -Ra[i] : Ra[i];
      w.Rab[slot][1][i] = nb ? -Rb[i] : Rb[i];
    }
    for (int i = 0; i < 3; ++i) w.tu[slot][i] = U[i * 3 + 2];
  }
  wsync();
  // lane per (E, candidate): error of the decomposition on the sample
  const bool act = lane < 4 * ne;
  double err = DBL_MAX;
  double R[9], t[3];
  if (act) {
    const int e = lane >> 2, cand = lane & 3;
    for (int i = 0; i < 9; ++i) R[i] = w.Rab[e][cand >> 1][i];
    const double sg = (cand & 1) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i) t[i] = sg * w.tu[e][i];
    err = 0.0;
    for (int i = 0; i < 5; ++i) err += model_error(R, t, w.f1 + 3 * i, w.f2 + 3 * i);
  }
  // the first minimum in (E, candidate) order among errors < DBL_MAX
  const bool valid = act && err < DBL_MAX;
  double mn = valid ? err : DBL_MAX;
  for (int off = 32; off > 0; off >>= 1) mn = fmin(mn, __shfl_xor(mn, off, 64));
  const unsigned long long wm = __ballot(valid && err == mn);
  if (lane == 0) w.ok = wm ? 1 : 0;
  if (wm && lane == __ffsll((long long)wm) - 1) {
    for (int i = 0; i < 9; ++i) w.mR[i] = R[i];
    for (int i = 0; i < 3; ++i) w.mt[i] = t[i];
  }
  wsync();
}

// ------------------------------------------ 5-point (Stewenius 2006) --
// oracle/lcd_oracle.c orc_fivept_stewenius: action matrix of x on the
// basis [x^2, xy, xz, y^2, yz, z^2, x, y, z, 1] after the graded
// Gauss-Jordan, EISPACK elmhes + hqr eigenvalues, complex eigenvectors, E from the
// real part of each solution (conjugate pairs once). The Hessenberg
// reduction and the QR iteration run on several hypotheses' matrices at once
// (grp_hessenberg / grp_hqr below); the eigenvector solves are
// column-per-lane complex LUs with the same per-element operations.
struct cplx_d {
  double re, im;
};
__device__ __forceinline__ cplx_d c_mul(cplx_d a, cplx_d b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ cplx_d c_sub(cplx_d a, cplx_d b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx_d c_div(cplx_d a, cplx_d d) {
  cplx_d r;
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
__device__ __forceinline__ double c_abs1(cplx_d a) { return fabs(a.re) + fabs(a.im); }

// Eigenvectors normalised to v9 = 1 for up to 6 eigenvalues at once: lanes
// 10g..10g+9 solve the eigenvalue of group g, lane 10g+c holding column c of
// M - lam I (mcol = column c of its group's M; eigvec10's LU with partial
// pivoting, per element the same operations; the column broadcasts are group
// shuffles). Returns this group's (v6, v7, v8) real parts; ok = 0 on a zero
// pivot.
__device__ __forceinline__ cplx_d shfl_c(cplx_d v, int src) { return {__shfl(v.re, src, 64), __shfl(v.im, src, 64)}; }
__device__ __forceinline__ int eigvec_col(const double mcol[10], int lane, cplx_d lam, double xyz[3]) {
  lane = fresh_lane(lane);
  const int g0 = (lane / 10) * 10, c = lane - g0 < 10 ? lane - g0 : 9;
  cplx_d b[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    b[i].re = mcol[i];
    b[i].im = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 10; ++i)
    if (i == c) b[i] = c_sub(b[i], lam);
  int ok = 1;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    cplx_d col[10];
#pragma unroll
    for (int i = k; i < 10; ++i) col[i] = shfl_c(b[i], g0 + k);
    int p = k;
    double pa = c_abs1(col[k]);
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (c_abs1(col[i]) > pa) { p = i; pa = c_abs1(col[i]); }
    if (pa == 0.0) ok = 0;
    cplx_d bk = b[k], bp = b[k], ck = col[k], cp = col[k];
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == p) { bp = b[i]; cp = col[i]; }
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == p) { b[i] = bk; col[i] = ck; }
    b[k] = bp;
    col[k] = cp;
    // the multiplier of row i, col[i] / col[k], is formed once, by lane g0 + i,
    // and broadcast (the same division, so the same bits in every lane)
    cplx_d cm = col[k];
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == c) cm = col[i];
    const cplx_d fm = c_div(cm, col[k]);
#pragma unroll
    for (int i = k + 1; i < 10; ++i) {
      const cplx_d f = shfl_c(fm, g0 + i);
      if (c > k) b[i] = c_sub(b[i], c_mul(f, b[k]));
    }
  }
  cplx_d v[10];
  v[9].re = 1.0;
  v[9].im = 0.0;
#pragma unroll
  for (int i = 8; i >= 0; --i) {
    cplx_d s = {0.0, 0.0};
#pragma unroll
    for (int j = i + 1; j < 10; ++j) s = c_sub(s, c_mul(shfl_c(b[i], g0 + j), v[j]));
    v[i] = c_div(s, shfl_c(b[i], g0 + i));
  }
  xyz[0] = v[6].re;
  xyz[1] = v[7].re;
  xyz[2] = v[8].re;
  return ok;
}

// eigvec_col for a real eigenvalue (lam.im == 0): the complex LU's operations
// with every imaginary part zero, in real arithmetic — the same real parts
// bit for bit (x - 0 * y = x, |re| + 0 = |re|, Smith's quotient by (d, 0) is
// re / d; lcd.hip is built without contraction), at half the shuffles and a
// quarter of the arithmetic.
__device__ __forceinline__ int eigvec_col_real(const double mcol[10], int lane, double lam, double xyz[3]) {
  lane = fresh_lane(lane);
  const int g0 = (lane / 10) * 10, c = lane - g0 < 10 ? lane - g0 : 9;
  double b[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) b[i] = (i == c) ? mcol[i] - lam : mcol[i];
  int ok = 1;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    double col[10];
#pragma unroll
    for (int i = k; i < 10; ++i) col[i] = __shfl(b[i], g0 + k, 64);
    int p = k;
    double pa = fabs(col[k]);
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (fabs(col[i]) > pa) { p = i; pa = fabs(col[i]); }
    if (pa == 0.0) ok = 0;
    double bk = b[k], bp = b[k], ck = col[k], cp = col[k];
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == p) { bp = b[i]; cp = col[i]; }
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == p) { b[i] = bk; col[i] = ck; }
    b[k] = bp;
    col[k] = cp;
    double cm = col[k];
#pragma unroll
    for (int i = k + 1; i < 10; ++i)
      if (i == c) cm = col[i];
    const double fm = cm / col[k];
#pragma unroll
    for (int i = k + 1; i < 10; ++i) {
      const double f = __shfl(fm, g0 + i, 64);
      if (c > k) b[i] = b[i] - f * b[k];
    }
  }
  double v[10];
  v[9] = 1.0;
#pragma unroll
  for (int i = 8; i >= 0; --i) {
    double s = 0.0;
#pragma unroll
    for (int j = i + 1; j < 10; ++j) s = s - __shfl(b[i], g0 + j, 64) * v[j];
    v[i] = s / __shfl(b[i], g0 + i, 64);
  }
  xyz[0] = v[6];
  xyz[1] = v[7];
  xyz[2] = v[8];
  return ok;
}

// ------------------------------------- batched Stewenius eigenvalues ---
// k_ransac_coop<STEW = true> takes a candidate's hypotheses SG at a time in
// the serial loop's order: the null space, system and Gauss-Jordan of each
// (cooperative, 64 lanes), then the Hessenberg reduction and the QR iteration
// of the SG action matrices together, one group of GL lanes per matrix, then
// the rest of each hypothesis (eigenvectors, decomposition, scoring) one at a
// time with the serial loop's stopping rule, so hypotheses past the stop are
// computed but never scored. The eigenvalue stage is a chain of scalar steps
// (the elimination and QR pivots, ~8 divisions and a square root per QR
// step) that every lane of the cooperative form repeats; in groups each
// instruction advances SG matrices (the per-element operations and their
// order are the serial code's: bit-identical results). Counters behind the
// choice: profiles/r03/lcd/.
#ifndef KMX_SG
#define KMX_SG 6
#endif
constexpr int SG = KMX_SG, GL = SG <= 4 ? 16 : 10;
static_assert(SG * GL <= RS_BLOCK && GL >= 10, "groups");
// LDS: the matrices the groups work on and their eigenvalues; rows 0-5 of each
// action matrix and each null space (needed again by the eigenvector and
// essential-matrix steps) wait in the candidate's global scratch (STASH
// doubles per candidate after its compact bearings), so the batch costs 5.8
// KB of LDS per wave at SG = 6
constexpr int MAXP = SG * 10;  // solutions of one batch
struct StewBatch {
  double H[SG][10][10];
  double wr[SG][10], wi[SG][10];
  double mR[SG][9], mt[SG][3];  // each hypothesis's model
  double f1[SG][15], f2[SG][15];  // each hypothesis's sample bearings
  int ok[SG];                   // Gauss-Jordan and QR iteration succeeded
  int mok[SG];                  // a model was found
  unsigned char pb[MAXP], ps[MAXP];  // the batch's solutions: hypothesis, eigenvalue
  unsigned char qo[MAXP];            // solution indices in eigenvector order (real first)
};
constexpr int STASH_H = 96;  // per hypothesis: C6 (rows 0-5 of M, 60) + N (36)
constexpr int GJW = 3;       // hypotheses per batched Gauss-Jordan (groups of 20 lanes)
// + the batch's essentials, + GJW staged 10 x 20 systems
constexpr int STASH = SG * STASH_H + MAXP * 9 + GJW * 200;

// The highest group-local lane whose pred holds (-1: none).
__device__ __forceinline__ int grp_top(bool pred, int g) {
  const unsigned long long b = __ballot(pred);
  const unsigned long long gm = (b >> (GL * g)) & ((1ull << GL) - 1ull);
  return gm ? 63 - __clzll(gm) : -1;
}
__device__ __forceinline__ double grp_bcast(double v, int g, int src) { return __shfl(v, g * GL + src, 64); }
// A broadcast from a fixed group lane: with 16-lane groups (SG <= 4) one DPP
// row_newbcast move per 32-bit half (each group is a DPP row), else a shuffle.
// Measured (profiles/r04/lcd/sg4_dpp/): SG = 4 with DPP broadcasts 1.05-1.07e6
// candidates/s back to back, with shuffles 1.04-1.05e6, SG = 6 (the default,
// shuffles) 1.18e6: six matrices per pass outweigh the cheaper broadcasts.
template <int SRC>
__device__ __forceinline__ double grp_bcast_c(double v, int g) {
  if constexpr (GL == 16) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x150 + SRC, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x150 + SRC, 0xf, 0xf, false);
    (void)g;
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  }
  return __shfl(v, g * GL + SRC, 64);
}

// EISPACK ELMHES (Smith et al., EISPACK Guide, 1976; netlib eispack/elmhes.f;
// oracle/lcd_oracle.c hessenberg10) on sb.H[g] for every group g that is `on`:
// the pivot search and the multipliers are formed by the group's lanes from
// LDS reads in the serial order; each row / column update is one lane per
// element (the serial loop's element operations, same order of the dependent
// steps).
__device__ void grp_hessenberg(StewBatch& sb, int lane, bool on) {
  lane = fresh_lane(lane);
  const int g = lane / GL, gl = lane - g * GL;
  double (*a)[10] = sb.H[g < SG ? g : 0];
  const int n = 10, la = n - 2;
  for (int m = 1; m <= la; ++m) {
    const int mm1 = m - 1;
    double x = 0.0;
    int piv = m;
    for (int j = m; j < n; ++j) {
      const double v = a[j][mm1];
      if (fabs(v) <= fabs(x)) continue;
      x = v;
      piv = j;
    }
    wsync();
    const bool sw = on && piv != m;
    if (sw && gl >= mm1 && gl < n) { const double y = a[piv][gl]; a[piv][gl] = a[m][gl]; a[m][gl] = y; }
    wsync();
    if (sw && gl < n) { const double y = a[gl][piv]; a[gl][piv] = a[gl][m]; a[gl][m] = y; }
    wsync();
    const bool go = on && x != 0.0;
    for (int i = m + 1; i < n; ++i) {
      double y = a[i][mm1];
      const bool gy = go && y != 0.0;
      if (gy) y = y / x;
      wsync();
      if (gy && gl == 0) a[i][mm1] = y;
      if (gy && gl >= m && gl < n) a[i][gl] = a[i][gl] - y * a[m][gl];
      wsync();
      if (gy && gl < n) a[gl][m] = a[gl][m] + y * a[gl][i];
      wsync();
    }
  }
  if (on && gl >= 2 && gl < n)
    for (int j = 0; j < gl - 1; ++j) a[gl][j] = 0.0;
  wsync();
}

// EISPACK HQR (netlib eispack/hqr.f; oracle/lcd_oracle.c hqr10, the same
// loops and names) per group: each group's state (en, its, itn, t) advances
// one step per pass — deflation of one or two roots, or one double QR sweep —
// and the pass repeats while any group is working. The search for a
// negligible subdiagonal and the search for the sweep's start row m evaluate
// all candidates at once (lane per candidate; the serial loop's pick = the
// highest index whose test holds), the row and column modifications of the
// double QR step are one lane per column / row. Eigenvalues to sb.wr / sb.wi
// (a complex pair: wi(na) = +, wi(en) = -); sb.ok[g] = 0 when the group's
// 30 n sweeps ran out.
// ONE: only group 0 works (a batch of one hypothesis: the spread form's lone
// waves): the broadcasts are readlanes of group 0's lanes (scalar, no LDS
// round trip) and every search reads group 0's ballot bits, so the source
// lanes are wave-uniform; the other groups' lanes compute nothing that is
// kept. The same operations on the same values: the same bits.
template <bool ONE, int SRC>
__device__ __forceinline__ double hq_bc(double v, int g) {
  if constexpr (ONE) return rdlane(v, SRC);
  else return grp_bcast_c<SRC>(v, g);
}
template <bool ONE = false>
__device__ void grp_hqr(StewBatch& sb, int lane, bool on) {
  lane = fresh_lane(lane);
  const int g = lane / GL, gl = lane - g * GL;
  const int gs = ONE ? 0 : g;  // the group whose ballot bits a search reads
  double (*h)[10] = sb.H[g < SG ? g : 0];
  const int n = 10;
  double norm = 0.0;
  for (int i = 0, k = 0; i < n; k = i, ++i)
    for (int j = k; j < n; ++j) norm += fabs(h[i][j]);
  int en = on ? n - 1 : -1, itn = 30 * n, its = 0;
  bool fail = false;
  double t = 0.0;
  while (__ballot(en >= 0 && !fail)) {
    const bool act = en >= 0 && !fail;
    const int na = en - 1, enm2 = na - 1;
    bool hit = false;  // single small subdiagonal element: h(l,l-1), l = en .. 1
    if (act && gl >= 1 && gl <= en) {
      double s = fabs(h[gl - 1][gl - 1]) + fabs(h[gl][gl]);
      if (s == 0.0) s = norm;
      const double tst1 = s, tst2 = tst1 + fabs(h[gl][gl - 1]);
      hit = tst2 == tst1;
    }
    int l = grp_top(hit, gs);
    if (l < 0) l = 0;
    bool sweep = false;
    double x = 0.0, y = 0.0, wv = 0.0;
    if (act) {
      x = h[en][en];
      if (l == en) {  // one root
        if (gl == 0) { sb.wr[g][en] = x + t; sb.wi[g][en] = 0.0; }
        en = na;
        its = 0;
      } else {
        y = h[na][na];
        wv = h[en][na] * h[na][en];
        if (l == na) {  // two roots
          const double p = (y - x) / 2.0, q = p * p + wv;
          double zz = sqrt(fabs(q));
          x = x + t;
          if (gl == 0) {
            if (q >= 0.0) {
              zz = p + (p >= 0.0 ? fabs(zz) : -fabs(zz));
              sb.wr[g][na] = x + zz;
              sb.wr[g][en] = sb.wr[g][na];
              if (zz != 0.0) sb.wr[g][en] = x - wv / zz;
              sb.wi[g][na] = 0.0;
              sb.wi[g][en] = 0.0;
            } else {
              sb.wr[g][na] = x + p;
              sb.wr[g][en] = x + p;
              sb.wi[g][na] = zz;
              sb.wi[g][en] = -zz;
            }
          }
          en = enm2;
          its = 0;
        } else if (itn == 0) {
          fail = true;
        } else {
          sweep = true;
        }
      }
    }
    const bool exc = sweep && (its == 10 || its == 20);  // exceptional shift
    if (exc) t = t + x;
    wsync();
    if (exc && gl <= en) h[gl][gl] = h[gl][gl] - x;
    wsync();
    if (exc) {
      const double s = fabs(h[en][na]) + fabs(h[na][enm2]);
      x = 0.75 * s;
      y = x;
      wv = -0.4375 * s * s;
    }
    if (sweep) {
      ++its;
      --itn;
    }
    // the sweep's start: the largest m in [l, enm2] with m == l or two
    // consecutive small subdiagonal elements (lane per m)
    bool stop = false;
    double pm = 0.0, qm = 0.0, rm = 0.0;
    if (sweep && gl >= l && gl <= enm2) {
      const int m = gl;
      const double zz = h[m][m];
      rm = x - zz;
      double s = y - zz;
      pm = (rm * s - wv) / h[m + 1][m] + h[m][m + 1];
      qm = h[m + 1][m + 1] - zz - rm - s;
      rm = h[m + 2][m + 1];
      s = fabs(pm) + fabs(qm) + fabs(rm);
      pm = pm / s;
      qm = qm / s;
      rm = rm / s;
      if (m == l) {
        stop = true;
      } else {
        const double tst1 = fabs(pm) * (fabs(h[m - 1][m - 1]) + fabs(zz) + fabs(h[m + 1][m + 1]));
        const double tst2 = tst1 + fabs(h[m][m - 1]) * (fabs(qm) + fabs(rm));
        stop = tst2 == tst1;
      }
    }
    int m = grp_top(stop, gs);  // lane l always stops
    if (m < 0) m = 0;
    double p, q, r, zz = 0.0;
    if constexpr (ONE) {
      p = rdlane(pm, m);
      q = rdlane(qm, m);
      r = rdlane(rm, m);
    } else {
      p = grp_bcast(pm, g, m);
      q = grp_bcast(qm, g, m);
      r = grp_bcast(rm, g, m);
    }
    wsync();
    if (sweep && gl >= m + 2 && gl <= en) {
      h[gl][gl - 2] = 0.0;
      if (gl != m + 2) h[gl][gl - 3] = 0.0;
    }
    wsync();
    for (int kk = 0; __ballot(sweep && m + kk <= na); ++kk) {  // double QR step on rows l..en, columns m..en
      const int k = m + kk;
      bool go = sweep && k <= na;
      const bool notlas = k != na;
      if (go && k != m) {
        p = h[k][k - 1];
        q = h[k + 1][k - 1];
        r = 0.0;
        if (notlas) r = h[k + 2][k - 1];
        x = fabs(p) + fabs(q) + fabs(r);
        if (x == 0.0) {
          go = false;
        } else {  // p / x, q / x, r / x: one quotient per lane 0-2 of the group, broadcast
          const double quo = (gl == 0 ? p : gl == 1 ? q : r) / x;
          p = hq_bc<ONE, 0>(quo, g);
          q = hq_bc<ONE, 1>(quo, g);
          r = hq_bc<ONE, 2>(quo, g);
        }
      }
      double s = 0.0;
      if (go) {
        const double sq = sqrt(p * p + q * q + r * r);
        s = p >= 0.0 ? sq : -sq;
      }
      wsync();
      if (go && gl == 0) {
        if (k == m) {
          if (l != m) h[k][k - 1] = -h[k][k - 1];
        } else {
          h[k][k - 1] = -s * x;
        }
      }
      if (go) {  // p / s, q / s, r / s, q / p, r / p: lanes 0-4 of the group, broadcast
        p = p + s;
        const double quo = (gl == 0 ? p : gl == 1 || gl == 3 ? q : r) / (gl < 3 ? s : p);
        x = hq_bc<ONE, 0>(quo, g);
        y = hq_bc<ONE, 1>(quo, g);
        zz = hq_bc<ONE, 2>(quo, g);
        q = hq_bc<ONE, 3>(quo, g);
        r = hq_bc<ONE, 4>(quo, g);
      }
      if (go && gl >= k && gl <= en) {  // row modification, column j = gl
        const int j = gl;
        if (notlas) {
          const double pp = h[k][j] + q * h[k + 1][j] + r * h[k + 2][j];
          h[k][j] = h[k][j] - pp * x;
          h[k + 1][j] = h[k + 1][j] - pp * y;
          h[k + 2][j] = h[k + 2][j] - pp * zz;
        } else {
          const double pp = h[k][j] + q * h[k + 1][j];
          h[k][j] = h[k][j] - pp * x;
          h[k + 1][j] = h[k + 1][j] - pp * y;
        }
      }
      wsync();
      const int jmax = en < k + 3 ? en : k + 3;
      if (go && gl >= l && gl <= jmax) {  // column modification, row i = gl
        const int i = gl;
        if (notlas) {
          const double pp = x * h[i][k] + y * h[i][k + 1] + zz * h[i][k + 2];
          h[i][k] = h[i][k] - pp;
          h[i][k + 1] = h[i][k + 1] - pp * q;
          h[i][k + 2] = h[i][k + 2] - pp * r;
        } else {
          const double pp = x * h[i][k] + y * h[i][k + 1];
          h[i][k] = h[i][k] - pp;
          h[i][k + 1] = h[i][k + 1] - pp * q;
        }
      }
      wsync();
    }
  }
  if (on && fail && gl == 0) sb.ok[g] = 0;
  wsync();
}

// Entry (i, j) of the action matrix of x after coop_gj(graded) (w.A = [I | C]
// in graded order): rows 0-5 are -C, rows 6-9 unit entries (oracle
// orc_fivept_stewenius).
__device__ __forceinline__ double action_entry(const double* C6, int i, int j) {
  double v = (i < 6) ? C6[i * 10 + j] : 0.0;
  if ((i == 6 && j == 0) || (i == 7 && j == 1) || (i == 8 && j == 2) || (i == 9 && j == 6)) v = 1.0;
  return v;
}

// The models of a batch after grp_hqr (orc_fivept_stewenius + model_from_sample
// for each hypothesis b < nb, all at once): the solutions of every hypothesis
// whose eigenvalues exist (eigenvalue order, a conjugate pair once) are listed
// in (b, solution) order; their eigenvectors six at a time (eigvec_col, the
// column of the hypothesis's action matrix rebuilt from the stash) and
// essentials (stash, STASH_E); then one lane per essential decomposes it and
// scores its 4 (R, t) candidates on its hypothesis's sample in candidate
// order; each hypothesis takes the first minimum in (essential, candidate)
// order, as coop_decompose does for one. sb.mok[b] = 0: no model.
__device__ __forceinline__ void stew_models(StewBatch& sb, double* stash, int lane, const double* F1, const double* F2,
                                            const short* tab, int p0, int nb, bool prof) {
  lane = fresh_lane(lane);
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  int np;
  int nre;  // the real solutions come first in the eigenvector order (sb.qo)
  {  // solution list
    const int b = lane / 10, s = lane - 10 * b;
    const bool sol = lane < 10 * nb && sb.ok[b < SG ? b : 0] && !(sb.wi[b < SG ? b : 0][s] < 0.0);
    const bool re = sol && sb.wi[b < SG ? b : 0][s] == 0.0;
    const unsigned long long m = __ballot(sol), mr = __ballot(re);
    if (sol) {
      const int k = __popcll(m & ((1ull << lane) - 1ull));
      sb.pb[k] = (unsigned char)b;
      sb.ps[k] = (unsigned char)s;
      // eigenvector order: real solutions first (real LU), then the complex ones
      const int o = re ? __popcll(mr & ((1ull << lane) - 1ull))
                       : __popcll(mr) + __popcll((m & ~mr) & ((1ull << lane) - 1ull));
      sb.qo[o] = (unsigned char)k;
    }
    np = __popcll(m);
    nre = __popcll(mr);
  }
  wsync();
  double* Es = stash + SG * STASH_H;
  unsigned long long pok = 0;  // bit k: solution k gave an essential
  // six solutions at a time in eigenvector order: batches [0, nre) real, then
  // [nre, np) complex (a batch never mixes them; results land at the solution's
  // list index, so the order they are computed in changes nothing)
  for (int q0 = 0; q0 < np;) {
    const bool real = q0 < nre;
    const int qend = real ? nre : np, qn = min(6, qend - q0);
    const int g = lane / 10, g0 = g * 10, c = lane - g0;
    const bool act = g < qn;
    const int pi = act ? sb.qo[q0 + g] : 0;
    const int b = act ? sb.pb[pi] : 0, si = act ? sb.ps[pi] : 0;
    const double* st = stash + b * STASH_H;
    const int cc = c < 10 ? c : 9;
    double mcol[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) mcol[i] = action_entry(st, i, cc);
    double xyz[3] = {0.0, 0.0, 0.0};
    const int okv = real ? eigvec_col_real(mcol, lane, act ? sb.wr[b][si] : 0.0, xyz)
                         : eigvec_col(mcol, lane, cplx_d{act ? sb.wr[b][si] : 0.0, act ? sb.wi[b][si] : 0.0}, xyz);
    // lane 10g + e (e < 9): entry e of E; the norm over the group's 9 entries in order
    const double* Nb = st + 60;
    const double e = (c < 9) ? xyz[0] * Nb[c] + xyz[1] * Nb[9 + c] + xyz[2] * Nb[18 + c] + Nb[27 + c] : 0.0;
    double nn = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const double ei = __shfl(e, g0 + i < 64 ? g0 + i : 63, 64);
      nn += ei * ei;
    }
    nn = sqrt(nn);
    const bool good = act && okv && nn > 0.0 && isfinite(nn);
    if (good && c < 9) Es[pi * 9 + c] = e / nn;
    const unsigned long long gm = __ballot(good && c == 0);
#pragma unroll
    for (int gg = 0; gg < 6; ++gg)
      if ((gm >> (10 * gg)) & 1ull) pok |= 1ull << sb.qo[q0 + gg];
    q0 += qn;
  }
  __threadfence_block();  // Es is read back by other lanes of this wave
  wsync();
  KMX_PT(9);
  // lane per essential: decomposition and its best candidate on the sample
  const bool eact = lane < np && ((pok >> lane) & 1ull);
  const int eb = eact ? sb.pb[lane] : 0;
  bool valid = false;
  double best = DBL_MAX, bR[9], bt[3];
  if (eact) {
    double Eo[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) Eo[i] = Es[lane * 9 + i];
    double U[9], sv[3], V[9];
    svd3(Eo, U, sv, V);
    const double* f1 = sb.f1[eb];
    const double* f2 = sb.f2[eb];
    // the two rotations one after the other (Ra: candidates 0, 1; Rb: 2, 3),
    // so only one is live: Ra = (U1, -U0, U2) V^T, Rb = (-U1, U0, U2) V^T
    // (the negations are exact: the same bits as forming both at once)
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      double Rh[9];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          const double u0 = h ? -U[i * 3 + 1] : U[i * 3 + 1], u1 = h ? U[i * 3 + 0] : -U[i * 3 + 0],
                       u2 = U[i * 3 + 2];
          Rh[i * 3 + j] = u0 * V[j * 3 + 0] + u1 * V[j * 3 + 1] + u2 * V[j * 3 + 2];
        }
      const bool neg = det3(Rh) < 0.0;
      for (int i = 0; i < 9; ++i) Rh[i] = neg ? -Rh[i] : Rh[i];
      for (int cs = 0; cs < 2; ++cs) {
        double t[3];
        const double sg = cs ? -1.0 : 1.0;
        for (int i = 0; i < 3; ++i) t[i] = sg * U[i * 3 + 2];
        double err = 0.0;
        for (int i = 0; i < 5; ++i) err += model_error(Rh, t, f1 + 3 * i, f2 + 3 * i);
        if (err < DBL_MAX && (!valid || err < best)) {
          valid = true;
          best = err;
          for (int i = 0; i < 9; ++i) bR[i] = Rh[i];
          for (int i = 0; i < 3; ++i) bt[i] = t[i];
        }
      }
    }
  }
  for (int b = 0; b < nb; ++b) {  // each hypothesis: the first minimum over its essentials
    const bool inb = valid && eb == b;
    double mn = inb ? best : DBL_MAX;
    for (int off = 32; off > 0; off >>= 1) mn = fmin(mn, __shfl_xor(mn, off, 64));
    const unsigned long long wm = __ballot(inb && best == mn);
    if (lane == 0) sb.mok[b] = wm ? 1 : 0;
    if (wm && lane == __ffsll((long long)wm) - 1) {
      for (int i = 0; i < 9; ++i) sb.mR[b][i] = bR[i];
      for (int i = 0; i < 3; ++i) sb.mt[b][i] = bt[i];
    }
  }
  wsync();
  KMX_PT(10);
}

// The sample's bearings, the null space and the 10x20 system (both solvers).
template <typename WS>
__device__ __forceinline__ void coop_prepare(WS& w, int lane, const double* F1, const double* F2, int N,
                                             const short* smp, bool prof, double* A) {
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  if (lane < 15) {
    const int i = lane / 3, c = lane % 3;
    w.f1[lane] = F1[(size_t)c * N + smp[i]];
    w.f2[lane] = F2[(size_t)c * N + smp[i]];
  }
  wsync();
  KMX_PT(0);
  coop_nullspace(w, lane);
  KMX_PT(1);
  coop_system(w, lane, A);
  KMX_PT(2);
}

// One Nister hypothesis: sample -> models (w.ok, w.mR, w.mt).
__device__ __forceinline__ void coop_hypothesis(CoopWS& w, int lane, const double* F1, const double* F2, int N,
                                                const short* smp, bool prof) {
  coop_prepare(w, lane, F1, F2, N, smp, prof, &w.A[0][0]);
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  if (!coop_gj(w, lane, false)) {
    if (lane == 0) w.ok = 0;
    wsync();
    return;
  }
  KMX_PT(3);
  coop_roots(w, lane, prof);
  KMX_PT(4);
  if (w.nr == 0) {
    if (lane == 0) w.ok = 0;
    wsync();
    return;
  }
  coop_models(w, lane);
  KMX_PT(5);
}

// Stewenius: the hypotheses p0 .. p0 + nb - 1 up to their action matrices,
// stashed in sb (one at a time, 64 lanes), then their eigenvalues together.
// coop_gj for GJW systems at once: group g (lanes 20g .. 20g + 19) eliminates
// the system staged at A (row-major 10 x 20) with lane 20g + c holding graded
// column c, the column-k broadcasts a group shuffle; per element the
// operations of coop_gj in its order (the same bits). Returns the group's
// success (0: a zero pivot; the group's later values are then unused).
__device__ __forceinline__ int grp_gj(const double* A, int cl, int g0, double a[10]) {
  const int src = GORD_D[cl];
#pragma unroll
  for (int i = 0; i < 10; ++i) a[i] = A[i * 20 + src];
  int ok = 1;
  for (int k = 0; k < 10; ++k) {
    double col[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) col[i] = __shfl(a[i], g0 + k, 64);
    int p = k;
    double pv = 0.0, pa = -1.0, ck = 0.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (i == k) { ck = col[i]; pv = ck; pa = fabs(ck); }
      else if (i > k && fabs(col[i]) > pa) { p = i; pv = col[i]; pa = fabs(col[i]); }
    }
    if (pv == 0.0) ok = 0;
    const double inv = 1.0 / pv;
    double ak = 0.0, ap = 0.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      ak = (i == k) ? a[i] : ak;
      ap = (i == p) ? a[i] : ap;
    }
    const double rk = ap * inv;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (i == k) {
        a[i] = rk;
      } else {
        double ai = (i == p) ? ak : a[i];
        const double f = (i == p) ? ck : col[i];
        if (f != 0.0) ai -= f * rk;
        a[i] = ai;
      }
    }
  }
  return ok;
}

// Stewenius: the hypotheses p0 .. p0 + nb - 1 up to their action matrices
// (null space and system one at a time, 64 lanes; Gauss-Jordan GJW at a time
// from systems staged in the wave's scratch), stashed in sb, then their
// eigenvalues together.
template <bool ALLOW_ONE = false, typename WS>
__device__ __forceinline__ void stew_batch(WS& w, StewBatch& sb, double* stash, int lane, const double* F1,
                                           const double* F2, int N, const short* tab, int p0, int nb, bool prof) {
  double* Ab = stash + SG * STASH_H + MAXP * 9;
  for (int b0 = 0; b0 < nb; b0 += GJW) {
    const int nw = min(GJW, nb - b0);
    for (int u = 0; u < nw; ++u) {
      const int b = b0 + u;
      coop_prepare(w, lane, F1, F2, N, tab + (size_t)(p0 + b) * 5, prof, Ab + u * 200);
      double* st = stash + b * STASH_H;
      if (lane < 36) st[60 + lane] = (&w.N[0][0])[lane];
      if (lane < 15) {
        sb.f1[b][lane] = w.f1[lane];
        sb.f2[b][lane] = w.f2[lane];
      }
      __threadfence_block();  // the staged system is read by other lanes of this wave
      wsync();
    }
    const int gg = lane / 20, g = gg < nw ? gg : 0, cl = lane - gg * 20 < 20 ? lane - gg * 20 : 19;
    const bool gact = gg < nw;
    double a[10];
    const int okg = grp_gj(Ab + g * 200, cl, g * 20, a);
    if (gact && okg) {
      const int b = b0 + gg;
      double* st = stash + b * STASH_H;
      if (cl >= 10) {  // rows 0-5 of the action matrix: -C from columns 10-19
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const double v = -a[i];
          st[i * 10 + (cl - 10)] = v;
          sb.H[b][i][cl - 10] = v;
        }
      } else {  // rows 6-9: unit entries
#pragma unroll
        for (int i = 6; i < 10; ++i) sb.H[b][i][cl] = action_entry(nullptr, i, cl);
      }
    }
    if (gact && cl == 0 && lane - gg * 20 == 0) sb.ok[b0 + gg] = okg;
    __threadfence_block();
    wsync();
  }
  __threadfence_block();  // the stash is read back by this wave (stew_models)
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  const int g = lane / GL;
  const bool on = g < nb && sb.ok[g];
  grp_hessenberg(sb, lane, on);
  KMX_PT(7);
  if (ALLOW_ONE && nb == 1) grp_hqr<true>(sb, lane, on);
  else grp_hqr<false>(sb, lane, on);
  KMX_PT(8);
}

// The candidate's result after its RANSAC loop (shared by the work-queue
// kernel and the spread form's k_rs_finish): the best model's inliers (and
// mask), then the 1-point 3D-3D recovery (and refine_pose), or the hand-over
// to k_recover. w.bestm holds the best model when `have`.
// WAVE: the 1-point recovery's loops by the whole wave with its data staged
// in `lds` (tail_lds_doubles(N) doubles; k_rs_finish's dynamic LDS).
__host__ __device__ constexpr size_t tail_lds_doubles(int N) { return 3 * ((size_t)N + 4) + ((size_t)N + 15) / 8 + 6 * (size_t)N; }
struct NoCount {  // the work-queue kernel: no multi-wave count
  __device__ int operator()(const double*, const unsigned char*, int, double) const { return -1; }
};
// Not inlined: the tail runs once per candidate, and as a call of its own its
// registers are allocated apart from the hypothesis loop's, so the Stewenius
// work queue fits 128 VGPRs (four waves per SIMD) with 200 spilled instead of
// 308 inlined; same box, 20k candidates: 1.514e6 -> 1.543e6 candidates/s, the
// hard leg 7.89e4 -> 8.24e4 (profiles/r06/lcd_lb4/).
template <bool WAVE, typename WS, typename Count = NoCount>
__device__ __noinline__ void ransac_tail(int c, WS& w, double* F1, double* F2, const double* points, int N,
                                            int q, int m, const int2* pl, int K, const RsParams& P,
                                            kmx_lcd_result* R_, unsigned char* mask, int have, int iterations,
                                            int lane, double* lds = nullptr, Count&& count_best = Count{}) {
  const bool st2d = (P.stages & KMX_LCD_STAGE_2D2D) != 0;
  auto pair_error = [&](const double* R, const double* t, int j) {
    const double a[3] = {F1[j], F1[N + j], F1[2 * N + j]}, b[3] = {F2[j], F2[N + j], F2[2 * N + j]};
    return model_error(R, t, a, b);
  };
  if (!have && st2d) {
    if (lane == 0) {
      kmx_lcd_result r = {};
      r.n_matches = K;
      r.iterations_2d2d = iterations;
      *R_ = r;
    }
    return;
  }
  double Rb[9], tb[3];
  if (st2d) {
    for (int i = 0; i < 9; ++i) Rb[i] = w.bestm[i];
    for (int i = 0; i < 3; ++i) tb[i] = w.bestm[9 + i];
  } else {  // the caller's 2D-2D pose (only the 1-point recovery reads it)
    for (int i = 0; i < 12; ++i) (i < 9 ? Rb[i] : tb[i - 9]) = P.prior ? P.prior[(size_t)c * 12 + i] : (i % 4 == 0 && i < 9 ? 1.0 : 0.0);
  }
  // a pair's 2D-2D inlier test: the best model's, or every pair without the stage
  auto inl2d = [&](int j) { return (j < K) && (!st2d || pair_error(Rb, tb, j) < P.thr2d); };
  int n_in = 0;
  for (int j0 = 0; j0 < K; j0 += RS_BLOCK) {
    const int j = j0 + lane;
    const bool in = inl2d(j);
    if (j < K && mask) mask[j] = in ? 1 : 0;
    n_in += __popcll(__ballot(in));
  }
  kmx_lcd_result r = {};
  r.n_matches = K;
  r.mono_inliers = n_in;
  r.iterations_2d2d = iterations;
  for (int i = 0; i < 9; ++i) r.T_query_match[i] = Rb[i];
  for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = tb[i];
  if (st2d && n_in < P.min2d) {
    if (lane == 0) *R_ = r;
    return;
  }
  if (!(P.stages & KMX_LCD_STAGE_RECOVER)) {  // geometricVerificationNister alone
    r.accepted = 1;
    if (lane == 0) *R_ = r;
    return;
  }
  if (P.pnp) {
    if (P.nrec) {  // ordered sampler: the host sizes the recovery's sample row
      int n2 = 0;
      for (int j0 = 0; j0 < K; j0 += RS_BLOCK) {
        const int j = j0 + lane;
        bool v = inl2d(j);
        if (v) {
          const int2 pr = pl[j];
          const double* a = points + ((size_t)q * N + pr.x) * 3;
          const double* b = points + ((size_t)m * N + pr.y) * 3;
          v = !(isnan(a[0]) || isnan(a[1]) || isnan(a[2]) || isnan(b[0]) || isnan(b[1]) || isnan(b[2]));
        }
        n2 += __popcll(__ballot(v));
      }
      if (lane == 0) P.nrec[c] = n2;
    }
    if (lane == 0) {
      for (int i = 0; i < 12; ++i) r.T_query_match[i] = 0.0;
      *R_ = r;
    }
    return;
  }
  // 1-point 3D-3D given the rotation over the 2D-2D inliers (pair order):
  // T_j = p_q - R p_m; the largest consistent set (ties: smallest index)
  // reuses F2's scratch slot for T and the workspace for the index list.
  double* T = F2;
  wsync();
  int n3 = 0;
  for (int j0 = 0; j0 < K; j0 += RS_BLOCK) {  // compact inlier positions in pair order
    const int j = j0 + lane;
    const bool in = inl2d(j);
    const unsigned long long bm = __ballot(in);
    const int pos = n3 + __popcll(bm & ((1ull << lane) - 1ull));
    if (in) reinterpret_cast<int*>(F1)[pos] = j;  // F1 rows < j0 + 64 are no longer read
    n3 += __popcll(bm);
    wsync();
  }
  const int* idx = reinterpret_cast<const int*>(F1);
  unsigned char* valid = reinterpret_cast<unsigned char*>(F1) + sizeof(int) * (size_t)N;
  // note: F1's first N ints hold idx; valid bytes follow within F1's 3N doubles
  wsync();
  // (WAVE: four inliers per lane per pass, the idx -> pair -> point loads of
  // the pass issued before their uses: three dependent round trips per pass
  // instead of per inlier)
  constexpr int TU = WAVE ? 4 : 1;
  for (int k0 = lane; k0 < n3; k0 += TU * RS_BLOCK) {
    int jj[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) jj[u] = idx[min(k0 + u * RS_BLOCK, n3 - 1)];
    int2 pr[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) pr[u] = pl[jj[u]];
    double a[TU][3], b[TU][3];
#pragma unroll
    for (int u = 0; u < TU; ++u)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        a[u][i] = points[((size_t)q * N + pr[u].x) * 3 + i];
        b[u][i] = points[((size_t)m * N + pr[u].y) * 3 + i];
      }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int k = k0 + u * RS_BLOCK;
      if (k >= n3) break;
      const bool v = !(isnan(a[u][0]) || isnan(a[u][1]) || isnan(a[u][2]) || isnan(b[u][0]) || isnan(b[u][1]) ||
                       isnan(b[u][2]));
      valid[k] = v ? 1 : 0;
      for (int i = 0; i < 3; ++i)
        T[3 * k + i] = a[u][i] - (Rb[i * 3 + 0] * b[u][0] + Rb[i * 3 + 1] * b[u][1] + Rb[i * 3 + 2] * b[u][2]);
    }
  }
  __threadfence_block();
  wsync();
  if constexpr (!WAVE) {  // one lane's serial loops (the work-queue kernel: other waves fill the CU meanwhile)
  const double thr2 = P.thr3d * P.thr3d;
  int my_best = -1, my_cnt = 0;
  for (int i = lane; i < n3; i += RS_BLOCK) {
    if (!valid[i]) continue;
    int cc = 0;
    for (int j = 0; j < n3; ++j) {
      if (!valid[j]) continue;
      const double dx = T[3 * j] - T[3 * i], dy = T[3 * j + 1] - T[3 * i + 1], dz = T[3 * j + 2] - T[3 * i + 2];
      if (dx * dx + dy * dy + dz * dz < thr2) ++cc;
    }
    if (cc > my_cnt) { my_cnt = cc; my_best = i; }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const int oc = __shfl_xor(my_cnt, off, 64);
    const int ob = __shfl_xor(my_best, off, 64);
    if (oc > my_cnt || (oc == my_cnt && ob >= 0 && (my_best < 0 || ob < my_best))) {
      my_cnt = oc;
      my_best = ob;
    }
  }
  if (lane == 0) {
    const int best = my_best;
    if (best >= 0) {
      int cc = 0;
      double s[3] = {0.0, 0.0, 0.0};
      for (int j = 0; j < n3; ++j) {
        int in = 0;
        if (valid[j]) {
          const double dx = T[3 * j] - T[3 * best], dy = T[3 * j + 1] - T[3 * best + 1], dz = T[3 * j + 2] - T[3 * best + 2];
          in = dx * dx + dy * dy + dz * dz < thr2;
        }
        if (in) {
          for (int i = 0; i < 3; ++i) s[i] += T[3 * j + i];
          ++cc;
          if (mask) mask[idx[j]] |= 2;
        }
      }
      for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = s[i] / (double)cc;
      r.stereo_inliers = cc;
      r.accepted = (cc >= P.min3d) ? 1 : 0;
      if (r.accepted && P.refine) {  // the inliers again: valid and within thr3d of the best translation
        refit_3d3d(
            n3,
            [&](int j, double* pq, double* pm) {
              if (!valid[j]) return false;
              const double dx = T[3 * j] - T[3 * best], dy = T[3 * j + 1] - T[3 * best + 1],
                           dz = T[3 * j + 2] - T[3 * best + 2];
              if (!(dx * dx + dy * dy + dz * dz < thr2)) return false;
              const int2 pr = pl[idx[j]];
              const double* a = points + ((size_t)q * N + pr.x) * 3;
              const double* b = points + ((size_t)m * N + pr.y) * 3;
              for (int k = 0; k < 3; ++k) { pq[k] = a[k]; pm[k] = b[k]; }
              return true;
            },
            r.T_query_match, r.T_query_match + 9);
      }
    } else {
      for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = 0.0;
    }
    *R_ = r;
  }
  } else {  // the same sums by the whole wave (the spread form's latency path: k_rs_finish)
  // (KMX_RS_PROF=3, diagnostic: g_phase[11..13] = count, final pass, refit; [14] n3, [15] calls)
  const bool prof = P.prof == 3;
  unsigned long long t_prev = prof ? wall_clock64() : 0;
  if (prof && lane == 0) {
    atomicAdd(&g_phase[15], 1ull);
    atomicAdd(&g_phase[14], (unsigned long long)n3);
  }
  const double thr2 = P.thr3d * P.thr3d;
  // T and valid staged in LDS (each lane copies the entries it wrote), then
  // the largest consistent set (count_best: every wave of k_rs_finish's
  // workgroup counts a block of i against a range of j; the ties and the
  // first maximum as below)
  double* Tl = lds;                                                              // [N + 4][3]
  unsigned char* vl = reinterpret_cast<unsigned char*>(lds + 3 * ((size_t)N + 4));  // [N + 4]
  double* Pc = lds + 3 * ((size_t)N + 4) + ((size_t)N + 15) / 8;                 // [N][6]: compacted inliers
  for (int k = lane; k < n3; k += RS_BLOCK) {
    for (int i = 0; i < 3; ++i) Tl[3 * k + i] = T[3 * k + i];
    vl[k] = valid[k];
  }
  for (int k = n3 + lane; k < ((n3 + 3) & ~3); k += RS_BLOCK) {  // the last quad's padding
    for (int i = 0; i < 3; ++i) Tl[3 * k + i] = 0.0;
    vl[k] = 0;
  }
  wsync();
  const int best = count_best(Tl, vl, n3, thr2);  // the same in every lane
  KMX_PT(11);
  if (best >= 0) {
    // the inliers of the best translation, compacted in pair order into Pc
    // (T_j, and with refine_pose their two points) by ballot prefix sums; the
    // ordered sums then run over contiguous LDS (every lane the same adds in
    // the serial order, four loads ahead)
    const double tb[3] = {Tl[3 * best], Tl[3 * best + 1], Tl[3 * best + 2]};
    const bool refine = P.refine != 0;
    int cc = 0;
    // four passes of the wave at a time, their idx -> pair -> point loads
    // issued before the passes' ballots (three dependent round trips per four
    // passes instead of per pass)
    constexpr int FU = 4;
    for (int j00 = 0; j00 < n3; j00 += FU * RS_BLOCK) {
      int jx[FU];
      int2 pr[FU];
      double pa[FU][3], pb[FU][3];
#pragma unroll
      for (int u = 0; u < FU; ++u) jx[u] = idx[min(j00 + u * RS_BLOCK + lane, n3 - 1)];
      if (refine) {
#pragma unroll
        for (int u = 0; u < FU; ++u) pr[u] = pl[jx[u]];
#pragma unroll
        for (int u = 0; u < FU; ++u)
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            pa[u][k] = points[((size_t)q * N + pr[u].x) * 3 + k];
            pb[u][k] = points[((size_t)m * N + pr[u].y) * 3 + k];
          }
      }
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const int j0 = j00 + u * RS_BLOCK;
        if (j0 >= n3) break;
        const int j = j0 + lane;
        bool in = false;
        double tj[3] = {0.0, 0.0, 0.0};
        if (j < n3 && vl[j]) {
          for (int k = 0; k < 3; ++k) tj[k] = Tl[3 * j + k];
          const double dx = tj[0] - tb[0], dy = tj[1] - tb[1], dz = tj[2] - tb[2];
          in = dx * dx + dy * dy + dz * dz < thr2;
        }
        if (j < n3 && mask) mask[jx[u]] = in ? 3 : 1;  // idx lists 2D-2D inliers (mask 1): | 2
        const unsigned long long im = __ballot(in);
        if (in) {
          const int pos = cc + __popcll(im & ((1ull << lane) - 1ull));
          double* o = Pc + 6 * (size_t)pos;
          if (refine) {
            for (int k = 0; k < 3; ++k) {
              o[k] = pa[u][k];
              o[3 + k] = pb[u][k];
            }
          } else {
            for (int k = 0; k < 3; ++k) o[k] = tj[k];
          }
        }
        cc += __popcll(im);
      }
    }
    wsync();
    // Each ordered sum below is one lane's serial chain (the serial loop's
    // adds in its order, so the same bits), the chains on different lanes,
    // and each lane's operands loaded eight inliers ahead of its adds (LDS
    // loads were one latency per inlier on the chain); the results reach every
    // lane by readlane.
    constexpr int AH = 8;
    double s3[3] = {0.0, 0.0, 0.0};
    {
      const int i = lane < 3 ? lane : 0;
      double acc = 0.0;
      for (int k0 = 0; k0 < cc; k0 += AH) {
        double v[AH];
        const int kn = min(AH, cc - k0);
        if (!refine) {
#pragma unroll
          for (int u = 0; u < AH; ++u) v[u] = u < kn ? Pc[6 * (k0 + u) + i] : 0.0;
        } else {  // T_j = p_q - R p_m again from the staged points (the expression T was formed by)
#pragma unroll
          for (int u = 0; u < AH; ++u) {
            const double* a = Pc + 6 * (k0 + (u < kn ? u : 0));
            const double* b = a + 3;
            v[u] = a[i] - (Rb[i * 3 + 0] * b[0] + Rb[i * 3 + 1] * b[1] + Rb[i * 3 + 2] * b[2]);
          }
        }
#pragma unroll
        for (int u = 0; u < AH; ++u)
          if (u < kn) acc += v[u];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) s3[c] = rdlane(acc, c);
    }
    for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = s3[i] / (double)cc;
    r.stereo_inliers = cc;
    r.accepted = (cc >= P.min3d) ? 1 : 0;
    KMX_PT(12);
    if (r.accepted && refine) {  // refit_3d3d's sums over the same inliers, in its order
      // centroids: lane c < 6 sums coordinate c of the staged (p_q, p_m) pairs
      double cq3[3], cm3[3];
      {
        const int c = lane < 6 ? lane : 0;
        double acc = 0.0;
        for (int k0 = 0; k0 < cc; k0 += AH) {
          double v[AH];
          const int kn = min(AH, cc - k0);
#pragma unroll
          for (int u = 0; u < AH; ++u) v[u] = u < kn ? Pc[6 * (k0 + u) + c] : 0.0;
#pragma unroll
          for (int u = 0; u < AH; ++u)
            if (u < kn) acc += v[u];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          cq3[i] = rdlane(acc, i) / (double)cc;
          cm3[i] = rdlane(acc, 3 + i) / (double)cc;
        }
      }
      // H[a][b] = sum dm[a] dq[b]: lane 3a + b < 9 its entry's chain
      double H[9];
      {
        const int e = lane < 9 ? lane : 0, a = e / 3, b = e - 3 * a;
        const double ca = a == 0 ? cm3[0] : (a == 1 ? cm3[1] : cm3[2]);
        const double cb = b == 0 ? cq3[0] : (b == 1 ? cq3[1] : cq3[2]);
        double acc = 0.0;
        for (int k0 = 0; k0 < cc; k0 += AH) {
          double vm[AH], vq[AH];
          const int kn = min(AH, cc - k0);
#pragma unroll
          for (int u = 0; u < AH; ++u) {
            const int k = k0 + (u < kn ? u : 0);
            vq[u] = Pc[6 * k + b];
            vm[u] = Pc[6 * k + 3 + a];
          }
#pragma unroll
          for (int u = 0; u < AH; ++u)
            if (u < kn) acc += (vm[u] - ca) * (vq[u] - cb);
        }
#pragma unroll
        for (int x = 0; x < 9; ++x) H[x] = rdlane(acc, x);
      }
      double U[9], sv[3], V[9], Rr[9];
      svd3(H, U, sv, V);
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
          Rr[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
      if (det3(Rr) < 0.0) {
        for (int a = 0; a < 3; ++a) V[a * 3 + 2] = -V[a * 3 + 2];
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b)
            Rr[a * 3 + b] = V[a * 3 + 0] * U[b * 3 + 0] + V[a * 3 + 1] * U[b * 3 + 1] + V[a * 3 + 2] * U[b * 3 + 2];
      }
      for (int a = 0; a < 9; ++a) r.T_query_match[a] = Rr[a];
      for (int a = 0; a < 3; ++a)
        r.T_query_match[9 + a] = cq3[a] - (Rr[a * 3 + 0] * cm3[0] + Rr[a * 3 + 1] * cm3[1] + Rr[a * 3 + 2] * cm3[2]);
      KMX_PT(13);
    }
  } else {
    for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = 0.0;
  }
  if (lane == 0) *R_ = r;
  }
}

// One candidate's 2D-2D RANSAC and 3D-3D recovery by the calling wave; F1 is
// the wave's global scratch (6 N + STASH doubles).
template <bool STEW, typename WS, typename SB>
__device__ __forceinline__ void ransac_candidate(int c, WS& w, SB& sb, double* F1, const double* bearings,
                                                 const double* points, int N, const int* cq, const int* cm,
                                                 const int2* pairs, const int* Kin, const short* table,
                                                 const RsParams& P, kmx_lcd_result* res, unsigned char* masks) {
  const int lane = fresh_lane(threadIdx.x);
  const WaveStamp stamp(c, P.prof == 2);
  const int K = Kin[c];
  const int q = cq[c], m = cm[c];
  unsigned char* mask = masks ? masks + (size_t)c * N : nullptr;
  kmx_lcd_result* R_ = res + c;
  for (int j = lane; j < N && mask; j += RS_BLOCK) mask[j] = 0;
  const bool st2d = (P.stages & KMX_LCD_STAGE_2D2D) != 0;
  if (K < 5 && st2d) {
    if (P.hyps && lane == 0) P.hyps[c] = 0;
    if (lane == 0) {
      kmx_lcd_result r = {};
      r.n_matches = K;
      *R_ = r;
    }
    return;
  }
  // compact bearings of the match pairs (global scratch, L1/L2 resident), one
  // component per row of N (F1[k][j]): the scoring loops' loads are coalesced
  double* stash = F1 + 6 * N;  // Stewenius: the batch's action matrices and null spaces
  double* F2 = F1 + 3 * N;
  const int2* pl = pairs + (size_t)c * N;
  for (int j = lane; j < K; j += RS_BLOCK) {
    const int2 pr = pl[j];
    for (int k = 0; k < 3; ++k) {
      F1[(size_t)k * N + j] = bearings[((size_t)q * N + pr.x) * 3 + k];
      F2[(size_t)k * N + j] = bearings[((size_t)m * N + pr.y) * 3 + k];
    }
  }
  // pair j's error under the model (R, t)
  auto pair_error = [&](const double* R, const double* t, int j) {
    const double a[3] = {F1[j], F1[N + j], F1[2 * N + j]}, b[3] = {F2[j], F2[N + j], F2[2 * N + j]};
    return model_error(R, t, a, b);
  };
  for (int t = lane; t < 40; t += RS_BLOCK) (&w.t11[0][0][0])[t] = (&T11[0][0][0])[t];
  for (int t = lane; t < 120; t += RS_BLOCK) (&w.t21[0][0][0])[t] = (&T21[0][0][0])[t];
  __threadfence_block();
  wsync();
  int iterations = 0, skipped = 0, best_cnt = -INT_MAX, have = 0;
  double kk = 1.0;
  const int max_skip = P.max_iter * 10;
  const short* tab = P.tab_fixed ? table : table + (size_t)(K - 5) * P.pmax * 5;
  const bool prof = (c < 64) && P.prof == 1;
  bool done = !st2d;  // without the 2D-2D stage every pair is an inlier of the caller's pose
  // the serial loop's bookkeeping of one hypothesis's model (w.ok, w.mR, w.mt):
  // a failed solve counts as skipped; otherwise its inliers, the best model and
  // the adaptive iteration bound, and the iteration count
  auto account = [&](bool ok, const double* mR, const double* mt) {
    unsigned long long t_prev = prof ? wall_clock64() : 0;
    if (!ok) {
      ++skipped;
      wsync();
      return;
    }
    double Rm[9], tm[3];
    for (int i = 0; i < 9; ++i) Rm[i] = mR[i];
    for (int i = 0; i < 3; ++i) tm[i] = mt[i];
    int cnt = 0;
    for (int j0 = 0; j0 < K; j0 += RS_BLOCK) {
      const int j = j0 + lane;
      const bool in = (j < K) && pair_error(Rm, tm, j) < P.thr2d;
      cnt += __popcll(__ballot(in));
    }
    KMX_PT(6);
    if (cnt > best_cnt) {
      best_cnt = cnt;
      if (lane == 0) {
        for (int i = 0; i < 9; ++i) w.bestm[i] = Rm[i];
        for (int i = 0; i < 3; ++i) w.bestm[9 + i] = tm[i];
      }
      have = 1;
      const double wr = (double)cnt / (double)K;
      double p_no = 1.0 - pow(wr, 5.0);
      p_no = fmax(DBL_EPSILON, p_no);
      p_no = fmin(1.0 - DBL_EPSILON, p_no);
      kk = log(1.0 - P.prob) / log(p_no);
    }
    ++iterations;
    wsync();
    if (iterations > P.max_iter) done = true;
  };
  if (!st2d) {
  } else if constexpr (STEW) {
    // SG hypotheses' eigenvalues at a time, then each hypothesis in order under
    // the serial loop's tests (a batch may run past the stop: those are never
    // scored, so the results are the one-at-a-time loop's)
    int nb = SG;
    for (int p0 = 0; p0 < P.pmax && !done; p0 += nb) {
      if (!(iterations < kk && skipped < max_skip)) break;  // uniform
      // once a model exists, the serial loop scores at most ceil(kk) -
      // iterations more hypotheses (kk only falls), plus any that fail to give
      // a model (a later batch takes those): a batch no longer computes the
      // hypotheses past that bound (up to SG - 1 of them in a candidate's last
      // batch)
      int want = SG;
      if (have) {
        const double rem = ceil(kk) - (double)iterations;
        want = rem < 1.0 ? 1 : (rem < (double)SG ? (int)rem : SG);
      }
      nb = min(want, P.pmax - p0);
      stew_batch(w, sb, stash, lane, F1, F2, N, tab, p0, nb, prof);
      stew_models(sb, stash, lane, F1, F2, tab, p0, nb, prof);
      for (int b = 0; b < nb && !done; ++b) {
        if (!(iterations < kk && skipped < max_skip)) {
          done = true;
          break;
        }
        account(sb.mok[b] != 0, sb.mR[b], sb.mt[b]);
      }
    }
  } else {
    for (int p = 0; p < P.pmax && !done; ++p) {
      if (!(iterations < kk && skipped < max_skip)) break;  // uniform
      coop_hypothesis(w, lane, F1, F2, N, tab + (size_t)p * 5, prof);
      account(w.ok != 0, w.mR, w.mt);
    }
  }
  if (P.hyps && lane == 0) P.hyps[c] = iterations + skipped;
  ransac_tail<false>(c, w, F1, F2, points, N, q, m, pl, K, P, R_, mask, have, iterations, lane);
}



// k_ransac_coop: a work queue over the candidates. The launch holds as many
// one-wave workgroups as are resident at once; each wave takes the next
// candidate from a counter until none is left (every wave reaches the exit
// test). The candidates' costs differ by orders of magnitude (no RANSAC below
// 5 matches; ~30 hypotheses for a true loop closure; up to max_iter), so a
// static candidate -> workgroup map leaves slots idle: with the synthetic
// pools' alternating true / false pairs the statically dispatched form kept
// only half of the 12 waves per CU busy (profiles/r03/lcd/occupancy/). The
// scratch is per wave (blockIdx), reused from candidate to candidate.
template <int LB, bool STEW>
__global__ __launch_bounds__(RS_BLOCK, LB) void k_ransac_coop(const double* bearings, const double* points, int N,
                                                          const int* cq, const int* cm, const int2* pairs,
                                                          const int* Kin, const short* table, RsParams P,
                                                          kmx_lcd_result* res, unsigned char* masks,
                                                          double* fbuf, int n, int* next, const int* order) {
  __shared__ typename std::conditional<STEW, CoopWSS, CoopWS>::type w;
  __shared__ typename std::conditional<STEW, StewBatch, int>::type sb;  // Stewenius: the batch
  double* F1 = fbuf + (size_t)blockIdx.x * (6 * N + STASH);
  for (;;) {
    int c = 0;
    if (threadIdx.x == 0) c = atomicAdd(next, 1);
    c = __shfl(c, 0, 64);
    if (c >= n) break;
    if (order) c = order[c];  // the queue in the given order (longest first)
    ransac_candidate<STEW>(c, w, sb, F1, bearings, points, N, cq, cm, pairs, Kin, table, P, res, masks);
    __threadfence_block();
    wsync();
  }
}

// ------------------------------------------------- spread form (small calls) --
// A call of a few candidates (the reference's verification thread checks ONE
// candidate per call: verifyLoopSpin -> geometricVerificationNister,
// drawio:2638-2657) would leave one wave working through up to max_iter
// hypotheses while the rest of the device idles (a look-alike candidate that
// fails geometry runs all 500 iterations: ~20 ms on one wave against ~10 ms
// for one CPU thread). The hypotheses of one candidate do not depend on each
// other — each pass p takes its sample from the sampler table row and gives a
// model (or none) and that model's inlier count — only the serial loop's
// control does (the iteration bound kk from the best count so far, the skip
// count, the stop). So the spread form
//   1. computes a range of hypotheses of every candidate on many waves at once
//      (k_rs_hyps: SG per wave for Stewenius, as one batch of the work-queue
//      kernel; per hypothesis the same operations, so the same bits), scoring
//      each model over the candidate's pairs;
//   2. replays the serial loop's control over them in order (rs_replay_c, by the
//      range's last wave per candidate: the
//      `account` arithmetic of ransac_candidate, one thread per candidate),
//      stopping where the serial loop stops;
//   3. computes the next range only for candidates whose replay ran past the
//      computed ones (ranges grow: 66, then 444, then 1500 ... passes);
//   4. finishes each candidate from the replayed state (k_rs_finish: the best
//      model's inliers and the 3D-3D recovery, ransac_tail).
// Results are the serial loop's bit for bit (tests/test_lcd_spread_gpu.py);
// hypotheses past a candidate's stop inside a range are computed and never
// counted. Used by the synchronous calls for n <= spread_max candidates
// (KMX_LCD_SPREAD, default 8; 0 turns it off).
struct HypOut {
  double m[12];  // R (row-major), t
  int ok, cnt;   // a model was found; its inliers among the candidate's pairs
};
struct RsState {  // the serial loop's control between passes
  double kk;
  double best[12];
  int iterations, skipped, best_cnt, have, done, p_next;
};
constexpr int SPREAD_PER_NISTER = 2;  // Nister hypotheses per wave (one at a time)

// Candidate c's serial-loop state before its first range, and its wave
// arrival counter (k_rs_hyps: the last wave of a range replays it).
__device__ __forceinline__ void rs_init_c(RsState* st, unsigned* hcnt, int c, int stages) {
  RsState s;
  s.kk = 1.0;
  for (int i = 0; i < 12; ++i) s.best[i] = 0.0;
  s.iterations = s.skipped = s.have = s.p_next = 0;
  s.best_cnt = -INT_MAX;
  s.done = (stages & KMX_LCD_STAGE_2D2D) ? 0 : 1;
  st[c] = s;
  hcnt[c] = 0u;
}
__global__ void k_rs_init(RsState* st, unsigned* hcnt, int n, int stages, unsigned* more, int nmore) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nmore) more[c] = 0u;  // the ranges' flags (the replay)
  if (c < n) rs_init_c(st, hcnt, c, stages);
}

// The candidate's compact bearings (ransac_candidate's layout) and the LDS
// constant tables, by the calling wave.
template <typename WS>
__device__ __forceinline__ void rs_compact(WS& w, double* F1, const double* bearings, int N, int q, int m,
                                           const int2* pl, int K, int lane) {
  double* F2 = F1 + 3 * N;
  // four pairs per lane per pass, every load of the pass issued before its
  // stores (the stores may alias the bearings for the compiler, which then
  // kept one dependent pair -> bearing round trip per pair: ~7 us of a lone
  // wave's hypothesis at K = 350)
  constexpr int U = 4;
  for (int j0 = lane; j0 < K; j0 += U * RS_BLOCK) {
    int2 pr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) pr[u] = pl[min(j0 + u * RS_BLOCK, K - 1)];
    double a[U][3], b[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a[u][k] = bearings[((size_t)q * N + pr[u].x) * 3 + k];
        b[u][k] = bearings[((size_t)m * N + pr[u].y) * 3 + k];
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * RS_BLOCK;
      if (j < K)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          F1[(size_t)k * N + j] = a[u][k];
          F2[(size_t)k * N + j] = b[u][k];
        }
    }
  }
  for (int t = lane; t < 40; t += RS_BLOCK) (&w.t11[0][0][0])[t] = (&T11[0][0][0])[t];
  for (int t = lane; t < 120; t += RS_BLOCK) (&w.t21[0][0][0])[t] = (&T21[0][0][0])[t];
  __threadfence_block();
  wsync();
}

__device__ __forceinline__ void rs_replay_c(int c, int lane, const int* Kin, const RsParams& P, RsState* st,
                                            const HypOut* hout, int pb, unsigned* more);
// The last of a candidate's G waves to finish (hcnt: an agent-scope arrival
// counter, every wave's HypOut stores fenced before its arrival) replays the
// serial loop over the range at once: no k_rs_replay launch behind the range.
// Hypotheses [pa, pb) of every candidate still running: wave b works on
// candidate b / G, hypotheses pa + (b % G) * per ... (+ per).
template <bool STEW>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_hyps(const double* bearings, int N, const int* cq, const int* cm,
                                                      const int2* pairs, const int* Kin, const short* table,
                                                      RsParams P, RsState* st, HypOut* hout, int pa, int pb,
                                                      int G, int per, double* fbuf, unsigned* hcnt, unsigned* more) {
  __shared__ typename std::conditional<STEW, CoopWSS, CoopWS>::type w;
  __shared__ typename std::conditional<STEW, StewBatch, int>::type sb;
  const int c = blockIdx.x / G, g = blockIdx.x % G;
  const int lane = fresh_lane(threadIdx.x);
  [&]() {
  const int K = Kin[c];
  if (K < 5 || st[c].done) return;
  const int p_lo = pa + g * per, p_hi = min(min(p_lo + per, pb), P.pmax);
  if (p_lo >= p_hi) return;
  double* F1 = fbuf + (size_t)blockIdx.x * (6 * N + STASH);
  double* F2 = F1 + 3 * N;
  double* stash = F1 + 6 * N;
  // KMX_RS_PROF=1 (diagnostic): the solver's phase timers as in k_ransac_coop,
  // plus g_phase[11] the wave's whole time, [12] the compaction, [13] the
  // scoring, [15] waves (scripts/lcd_single.py)
  const bool prof = P.prof == 1;
  const unsigned long long t_wave = prof ? wall_clock64() : 0;
  unsigned long long t_prev = t_wave;
  rs_compact(w, F1, bearings, N, cq[c], cm[c], pairs + (size_t)c * N, K, lane);
  KMX_PT(12);
  const short* tab = table + (size_t)(K - 5) * P.pmax * 5;
  HypOut* ho = hout + (size_t)c * P.pmax;
  auto emit = [&](int p, bool ok, const double* mR, const double* mt) {
    int cnt = 0;
    if (ok) {
      double Rm[9], tm[3];
      for (int i = 0; i < 9; ++i) Rm[i] = mR[i];
      for (int i = 0; i < 3; ++i) tm[i] = mt[i];
      for (int j0 = 0; j0 < K; j0 += RS_BLOCK) {  // account()'s count, the same expression
        const int j = j0 + lane;
        bool in = false;
        if (j < K) {
          const double a[3] = {F1[j], F1[N + j], F1[2 * N + j]}, b[3] = {F2[j], F2[N + j], F2[2 * N + j]};
          in = model_error(Rm, tm, a, b) < P.thr2d;
        }
        cnt += __popcll(__ballot(in));
      }
      if (lane < 12) ho[p].m[lane] = lane < 9 ? Rm[lane] : tm[lane - 9];
    }
    if (lane == 0) {
      ho[p].ok = ok ? 1 : 0;
      ho[p].cnt = cnt;
    }
    wsync();
  };
  if constexpr (STEW) {
    const int nb = p_hi - p_lo;
    stew_batch<true>(w, sb, stash, lane, F1, F2, N, tab, p_lo, nb, prof);
    stew_models(sb, stash, lane, F1, F2, tab, p_lo, nb, prof);
    if (prof && lane == 0) t_prev = wall_clock64();
    for (int b = 0; b < nb; ++b) emit(p_lo + b, sb.mok[b] != 0, sb.mR[b], sb.mt[b]);
  } else {
    for (int p = p_lo; p < p_hi; ++p) {
      coop_hypothesis(w, lane, F1, F2, N, tab + (size_t)p * 5, prof);
      if (prof && lane == 0) t_prev = wall_clock64();
      emit(p, w.ok != 0, w.mR, w.mt);
    }
  }
  KMX_PT(13);
  if (prof && lane == 0) {
    atomicAdd(&g_phase[11], wall_clock64() - t_wave);
    atomicAdd(&g_phase[15], 1ull);
  }
  }();
  __threadfence();
  unsigned last = 0;
  if (lane == 0) last = atomicAdd(hcnt + c, 1u) == (unsigned)(G - 1);
  last = __shfl(last, 0, 64);
  if (!last) return;
  __threadfence();
  if (lane == 0) hcnt[c] = 0u;  // the next range's count starts at zero
  rs_replay_c(c, lane, Kin, P, st, hout, pb, more);
}

// The serial loop's control (ransac_candidate: the stop test, then account)
// over the computed hypotheses [p_next, pb), one wave per candidate: the
// lanes load 64 hypotheses' (ok, count) at once and every lane runs the
// control over them in order from readlane broadcasts (the same operations
// on the same values as one thread: the same state), so the serial chain has
// no dependent global load per hypothesis (one thread per candidate spent
// ~0.3 us per hypothesis waiting for it: 136 us for a 444-hypothesis range).
// The best model's 12 values are copied once, after the scan.
__device__ __forceinline__ void rs_replay_c(int c, int lane, const int* Kin, const RsParams& P, RsState* st,
                                            const HypOut* hout, int pb, unsigned* more) {
  RsState* sp = st + c;
  if (sp->done) return;
  const int K = Kin[c];
  if (K < 5) {
    if (lane == 0) sp->done = 1;
    return;
  }
  // the control state in scalars (wave-uniform)
  double kk = sp->kk;
  int iterations = sp->iterations, skipped = sp->skipped, best_cnt = sp->best_cnt, have = sp->have;
  int p_next = sp->p_next, done = 0;
  const int max_skip = P.max_iter * 10;
  const HypOut* ho = hout + (size_t)c * P.pmax;
  int bestp = -1;  // the hypothesis whose model becomes the best
  for (bool run = true; run;) {
    const int p0 = p_next, p = p0 + lane;
    int okl = 0, cntl = 0;
    if (p < pb && p < P.pmax) {
      okl = ho[p].ok;
      cntl = ho[p].cnt;
    }
    for (int jj = 0; jj < 64; ++jj) {
      if (p_next >= P.pmax || !(iterations < kk && skipped < max_skip)) {
        done = 1;
        run = false;
        break;
      }
      if (p_next >= pb) {  // past the computed hypotheses: the next pass
        run = false;
        break;
      }
      const int ok = __builtin_amdgcn_readlane(okl, jj), cnt = __builtin_amdgcn_readlane(cntl, jj);
      ++p_next;
      if (!ok) {
        ++skipped;
        continue;
      }
      if (cnt > best_cnt) {
        best_cnt = cnt;
        bestp = p0 + jj;
        have = 1;
        const double wr = (double)cnt / (double)K;
        double p_no = 1.0 - pow(wr, 5.0);
        p_no = fmax(DBL_EPSILON, p_no);
        p_no = fmin(1.0 - DBL_EPSILON, p_no);
        kk = log(1.0 - P.prob) / log(p_no);
      }
      ++iterations;
      if (iterations > P.max_iter) {
        done = 1;
        run = false;
        break;
      }
    }
  }
  if (lane < 12 && bestp >= 0) sp->best[lane] = ho[bestp].m[lane];
  if (lane == 0) {
    sp->kk = kk;
    sp->iterations = iterations;
    sp->skipped = skipped;
    sp->best_cnt = best_cnt;
    sp->have = have;
    sp->p_next = p_next;
    sp->done = done;
    if (!done) atomicOr(more, 1u);
  }
}

// Each candidate's result from its replayed loop: one workgroup of RS_FIN
// waves per candidate. Wave 0 runs ransac_tail<true>; the 1-point
// recovery's largest consistent set — n3^2 distance tests over the 2D-2D
// inliers, the tail's longest loop on a lone wave — is counted by every wave:
// wave v takes the 64 inliers i of block v % n_ib against the j of range
// v / n_ib, adds its integer counts into LDS (any order: the same counts), and
// wave 0 then takes the first maximum over the valid i (the serial loop's
// pick). Waves 1.. wait at the first barrier and leave when wave 0 reached no
// count (`fin_go` < 0: no model, too few inliers, no recovery stage, PnP).
// `skip` (the speculative finish of a spread call): the range's `more` word;
// set, the candidates are not done and the workgroup leaves at once.
constexpr int RS_FIN = 8;
__device__ __forceinline__ void fin_count(const double* Tl, const unsigned char* vl, int n3, double thr2, int* cnt,
                                          int wave, int lane) {
  const int n_ib = (n3 + RS_BLOCK - 1) / RS_BLOCK;
  if (n_ib == 0) return;
  const int n_jc = max(1, RS_FIN / n_ib);
  const int ib = wave % n_ib, jc = wave / n_ib;
  if (jc >= n_jc) return;
  const int n3p = (n3 + 3) & ~3;  // entries n3 .. n3 + 3 are invalid padding
  const int jlen = (((n3p + n_jc - 1) / n_jc) + 3) & ~3;
  const int j0 = jc * jlen, j1 = min(n3p, j0 + jlen);
  const int i = ib * RS_BLOCK + lane;
  double ti[3] = {0.0, 0.0, 0.0};
  if (i < n3)
    for (int k = 0; k < 3; ++k) ti[k] = Tl[3 * i + k];
  int c4[4] = {0, 0, 0, 0};
  for (int j = j0; j < j1; j += 4) {
    const unsigned v4 = *reinterpret_cast<const unsigned*>(vl + j);
    // branch-free (a valid-byte test as a branch serialised the four chains)
    double d2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double* t = Tl + 3 * (j + u);
      const double dx = t[0] - ti[0], dy = t[1] - ti[1], dz = t[2] - ti[2];
      d2[u] = dx * dx + dy * dy + dz * dz;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) c4[u] += (int)((v4 >> (8 * u)) & 1u) & (d2[u] < thr2 ? 1 : 0);
  }
  if (i < n3 && j0 < j1) atomicAdd(cnt + i, (c4[0] + c4[1]) + (c4[2] + c4[3]));
}
__global__ __launch_bounds__(RS_BLOCK * RS_FIN) void k_rs_finish(const double* bearings, const double* points, int N,
                                                                 const int* cq, const int* cm, const int2* pairs,
                                                                 const int* Kin, RsParams P, const RsState* st,
                                                                 kmx_lcd_result* res, unsigned char* masks,
                                                                 double* fbuf, const unsigned* skip,
                                                                 unsigned* skip_host, unsigned* done, unsigned seq) {
  __shared__ CoopWS w;
  __shared__ int fin_go;
  __shared__ int cnt[MAX_FEATS];
  extern __shared__ double tail_lds[];  // tail_lds_doubles(N)
  if (skip) {
    const unsigned sk = *skip;
    // the word the host reads after the call (coherent host memory: no copy)
    if (skip_host && blockIdx.x == 0 && threadIdx.x == 0) *skip_host = sk;
    if (sk) {  // (uniform over the launch)
      if (done && threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
  }
  const int wave = threadIdx.x / RS_BLOCK;
  const int lane = fresh_lane(threadIdx.x % RS_BLOCK);
  if (wave > 0) {
    __syncthreads();  // A: wave 0 staged T (fin_go = n3) or reached no count (-1)
    const int n3 = fin_go;
    if (n3 < 0) return;
    const double* Tl = tail_lds;
    const unsigned char* vl = reinterpret_cast<const unsigned char*>(tail_lds + 3 * ((size_t)N + 4));
    fin_count(Tl, vl, n3, P.thr3d * P.thr3d, cnt, wave, lane);
    __syncthreads();  // B
    return;
  }
  bool met = false;
  auto count_best = [&](const double* Tl, const unsigned char* vl, int n3, double thr2) -> int {
    met = true;
    for (int k = lane; k < n3; k += RS_BLOCK) cnt[k] = 0;
    if (lane == 0) fin_go = n3;
    __syncthreads();  // A
    fin_count(Tl, vl, n3, thr2, cnt, 0, lane);
    __syncthreads();  // B
    int my_best = -1, my_cnt = 0;
    for (int i = lane; i < n3; i += RS_BLOCK) {
      const int cc = cnt[i];
      if (vl[i] && cc > my_cnt) { my_cnt = cc; my_best = i; }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const int oc = __shfl_xor(my_cnt, off, 64);
      const int ob = __shfl_xor(my_best, off, 64);
      if (oc > my_cnt || (oc == my_cnt && ob >= 0 && (my_best < 0 || ob < my_best))) {
        my_cnt = oc;
        my_best = ob;
      }
    }
    return my_best;
  };
  [&]() {
    const int c = blockIdx.x;
    const int K = Kin[c];
    const int q = cq[c], m = cm[c];
    unsigned char* mask = masks ? masks + (size_t)c * N : nullptr;
    kmx_lcd_result* R_ = res + c;
    for (int j = lane; j < N && mask; j += RS_BLOCK) mask[j] = 0;
    const bool st2d = (P.stages & KMX_LCD_STAGE_2D2D) != 0;
    if (K < 5 && st2d) {
      if (lane == 0) {
        kmx_lcd_result r = {};
        r.n_matches = K;
        *R_ = r;
      }
      return;
    }
    double* F1 = fbuf + (size_t)blockIdx.x * (6 * N + STASH);
    const int2* pl = pairs + (size_t)c * N;
    rs_compact(w, F1, bearings, N, q, m, pl, K, lane);
    const RsState s = st[c];
    if (lane < 12) w.bestm[lane] = s.best[lane];
    __threadfence_block();
    wsync();
    ransac_tail<true>(c, w, F1, F1 + 3 * N, points, N, q, m, pl, K, P, R_, mask, s.have, s.iterations, lane, tail_lds,
                      count_best);
  }();
  if (!met) {
    if (lane == 0) fin_go = -1;
    __syncthreads();  // A for the waves that wait to count
  }
  // a one-candidate call's completion word (wait_done): wave 0 wrote the
  // result and the mask; its stores are complete before lane 0's release
  if (done) {
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Arun 3-point model (oracle arun_model): centroids, H = sum dm dq^T, Kabsch
// with svd3, t = c_q - R c_m (p_q = R p_m + t).
__device__ void arun_model(const double* sq, const double* sm, double R[9], double t[3]) {
  double cq[3] = {0.0, 0.0, 0.0}, cm[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < 3; ++i)
    for (int c = 0; c < 3; ++c) {
      cq[c] += sq[3 * i + c];
      cm[c] += sm[3 * i + c];
    }
  for (int c = 0; c < 3; ++c) {
    cq[c] /= 3.0;
    cm[c] /= 3.0;
  }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    double dq[3], dm[3];
    for (int c = 0; c < 3; ++c) {
      dq[c] = sq[3 * i + c] - cq[c];
      dm[c] = sm[3 * i + c] - cm[c];
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
__device__ double arun_error(const double R[9], const double t[3], const double pq[3], const double pm[3]) {
  double d[3];
  for (int a = 0; a < 3; ++a) d[a] = pq[a] - (R[a * 3 + 0] * pm[0] + R[a * 3 + 1] * pm[1] + R[a * 3 + 2] * pm[2] + t[a]);
  return sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
}

// Pose recovery after the 2D-2D RANSAC, on its inliers whose stereo points
// are valid (pair-list order), one wavefront per candidate, one hypothesis
// per lane, the serial control replayed by lane 0 exactly as in k_ransac:
//   PNP:  pose_recovery_type 1, opengv AbsolutePoseSacProblem with EPnP
//         (sample 6): query bearings (A) against match-frame points (B);
//   !PNP: ransac_use_1point_3d3d 0, PointCloudSacProblem with Arun
//         (sample 3): query points (A) against match points (B).
template <bool PNP>
__global__ __launch_bounds__(RS_BLOCK) void k_recover(const double* bearings, const double* points, int N,
                                                      const int* cq, const int* cm, const int2* pairs, const int* Kin,
                                                      const short* table, PnpParams P, kmx_lcd_result* res,
                                                      unsigned char* masks) {
  constexpr int S = PNP ? PNP_S : 3;
  extern __shared__ __attribute__((aligned(16))) double sm_d[];
  const int c = xcd_candidate(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  kmx_lcd_result* R_ = res + c;
  if (R_->mono_inliers < P.min2d) {
    if (P.hyps && lane == 0) P.hyps[c] = 0;
    return;
  }
  const int K = Kin[c];
  const int q = cq[c], m = cm[c];
  double* Aq = sm_d;                  // [n2][3]
  double* Bm = Aq + 3 * N;            // [n2][3]
  double* models = Bm + 3 * N;        // [64][12]
  double* bestm = models + 64 * 12;   // [12]
  int* okc = reinterpret_cast<int*>(bestm + 12);
  int* cnt = okc + 64;
  int* ctrl = cnt + 64;               // [4]
  int* id2 = ctrl + 4;                // [n2]
  unsigned char* mask = masks + (size_t)c * N;
  const int2* pl = pairs + (size_t)c * N;
  if (lane == 0) {
    int n2 = 0;
    for (int j = 0; j < K; ++j) {
      if (!(mask[j] & 1)) continue;
      const int2 pr = pl[j];
      const double* a = points + ((size_t)q * N + pr.x) * 3;
      const double* b = points + ((size_t)m * N + pr.y) * 3;
      if (isnan(a[0]) || isnan(a[1]) || isnan(a[2]) || isnan(b[0]) || isnan(b[1]) || isnan(b[2])) continue;
      const double* av = PNP ? bearings + ((size_t)q * N + pr.x) * 3 : a;
      for (int k = 0; k < 3; ++k) {
        Aq[3 * n2 + k] = av[k];
        Bm[3 * n2 + k] = b[k];
      }
      id2[n2++] = j;
    }
    ctrl[3] = n2;
    ctrl[1] = 0;
  }
  __syncthreads();
  const int n2 = ctrl[3];
  auto err = [&](const double R[9], const double t[3], int j) {
    return PNP ? pnp_error(R, t, Bm + 3 * j, Aq + 3 * j) : arun_error(R, t, Aq + 3 * j, Bm + 3 * j);
  };
  int iterations = 0, skipped = 0, best_cnt = -INT_MAX, have = 0;
  double kk = 1.0;
  const int max_skip = P.max_iter * 10;
  if (n2 >= S) {
    const short* tab = P.tab_fixed ? table : table + (size_t)(n2 - S) * P.pmax * S;
    for (int base = 0;; base += RS_BLOCK) {
      const int p = base + lane;
      int ok = 0, count = 0;
      double Rm[9], tm[3];
      if (p < P.pmax) {
        double sa[3 * S], sb[3 * S];
        for (int i = 0; i < S; ++i) {
          const int id = tab[(size_t)p * S + i];
          for (int k = 0; k < 3; ++k) {
            sa[3 * i + k] = Aq[3 * id + k];
            sb[3 * i + k] = Bm[3 * id + k];
          }
        }
        if (PNP) {
          ok = epnp6(sb, sa, Rm, tm);
        } else {
          arun_model(sa, sb, Rm, tm);
          ok = 1;
        }
        if (ok)
          for (int j = 0; j < n2; ++j)
            if (err(Rm, tm, j) < P.thr) ++count;
      }
      okc[lane] = ok;
      cnt[lane] = count;
      if (ok) {
        for (int i = 0; i < 9; ++i) models[lane * 12 + i] = Rm[i];
        for (int i = 0; i < 3; ++i) models[lane * 12 + 9 + i] = tm[i];
      }
      __syncthreads();
      if (lane == 0) {
        int done = 0;
        for (int l = 0; l < RS_BLOCK; ++l) {
          if (!(iterations < kk && skipped < max_skip) || base + l >= P.pmax) { done = 1; break; }
          if (!okc[l]) { ++skipped; continue; }
          if (cnt[l] > best_cnt) {
            best_cnt = cnt[l];
            for (int i = 0; i < 12; ++i) bestm[i] = models[l * 12 + i];
            have = 1;
            const double w = (double)cnt[l] / (double)n2;
            double p_no = 1.0 - pow(w, (double)S);
            p_no = fmax(DBL_EPSILON, p_no);
            p_no = fmin(1.0 - DBL_EPSILON, p_no);
            kk = log(1.0 - P.prob) / log(p_no);
          }
          ++iterations;
          if (iterations > P.max_iter) { done = 1; break; }
        }
        if (!done && base + RS_BLOCK >= P.pmax) done = 1;
        ctrl[0] = done;
        ctrl[1] = have;
      }
      __syncthreads();
      if (ctrl[0]) break;
    }
  }
  __syncthreads();
  if (P.hyps && lane == 0) P.hyps[c] = iterations + skipped;
  const int have_model = ctrl[1];
  int np = 0;
  double Ro[9], to[3];
  if (have_model) {
    for (int i = 0; i < 9; ++i) Ro[i] = bestm[i];
    for (int i = 0; i < 3; ++i) to[i] = bestm[9 + i];
    for (int j0 = 0; j0 < n2; j0 += RS_BLOCK) {
      const int j = j0 + lane;
      const bool in = (j < n2) && err(Ro, to, j) < P.thr;
      if (in) mask[id2[j]] |= 2;
      np += __popcll(__ballot(in));
    }
  }
  if (lane == 0) {
    kmx_lcd_result r = *R_;
    if (PNP) {
      r.pnp_inliers = np;
      if (have_model) {  // camera pose in the match frame -> T_query_match
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) r.T_query_match[a * 3 + b] = Ro[b * 3 + a];
        for (int a = 0; a < 3; ++a)
          r.T_query_match[9 + a] = -(Ro[0 * 3 + a] * to[0] + Ro[1 * 3 + a] * to[1] + Ro[2 * 3 + a] * to[2]);
      }
      r.accepted = (have_model && np >= P.min_pnp) ? 1 : 0;
    } else {
      r.stereo_inliers = np;
      if (have_model) {
        for (int i = 0; i < 9; ++i) r.T_query_match[i] = Ro[i];
        for (int i = 0; i < 3; ++i) r.T_query_match[9 + i] = to[i];
      }
      r.accepted = (have_model && np >= P.min_pnp) ? 1 : 0;
      if (r.accepted && P.refine)
        refit_3d3d(
            n2,
            [&](int j, double* pq, double* pm) {
              if (!(err(Ro, to, j) < P.thr)) return false;
              for (int k = 0; k < 3; ++k) { pq[k] = Aq[3 * j + k]; pm[k] = Bm[3 * j + k]; }
              return true;
            },
            r.T_query_match, r.T_query_match + 9);
    }
    *R_ = r;
  }
}

}  // namespace

// ============================================================== handle ====
struct kmx_lcd {
  kmx_lcd_params P{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // frame pool: F resident frames of N feature slots, device capacity capF frames
  int F = 0, N = 0, capF = 0;
  std::vector<int> h_nfeat;  // host copy of the feature counts (argument checks)
  uint32_t* d_desc = nullptr;
  double* d_bear = nullptr;
  double* d_pts = nullptr;
  int* d_nfeat = nullptr;
  // sampler tables, built for rows K in [S, table_N] (they depend only on the
  // parameters and N, so frames can be added without rebuilding them)
  short* d_table = nullptr;
  short* d_table_rec = nullptr;  // samples of the recovery RANSAC (6: PnP, 3: Arun), built when used
  int table_N = 0;
  int pmax = 0;
  // candidate buffers: LCD_SLOTS slots, used by successive calls in turn, so
  // a call's kNN2 (on kstream) can run while earlier calls' RANSACs drain;
  // d_cq .. d_order below point into the current slot
  int cap = 0, cur = 0;  // cap: the current slot's capacity
  // Each slot's RANSAC can run on its own stream (slot 0: the handle's
  // stream, slot s > 0: rsx[s]) with its own work-queue counter and per-wave
  // scratch, so the next calls' RANSACs take the CUs the previous call's
  // drain (its last candidates, finishing alone) leaves idle.
  struct Slot {
    int *cq = nullptr, *cm = nullptr, *K = nullptr, *hyps = nullptr, *nrec = nullptr, *order = nullptr;
    int2* pairs = nullptr;
    kmx_lcd_result* res = nullptr;
    unsigned char* mask = nullptr;
    double* prior = nullptr;
    double* fbuf = nullptr;
    int* next = nullptr;
    int cap = 0;  // candidates the slot's buffers hold (0: not allocated yet)
  } slot[LCD_SLOTS];
  hipStream_t rsx[LCD_SLOTS] = {};  // rsx[s]: slot s's RANSAC stream (s > 0)
  bool rs_conc = true;              // KMX_LCD_RSX=0: every slot on the handle's stream (A/B switch)
  bool rs_small = false;            // this call runs its slots' RANSACs concurrently (the size cut)
  bool rs_on = false;               // this call's slot runs on rsx[cur]
  int cus = 0;
  hipStream_t kstream = nullptr;  // kNN2 of kmx_lcd_verify / _async
  hipEvent_t ev_knn[LCD_SLOTS] = {}, ev_rs[LCD_SLOTS] = {};
  bool ev_rs_set[LCD_SLOTS] = {};
  int *d_cq = nullptr, *d_cm = nullptr, *d_K = nullptr;
  int2* d_pairs = nullptr;
  kmx_lcd_result* d_res = nullptr;
  unsigned char* d_mask = nullptr;
  double* d_fbuf = nullptr;  // [slots][6 N + STASH] compact match bearings + Stewenius stash, per k_ransac_coop wave
  int* d_next = nullptr;     // k_ransac_coop's work-queue counter
  double* d_prior = nullptr;  // the current slot's T_prior rows (kmx_lcd_verify_matches)
  // ordered sampler (rng_stream 1): the verification thread's engine, one
  // candidate's sample row, the passes each problem drew, recovery sizes
  std::mt19937 stream_rng;
  short* d_row = nullptr;
  int *d_hyps = nullptr, *d_nrec = nullptr;
  int* d_order = nullptr;  // k_order's queue order (KMX_LCD_ORDER)
  // spread form (synchronous calls of <= spread_max candidates; lcd.hip k_rs_*)
  int spread_max = 8;
  int spread_cap = 0;
  RsState* d_st = nullptr;
  HypOut* d_hout = nullptr;
  double* d_sfbuf = nullptr;
  unsigned* d_more = nullptr;  // [more_cap] one word per range: some candidate needs the next range
  unsigned* d_hcnt = nullptr;  // [spread_cap] k_rs_hyps' wave arrivals per candidate (zero between ranges)
  int more_cap = 0;
  unsigned* h_more = nullptr;  // pinned copy of the word just read
  unsigned* z_more = nullptr;  // its device pointer (looked up once)
  // a one-candidate call's completion word (mapped; wait_done) and its sequence
  unsigned* h_done = nullptr;
  unsigned* z_done = nullptr;
  unsigned done_seq = 0;
  bool spin_wait = true;  // KMX_LCD_SPINWAIT=0: hipStreamSynchronize instead
  // k_knn2s (synchronous calls of <= KS_MAX candidates): per-query results and
  // the per-candidate arrival counters (zero between calls; KMX_LCD_KSPLIT=0: off)
  bool knn_split = true;
  // k_knn2q (4 queries per thread) for the Hamming matcher at N <= 512
  // (configs[2], same box: 6.72 vs 7.01 ms per 50k kNN2, 1.442e6 vs 1.416e6
  // candidates/s); the L1 matcher stays on k_knn2 (4.33 vs 4.16 ms: the
  // two-wave candidates run five waves per SIMD instead of eight, and the
  // v_sad_u8 chains need them). KMX_LCD_KNNQ=0: k_knn2 for both.
  bool knn_q = true;
  int* d_kqb = nullptr;
  unsigned* d_kcnt = nullptr;
  int kqb_N = 0;
  // pinned staging of the synchronous one-candidate calls (kmx_lcd_match,
  // kmx_lcd_verify_matches): every input in one host-to-device copy, every
  // output through pinned memory (a pageable copy is a blocking staged copy
  // each; the call-for-call chain made five to seven of them per call)
  size_t io_cap = 0;
  // small frame uploads (add_frames: one keyframe per call) are staged here
  // (pinned, mapped) and scattered into the pool by one kernel that reads the
  // mapped pages, instead of four pageable copies
  char* h_fst = nullptr;
  char* z_fst = nullptr;
  size_t fst_cap = 0;
  char* h_io = nullptr;  // pinned host, coherent and mapped
  char* z_io = nullptr;  // h_io's device pointer: the small synchronous calls' kernels read their
                         // inputs and write their outputs there (zero-copy: no blit per copy)
  char* d_io = nullptr;
  int prof = 0;              // KMX_RS_PROF: phase timers in k_ransac_coop
  // kmx_lcd_enable_timing: events around the kNN2 and the RANSAC launches
  bool timing = false;
  bool ev_ok = false;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
};

namespace {

void sync_rsx(kmx_lcd* h) {
  for (hipStream_t x : h->rsx)
    if (x) (void)hipStreamSynchronize(x);
}
void lcd_free_frames(kmx_lcd* h) {
  if (h->stream) (void)hipStreamSynchronize(h->stream);  // a verification in flight may read the pool
  sync_rsx(h);
  if (h->kstream) (void)hipStreamSynchronize(h->kstream);
  void* p[] = {h->d_desc, h->d_bear, h->d_pts, h->d_nfeat};
  for (void* x : p)
    if (x) (void)hipFree(x);
  h->d_desc = nullptr; h->d_bear = h->d_pts = nullptr; h->d_nfeat = nullptr;
  h->F = h->capF = 0;
  h->h_nfeat.clear();
}
void lcd_free_tables(kmx_lcd* h) {
  if (h->d_table) (void)hipFree(h->d_table);
  if (h->d_table_rec) (void)hipFree(h->d_table_rec);
  h->d_table = h->d_table_rec = nullptr;
  h->table_N = 0;
}
void lcd_free_cand(kmx_lcd* h) {
  if (h->stream) (void)hipStreamSynchronize(h->stream);  // in-flight calls may still use the buffers
  sync_rsx(h);
  if (h->kstream) (void)hipStreamSynchronize(h->kstream);
  for (auto& sl : h->slot) {
    void* p[] = {sl.cq, sl.cm, sl.K, sl.hyps, sl.nrec, sl.order, sl.pairs, sl.res, sl.mask, sl.prior, sl.fbuf, sl.next};
    for (void* x : p)
      if (x) (void)hipFree(x);
    sl = kmx_lcd::Slot{};
  }
  h->d_cq = h->d_cm = h->d_K = nullptr; h->d_pairs = nullptr; h->d_res = nullptr; h->d_mask = nullptr;
  h->d_fbuf = nullptr;
  h->d_next = h->d_hyps = h->d_nrec = nullptr;
  h->d_prior = nullptr;
  h->d_order = nullptr;
  for (bool& e : h->ev_rs_set) e = false;
  h->cap = 0;
  void* q[] = {h->d_st, h->d_hout, h->d_sfbuf, h->d_more, h->d_kqb, h->d_kcnt, h->d_hcnt};
  for (void* x : q)
    if (x) (void)hipFree(x);
  if (h->h_more) (void)hipHostFree(h->h_more);
  h->d_st = nullptr; h->d_hout = nullptr; h->d_sfbuf = nullptr; h->d_more = nullptr; h->h_more = nullptr; h->z_more = nullptr;
  h->d_kqb = nullptr; h->d_kcnt = nullptr; h->kqb_N = 0; h->d_hcnt = nullptr;
  h->spread_cap = 0;
  h->more_cap = 0;
}
// Pinned host + device staging of at least `bytes` (grow-only; the callers
// are synchronous, so the previous call's copies have completed).
int io_reserve(kmx_lcd* h, size_t bytes) {
  if (bytes <= h->io_cap) return 0;
  if (h->stream) KMX_HIP(hipStreamSynchronize(h->stream));
  sync_rsx(h);
  if (h->h_io) (void)hipHostFree(h->h_io);
  if (h->d_io) (void)hipFree(h->d_io);
  h->h_io = nullptr; h->d_io = nullptr; h->z_io = nullptr;
  h->io_cap = 0;
  const size_t cap = std::max<size_t>(bytes, 256 * 1024);
  KMX_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_io), cap, hipHostMallocMapped | hipHostMallocCoherent));
  KMX_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->z_io), h->h_io, 0));
  KMX_HIP(hipMalloc(reinterpret_cast<void**>(&h->d_io), cap));
  h->io_cap = cap;
  return 0;
}
// One-candidate calls (the reference's verifyLoopSpin pattern) end in a kernel
// that stores a fresh sequence number to a mapped word after its outputs
// (system-scope release): spinning on that word returns ~6 us sooner than
// hipStreamSynchronize, which also waits for the dispatch's end-of-kernel
// signal (scripts/probe/sync_latency.hip: 30.5 vs 36.2 us around a 25-us
// kernel). next_done gives the word and the sequence (nullptr: not used).
unsigned* next_done(kmx_lcd* h, unsigned* seq) {
  if (!h->spin_wait) return nullptr;
  if (!h->h_done) {
    if (hipHostMalloc(reinterpret_cast<void**>(&h->h_done), 64, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&h->z_done), h->h_done, 0) != hipSuccess) {
      if (h->h_done) (void)hipHostFree(h->h_done);
      h->h_done = h->z_done = nullptr;
      h->spin_wait = false;
      return nullptr;
    }
    __atomic_store_n(h->h_done, 0u, __ATOMIC_RELEASE);
  }
  *seq = ++h->done_seq == 0 ? ++h->done_seq : h->done_seq;  // never 0
  return h->z_done;
}
// Wait for `seq` in the completion word; past 2 s of spinning, synchronise
// the stream (a faulted or hung kernel surfaces there) and require the word.
int wait_done(kmx_lcd* h, hipStream_t st, unsigned seq) {
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) != seq) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      KMX_HIP(hipStreamSynchronize(st));
      KMX_CHECK(__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) == seq, KMX_EHIP,
                "a one-candidate call's kernel finished without its completion word");
      return 0;
    }
  }
  return 0;
}
inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
// The next call's slot: its buffers become d_cq .. d_order.
void use_next_slot(kmx_lcd* h) {
  h->cur = (h->cur + 1) % LCD_SLOTS;
  const kmx_lcd::Slot& sl = h->slot[h->cur];
  h->d_cq = sl.cq; h->d_cm = sl.cm; h->d_K = sl.K; h->d_hyps = sl.hyps; h->d_nrec = sl.nrec; h->d_order = sl.order;
  h->d_pairs = sl.pairs; h->d_res = sl.res; h->d_mask = sl.mask; h->d_prior = sl.prior;
  h->d_fbuf = sl.fbuf; h->d_next = sl.next;
  h->cap = sl.cap;
}
// The current slot's RANSAC stream: everything a call does on its slot's
// buffers after the kNN2 runs there.
// Slots s > 0 go on rsx[s] for calls of fewer than 96 candidates per CU (8
// per resident RANSAC wave): there the previous call's drain is a large part
// of a call and the kNN2 alone does not fill it (2k candidates, two slots:
// 6.5 -> 3.8 ms per back-to-back call, 20k: 16.9 -> 15.1 ms); at configs[2]'s
// 50k the kNN2 already fills it and the overlap cost 1.6 %
// (profiles/r04/lcd/two_stream). A larger call's kNN2 also waits for the
// RANSAC two calls back, as with two slots: run further ahead, the kNN2s took
// CUs from the RANSAC (four slots without it: 50k steps up to 3 % slower).
hipStream_t rs_stream(const kmx_lcd* h) { return h->rs_on ? h->rsx[h->cur] : h->stream; }
// The current slot's last work may be on another stream (the choice is per
// call): calls that write the slot's buffers from rs_stream wait for it.
int rs_wait_slot(kmx_lcd* h) {
  if (h->ev_rs_set[h->cur]) KMX_HIP(hipStreamWaitEvent(rs_stream(h), h->ev_rs[h->cur], 0));
  return 0;
}
void lcd_free_pairs(kmx_lcd* h) {
  void* p[] = {h->d_row};
  for (void* x : p)
    if (x) (void)hipFree(x);
  h->d_row = nullptr;
  if (h->h_io) (void)hipHostFree(h->h_io);
  if (h->d_io) (void)hipFree(h->d_io);
  h->h_io = nullptr; h->d_io = nullptr; h->z_io = nullptr;
  h->io_cap = 0;
  if (h->h_fst) (void)hipHostFree(h->h_fst);
  h->h_fst = h->z_fst = nullptr;
  h->fst_cap = 0;
  if (h->h_done) (void)hipHostFree(h->h_done);
  h->h_done = h->z_done = nullptr;
}

// One pass of opengv's drawIndexSample: S swaps of the persistent shuffle over
// the problem's K indices, each by std::uniform_int_distribution<int>(0,
// INT_MAX) over std::mt19937 (GCC-9 rejection or GCC-11 x >> 1).
inline int sampler_draw(std::mt19937& rng, int variant) {
  uint32_t x;
  if (variant == KMX_RNG_GCC11) {
    x = (uint32_t)rng() >> 1;
  } else {
    do x = (uint32_t)rng();
    while (x >= 0x80000000u);
  }
  return (int)x;
}
void sample_row(std::mt19937& rng, int variant, int K, int pmax, int S, short* out) {
  std::vector<int> sh(K);
  for (int i = 0; i < K; ++i) sh[i] = i;
  for (int p = 0; p < pmax; ++p) {
    for (int i = 0; i < S; ++i) {
      const int j = i + (int)((size_t)sampler_draw(rng, variant) % (size_t)(K - i));
      std::swap(sh[i], sh[j]);
    }
    for (int i = 0; i < S; ++i) out[(size_t)p * S + i] = (short)sh[i];
  }
}

// opengv sampler table: for every K in [S, N], the S indices drawn by each of
// the first pmax passes (std::mt19937 seeded per problem). Rows are
// independent, so they are built on a few host threads.
void build_table(const kmx_lcd_params& P, int N, int pmax, std::vector<short>& tab, int S = 5) {
  const int rows = std::max(N - S + 1, 1);
  tab.assign((size_t)rows * pmax * S, 0);
  const int nt = std::max(1, std::min(8, rows / 32));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int K = S + t; K <= N; K += nt) {
        std::mt19937 rng(P.ransac_seed);
        sample_row(rng, P.rng_variant, K, pmax, S, tab.data() + (size_t)(K - S) * pmax * S);
      }
    });
  for (auto& x : th) x.join();
}

bool rec_sampled(const kmx_lcd_params& P) { return P.pose_recovery_type == 1 || !P.use_1point_3d3d; }
int rec_S(const kmx_lcd_params& P) { return P.pose_recovery_type == 1 ? PNP_S : 3; }

// Sampler tables for the pool's N (kept across set_frames / add_frames with the
// same N). The ordered sampler draws its rows per candidate instead.
int ensure_tables(kmx_lcd* h) {
  // every pass the serial loop can reach: (max_iter + 1) iterations + 10 * max_iter skips
  h->pmax = h->P.ransac_max_iterations + 1 + 10 * h->P.ransac_max_iterations;
  if (h->P.rng_stream) {
    if (!h->d_row) KMX_HIP(hipMalloc(&h->d_row, sizeof(short) * (size_t)h->pmax * PNP_S));
    return 0;
  }
  if (h->table_N == h->N && h->d_table) return 0;
  lcd_free_tables(h);
  std::vector<short> tab;
  build_table(h->P, h->N, h->pmax, tab);
  KMX_HIP(hipMalloc(&h->d_table, sizeof(short) * tab.size()));
  KMX_HIP(hipMemcpy(h->d_table, tab.data(), sizeof(short) * tab.size(), hipMemcpyHostToDevice));
  if (rec_sampled(h->P)) {
    build_table(h->P, h->N, h->pmax, tab, rec_S(h->P));
    KMX_HIP(hipMalloc(&h->d_table_rec, sizeof(short) * tab.size()));
    KMX_HIP(hipMemcpy(h->d_table_rec, tab.data(), sizeof(short) * tab.size(), hipMemcpyHostToDevice));
  }
  h->table_N = h->N;
  return 0;
}

// True while an earlier call may still run on some slot (an async call's
// RANSAC or kNN2 not yet complete).
bool slots_busy(kmx_lcd* h) {
  for (int s = 0; s < LCD_SLOTS; ++s)
    if (h->ev_rs_set[s] && hipEventQuery(h->ev_rs[s]) != hipSuccess) return true;
  return h->kstream && hipStreamQuery(h->kstream) != hipSuccess;
}
// The call's slot, with buffers for n candidates. Slots are allocated (and
// grown) one at a time, when a call first lands on them: a synchronous call
// with nothing in flight takes slot 0, so callers that never overlap calls
// hold one slot's buffers, not LCD_SLOTS; async calls rotate through all.
int ensure_cap(kmx_lcd* h, int n, bool async) {
  if (!async && !slots_busy(h)) h->cur = LCD_SLOTS - 1;  // use_next_slot -> slot 0
  use_next_slot(h);
  kmx_lcd::Slot& sl = h->slot[h->cur];
  if (n > sl.cap) {
    // the slot's last call may still be in flight on any stream
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    sync_rsx(h);
    if (h->kstream) (void)hipStreamSynchronize(h->kstream);
    void* p[] = {sl.cq, sl.cm, sl.K, sl.hyps, sl.nrec, sl.order, sl.pairs, sl.res, sl.mask, sl.prior, sl.fbuf, sl.next};
    for (void* x : p)
      if (x) (void)hipFree(x);
    sl = kmx_lcd::Slot{};
    h->ev_rs_set[h->cur] = false;
    const int cap = std::max(n, 1024);
    bool ok =
           hipMalloc(&sl.fbuf, sizeof(double) * (6 * (size_t)h->N + STASH) * std::min(cap, RS_MAX_SLOTS)) ==
               hipSuccess &&
           hipMalloc(&sl.next, sizeof(int)) == hipSuccess &&
           hipMalloc(&sl.cq, sizeof(int) * cap) == hipSuccess && hipMalloc(&sl.cm, sizeof(int) * cap) == hipSuccess &&
           hipMalloc(&sl.K, sizeof(int) * cap) == hipSuccess &&
           hipMalloc(&sl.pairs, sizeof(int2) * (size_t)cap * h->N) == hipSuccess &&
           hipMalloc(&sl.res, sizeof(kmx_lcd_result) * cap) == hipSuccess &&
           hipMalloc(&sl.mask, (size_t)cap * h->N) == hipSuccess && hipMalloc(&sl.hyps, sizeof(int) * cap) == hipSuccess &&
           hipMalloc(&sl.nrec, sizeof(int) * cap) == hipSuccess &&
           hipMalloc(&sl.prior, sizeof(double) * 12 * (size_t)cap) == hipSuccess &&
           hipMalloc(&sl.order, sizeof(int) * cap) == hipSuccess;
    if (!ok) {
      lcd_free_cand(h);
      return kmx::fail(KMX_ENOMEM, "candidate buffers");
    }
    sl.cap = cap;
    h->cur = (h->cur + LCD_SLOTS - 1) % LCD_SLOTS;
    use_next_slot(h);  // re-point d_cq .. d_order at the new buffers
  }
  if (!h->cus) KMX_HIP(hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, h->device));
  h->rs_small = h->rs_conc && (int64_t)n < 96LL * h->cus;
  h->rs_on = h->cur != 0 && h->rs_small;
  return 0;
}

// CSR correspondences -> the per-candidate pair rows of k_ransac_coop
// (pairs[c][k], K[c]); one workgroup per candidate, which also moves the
// candidate's frame ids (and its prior) from the staging block to the slot.
// st != null (a spread-form call): also the spread form's initial state of
// candidate c and, over the grid, the ranges' more words (k_rs_init's work).
__global__ __launch_bounds__(256) void k_scatter_pairs(const int64_t* mptr, const int* iq, const int* im, int N,
                                                       int2* pairs, int* Kout, const int* cq_in, const int* cm_in,
                                                       const double* prior_in, int* cq, int* cm, double* prior,
                                                       RsState* st, unsigned* hcnt, int stages, unsigned* more,
                                                       int nmore) {
  const int c = blockIdx.x;
  if (st) {
    if (threadIdx.x == 0) rs_init_c(st, hcnt, c, stages);
    for (int i = c * blockDim.x + threadIdx.x; i < nmore; i += gridDim.x * blockDim.x) more[i] = 0u;
  }
  const int64_t b = mptr[c];
  const int K = (int)(mptr[c + 1] - b);
  for (int k = threadIdx.x; k < K; k += blockDim.x) pairs[(size_t)c * N + k] = make_int2(iq[b + k], im[b + k]);
  if (threadIdx.x == 0) {
    Kout[c] = K;
    cq[c] = cq_in[c];
    cm[c] = cm_in[c];
  }
  if (prior_in && threadIdx.x < 12) prior[12 * (size_t)c + threadIdx.x] = prior_in[12 * (size_t)c + threadIdx.x];
}

RsParams rs_params(const kmx_lcd* h, int stages) {
  RsParams rp{};
  rp.thr2d = h->P.ransac_threshold_2d2d;
  rp.thr3d = h->P.ransac_threshold_3d3d;
  rp.prob = h->P.ransac_probability;
  rp.max_iter = h->P.ransac_max_iterations;
  rp.min2d = h->P.min_2d2d_inliers;
  rp.min3d = h->P.min_3d3d_inliers;
  rp.pmax = h->pmax;
  rp.pnp = rec_sampled(h->P) ? 1 : 0;  // k_recover takes over
  rp.prof = h->prof;
  rp.algo = h->P.algorithm_2d2d;
  rp.refine = h->P.refine_pose && h->P.pose_recovery_type == 0 ? 1 : 0;
  rp.stages = stages;
  rp.prior = h->d_prior;
  return rp;
}
PnpParams pnp_params(const kmx_lcd* h, int stages) {
  const bool pnp = h->P.pose_recovery_type == 1;
  PnpParams pp{};
  pp.thr = pnp ? h->P.ransac_threshold_2d3d : h->P.ransac_threshold_3d3d;
  pp.prob = h->P.ransac_probability;
  pp.max_iter = h->P.ransac_max_iterations;
  // without the 2D-2D stage the caller's pairs are the inliers: recover whatever K is
  pp.min2d = (stages & KMX_LCD_STAGE_2D2D) ? h->P.min_2d2d_inliers : 0;
  pp.min_pnp = pnp ? h->P.min_2d3d_inliers : h->P.min_3d3d_inliers;
  pp.refine = !pnp && h->P.refine_pose ? 1 : 0;
  pp.pmax = h->pmax;
  return pp;
}

// The work queue's order: candidates by match count K, largest first (a
// counting sort in one workgroup; ties in any order — each candidate's result
// does not depend on when it is taken). KMX_LCD_ORDER=1 (A/B).
__global__ __launch_bounds__(1024) void k_order(const int* K, int n, int N, int* order) {
  __shared__ int hist[MAX_FEATS + 1];
  for (int k = threadIdx.x; k <= N; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += blockDim.x) atomicAdd(&hist[min(max(K[c], 0), N)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {  // start of each K's range, largest K first
    int acc = 0;
    for (int k = N; k >= 0; --k) {
      const int v = hist[k];
      hist[k] = acc;
      acc += v;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += blockDim.x) order[atomicAdd(&hist[min(max(K[c], 0), N)], 1)] = c;
}

// k_ransac_coop over candidates [0, n) of the (offset) candidate arrays.
int launch_ransac(kmx_lcd* h, int n, const RsParams& rp, const short* table, int c0, bool masks) {
  // minimum waves per SIMD: Stewenius 3 (the batch's LDS, 12.6 KB per wave,
  // admits 12 waves per CU; 168 VGPRs), Nister 4 — the measured best register
  // budgets. The <2, true> and <3, false> instantiations are compiled but never
  // launched: with them in the module the backend's code for the launched
  // <3, true> spills 118 VGPRs (412 B scratch per lane) instead of 396 (972 B)
  // — same source, every callee inlined in both builds, a different inlining
  // order (measured with -Rpass-analysis=kernel-resource-usage, round 4; the
  // RANSAC step took ~11 % longer without them).
  const bool stew = rp.algo == KMX_ALGO_STEWENIUS;
  // four waves per SIMD for both solvers (Stewenius: 128 VGPRs and 10.2 KB of
  // LDS, 16 per CU; no other Stewenius instance is compiled, so the tail's
  // call sees only this bound)
  auto kc = stew ? k_ransac_coop<4, true> : k_ransac_coop<4, false>;
  if (rp.pmax < 0) kc = k_ransac_coop<3, false>;  // never: keeps the Nister 3-wave form compiled
  // one wave per resident slot (<= RS_MAX_SLOTS: the scratch is sized for it)
  int per_cu = 0, dev = 0, cus = 0;
  KMX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kc, RS_BLOCK, 0));
  KMX_HIP(hipGetDevice(&dev));
  KMX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int slots = std::max(1, std::min({n, std::max(per_cu, 1) * cus, RS_MAX_SLOTS, h->cap}));
  KMX_HIP(hipMemsetAsync(h->d_next, 0, sizeof(int), rs_stream(h)));
  RsParams p = rp;
  if (p.prior) p.prior += (size_t)c0 * 12;
  if (p.hyps) p.hyps += c0;
  if (p.nrec) p.nrec += c0;
  const char* ov = std::getenv("KMX_LCD_ORDER");
  const bool longest_first = ov && std::atoi(ov) == 1;
  const int* order = nullptr;
  if (longest_first && n > 1 && c0 == 0) {
    hipLaunchKernelGGL(k_order, dim3(1), dim3(1024), 0, rs_stream(h), (const int*)h->d_K, n, h->N, h->d_order);
    order = h->d_order;
  }
  hipLaunchKernelGGL(kc, dim3(slots), dim3(RS_BLOCK), 0, rs_stream(h), (const double*)h->d_bear,
                     (const double*)h->d_pts, h->N, (const int*)h->d_cq + c0, (const int*)h->d_cm + c0,
                     (const int2*)h->d_pairs + (size_t)c0 * h->N, (const int*)h->d_K + c0, table, p, h->d_res + c0,
                     masks ? h->d_mask + (size_t)c0 * h->N : nullptr, h->d_fbuf, n, h->d_next, order);
  return 0;
}
int launch_recover(kmx_lcd* h, int n, const PnpParams& pp, const short* table, int c0) {
  const bool pnp = h->P.pose_recovery_type == 1;
  const size_t smem = sizeof(double) * (6 * (size_t)h->N + 64 * 12 + 12) + sizeof(int) * (64 + 64 + 4 + (size_t)h->N);
  PnpParams p = pp;
  if (p.hyps) p.hyps += c0;
  hipLaunchKernelGGL(pnp ? k_recover<true> : k_recover<false>, dim3(n), dim3(RS_BLOCK), smem, rs_stream(h),
                     (const double*)h->d_bear, (const double*)h->d_pts, h->N, (const int*)h->d_cq + c0,
                     (const int*)h->d_cm + c0, (const int2*)h->d_pairs + (size_t)c0 * h->N, (const int*)h->d_K + c0,
                     table, p, h->d_res + c0, h->d_mask + (size_t)c0 * h->N);
  return 0;
}

// The ordered sampler (rng_stream 1): candidates one after the other, each
// RANSAC problem drawing from the handle's engine where the previous problem
// left it — a chain through every candidate (the k-th problem's first sample
// depends on how many passes problem k-1 drew, known only when it ends), so
// this path is serial by construction: per problem the host draws the
// problem's sample row from a copy of the engine, the kernel runs that one
// problem, and the engine then advances by the passes the serial loop drew.
int verify_ordered(kmx_lcd* h, int n, int stages, bool masks) {
  std::vector<int> K(n);
  KMX_HIP(hipMemcpyAsync(K.data(), h->d_K, sizeof(int) * n, hipMemcpyDeviceToHost, rs_stream(h)));
  KMX_HIP(hipStreamSynchronize(rs_stream(h)));
  RsParams rp = rs_params(h, stages);
  rp.tab_fixed = 1;
  rp.hyps = h->d_hyps;
  rp.nrec = rec_sampled(h->P) ? h->d_nrec : nullptr;
  PnpParams pp = pnp_params(h, stages);
  pp.tab_fixed = 1;
  pp.hyps = h->d_hyps;
  const int v = h->P.rng_variant;
  std::vector<short> row((size_t)h->pmax * PNP_S);
  auto advance = [&](int passes, int S) {
    for (long i = 0; i < (long)passes * S; ++i) (void)sampler_draw(h->stream_rng, v);
  };
  for (int c = 0; c < n; ++c) {
    const bool st2d = (stages & KMX_LCD_STAGE_2D2D) != 0;
    if (st2d && K[c] >= 5) {
      std::mt19937 probe = h->stream_rng;
      sample_row(probe, v, K[c], h->pmax, 5, row.data());
      KMX_HIP(hipMemcpyAsync(h->d_row, row.data(), sizeof(short) * (size_t)h->pmax * 5, hipMemcpyHostToDevice,
                             rs_stream(h)));
    }
    if (int rc = launch_ransac(h, 1, rp, h->d_row, c, masks || rp.pnp)) return rc;
    int got[2] = {0, 0};
    KMX_HIP(hipMemcpyAsync(&got[0], h->d_hyps + c, sizeof(int), hipMemcpyDeviceToHost, rs_stream(h)));
    if (rp.nrec) KMX_HIP(hipMemcpyAsync(&got[1], h->d_nrec + c, sizeof(int), hipMemcpyDeviceToHost, rs_stream(h)));
    KMX_HIP(hipStreamSynchronize(rs_stream(h)));
    if (st2d && K[c] >= 5) advance(got[0], 5);
    if (!rp.pnp || !(stages & KMX_LCD_STAGE_RECOVER)) continue;
    kmx_lcd_result r{};
    KMX_HIP(hipMemcpyAsync(&r, h->d_res + c, sizeof(r), hipMemcpyDeviceToHost, rs_stream(h)));
    KMX_HIP(hipStreamSynchronize(rs_stream(h)));
    if (r.mono_inliers < pp.min2d) continue;
    const int S = rec_S(h->P), n2 = got[1];
    if (n2 >= S) {
      std::mt19937 probe = h->stream_rng;
      sample_row(probe, v, n2, h->pmax, S, row.data());
      KMX_HIP(hipMemcpyAsync(h->d_row, row.data(), sizeof(short) * (size_t)h->pmax * S, hipMemcpyHostToDevice,
                             rs_stream(h)));
    }
    if (int rc = launch_recover(h, 1, pp, h->d_row, c)) return rc;
    int hy = 0;
    KMX_HIP(hipMemcpyAsync(&hy, h->d_hyps + c, sizeof(int), hipMemcpyDeviceToHost, rs_stream(h)));
    KMX_HIP(hipStreamSynchronize(rs_stream(h)));
    if (n2 >= S) advance(hy, S);
  }
  return 0;
}

// The spread form (see k_rs_hyps): hypothesis ranges of growing size on many
// waves, the serial control replayed after each, until every candidate's loop
// has stopped; then the candidates' results. Synchronous (the host reads
// whether a candidate needs another range). With `copy_out` (the caller's
// result copies) the finish is enqueued speculatively behind the first
// range, gated on the device by the range's `more` word, with the copies
// after it: a call whose candidates all stop inside the first range (a true
// loop closure: ~30 of 66 or 510 hypotheses) then costs one host round trip
// instead of two, and *copied says the results are on their way.
constexpr int SPREAD_WAVES = 1024;  // waves of one k_rs_hyps launch at most
// res_dst / mask_dst (zero-copy callers): where k_rs_finish writes the results
// and masks (host-mapped memory) in place of the slot's device buffers; the
// speculative finish then also writes the range's `more` word to h_more.
// The spread form's buffers for n candidates (grow-only).
int spread_alloc(kmx_lcd* h, int n) {
  hipStream_t st = rs_stream(h);
  if (n > h->spread_cap) {
    void* q[] = {h->d_st, h->d_hout, h->d_sfbuf, h->d_hcnt};
    KMX_HIP(hipStreamSynchronize(st));
    for (void* x : q)
      if (x) (void)hipFree(x);
    h->d_st = nullptr; h->d_hout = nullptr; h->d_sfbuf = nullptr; h->d_hcnt = nullptr;
    h->spread_cap = 0;
    const int cap = std::max(n, h->spread_max);
    KMX_HIP(hipMalloc(&h->d_st, sizeof(RsState) * cap));
    KMX_HIP(hipMalloc(&h->d_hcnt, sizeof(unsigned) * cap));
    KMX_HIP(hipMalloc(&h->d_hout, sizeof(HypOut) * (size_t)cap * h->pmax));
    KMX_HIP(hipMalloc(&h->d_sfbuf, sizeof(double) * (6 * (size_t)h->N + STASH) * std::max(SPREAD_WAVES, cap)));
    h->spread_cap = cap;
  }
  if (h->pmax + 1 > h->more_cap) {  // every range advances by >= 1 pass: at most pmax ranges
    KMX_HIP(hipStreamSynchronize(st));
    if (h->d_more) (void)hipFree(h->d_more);
    h->d_more = nullptr;
    h->more_cap = 0;
    KMX_HIP(hipMalloc(&h->d_more, sizeof(unsigned) * (h->pmax + 1)));
    h->more_cap = h->pmax + 1;
  }
  if (!h->h_more) {
    KMX_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_more), sizeof(unsigned),
                          hipHostMallocMapped | hipHostMallocCoherent));
    KMX_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->z_more), h->h_more, 0));
  }
  return 0;
}
// inited: the caller's k_scatter_pairs already initialised the state (no k_rs_init launch)
// fseq (a zero-copy call of one candidate): the sequence its last kernel
// stores to the completion word, for the caller's wait_done (0: none).
int ransac_spread(kmx_lcd* h, int n, int stages, bool want_masks, const std::function<int()>* copy_out = nullptr,
                  bool* copied = nullptr, kmx_lcd_result* res_dst = nullptr, unsigned char* mask_dst = nullptr,
                  bool inited = false, unsigned* fseq = nullptr) {
  const RsParams rp = rs_params(h, stages);
  const bool masks = want_masks || rp.pnp;
  hipStream_t st = rs_stream(h);
  if (int rc = spread_alloc(h, n)) return rc;
  const bool stew = rp.algo == KMX_ALGO_STEWENIUS;
  const int per_max = stew ? SG : SPREAD_PER_NISTER;
  if (!inited)
    hipLaunchKernelGGL(k_rs_init, dim3((std::max(n, h->more_cap) + 63) / 64), dim3(64), 0, st, h->d_st, h->d_hcnt, n,
                       stages, h->d_more, h->more_cap);
  int pa = 0;
  // the first range: a true loop closure's loop (~30 iterations) in one pass;
  // where the launch has the waves for it (one or two candidates), a whole
  // 500-iteration loop (510) at once — one hypothesis per wave costs the
  // same latency, and a look-alike then needs one range, not two
  int range = (int64_t)n * 510 <= SPREAD_WAVES ? 510 : 66;
  const size_t tail_bytes = sizeof(double) * tail_lds_doubles(h->N);
  if (tail_bytes > 65536 - 16384)  // (max_feats near 1024: 75 KB, + 8.8 KB static: workspace, counts)
    KMX_HIP(hipFuncSetAttribute((const void*)k_rs_finish, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tail_bytes));
  const bool zc = res_dst != nullptr;
  unsigned* z_more = zc ? h->z_more : nullptr;
  if (fseq) *fseq = 0;
  const bool one = zc && n == 1 && fseq;  // a one-candidate call: its finishes store the completion word
  auto finish = [&](const unsigned* skip, unsigned* seq_out) {
    unsigned seq = 0;
    unsigned* done = one && seq_out ? next_done(h, &seq) : nullptr;
    if (seq_out) *seq_out = done ? seq : 0;
    hipLaunchKernelGGL(k_rs_finish, dim3(n), dim3(RS_BLOCK * RS_FIN), tail_bytes, st,
                       (const double*)h->d_bear, (const double*)h->d_pts,
                       h->N, (const int*)h->d_cq, (const int*)h->d_cm, (const int2*)h->d_pairs, (const int*)h->d_K, rp,
                       (const RsState*)h->d_st, zc ? res_dst : h->d_res,
                       masks ? (zc && mask_dst ? mask_dst : h->d_mask) : nullptr, h->d_sfbuf, skip,
                       skip && zc ? z_more : nullptr, done, seq);
  };
  const bool spec = copy_out && copied && !rp.pnp;
  if (copied) *copied = false;
  for (int it = 0; pa < h->pmax && (stages & KMX_LCD_STAGE_2D2D); ++it) {  // (recovery alone: no hypotheses)
    // hypotheses per wave: as few as the launch's waves allow (one wave
    // works through its hypotheses one after another; the batch of SG
    // Stewenius hypotheses per wave only pays where waves are short)
    const int per = std::max(1, std::min(per_max, (int)(((int64_t)n * range + SPREAD_WAVES - 1) / SPREAD_WAVES)));
    int G = (range + per - 1) / per;
    G = std::max(1, std::min(G, SPREAD_WAVES / n));
    const int pb = std::min(pa + G * per, h->pmax);
    hipLaunchKernelGGL(stew ? k_rs_hyps<true> : k_rs_hyps<false>, dim3(n * G), dim3(RS_BLOCK), 0, st,
                       (const double*)h->d_bear, h->N, (const int*)h->d_cq, (const int*)h->d_cm,
                       (const int2*)h->d_pairs, (const int*)h->d_K, (const short*)h->d_table, rp,
                       h->d_st, h->d_hout, pa, pb, G, per, h->d_sfbuf, h->d_hcnt, h->d_more + it);
    const bool zc_more = spec && it == 0 && zc;  // the speculative finish writes the word itself
    unsigned sseq = 0;
    if (spec && it == 0) {
      finish(h->d_more, zc_more ? &sseq : nullptr);
      if (int rc = (*copy_out)()) return rc;
    }
    if (!zc_more) KMX_HIP(hipMemcpyAsync(h->h_more, h->d_more + it, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    if (sseq) {  // the finish stored the more word before its completion word
      if (int rc = wait_done(h, st, sseq)) return rc;
    } else {
      KMX_HIP(hipStreamSynchronize(st));
    }
    if (!*h->h_more) {
      if (spec && it == 0) {
        *copied = true;
        if (fseq) *fseq = sseq;
        KMX_HIP(hipGetLastError());
        return 0;
      }
      break;
    }
    pa = pb;
    range = pa < 510 ? 510 - pa : 1500;  // then the rest of a 500-iteration loop, then its skips
  }
  finish(nullptr, fseq);
  if (rp.pnp && (stages & KMX_LCD_STAGE_RECOVER))
    if (int rc = launch_recover(h, n, pnp_params(h, stages), h->d_table_rec, 0)) return rc;
  KMX_HIP(hipGetLastError());
  return 0;
}

// Everything after the pair rows d_pairs / d_K exist: RANSAC, then recovery.
// sync_ok: the caller synchronises on the results (kmx_lcd_verify,
// kmx_lcd_verify_matches), so a small call may take the spread form.
int enqueue_ransac(kmx_lcd* h, int n, int stages, bool want_masks, bool sync_ok = false,
                   const std::function<int()>* copy_out = nullptr, bool* copied = nullptr,
                   kmx_lcd_result* res_dst = nullptr, unsigned char* mask_dst = nullptr, bool inited = false,
                   unsigned* fseq = nullptr) {
  if (copied) *copied = false;
  if (fseq) *fseq = 0;
  if (h->P.rng_stream) return verify_ordered(h, n, stages, want_masks);
  if (sync_ok && n > 0 && n <= h->spread_max)
    return ransac_spread(h, n, stages, want_masks, copy_out, copied, res_dst, mask_dst, inited, fseq);
  const RsParams rp = rs_params(h, stages);
  if (int rc = launch_ransac(h, n, rp, h->d_table, 0, want_masks || rp.pnp)) return rc;
  if (rp.pnp && (stages & KMX_LCD_STAGE_RECOVER))
    if (int rc = launch_recover(h, n, pnp_params(h, stages), h->d_table_rec, 0)) return rc;
  return 0;
}

// The side stream may write the current slot once the last RANSAC that read it
// (LCD_SLOTS calls back) is done; the candidate uploads then go on it.
int slot_upload(kmx_lcd* h, int n, const int32_t* cq, const int32_t* cm) {
  const int s = h->cur, s2 = (s + LCD_SLOTS - 2) % LCD_SLOTS;
  if (h->ev_rs_set[s]) KMX_HIP(hipStreamWaitEvent(h->kstream, h->ev_rs[s], 0));
  if (!h->rs_small && h->ev_rs_set[s2]) KMX_HIP(hipStreamWaitEvent(h->kstream, h->ev_rs[s2], 0));
  KMX_HIP(hipMemcpyAsync(h->d_cq, cq, sizeof(int) * n, hipMemcpyHostToDevice, h->kstream));
  KMX_HIP(hipMemcpyAsync(h->d_cm, cm, sizeof(int) * n, hipMemcpyHostToDevice, h->kstream));
  return 0;
}
// The kNN2 of n candidates (ids at dcq / dcm) on stream st: k_knn2, or for a
// synchronous call of <= KS_MAX candidates the split form k_knn2s (same rows).
constexpr int KS_MAX = 64;
int launch_knn2(kmx_lcd* h, int n, const int* dcq, const int* dcm, hipStream_t st, bool sync_call,
                int2* pairs_dst = nullptr, int* k_dst = nullptr, unsigned* done = nullptr, unsigned seq = 0) {
  if (sync_call && h->knn_split && n <= KS_MAX) {
    if (h->kqb_N < h->N) {
      KMX_HIP(hipStreamSynchronize(st));
      if (h->d_kqb) (void)hipFree(h->d_kqb);
      h->d_kqb = nullptr;
      h->kqb_N = 0;
      KMX_HIP(hipMalloc(&h->d_kqb, sizeof(int) * (size_t)KS_MAX * h->N));
      h->kqb_N = h->N;
    }
    if (!h->d_kcnt) {
      KMX_HIP(hipMalloc(&h->d_kcnt, sizeof(unsigned) * KS_MAX));
      KMX_HIP(hipMemsetAsync(h->d_kcnt, 0, sizeof(unsigned) * KS_MAX, st));
    }
    const int S = (h->N + KS_Q - 1) / KS_Q;
    const size_t smem = (size_t)h->N * 32 + sizeof(uint32_t) * 4 * KS_Q * 2 + sizeof(int) * (KNN_BLOCK + 1);
    hipLaunchKernelGGL(h->P.norm == KMX_NORM_HAMMING ? k_knn2s<true> : k_knn2s<false>, dim3(n * S), dim3(KNN_BLOCK),
                       smem, st, (const uint32_t*)h->d_desc, (const int*)h->d_nfeat, h->N, dcq, dcm,
                       h->P.lowe_ratio, pairs_dst ? pairs_dst : h->d_pairs, k_dst ? k_dst : h->d_K, h->d_kqb,
                       h->d_kcnt, S, done, seq);
  } else if (h->knn_q && h->P.norm == KMX_NORM_HAMMING && h->N <= KQ_BLOCK * KQ_Q) {
    hipLaunchKernelGGL(k_knn2q<true>, dim3(n), dim3(KQ_BLOCK),
                       (size_t)h->N * 32, st, (const uint32_t*)h->d_desc, (const int*)h->d_nfeat, h->N, dcq, dcm,
                       h->P.lowe_ratio, pairs_dst ? pairs_dst : h->d_pairs, k_dst ? k_dst : h->d_K);
  } else {
    hipLaunchKernelGGL(k_knn2, dim3(n), dim3(KNN_BLOCK), (size_t)h->N * 32 + sizeof(int) * (KNN_BLOCK + 1), st,
                       (const uint32_t*)h->d_desc, (const int*)h->d_nfeat, h->N, dcq, dcm, h->P.norm,
                       h->P.lowe_ratio, pairs_dst ? pairs_dst : h->d_pairs, k_dst ? k_dst : h->d_K);
  }
  return 0;
}

// kNN2 of the current slot on the side stream, the RANSAC on the handle's
// stream behind it: a call's kNN2 runs in the previous call's RANSAC tail
// (the work-queue RANSAC holds every wave slot until its queue drains, so the
// kNN2 workgroups start as its last waves leave), off the critical path.
int enqueue_verify(kmx_lcd* h, int n, bool want_masks, bool sync_ok = false) {
  if (n == 0) return 0;
  const int s = h->cur;
  if (h->timing) {
    if (!h->ev_ok) {
      for (auto& e : h->ev) KMX_HIP(hipEventCreate(&e));
      h->ev_ok = true;
    }
    KMX_HIP(hipEventRecord(h->ev[0], h->kstream));
  }
  if (int rc = launch_knn2(h, n, h->d_cq, h->d_cm, h->kstream, sync_ok)) return rc;
  if (h->timing) KMX_HIP(hipEventRecord(h->ev[1], h->kstream));
  KMX_HIP(hipEventRecord(h->ev_knn[s], h->kstream));
  KMX_HIP(hipStreamWaitEvent(rs_stream(h), h->ev_knn[s], 0));
  if (int rc = enqueue_ransac(h, n, KMX_LCD_STAGE_2D2D | KMX_LCD_STAGE_RECOVER, want_masks, sync_ok)) return rc;
  if (h->timing) KMX_HIP(hipEventRecord(h->ev[2], rs_stream(h)));
  KMX_HIP(hipEventRecord(h->ev_rs[s], rs_stream(h)));
  h->ev_rs_set[s] = true;
  KMX_HIP(hipGetLastError());
  return 0;
}
// Calls that work on the current slot from the handle's stream only (match,
// verify_matches): they end with its RANSAC-done event too.
int mark_slot(kmx_lcd* h) {
  KMX_HIP(hipEventRecord(h->ev_rs[h->cur], rs_stream(h)));
  h->ev_rs_set[h->cur] = true;
  return 0;
}

// Device pool of at least `need` frames of N slots: capacity doubling, the
// resident frames copied device to device (never re-uploaded).
int grow_pool(kmx_lcd* h, int need) {
  if (need <= h->capF) return 0;
  const int cap = std::max({need, 2 * h->capF, 64});
  const size_t FN = (size_t)cap * h->N, old = (size_t)h->F * h->N;
  uint32_t* desc = nullptr;
  double *bear = nullptr, *pts = nullptr;
  int* nf = nullptr;
  if (hipMalloc(&desc, FN * 32) != hipSuccess || hipMalloc(&bear, FN * 3 * sizeof(double)) != hipSuccess ||
      hipMalloc(&pts, FN * 3 * sizeof(double)) != hipSuccess || hipMalloc(&nf, sizeof(int) * cap) != hipSuccess) {
    for (void* x : {(void*)desc, (void*)bear, (void*)pts, (void*)nf})
      if (x) (void)hipFree(x);
    return kmx::fail(KMX_ENOMEM, "frame pool");
  }
  KMX_HIP(hipStreamSynchronize(h->kstream));  // a kNN2 in flight may read the old pool
  for (hipStream_t x : h->rsx)  // and the slots' RANSACs (slot 0's is on h->stream, below)
    if (x) KMX_HIP(hipStreamSynchronize(x));
  if (h->F) {
    KMX_HIP(hipMemcpyAsync(desc, h->d_desc, old * 32, hipMemcpyDeviceToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(bear, h->d_bear, old * 3 * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(pts, h->d_pts, old * 3 * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(nf, h->d_nfeat, sizeof(int) * h->F, hipMemcpyDeviceToDevice, h->stream));
    KMX_HIP(hipStreamSynchronize(h->stream));
  }
  for (void* x : {(void*)h->d_desc, (void*)h->d_bear, (void*)h->d_pts, (void*)h->d_nfeat})
    if (x) (void)hipFree(x);
  h->d_desc = desc;
  h->d_bear = bear;
  h->d_pts = pts;
  h->d_nfeat = nf;
  h->capF = cap;
  return 0;
}

// The staged frames (mapped host pages: desc | bearings | points | n_feats)
// into the pool: 8-B words, n_feats 4-B.
__global__ __launch_bounds__(256) void k_put_frames(const unsigned long long* src, size_t w_desc, size_t w_bear,
                                                    unsigned long long* desc, unsigned long long* bear,
                                                    unsigned long long* pts, const int* nf_src, int* nf, int n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t tot = w_desc + 2 * w_bear;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
    const unsigned long long v = src[i];
    if (i < w_desc) desc[i] = v;
    else if (i < w_desc + w_bear) bear[i - w_desc] = v;
    else pts[i - w_desc - w_bear] = v;
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n; i += stride) nf[i] = nf_src[i];
}
constexpr size_t FRAME_STAGE_MAX = 16u << 20;  // larger uploads (set_pool) copy from the caller's pages

// Frames [F, F + n) from host arrays (desc [n][N][32], bearings / points
// [n][N][3]); the caller has grown the pool.
int upload_frames(kmx_lcd* h, int n, const int32_t* n_feats, const uint8_t* desc, const double* bearings,
                  const double* points) {
  const size_t at = (size_t)h->F * h->N, FN = (size_t)n * h->N;
  const size_t b_desc = FN * 32, b_bear = FN * 3 * sizeof(double), b_nf = sizeof(int) * n;
  const size_t b_all = b_desc + 2 * b_bear + b_nf;
  if (b_all <= FRAME_STAGE_MAX) {
    if (b_all > h->fst_cap) {  // grow-only; the previous upload has completed (synchronised below)
      if (h->h_fst) (void)hipHostFree(h->h_fst);
      h->h_fst = h->z_fst = nullptr;
      h->fst_cap = 0;
      const size_t cap = std::max<size_t>(b_all, 256 * 1024);
      KMX_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_fst), cap, hipHostMallocMapped | hipHostMallocCoherent));
      KMX_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->z_fst), h->h_fst, 0));
      h->fst_cap = cap;
    }
    std::memcpy(h->h_fst, desc, b_desc);
    std::memcpy(h->h_fst + b_desc, bearings, b_bear);
    std::memcpy(h->h_fst + b_desc + b_bear, points, b_bear);
    std::memcpy(h->h_fst + b_desc + 2 * b_bear, n_feats, b_nf);
    const size_t words = (b_desc + 2 * b_bear) / 8;
    const int blocks = (int)std::min<size_t>((words + 255) / 256, 1024);
    hipLaunchKernelGGL(k_put_frames, dim3(std::max(blocks, 1)), dim3(256), 0, h->stream,
                       reinterpret_cast<const unsigned long long*>(h->z_fst), b_desc / 8, b_bear / 8,
                       reinterpret_cast<unsigned long long*>(reinterpret_cast<uint8_t*>(h->d_desc) + at * 32),
                       reinterpret_cast<unsigned long long*>(h->d_bear + at * 3),
                       reinterpret_cast<unsigned long long*>(h->d_pts + at * 3),
                       reinterpret_cast<const int*>(h->z_fst + b_desc + 2 * b_bear), h->d_nfeat + h->F, n);
    KMX_HIP(hipGetLastError());
    KMX_HIP(hipStreamSynchronize(h->stream));  // the staging area is reused by the next call
    h->h_nfeat.insert(h->h_nfeat.end(), n_feats, n_feats + n);
    h->F += n;
    return 0;
  }
  KMX_HIP(hipMemcpyAsync(reinterpret_cast<uint8_t*>(h->d_desc) + at * 32, desc, FN * 32, hipMemcpyHostToDevice,
                         h->stream));
  KMX_HIP(hipMemcpyAsync(h->d_bear + at * 3, bearings, FN * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipMemcpyAsync(h->d_pts + at * 3, points, FN * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipMemcpyAsync(h->d_nfeat + h->F, n_feats, sizeof(int) * n, hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));  // the host arrays may go away after return
  h->h_nfeat.insert(h->h_nfeat.end(), n_feats, n_feats + n);
  h->F += n;
  return 0;
}

}  // namespace

extern "C" int kmx_lcd_create(const kmx_lcd_params* params, int device, kmx_lcd** out) {
  KMX_GUARD_BEGIN
  KMX_CHECK(params && out, KMX_EINVAL, "null argument");
  KMX_CHECK(params->norm == KMX_NORM_L1 || params->norm == KMX_NORM_HAMMING, KMX_EINVAL, "bad norm");
  KMX_CHECK(params->rng_variant == KMX_RNG_GCC9 || params->rng_variant == KMX_RNG_GCC11, KMX_EINVAL,
            "bad rng variant");
  KMX_CHECK(params->ransac_randomize == 0, KMX_EUNSUP, "ransac_randomize = 1 is not reproducible; use 0");
  KMX_CHECK(params->use_1point_3d3d == 0 || params->use_1point_3d3d == 1, KMX_EINVAL, "use_1point_3d3d is 0 or 1");
  KMX_CHECK(params->algorithm_2d2d == KMX_ALGO_STEWENIUS || params->algorithm_2d2d == KMX_ALGO_NISTER, KMX_EUNSUP,
            "ransac_2d2d_algorithm: 0 (Stewenius) and 1 (Nister) are built");
  KMX_CHECK(params->ransac_max_iterations > 0, KMX_EINVAL, "ransac_max_iterations must be > 0");
  KMX_CHECK(params->rng_stream == 0 || params->rng_stream == 1, KMX_EINVAL, "rng_stream is 0 or 1");
  int ndev = 0;
  KMX_HIP(hipGetDeviceCount(&ndev));
  KMX_CHECK(device >= 0 && device < ndev, KMX_EINVAL, "bad HIP device ordinal");
  KMX_HIP(hipSetDevice(device));
  kmx_lcd* h = new kmx_lcd();
  h->P = *params;
  h->device = device;
  h->stream_rng.seed(params->ransac_seed);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return kmx::fail(KMX_EHIP, "hipStreamCreate");
  }
  h->own_stream = true;
  if (const char* e = std::getenv("KMX_LCD_RSX")) h->rs_conc = std::atoi(e) != 0;
  if (const char* e = std::getenv("KMX_LCD_KSPLIT")) h->knn_split = std::atoi(e) != 0;
  if (const char* e = std::getenv("KMX_LCD_KNNQ")) h->knn_q = std::atoi(e) != 0;
  if (const char* e = std::getenv("KMX_LCD_SPINWAIT")) h->spin_wait = std::atoi(e) != 0;
  bool ok = hipStreamCreateWithFlags(&h->kstream, hipStreamNonBlocking) == hipSuccess;
  for (int i = 1; i < LCD_SLOTS && ok; ++i) ok = hipStreamCreateWithFlags(&h->rsx[i], hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; i < LCD_SLOTS && ok; ++i)
    ok = hipEventCreateWithFlags(&h->ev_knn[i], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&h->ev_rs[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    kmx_lcd_destroy(h);
    return kmx::fail(KMX_EHIP, "hipStreamCreate / hipEventCreate");
  }
  if (const char* v = std::getenv("KMX_RS_PROF")) h->prof = std::atoi(v);
  // KMX_LCD_SPREAD: the largest synchronous call that takes the spread form (0: never)
  if (const char* v = std::getenv("KMX_LCD_SPREAD")) h->spread_max = std::max(0, std::atoi(v));
  *out = h;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_lcd_destroy(kmx_lcd* h) {
  if (!h) return KMX_OK;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  sync_rsx(h);
  if (h->kstream) (void)hipStreamSynchronize(h->kstream);
  lcd_free_frames(h);
  lcd_free_tables(h);
  lcd_free_cand(h);
  lcd_free_pairs(h);
  if (h->ev_ok)
    for (auto e : h->ev) (void)hipEventDestroy(e);
  for (int i = 0; i < LCD_SLOTS; ++i) {
    if (h->ev_knn[i]) (void)hipEventDestroy(h->ev_knn[i]);
    if (h->ev_rs[i]) (void)hipEventDestroy(h->ev_rs[i]);
  }
  if (h->kstream) (void)hipStreamDestroy(h->kstream);
  for (hipStream_t x : h->rsx)
    if (x) (void)hipStreamDestroy(x);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return KMX_OK;
}

extern "C" int kmx_lcd_set_stream(kmx_lcd* h, void* s) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  if (h->kstream) KMX_HIP(hipStreamSynchronize(h->kstream));
  for (hipStream_t x : h->rsx)
    if (x) KMX_HIP(hipStreamSynchronize(x));
  if (h->stream) KMX_HIP(hipStreamSynchronize(h->stream));
  if (h->own_stream && h->stream) KMX_HIP(hipStreamDestroy(h->stream));
  h->own_stream = false;
  h->stream = reinterpret_cast<hipStream_t>(s);
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_lcd_set_frames(kmx_lcd* h, const kmx_lcd_batch_desc* pool) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h && pool, KMX_EINVAL, "null argument");
  KMX_CHECK(pool->n_frames > 0 && pool->max_feats >= 5 && pool->max_feats <= MAX_FEATS, KMX_EINVAL,
            "need n_frames > 0 and 5 <= max_feats <= 1024");
  KMX_CHECK(pool->n_feats && pool->desc && pool->bearings && pool->points, KMX_EINVAL, "null pool array");
  for (int f = 0; f < pool->n_frames; ++f)
    KMX_CHECK(pool->n_feats[f] >= 0 && pool->n_feats[f] <= pool->max_feats, KMX_EINVAL, "bad n_feats");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  if (pool->max_feats != h->N) lcd_free_cand(h);
  lcd_free_frames(h);
  h->N = pool->max_feats;
  if (int rc = grow_pool(h, pool->n_frames)) return rc;
  if (int rc = upload_frames(h, pool->n_frames, pool->n_feats, pool->desc, pool->bearings, pool->points)) return rc;
  return ensure_tables(h);
  KMX_GUARD_END
}

extern "C" int kmx_lcd_add_frames(kmx_lcd* h, int32_t n, int32_t max_feats, const int32_t* n_feats,
                                  const uint8_t* desc, const double* bearings, const double* points,
                                  int32_t* first_id) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_CHECK(n >= 0 && (n == 0 || (n_feats && desc && bearings && points)), KMX_EINVAL, "null frame array");
  KMX_CHECK(max_feats >= 5 && max_feats <= MAX_FEATS, KMX_EINVAL, "need 5 <= max_feats <= 1024");
  KMX_CHECK(h->F == 0 || max_feats == h->N, KMX_EINVAL, "max_feats differs from the resident pool's");
  for (int f = 0; f < n; ++f)
    KMX_CHECK(n_feats[f] >= 0 && n_feats[f] <= max_feats, KMX_EINVAL, "bad n_feats");
  KMX_CHECK((int64_t)h->F + n <= INT32_MAX, KMX_EINVAL, "frame ids exceed int32");
  KMX_HIP(hipSetDevice(h->device));
  if (h->F == 0 && max_feats != h->N) {
    KMX_HIP(hipStreamSynchronize(h->stream));
    lcd_free_cand(h);
    lcd_free_frames(h);
    h->N = max_feats;
  }
  if (first_id) *first_id = h->F;
  if (n == 0) return ensure_tables(h);
  if (int rc = grow_pool(h, h->F + n)) return rc;
  if (int rc = upload_frames(h, n, n_feats, desc, bearings, points)) return rc;
  return ensure_tables(h);
  KMX_GUARD_END
}

extern "C" int kmx_lcd_pool_info(kmx_lcd* h, int32_t* n_frames, int32_t* capacity, int32_t* max_feats) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  if (n_frames) *n_frames = h->F;
  if (capacity) *capacity = h->capF;
  if (max_feats) *max_feats = h->N;
  return KMX_OK;
}

static int check_cands(kmx_lcd* h, int32_t n, const int32_t* cq, const int32_t* cm) {
  KMX_CHECK(h && h->d_desc && h->F > 0, KMX_ESTATE, "no frames: set_frames or add_frames first");
  KMX_CHECK(n >= 0 && (n == 0 || (cq && cm)), KMX_EINVAL, "bad candidate arrays");
  for (int i = 0; i < n; ++i)
    KMX_CHECK(cq[i] >= 0 && cq[i] < h->F && cm[i] >= 0 && cm[i] < h->F, KMX_EINVAL, "candidate frame id out of range");
  return 0;
}

extern "C" int kmx_lcd_verify(kmx_lcd* h, int32_t n, const int32_t* cq, const int32_t* cm, kmx_lcd_result* results,
                              uint8_t* inlier_masks) {
  KMX_GUARD_BEGIN
  if (int rc = check_cands(h, n, cq, cm)) return rc;
  KMX_CHECK(results || n == 0, KMX_EINVAL, "null results");
  KMX_HIP(hipSetDevice(h->device));
  if (int rc = ensure_cap(h, n, false)) return rc;
  if (int rc = slot_upload(h, n, cq, cm)) return rc;
  if (int rc = enqueue_verify(h, n, inlier_masks != nullptr, true)) return rc;
  if (n) KMX_HIP(hipMemcpyAsync(results, h->d_res, sizeof(kmx_lcd_result) * n, hipMemcpyDeviceToHost, rs_stream(h)));
  if (n && inlier_masks)
    KMX_HIP(hipMemcpyAsync(inlier_masks, h->d_mask, (size_t)n * h->N, hipMemcpyDeviceToHost, rs_stream(h)));
  KMX_HIP(hipStreamSynchronize(rs_stream(h)));
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_lcd_verify_async(kmx_lcd* h, int32_t n, const int32_t* cq, const int32_t* cm) {
  KMX_GUARD_BEGIN
  if (int rc = check_cands(h, n, cq, cm)) return rc;
  KMX_HIP(hipSetDevice(h->device));
  if (int rc = ensure_cap(h, n, true)) return rc;
  if (int rc = slot_upload(h, n, cq, cm)) return rc;
  KMX_HIP(hipStreamSynchronize(h->kstream));  // host arrays may go away after return
  return enqueue_verify(h, n, false);
  KMX_GUARD_END
}

extern "C" int kmx_lcd_match(kmx_lcd* h, int32_t n, const int32_t* cq, const int32_t* cm, int32_t* pairs_out,
                             int32_t* k_out) {
  KMX_GUARD_BEGIN
  if (int rc = check_cands(h, n, cq, cm)) return rc;
  KMX_CHECK(n == 0 || (pairs_out && k_out), KMX_EINVAL, "null output");
  if (n == 0) return KMX_OK;
  KMX_HIP(hipSetDevice(h->device));
  if (int rc = ensure_cap(h, n, false)) return rc;
  if (int rc = rs_wait_slot(h)) return rc;
  // pinned staging: [cq][cm] in, [pairs][K] out. The split kNN2 (small calls)
  // reads the ids from the mapped staging and writes the rows there
  // (zero-copy); k_knn2 goes through the device buffers and copies.
  const size_t pb = sizeof(int2) * (size_t)n * h->N, kin = al16(sizeof(int) * n), o_out = 2 * kin;
  if (int rc = io_reserve(h, o_out + pb + kin)) return rc;
  std::memcpy(h->h_io, cq, sizeof(int) * n);
  std::memcpy(h->h_io + kin, cm, sizeof(int) * n);
  const bool zc = h->knn_split && n <= KS_MAX;
  unsigned seq = 0;
  unsigned* done = zc && n == 1 ? next_done(h, &seq) : nullptr;  // one candidate: spin on the completion word
  if (zc) {
    if (int rc = launch_knn2(h, n, (const int*)h->z_io, (const int*)(h->z_io + kin), rs_stream(h), true,
                             (int2*)(h->z_io + o_out), (int*)(h->z_io + o_out + pb), done, seq))
      return rc;
  } else {
    KMX_HIP(hipMemcpyAsync(h->d_io, h->h_io, 2 * kin, hipMemcpyHostToDevice, rs_stream(h)));
    if (int rc = launch_knn2(h, n, (const int*)h->d_io, (const int*)(h->d_io + kin), rs_stream(h), true)) return rc;
    KMX_HIP(hipMemcpyAsync(h->h_io + o_out, h->d_pairs, pb, hipMemcpyDeviceToHost, rs_stream(h)));
    KMX_HIP(hipMemcpyAsync(h->h_io + o_out + pb, h->d_K, sizeof(int) * n, hipMemcpyDeviceToHost, rs_stream(h)));
  }
  KMX_HIP(hipGetLastError());
  if (int rc = mark_slot(h)) return rc;
  if (done) {
    if (int rc = wait_done(h, rs_stream(h), seq)) return rc;
  } else {
    KMX_HIP(hipStreamSynchronize(rs_stream(h)));
  }
  std::memcpy(pairs_out, h->h_io + o_out, pb);
  std::memcpy(k_out, h->h_io + o_out + pb, sizeof(int) * n);
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_lcd_verify_matches(kmx_lcd* h, int32_t n, const int32_t* cq, const int32_t* cm,
                                      const int64_t* mptr, const int32_t* iq, const int32_t* im, int stages,
                                      const double* T_prior, kmx_lcd_result* results, uint8_t* inlier_masks) {
  KMX_GUARD_BEGIN
  if (int rc = check_cands(h, n, cq, cm)) return rc;
  KMX_CHECK(results || n == 0, KMX_EINVAL, "null results");
  KMX_CHECK(stages >= 1 && stages <= 3, KMX_EINVAL, "stages: a non-empty mask of KMX_LCD_STAGE_*");
  KMX_CHECK(n == 0 || mptr, KMX_EINVAL, "null mptr");
  const bool need_prior = !(stages & KMX_LCD_STAGE_2D2D) && (stages & KMX_LCD_STAGE_RECOVER) &&
                          h->P.pose_recovery_type == 0 && h->P.use_1point_3d3d;
  KMX_CHECK(!need_prior || T_prior, KMX_EINVAL,
            "the 1-point 3D-3D recovery without the 2D-2D stage needs T_prior (the 2D-2D rotation)");
  if (n == 0) return KMX_OK;
  const int64_t base = mptr[0];
  KMX_CHECK(base >= 0, KMX_EINVAL, "mptr[0] < 0");
  KMX_CHECK(mptr[n] == base || (iq && im), KMX_EINVAL, "null i_query / i_match with correspondences in mptr");
  for (int i = 0; i < n; ++i) {
    const int64_t K = mptr[i + 1] - mptr[i];
    KMX_CHECK(K >= 0 && K <= h->N, KMX_EINVAL, "a candidate has more pairs than max_feats (or mptr decreases)");
    const int nq = h->h_nfeat[cq[i]], nm = h->h_nfeat[cm[i]];
    for (int64_t k = mptr[i]; k < mptr[i + 1]; ++k)
      KMX_CHECK(iq[k] >= 0 && iq[k] < nq && im[k] >= 0 && im[k] < nm, KMX_EINVAL,
                "correspondence index outside its frame's features");
  }
  const size_t total = (size_t)(mptr[n] - base);
  KMX_HIP(hipSetDevice(h->device));
  if (int rc = ensure_cap(h, n, false)) return rc;
  if (int rc = rs_wait_slot(h)) return rc;
  // every input in one pinned block and one host-to-device copy:
  // [mptr - base][cq][cm][i_query][i_match][T_prior]; k_scatter_pairs moves
  // the candidates' ids and priors into the slot's buffers
  const size_t o_cq = al16(sizeof(int64_t) * (n + 1)), o_cm = o_cq + al16(sizeof(int) * n),
               o_iq = o_cm + al16(sizeof(int) * n), o_im = o_iq + al16(sizeof(int) * total),
               o_pr = o_im + al16(sizeof(int) * total), in_bytes = o_pr + (T_prior ? sizeof(double) * 12 * n : 0);
  const size_t rb = al16(sizeof(kmx_lcd_result) * n), out_bytes = rb + (inlier_masks ? (size_t)n * h->N : 0);
  const size_t o_out = al16(in_bytes);  // outputs after the inputs (zero-copy kernels read and write at once)
  if (int rc = io_reserve(h, o_out + out_bytes)) return rc;
  {
    int64_t* mp = reinterpret_cast<int64_t*>(h->h_io);
    for (int i = 0; i <= n; ++i) mp[i] = mptr[i] - base;
    std::memcpy(h->h_io + o_cq, cq, sizeof(int) * n);
    std::memcpy(h->h_io + o_cm, cm, sizeof(int) * n);
    if (total) {
      std::memcpy(h->h_io + o_iq, iq + base, sizeof(int) * total);
      std::memcpy(h->h_io + o_im, im + base, sizeof(int) * total);
    }
    if (T_prior) std::memcpy(h->h_io + o_pr, T_prior, sizeof(double) * 12 * n);
  }
  // a spread-form call (small, synchronous) reads its inputs from the mapped
  // staging and, without PnP (k_recover writes through the device buffers),
  // its finish writes the results there: no copy in either direction
  const bool spread = !h->P.rng_stream && n <= h->spread_max;
  const bool zc_out = spread && !rs_params(h, stages).pnp;
  const char* src = spread ? h->z_io : h->d_io;
  if (spread) {
    if (int rc = spread_alloc(h, n)) return rc;
  } else {
    KMX_HIP(hipMemcpyAsync(h->d_io, h->h_io, in_bytes, hipMemcpyHostToDevice, rs_stream(h)));
  }
  hipLaunchKernelGGL(k_scatter_pairs, dim3(n), dim3(256), 0, rs_stream(h), (const int64_t*)src,
                     (const int*)(src + o_iq), (const int*)(src + o_im), h->N, h->d_pairs, h->d_K,
                     (const int*)(src + o_cq), (const int*)(src + o_cm),
                     T_prior ? (const double*)(src + o_pr) : nullptr, h->d_cq, h->d_cm, h->d_prior,
                     spread ? h->d_st : nullptr, h->d_hcnt, stages, h->d_more, h->more_cap);
  KMX_HIP(hipGetLastError());
  const std::function<int()> copy_out = [&]() -> int {
    if (zc_out) return 0;
    KMX_HIP(hipMemcpyAsync(h->h_io + o_out, h->d_res, sizeof(kmx_lcd_result) * n, hipMemcpyDeviceToHost,
                           rs_stream(h)));
    if (inlier_masks)
      KMX_HIP(hipMemcpyAsync(h->h_io + o_out + rb, h->d_mask, (size_t)n * h->N, hipMemcpyDeviceToHost,
                             rs_stream(h)));
    return 0;
  };
  bool copied = false;
  unsigned fseq = 0;  // the last kernel's completion word (one zero-copy candidate)
  if (int rc = enqueue_ransac(h, n, stages, inlier_masks != nullptr, true, &copy_out, &copied,
                              zc_out ? reinterpret_cast<kmx_lcd_result*>(h->z_io + o_out) : nullptr,
                              zc_out && inlier_masks ? reinterpret_cast<unsigned char*>(h->z_io + o_out + rb) : nullptr,
                              spread, &fseq))
    return rc;
  KMX_HIP(hipGetLastError());
  if (!copied)
    if (int rc = copy_out()) return rc;
  if (int rc = mark_slot(h)) return rc;
  if (fseq) {
    if (int rc = wait_done(h, rs_stream(h), fseq)) return rc;
  } else {
    KMX_HIP(hipStreamSynchronize(rs_stream(h)));
  }
  std::memcpy(results, h->h_io + o_out, sizeof(kmx_lcd_result) * n);
  if (inlier_masks) std::memcpy(inlier_masks, h->h_io + o_out + rb, (size_t)n * h->N);
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_lcd_enable_timing(kmx_lcd* h, int enable) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  h->timing = enable != 0;
  return KMX_OK;
}

extern "C" int kmx_lcd_read_timing(kmx_lcd* h, double* knn_ms, double* ransac_ms) {
  KMX_CHECK(h && knn_ms && ransac_ms, KMX_EINVAL, "null argument");
  KMX_CHECK(h->ev_ok, KMX_ESTATE, "no evented verification yet (kmx_lcd_enable_timing)");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->kstream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  for (hipStream_t x : h->rsx)
    if (x) KMX_HIP(hipStreamSynchronize(x));
  float a = 0.f, b = 0.f;
  KMX_HIP(hipEventElapsedTime(&a, h->ev[0], h->ev[1]));
  KMX_HIP(hipEventElapsedTime(&b, h->ev[1], h->ev[2]));
  *knn_ms = a;
  *ransac_ms = b;
  return KMX_OK;
}

extern "C" int kmx_lcd_sync(kmx_lcd* h) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->kstream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  for (hipStream_t x : h->rsx)
    if (x) KMX_HIP(hipStreamSynchronize(x));
  return KMX_OK;
}

// Stand-alone computeMatchedIndices on two host descriptor sets (one
// candidate through the same kernel; uses a temporary context on device 0
// of the calling thread's current device).
extern "C" int kmx_lcd_knn2(int norm, double lowe_ratio, const uint8_t* q, int32_t nq, const uint8_t* mdesc,
                            int32_t nm, int32_t* pairs_out, int32_t* k) {
  KMX_GUARD_BEGIN
  KMX_CHECK(k && pairs_out && (nq == 0 || q) && (nm == 0 || mdesc), KMX_EINVAL, "null argument");
  KMX_CHECK(nq >= 0 && nm >= 0 && nq <= MAX_FEATS && nm <= MAX_FEATS, KMX_EINVAL, "at most 1024 descriptors");
  KMX_CHECK(norm == KMX_NORM_L1 || norm == KMX_NORM_HAMMING, KMX_EINVAL, "bad norm");
  const int N = std::max(std::max(nq, nm), 1);
  std::vector<uint8_t> pool((size_t)2 * N * 32, 0);
  if (nq) std::memcpy(pool.data(), q, (size_t)nq * 32);
  if (nm) std::memcpy(pool.data() + (size_t)N * 32, mdesc, (size_t)nm * 32);
  int nf[2] = {nq, nm}, cq = 0, cm = 1;
  uint32_t* d_desc = nullptr;
  int *d_nf = nullptr, *d_c = nullptr, *d_K = nullptr;
  int2* d_pairs = nullptr;
  auto cleanup = [&]() {
    if (d_desc) (void)hipFree(d_desc);
    if (d_nf) (void)hipFree(d_nf);
    if (d_c) (void)hipFree(d_c);
    if (d_K) (void)hipFree(d_K);
    if (d_pairs) (void)hipFree(d_pairs);
  };
  if (hipMalloc(&d_desc, pool.size()) != hipSuccess || hipMalloc(&d_nf, sizeof(nf)) != hipSuccess ||
      hipMalloc(&d_c, 2 * sizeof(int)) != hipSuccess || hipMalloc(&d_K, sizeof(int)) != hipSuccess ||
      hipMalloc(&d_pairs, sizeof(int2) * N) != hipSuccess) {
    cleanup();
    return kmx::fail(KMX_ENOMEM, "hipMalloc");
  }
  int cc[2] = {cq, cm};
  hipError_t e = hipMemcpy(d_desc, pool.data(), pool.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_nf, nf, sizeof(nf), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_c, cc, sizeof(cc), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_knn2, dim3(1), dim3(KNN_BLOCK), (size_t)N * 32 + sizeof(int) * (KNN_BLOCK + 1), 0,
                       (const uint32_t*)d_desc, (const int*)d_nf, N, (const int*)d_c, (const int*)(d_c + 1), norm,
                       lowe_ratio, d_pairs, d_K);
    e = hipGetLastError();
  }
  int K = 0;
  std::vector<int2> pr(N);
  if (e == hipSuccess) e = hipMemcpy(&K, d_K, sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && K > 0) e = hipMemcpy(pr.data(), d_pairs, sizeof(int2) * K, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return kmx::fail(KMX_EHIP, hipGetErrorString(e));
  for (int i = 0; i < K; ++i) {
    pairs_out[2 * i] = pr[i].x;
    pairs_out[2 * i + 1] = pr[i].y;
  }
  *k = K;
  return KMX_OK;
  KMX_GUARD_END
}

// Diagnostic (KMX_RS_PROF=2): the per-candidate wave start / end stamps of the
// last launch, n <= 65536 pairs.
extern "C" int kmx_lcd_debug_wave_stamps(unsigned long long* out, int n) {
  n = std::max(0, std::min(n, STAMPS));
  KMX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(unsigned long long) * 2 * n));
  return KMX_OK;
}

// Diagnostic: read (and reset) the k_ransac_coop phase timers (wall-clock ticks).
extern "C" int kmx_lcd_debug_phase_times(unsigned long long* out16) {
  KMX_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 16));
  unsigned long long z[16] = {};
  KMX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)));
  return KMX_OK;
}
