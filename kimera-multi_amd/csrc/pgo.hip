// pgo.hip — MI355X (gfx950) RBCD block updates on lifted SE(3) with GNC-TLS.
//
// Replaces dpgo's PGOAgent::iterate / updateMeasurementWeights hot path
// (drawio:2058-2066, 2215, 2513). Design:
//   * Every local robot block lives in HBM; all blocks are updated by the same
//     launches (batched RBCD). Workgroup tiles never straddle robots, so every
//     reduction is per robot and its control scalars (trust radius, tCG alpha /
//     beta, ...) live on the device in a Ctl record per robot. The host never
//     reads a scalar inside a round: the tCG loop is a fixed launch sequence and
//     finished robots' tiles exit at their first instruction.
//   * Thread <-> (pose, row): the Euclidean Hessian-vector product X -> XQ acts
//     on each of the r rows of a pose independently, so a lane owns one row
//     (4 doubles) of one pose and a pose is a group of r lanes of one wave.
//     Only the Stiefel projection / retraction need sums over the r rows, done
//     with in-group shuffles in a fixed order.
//   * Node-centric gather over a CSR incidence list (no atomics): every output
//     element accumulates its incident edges in increasing edge id, the same
//     order as the CPU restatement's edge loop (FMA contraction on: per-element
//     results agree with the oracle to ~1e-15; `make FPC=off` reproduces its
//     roundings).
//   * Reductions: one partial per workgroup tile, reduced in fixed order by a
//     one-workgroup control kernel that also runs the RTR / tCG scalar logic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <vector>

#include "common.h"

namespace {

constexpr int WAVES = 4;
// Minimum waves per SIMD for the gather kernels (k_grad / k_hess / k_cost):
// caps their VGPRs so enough waves are resident to hide the gather latency.
#ifndef KMX_LB_GATHER
#define KMX_LB_GATHER 5
#endif
constexpr int BLOCK = 64 * WAVES;
constexpr int NPART = 4;  // partial sums per tile
// per-kernel LDS reduction area: NPART x WAVES wave sums + the ticket flag
constexpr int RED_BYTES = 8 * NPART * WAVES + 16;

enum Phase { PH_IDLE = 0, PH_START = 1, PH_TCG = 2, PH_STEP = 3 };
enum Mode { MODE_INTERIOR = 0, MODE_BOUNDARY = 1 };
enum RedKind { RED_GRAD = 0, RED_HESS = 1, RED_UPDATE = 2, RED_COST = 3 };

struct Ctl {
  int phase, rtr_iter, tcg_iter, tcg_stop;
  int mode, accepted, commit, updated;
  int hessvecs, skipped, pad0, pad1;
  double Delta, f_init, gn_init, f_cur;
  double f_final, norm_r0, z_r, e_Pe;
  double e_Pd, d_Pd, alpha, beta;
  double coef, rho, chg_acc, rel_change;
};

struct Counters {
  unsigned long long edges_iters;
  unsigned long long block_updates;
  unsigned long long hessvecs;
  unsigned long long pad;
  double hess_alg_bytes;
  double pad2[3];
};

// Host-visible progress of one robot after a tCG step, written by the robot's
// k_reduce(RED_UPDATE) workgroup into host-mapped memory as ONE 64-bit word
// (seq << 1 | still-in-tCG): a single relaxed system-scope store needs no
// release fence, so no L2 writeback is forced. The host enqueues further tCG
// steps only while a robot is in tCG.
struct HostStatus {
  unsigned long long word;
};
__device__ __forceinline__ void post_status(HostStatus* hs, int l, unsigned long long seq, bool running) {
  __hip_atomic_store(&hs[l].word, (seq << 1) | (running ? 1ull : 0ull), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Params {
  int tcg_max, rtr_iters, use_precond, robust;
  double kappa, theta, Delta0, Delta_max, accept_rho, gn_tol, shift, barc;
};

struct Dev {
  int ntiles, L, nloc, npub;
  const int* tile_robot;
  const int* tile_p0;
  const int* tile_np;
  const int* rtile0;  // [L+1]
  const int* inc_ptr; // [nloc+1]
  const int2* inc;    // x = other (>=0 local pose, <0 -> public slot -1-x); y = edge | tail<<31
  double* irec;       // [ninc][16] per-incidence edge record in CSR order: R(9) t(3) w*kappa w*tau 0 0
  double* crec;       // [ninc][12] compact record (gather variant 3): R rows 0-1 (6) t(3) w*kappa w*tau
                      // {other, edge|tail<<31} — R row 2 = row 0 x row 1 (used only when every
                      // local measurement rotation satisfies that to 1e-12; see kmx_pgo_set_graph)
  double* ocrec;      // [m_own][12] compact records of the owner incidences only (each local edge
                      // once: the tail of a local-local edge, the local end of a shared one), CSR by pose
  const int* optr;    // [nloc+1] CSR pointers into ocrec
  const int2* eopos;  // [mloc] positions of each local edge in ocrec (a shared edge with both
                      // robots on this handle has two owner incidences; -1 = none)
  double* ekappa;     // [mloc] per local edge
  double* etau;
  double* ew;         // GNC weight
  const int2* eipos;  // [mloc] incidence positions (tail, head) of each local edge, -1 if not local
  const int2* cipos;  // [mloc] the same positions in crec (differs from eipos in the segment-major layout)
  const int* trec0;   // [ntiles] segment-major layout (rect): first crec record of each tile
  const int* torec0;  // [ntiles] ... and of ocrec
  int rect;           // crec / ocrec in segment-major order (gather G = 5/6 only)
  double* hrec;       // [ninc + 1][12] compact records in CSR order for the G = 9 Hessian gather
                      // (+ one zero pad record), null when that gather is off
  double* hD;         // [nloc][16] diagonal blocks of Q per pose (G = 9), written by k_precond
  double* hocrec;     // [m_own + 1][12] owner compact records in CSR order (G = 9 k_cost) + pad
  const int2* heopos; // [mloc] positions of each local edge in hocrec
  int dbg;            // diagnostic ablations (KMX_PGO_DBG; 0 in the product path)
  double *X, *Xt, *g, *r, *z, *eta, *del, *hd, *S, *Pinv, *pub;
  double* part;       // [ntiles][NPART]
  Ctl* ctl;
  Counters* cnt;
  unsigned* tickets;         // [L] per-robot arrival counters (zero between launches)
  const long long* m_robot;  // [L] local-problem edges per robot
  const int* n_robot;        // [L] poses per robot
  Params p;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sum over all BLOCK threads in fixed order; every thread gets the result.
__device__ __forceinline__ double block_sum(double v, double* lds) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) s += lds[w];
  return s;
}

// Sum of x over the R lanes of this lane's pose group, lane order 0..R-1
// (the order of the oracle's row loop); identical in every lane of the group.
template <int R>
__device__ __forceinline__ double gsum(double x, int base) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k) s += __shfl(x, base + k, 64);
  return s;
}

__device__ __forceinline__ void load4(const double* p, double v[4]) {
  const double2* q = reinterpret_cast<const double2*>(p);
  double2 a = q[0], b = q[1];
  v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}
__device__ __forceinline__ void store4(double* p, const double v[4]) {
  double2* q = reinterpret_cast<double2*>(p);
  q[0] = make_double2(v[0], v[1]);
  q[1] = make_double2(v[2], v[3]);
}

struct Edge {
  double R[9], t[3], wk, wt;
};
// Accumulate the contribution of one incidence to row a of pose `self`.
// vs = self row, vo = other endpoint row (zeros for a Hessian product across a
// shared edge). Expressions mirror oracle/dpgo_oracle.c edge_eval exactly.
// Returns the row's share of 1/2 w (kappa |E_R|^2 + tau E_t^2).
__device__ __forceinline__ double incidence_row(const Edge& E, bool self_tail, const double vs[4],
                                                const double vo[4], double acc[4]) {
  double ER[3], Et;
  if (self_tail) {  // self = i (tail), other = j (head)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      ER[c] = vo[c] - (vs[0] * E.R[0 * 3 + c] + vs[1] * E.R[1 * 3 + c] + vs[2] * E.R[2 * 3 + c]);
    Et = vo[3] - vs[3] - (vs[0] * E.t[0] + vs[1] * E.t[1] + vs[2] * E.t[2]);
#pragma unroll
    for (int c = 0; c < 3; ++c)
      acc[c] -= E.wk * (ER[0] * E.R[c * 3 + 0] + ER[1] * E.R[c * 3 + 1] + ER[2] * E.R[c * 3 + 2]) +
                E.wt * Et * E.t[c];
    acc[3] -= E.wt * Et;
  } else {  // self = j (head), other = i (tail)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      ER[c] = vs[c] - (vo[0] * E.R[0 * 3 + c] + vo[1] * E.R[1 * 3 + c] + vo[2] * E.R[2 * 3 + c]);
    Et = vs[3] - vo[3] - (vo[0] * E.t[0] + vo[1] * E.t[1] + vo[2] * E.t[2]);
    acc[0] += E.wk * ER[0];
    acc[1] += E.wk * ER[1];
    acc[2] += E.wk * ER[2];
    acc[3] += E.wt * Et;
  }
  return 0.5 * (E.wk * (ER[0] * ER[0] + ER[1] * ER[1] + ER[2] * ER[2]) + E.wt * Et * Et);
}

// S = sym(Y^T G_Y) for the pose group (9 entries, identical in all R lanes):
// the 6 distinct entries are group sums of the symmetrised products. Each sum
// is chained to the previous one (empty asm) so only one sum's R shuffles are
// in flight: interleaving all of them held ~90 VGPRs and capped k_hess at 3
// waves/SIMD.
//
// LDS = true (kernels that own a free BLOCK x 6-double LDS scratch `scr`): every
// lane writes its 6 products, then reads its group's R x 6 back and adds them
// in the same lane order, so the 6 sums cost one LDS round trip instead of 6
// chained shuffle chains. Only lanes of one wave exchange data (in-order LDS
// queue; no workgroup barrier).
template <int R, bool LDS = false>
__device__ __forceinline__ void group_symYtG(const double y[4], const double G[4], int base, double S[9],
                                             double* scr = nullptr) {
  if constexpr (LDS) {
    double* mine = scr + 6 * threadIdx.x;
    {
      int j = 0;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = c; k < 3; ++k) mine[j++] = 0.5 * (y[c] * G[k] + y[k] * G[c]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const double* grp = scr + 6 * ((threadIdx.x & ~63u) + base);
    double t[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = 0; m < R; ++m)
#pragma unroll
      for (int j = 0; j < 6; ++j) t[j] += grp[6 * m + j];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int j = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int k = c; k < 3; ++k, ++j) {
        S[c * 3 + k] = t[j];
        S[k * 3 + c] = t[j];
      }
  } else {
    double prev = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int k = c; k < 3; ++k) {
        double x = 0.5 * (y[c] * G[k] + y[k] * G[c]);
        asm volatile("" : "+v"(x) : "v"(prev));
        prev = gsum<R>(x, base);
        S[c * 3 + k] = prev;
        S[k * 3 + c] = prev;
      }
  }
}

// Tangent projection of row V at Y (group-cooperative): V_Y - Y sym(Y^T V_Y).
template <int R, bool LDS = false>
__device__ __forceinline__ void group_proj(const double y[4], const double V[4], int base, double out[4],
                                           double* scr = nullptr) {
  double S[9];
  group_symYtG<R, LDS>(y, V, base, S, scr);
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c] = V[c] - (y[0] * S[0 * 3 + c] + y[1] * S[1 * 3 + c] + y[2] * S[2 * 3 + c]);
  out[3] = V[3];
}

template <int R, bool LDS = false>
__device__ __forceinline__ void group_precon(const Dev& d, int pose, bool valid, const double y[4],
                                             const double V[4], int base, double out[4], double* scr = nullptr) {
  double buf[4] = {0.0, 0.0, 0.0, 0.0};
  if (d.p.use_precond) {
    const double* Pp = d.Pinv + 16 * (size_t)pose;
    if constexpr (LDS) {
      // the 128-VGPR kernels: all of P in flight at once (pose is a valid
      // index on every lane: lane_map clamps idle lanes to the tile's first pose)
      double P[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) load4(Pp + 4 * i, P + 4 * i);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) buf[k] = (i == 0) ? V[0] * P[k] : buf[k] + V[i] * P[4 * i + k];
    } else {
      // buf = V P, one 4-double row of P at a time (keeps 8 VGPRs of P live)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double Pr[4] = {0.0, 0.0, 0.0, 0.0};
        if (valid) load4(Pp + 4 * i, Pr);
        asm volatile("" : "+v"(Pr[0]), "+v"(Pr[1]), "+v"(Pr[2]), "+v"(Pr[3]) : "v"(buf[0]));
#pragma unroll
        for (int k = 0; k < 4; ++k) buf[k] = (i == 0) ? V[0] * Pr[k] : buf[k] + V[i] * Pr[k];
      }
    }
    group_proj<R, LDS>(y, buf, base, out, scr);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = V[k];
  }
}

// Riemannian Hessian row of V given the Euclidean Hessian row H:
// P_Y(H_Y - V_Y S) ; p-part H_p.
template <int R, bool LDS = false>
__device__ __forceinline__ void group_rhess(const double y[4], const double V[4], const double H[4],
                                            const double S[9], int base, double out[4], double* scr = nullptr) {
  double buf[4];
#pragma unroll
  for (int k = 0; k < 3; ++k) buf[k] = H[k] - (V[0] * S[0 * 3 + k] + V[1] * S[1 * 3 + k] + V[2] * S[2 * 3 + k]);
  buf[3] = H[3];
  group_proj<R, LDS>(y, buf, base, out, scr);
}

// QF retraction (modified Gram-Schmidt over the 3 columns, positive diagonal).
template <int R>
__device__ __forceinline__ void group_retract(const double x[4], const double v[4], int base, double out[4]) {
  double A[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) A[c] = x[c] + v[c];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int k = 0; k < c; ++k) {
      const double s = gsum<R>(A[k] * A[c], base);
      A[c] -= s * A[k];
    }
    const double nn = gsum<R>(A[c] * A[c], base);
    const double inv = 1.0 / sqrt(nn);
    A[c] *= inv;
  }
  out[0] = A[0]; out[1] = A[1]; out[2] = A[2];
  out[3] = x[3] + v[3];
}

struct Lane {
  int tile, l, w, ln, pw, a, base, pose;
  bool valid;
};
template <int R>
__device__ __forceinline__ Lane lane_map(const Dev& d) {
  constexpr int PPW = 64 / R;
  Lane L;
  // XCD-aware, bijective block -> tile remap (cdna_hip_programming.md T1):
  // blocks b and b + 8 share an XCD, so each XCD gets one contiguous range of
  // tiles — i.e. (about) one robot block, whose iterate then stays in that
  // XCD's 4 MiB L2 across the gathers of every kernel of the round.
  {
    const int nwg = gridDim.x, b = blockIdx.x;
    const int q = nwg >> 3, rr = nwg & 7, x = b & 7;
    L.tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  L.l = d.tile_robot[L.tile];
  L.w = threadIdx.x >> 6;
  L.ln = threadIdx.x & 63;
  L.pw = L.ln / R;
  L.a = L.ln - L.pw * R;
  L.base = L.pw * R;
  const int local = L.w * PPW + L.pw;
  L.valid = (L.pw < PPW) && (local < d.tile_np[L.tile]);
  L.pose = d.tile_p0[L.tile] + (L.valid ? local : 0);
  if (L.base + R > 64) L.base = 64 - R;  // idle tail lanes shuffle within range
  return L;
}

// ---------------------------------------------------------------- kernels --
// Direct variant (G = 0): each (pose, row) lane walks its pose's incidences
// with per-lane global loads (every lane of the pose loads the edge record).
struct EdgeRaw {
  double2 q[8];
};
__device__ __forceinline__ void edge_from_raw(const EdgeRaw& w, Edge& E) {
  E.R[0] = w.q[0].x; E.R[1] = w.q[0].y; E.R[2] = w.q[1].x; E.R[3] = w.q[1].y; E.R[4] = w.q[2].x;
  E.R[5] = w.q[2].y; E.R[6] = w.q[3].x; E.R[7] = w.q[3].y; E.R[8] = w.q[4].x;
  E.t[0] = w.q[4].y; E.t[1] = w.q[5].x; E.t[2] = w.q[5].y;
  E.wk = w.q[6].x;
  E.wt = w.q[6].y;
}

template <int R, bool PUB>
__device__ __forceinline__ void fetch_incidence(const Dev& d, const double* V, const double* pub, int a, int k,
                                                int2 in, EdgeRaw& w, double2& v0, double2& v1) {
  const double2* q2 = reinterpret_cast<const double2*>(d.irec + 16 * (size_t)k);
#pragma unroll
  for (int i = 0; i < 8; ++i) w.q[i] = q2[i];
  const int o = in.x;
  const double* base = (o >= 0) ? V + (size_t)o * 4 * R : (PUB ? pub + (size_t)(-1 - o) * 4 * R : V);
  const double2* b2 = reinterpret_cast<const double2*>(base + 4 * a);
  v0 = b2[0];
  v1 = b2[1];
  if (!PUB && o < 0) v0 = v1 = make_double2(0.0, 0.0);
}

// Direct variant (G = 0): each (pose, row) lane walks its pose's incidences in
// CSR order, software-pipelined: incidence k+1's edge record and neighbour row
// are in flight while k is computed, and the CSR entry of k+2 while k+1 loads.
template <int R, bool PUB>
__device__ __forceinline__ void lane_gather(const Dev& d, const Lane& L, const double* V, const double* pub,
                                            double acc[4], double* cost) {
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  if (!L.valid) return;
  double vs[4];
  load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
  const int k0 = d.inc_ptr[L.pose], k1 = d.inc_ptr[L.pose + 1];
  if (k0 >= k1) return;
  int2 inA = d.inc[k0];
  int2 inB = (k0 + 1 < k1) ? d.inc[k0 + 1] : inA;
  EdgeRaw wA, wB;
  double2 a0, a1, b0, b1;
  fetch_incidence<R, PUB>(d, V, pub, L.a, k0, inA, wA, a0, a1);
  for (int k = k0; k < k1; ++k) {
    const bool more = (k + 1 < k1);
    if (more) fetch_incidence<R, PUB>(d, V, pub, L.a, k + 1, inB, wB, b0, b1);
    const int2 inC = (k + 2 < k1) ? d.inc[k + 2] : inB;
    Edge E;
    edge_from_raw(wA, E);
    const double vo[4] = {a0.x, a0.y, a1.x, a1.y};
    const bool tail = (inA.y >> 31) & 1;
    const double c = incidence_row(E, tail, vs, vo, acc);
    if (cost) *cost += (inA.x >= 0) ? 0.5 * c : c;
    wA = wB;
    a0 = b0;
    a1 = b1;
    inA = inB;
    inB = inC;
  }
}

// Incidence-parallel tile gather (variant G = 1). A tile's poses are
// contiguous, so its incidences are one contiguous CSR range. The tile walks
// it in chunks of CI = 256 / r incidences:
//   * the tile's CSR entries and its own pose rows are staged in LDS once;
//   * per chunk, every edge record is loaded ONCE (8 lanes x 16 B) into LDS,
//     and lane (incidence i, row a) loads neighbour row a straight into
//     registers (r lanes read one contiguous 32r-byte pose row);
//   * lane (i, a) forms its incidence's contribution to row a of the self pose
//     and parks it in LDS; then each (pose, row) lane adds its pose's
//     contributions in CSR (= increasing edge id) order — the same order and
//     the same (exactly negated) terms as the oracle, so results stay bitwise
//     identical;
//   * the next chunk's loads are issued before the current chunk is computed.
template <int R>
struct Smem {
  static constexpr int PPW = 64 / R;
  static constexpr int TP = WAVES * PPW;           // poses per tile
  static constexpr int CI = BLOCK / R;             // incidences per chunk
  static constexpr int MAXI = 512;                 // CSR entries staged per segment
  static constexpr int inc_off = 0;                                   // int2[MAXI]
  static constexpr int ptr_off = inc_off + MAXI * 8;                  // int[TP + 1]
  static constexpr int x_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;  // double[TP][R][4]
  static constexpr int edge_off = x_off + TP * R * 32;                // double[CI][16]
  static constexpr int con_off = edge_off + CI * 128;                 // double[CI][R][4]
  static constexpr int red_off = con_off + CI * R * 32;               // double[WAVES] + flag
  static constexpr int bytes = red_off + RED_BYTES;
};

template <int R, bool PUB>
__device__ __forceinline__ void tile_gather(const Dev& d, const Lane& L, const double* V, const double* pub,
                                            double acc[4], double* cost, char* smem) {
  using SM = Smem<R>;
  constexpr int CI = SM::CI;
  constexpr int E_IT = (CI * 8 + BLOCK - 1) / BLOCK;
  int2* sinc = reinterpret_cast<int2*>(smem + SM::inc_off);
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  double* sx = reinterpret_cast<double*>(smem + SM::x_off);
  double* sedge = reinterpret_cast<double*>(smem + SM::edge_off);
  double* scon = reinterpret_cast<double*>(smem + SM::con_off);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = d.inc_ptr[p0], K1 = d.inc_ptr[p0 + np];
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  {
    const double2* src = reinterpret_cast<const double2*>(V + (size_t)p0 * 4 * R);
    double2* dst = reinterpret_cast<double2*>(sx);
    for (int q = tid; q < np * 2 * R; q += BLOCK) dst[q] = src[q];
  }
  int kp0 = 0, kp1 = 0;
  if (L.valid) {
    kp0 = d.inc_ptr[L.pose];
    kp1 = d.inc_ptr[L.pose + 1];
  }
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  const int ci = tid / R, ca = tid - ci * R;  // compute lane (incidence, row)
  double csum = 0.0;
  for (int seg = K0; seg < K1; seg += SM::MAXI) {
    const int nseg = min(SM::MAXI, K1 - seg);
    for (int q = tid; q < nseg; q += BLOCK) sinc[q] = d.inc[seg + q];
    __syncthreads();
    static_assert(E_IT <= 3, "edge staging assumes <= 3 pieces per lane");
    double2 eb0 = make_double2(0.0, 0.0), eb1 = eb0, eb2 = eb0, v0 = eb0, v1 = eb0;
#define KMX_LOAD_CHUNK(CB)                                                                         \
    {                                                                                              \
      const int n_ = min(CI, nseg - (CB));                                                         \
      const double2* er2 = reinterpret_cast<const double2*>(d.irec);                               \
      {                                                                                            \
        const int q = tid, qc = (q < n_ * 8) ? q : 0;                                              \
        eb0 = er2[16 / 2 * (size_t)(seg + (CB) + (qc >> 3)) + (qc & 7)];                          \
      }                                                                                            \
      if constexpr (E_IT > 1) {                                                                    \
        const int q = tid + BLOCK, qc = (q < n_ * 8) ? q : 0;                                      \
        eb1 = er2[16 / 2 * (size_t)(seg + (CB) + (qc >> 3)) + (qc & 7)];                          \
      }                                                                                            \
      if constexpr (E_IT > 2) {                                                                    \
        const int q = tid + 2 * BLOCK, qc = (q < n_ * 8) ? q : 0;                                  \
        eb2 = er2[16 / 2 * (size_t)(seg + (CB) + (qc >> 3)) + (qc & 7)];                          \
      }                                                                                            \
      const int ic = (ci < n_) ? ci : 0;                                                           \
      const int o = sinc[(CB) + ic].x;                                                             \
      const double* base = (o >= 0) ? V + (size_t)o * 4 * R : (PUB ? pub + (size_t)(-1 - o) * 4 * R : V); \
      const double2* b2 = reinterpret_cast<const double2*>(base + 4 * ca);                         \
      v0 = b2[0];                                                                                  \
      v1 = b2[1];                                                                                  \
      if (!PUB && o < 0) v0 = v1 = make_double2(0.0, 0.0);                                         \
    }
    KMX_LOAD_CHUNK(0)
    for (int cb = 0; cb < nseg; cb += CI) {
      const int n = min(CI, nseg - cb);
      if (tid < n * 8) reinterpret_cast<double2*>(sedge)[tid] = eb0;
      if (E_IT > 1 && tid + BLOCK < n * 8) reinterpret_cast<double2*>(sedge)[tid + BLOCK] = eb1;
      if (E_IT > 2 && tid + 2 * BLOCK < n * 8) reinterpret_cast<double2*>(sedge)[tid + 2 * BLOCK] = eb2;
      const double2 c0 = v0, c1 = v1;
      __syncthreads();
      if (cb + CI < nseg) KMX_LOAD_CHUNK(cb + CI)  // next chunk in flight during compute
      if (ci < n && tid < CI * R) {
        const int kk = (seg - K0) + cb + ci;  // tile-relative incidence index
        int lo = 0, hi = np;                  // self pose: sptr[lo] <= kk < sptr[lo + 1]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (sptr[mid] <= kk) lo = mid;
          else hi = mid;
        }
        const int2 in = sinc[cb + ci];
        const bool tail = (in.y >> 31) & 1;
        const double2* q2 = reinterpret_cast<const double2*>(sedge + 16 * ci);
        double2 w0 = q2[0], w1 = q2[1], w2 = q2[2], w3 = q2[3], w4 = q2[4], w5 = q2[5], w6 = q2[6];
        Edge E;
        E.R[0] = w0.x; E.R[1] = w0.y; E.R[2] = w1.x; E.R[3] = w1.y; E.R[4] = w2.x;
        E.R[5] = w2.y; E.R[6] = w3.x; E.R[7] = w3.y; E.R[8] = w4.x;
        E.t[0] = w4.y; E.t[1] = w5.x; E.t[2] = w5.y;
        E.wk = w6.x;
        E.wt = w6.y;
        double vs[4], vo[4] = {c0.x, c0.y, c1.x, c1.y}, con[4] = {0.0, 0.0, 0.0, 0.0};
        load4(sx + (lo * R + ca) * 4, vs);
        const double c = incidence_row(E, tail, vs, vo, con);
        csum += (in.x >= 0) ? 0.5 * c : c;
        store4(scon + (ci * R + ca) * 4, con);
      }
      __syncthreads();
      if (L.valid) {
        const int A = seg + cb;
        const int ka = max(kp0, A), kb = min(kp1, A + n);
        for (int k = ka; k < kb; ++k) {
          double cv[4];
          load4(scon + ((k - A) * R + L.a) * 4, cv);
          acc[0] += cv[0]; acc[1] += cv[1]; acc[2] += cv[2]; acc[3] += cv[3];
        }
      }
      __syncthreads();
    }
  }
  if (cost) *cost += csum;
#undef KMX_LOAD_CHUNK
}

// Plain direct variant (G = 2, diagnostic): no software pipelining.
template <int R, bool PUB>
__device__ __forceinline__ void lane_gather_plain(const Dev& d, const Lane& L, const double* V, const double* pub,
                                                  double acc[4], double* cost) {
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  if (!L.valid) return;
  double vs[4];
  load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
  const int k0 = d.inc_ptr[L.pose], k1 = d.inc_ptr[L.pose + 1];
  for (int k = k0; k < k1; ++k) {
    const int2 in = d.inc[k];
    EdgeRaw w;
    double2 b0, b1;
    fetch_incidence<R, PUB>(d, V, pub, L.a, k, in, w, b0, b1);
    Edge E;
    edge_from_raw(w, E);
    const double vo[4] = {b0.x, b0.y, b1.x, b1.y};
    const double c = incidence_row(E, (in.y >> 31) & 1, vs, vo, acc);
    if (cost) *cost += (in.x >= 0) ? 0.5 * c : c;
  }
}

// Compact-record variant (G = 3): 96-B records carry the neighbour index, so
// the incidence loop reads one record (6 x 16 B) and one neighbour row — no
// separate CSR entry — and the third rotation row is rebuilt as row0 x row1.
// OWN (cost only, G = 4): visit each edge once — the tail incidence of a
// local-local edge, or the only local incidence of a shared edge — from a
// second compact array holding just those records (half the record bytes).
__device__ __forceinline__ int2 unpack_int2(double v) {
  const long long b = __double_as_longlong(v);
  return make_int2((int)(b & 0xffffffffll), (int)(b >> 32));
}
__device__ __forceinline__ void edge_from_compact(const double2 q[6], Edge& E) {
  E.R[0] = q[0].x; E.R[1] = q[0].y; E.R[2] = q[1].x;
  E.R[3] = q[1].y; E.R[4] = q[2].x; E.R[5] = q[2].y;
  E.R[6] = E.R[1] * E.R[5] - E.R[2] * E.R[4];
  E.R[7] = E.R[2] * E.R[3] - E.R[0] * E.R[5];
  E.R[8] = E.R[0] * E.R[4] - E.R[1] * E.R[3];
  E.t[0] = q[3].x; E.t[1] = q[3].y; E.t[2] = q[4].x;
  E.wk = q[4].y;
  E.wt = q[5].x;
}

template <int R, bool PUB, bool OWN>
__device__ __forceinline__ void lane_gather_compact(const Dev& d, const Lane& L, const double* V,
                                                    const double* pub, double acc[4], double* cost) {
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  if (!L.valid) return;
  double vs[4];
  load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
  const int* ptr = OWN ? d.optr : d.inc_ptr;
  const double* rec = OWN ? d.ocrec : d.crec;
  const int k0 = ptr[L.pose], k1 = ptr[L.pose + 1];
  for (int k = k0; k < k1; ++k) {
    const double2* q2 = reinterpret_cast<const double2*>(rec + 12 * (size_t)k);
    double2 q[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = q2[i];
    const int2 in = unpack_int2(q[5].y);
    const int o = in.x;
    const double* base = (o >= 0) ? V + (size_t)o * 4 * R : (PUB ? pub + (size_t)(-1 - o) * 4 * R : V);
    const double2* b2 = reinterpret_cast<const double2*>(base + 4 * L.a);
    double2 v0 = b2[0], v1 = b2[1];
    if (!PUB && o < 0) v0 = v1 = make_double2(0.0, 0.0);
    Edge E;
    edge_from_compact(q, E);
    const double vo[4] = {v0.x, v0.y, v1.x, v1.y};
    const double c = incidence_row(E, (in.y >> 31) & 1, vs, vo, acc);
    if (cost) *cost += (OWN || o < 0) ? c : 0.5 * c;
  }
}

// Degree-balanced compact gather (G = 5; G = 6: owner-only cost). A tile's
// incidences are one contiguous CSR range; it is cut into TP equal segments,
// one per lane group, so every group walks ~the mean degree instead of the
// wave waiting for its highest-degree pose (capping the per-pose walk at the
// mean degree halves the gather time: k_gcap). A segment can
// span several poses; each (group, pose) partial is flushed to LDS: the
// first group of a pose writes A[pose], a group that starts inside a pose
// (the continuation) writes H[group]. The (pose, row) lanes then add
// A[pose] + H[g] for the pose's later segments in order, so the result is
// deterministic and independent of everything but the tiling.
template <int R, bool PUB, bool OWN>
__device__ __forceinline__ void tile_gather_bal(const Dev& d, const Lane& L, const double* V, const double* pub,
                                                double acc[4], double* cost, char* smem) {
  using SM = Smem<R>;
  constexpr int TP = SM::TP;
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);          // [TP + 1] tile-local CSR
  double* A = reinterpret_cast<double*>(smem + SM::x_off);         // [TP][R][4]
  double* H = reinterpret_cast<double*>(smem + SM::con_off);       // [TP][R][4]
  const int* ptr = OWN ? d.optr : d.inc_ptr;
  const double* rec = OWN ? d.ocrec : d.crec;
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = ptr[p0];
  const bool rect = d.rect != 0;
  const int rbase = rect ? (OWN ? d.torec0 : d.trec0)[L.tile] : 0;
  __syncthreads();  // LDS reuse across consecutive gathers in one kernel (k_eval)
  if (tid <= np) sptr[tid] = ptr[p0 + tid] - K0;
  if constexpr (!OWN)
    for (int i = tid; i < TP * R * 4; i += BLOCK) A[i] = 0.0;
  __syncthreads();
  const int n = sptr[np];
  const int S = max(1, (n + TP - 1) / TP);
  const int g = L.w * (64 / R) + L.pw;  // group = (wave, pose slot)
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  double csum = 0.0;
  const bool gvalid = (L.pw < 64 / R);
  const int s0 = gvalid ? g * S : n, s1 = gvalid ? min(s0 + S, n) : n;
  if (s0 < s1) {
    int lo = 0, hi = np;  // pose containing s0: sptr[lo] <= s0 < sptr[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sptr[mid] <= s0) lo = mid;
      else hi = mid;
    }
    while (sptr[lo + 1] <= s0) ++lo;  // skip zero-degree poses
    int p = lo;
    bool head = s0 > sptr[p];
    // self row of the current pose, and (prefetched) of the next pose with
    // incidences, so crossing a pose boundary does not wait on memory
    auto next_pose = [&](int q) {
      do ++q;
      while (q < np - 1 && sptr[q + 1] == sptr[q]);
      return q;
    };
    double vs[4], vn[4] = {0.0, 0.0, 0.0, 0.0};
    load4(V + (size_t)(p0 + p) * 4 * R + 4 * L.a, vs);
    int pn = next_pose(p);
    if (pn < np && sptr[pn] < s1) load4(V + (size_t)(p0 + pn) * 4 * R + 4 * L.a, vn);
    int pend = sptr[p + 1];
    for (int k = s0; k < s1; ++k) {
      if (k >= pend) {  // next pose: flush this one's partial
        if constexpr (!OWN) store4((head ? H + (g * R + L.a) * 4 : A + (p * R + L.a) * 4), part);
        part[0] = part[1] = part[2] = part[3] = 0.0;
        head = false;
        p = pn;
        pend = sptr[p + 1];
        vs[0] = vn[0]; vs[1] = vn[1]; vs[2] = vn[2]; vs[3] = vn[3];
        pn = next_pose(p);
        if (pn < np && sptr[pn] < s1) load4(V + (size_t)(p0 + pn) * 4 * R + 4 * L.a, vn);
      }
      // segment-major layout: step j of every group of the tile is one run of
      // consecutive records, so a wave's 12 groups read 1152 contiguous bytes
      const size_t ri = rect ? (size_t)rbase + (size_t)(k - s0) * TP + g : (size_t)(K0 + k);
      const double2* q2 = reinterpret_cast<const double2*>(rec + 12 * ri);
      double2 q[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) q[i] = q2[i];
      const int2 in = unpack_int2(q[5].y);
      const int o = in.x;
      const double* base = (o >= 0) ? V + (size_t)o * 4 * R : (PUB ? pub + (size_t)(-1 - o) * 4 * R : V);
      const double2* b2 = reinterpret_cast<const double2*>(base + 4 * L.a);
      double2 v0 = b2[0], v1 = b2[1];
      if (!PUB && o < 0) v0 = v1 = make_double2(0.0, 0.0);
      Edge E;
      edge_from_compact(q, E);
      const double vo[4] = {v0.x, v0.y, v1.x, v1.y};
      const double c = incidence_row(E, (in.y >> 31) & 1, vs, vo, part);
      csum += (OWN || o < 0) ? c : 0.5 * c;
    }
    if constexpr (!OWN) store4((head ? H + (g * R + L.a) * 4 : A + (p * R + L.a) * 4), part);
  }
  if (cost) *cost += csum;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  if constexpr (!OWN) {
    __syncthreads();
    if (L.valid) {
      const int p = L.pose - p0;
      load4(A + (p * R + L.a) * 4, acc);
      if (sptr[p + 1] > sptr[p]) {
        const int gf = sptr[p] / S, gl = (sptr[p + 1] - 1) / S;
        for (int gg = gf + 1; gg <= gl; ++gg) {
          double h[4];
          load4(H + (gg * R + L.a) * 4, h);
          acc[0] += h[0]; acc[1] += h[1]; acc[2] += h[2]; acc[3] += h[3];
        }
      }
    }
  }
}

// LDS-staged chunked gather (G = 7; G = 8: owner-only cost). The tile's
// incidences are cut into segments of SEG consecutive incidences; chunk c
// holds the NG = TP segments [c NG, (c + 1) NG), one per lane group. Per chunk:
//   * the chunk's compact records (one contiguous range, 96 B each) are
//     copied into LDS by the whole workgroup with full-line 16-B loads, so an
//     edge record crosses L2 -> L1 once instead of once per row lane and per
//     partially used line; the NEXT chunk's records are loaded into registers
//     while this chunk is computed (register-staged double buffer);
//   * every group reads its SEG neighbour indices from LDS and issues all SEG
//     neighbour-row loads at once, then consumes them in order;
//   * (group, pose) partials are flushed as in G = 5: the segment holding a
//     pose's first incidence writes A[pose], a segment that starts inside a
//     pose writes H[group]; after a barrier the (pose, row) lanes add their
//     pose's continuation segments of the chunk in segment order.
// Every pose's sum is therefore a fixed function of the tiling (deterministic).
template <int R, int SEG>
struct SmemL {
  static constexpr int PPW = 64 / R;
  static constexpr int TP = WAVES * PPW;  // poses per tile = lane groups per workgroup
  static constexpr int NG = TP;
  static constexpr int CH = NG * SEG;     // incidences per chunk
  static constexpr int NSL = (CH * 6 + BLOCK - 1) / BLOCK;  // 16-B staging slots per thread
  static constexpr int ptr_off = 0;                                      // int[TP + 1]
  static constexpr int a_off = ((TP + 1) * 4 + 15) / 16 * 16;            // double[TP][R][4]
  static constexpr int h_off = a_off + TP * R * 32;                      // double[NG][R][4]
  static constexpr int rec_off = h_off + NG * R * 32;                    // double[CH][12]
  static constexpr int red_off = rec_off + CH * 96;
  static constexpr int bytes = red_off + RED_BYTES;
};
#ifndef KMX_SEG
#define KMX_SEG 4
#endif
#ifndef KMX_GATHER_DEFAULT
#define KMX_GATHER_DEFAULT 5
#endif

template <int R, bool PUB, bool OWN, int SEG>
__device__ __forceinline__ void tile_gather_lds(const Dev& d, const Lane& L, const double* V, const double* pub,
                                                double acc[4], double* cost, char* smem) {
  using SM = SmemL<R, SEG>;
  constexpr int NG = SM::NG, CH = SM::CH, NSL = SM::NSL;
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  double* A = reinterpret_cast<double*>(smem + SM::a_off);
  double* H = reinterpret_cast<double*>(smem + SM::h_off);
  double2* lrec = reinterpret_cast<double2*>(smem + SM::rec_off);
  const int* ptr = OWN ? d.optr : d.inc_ptr;
  const double2* grec = reinterpret_cast<const double2*>(OWN ? d.ocrec : d.crec);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = ptr[p0];
  grec += (size_t)K0 * 6;
  __syncthreads();  // LDS reuse across consecutive gathers in one kernel (k_eval)
  if (tid <= np) sptr[tid] = ptr[p0 + tid] - K0;
  __syncthreads();
  const int n = sptr[np];
  const int nch = (n + CH - 1) / CH;
  const int g = L.w * (64 / R) + L.pw;
  const bool gvalid = (L.pw < 64 / R);
  double2 stg[NSL];
  auto issue = [&](int c) {
    const int base = c * CH * 6, cnt = min(CH, n - c * CH) * 6;
#pragma unroll
    for (int i = 0; i < NSL; ++i) {
      const int j = tid + i * BLOCK;
      if (j < cnt) stg[i] = grec[base + j];
    }
  };
  auto commit = [&](int c) {
    const int cnt = min(CH, n - c * CH) * 6;
#pragma unroll
    for (int i = 0; i < NSL; ++i) {
      const int j = tid + i * BLOCK;
      if (j < cnt) lrec[j] = stg[i];
    }
  };
  double csum = 0.0;
  if (nch > 0) issue(0);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();  // the previous chunk's records and H are no longer read
    commit(c);
    __syncthreads();
    const int s = c * NG + g;
    const int k0 = s * SEG, k1 = min(k0 + SEG, n);
    const bool work = gvalid && k0 < k1;
    double2 nb[SEG][2];
    if (work) {
#pragma unroll
      for (int j = 0; j < SEG; ++j) {
        nb[j][0] = nb[j][1] = make_double2(0.0, 0.0);
        if (k0 + j < k1) {
          const int o = unpack_int2(lrec[(k0 + j - c * CH) * 6 + 5].y).x;
          if (o >= 0 || PUB) {
            const double* base = (o >= 0) ? V + (size_t)o * 4 * R : pub + (size_t)(-1 - o) * 4 * R;
            const double2* b2 = reinterpret_cast<const double2*>(base + 4 * L.a);
            nb[j][0] = b2[0];
            nb[j][1] = b2[1];
          }
        }
      }
    }
    if (c + 1 < nch) issue(c + 1);  // next chunk's records fly while this one computes
    if (work) {
      int lo = 0, hi = np;  // pose containing k0: sptr[lo] <= k0 < sptr[lo + 1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (sptr[mid] <= k0) lo = mid;
        else hi = mid;
      }
      while (sptr[lo + 1] <= k0) ++lo;  // skip zero-degree poses
      int p = lo;
      bool head = k0 > sptr[p];
      int pend = sptr[p + 1];
      double vs[4];
      load4(V + (size_t)(p0 + p) * 4 * R + 4 * L.a, vs);
      double part[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int j = 0; j < SEG; ++j) {
        const int k = k0 + j;
        if (k < k1) {
          if (k >= pend) {  // next pose: flush this one's partial
            if constexpr (!OWN) store4((head ? H + (g * R + L.a) * 4 : A + (p * R + L.a) * 4), part);
            part[0] = part[1] = part[2] = part[3] = 0.0;
            head = false;
            do ++p;
            while (sptr[p + 1] <= k);
            pend = sptr[p + 1];
            load4(V + (size_t)(p0 + p) * 4 * R + 4 * L.a, vs);
          }
          const double2* q2 = lrec + (k - c * CH) * 6;
          double2 q[6];
#pragma unroll
          for (int i = 0; i < 6; ++i) q[i] = q2[i];
          Edge E;
          edge_from_compact(q, E);
          const int2 in = unpack_int2(q[5].y);
          const double vo[4] = {nb[j][0].x, nb[j][0].y, nb[j][1].x, nb[j][1].y};
          const double cc = incidence_row(E, (in.y >> 31) & 1, vs, vo, part);
          csum += (OWN || in.x < 0) ? cc : 0.5 * cc;
        }
      }
      if constexpr (!OWN) store4((head ? H + (g * R + L.a) * 4 : A + (p * R + L.a) * 4), part);
    }
    if constexpr (!OWN) {
      __syncthreads();
      if (L.valid) {  // fold this chunk's continuation segments of the lane's pose
        const int p = L.pose - p0;
        const int e0 = sptr[p], e1 = sptr[p + 1];
        if (e1 > e0) {
          const int sf = e0 / SEG, sl = (e1 - 1) / SEG;
          const int lo = max(sf + 1, c * NG), hi = min(sl, c * NG + NG - 1);
          if (lo <= hi) {
            double a4[4];
            load4(A + (p * R + L.a) * 4, a4);
            for (int ss = lo; ss <= hi; ++ss) {
              double h4[4];
              load4(H + ((ss - c * NG) * R + L.a) * 4, h4);
              a4[0] += h4[0]; a4[1] += h4[1]; a4[2] += h4[2]; a4[3] += h4[3];
            }
            store4(A + (p * R + L.a) * 4, a4);
          }
        }
      }
    }
  }
  if (cost) *cost += csum;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  if constexpr (!OWN) {
    if (L.valid) {
      const int p = L.pose - p0;
      if (sptr[p + 1] > sptr[p]) load4(A + (p * R + L.a) * 4, acc);  // the last fold's own writes
    }
  }
}

template <int R, int G, bool PUB>
__device__ __forceinline__ void gather(const Dev& d, const Lane& L, const double* V, const double* pub,
                                       double acc[4], double* cost, char* smem) {
  if constexpr (G == 0) lane_gather<R, PUB>(d, L, V, pub, acc, cost);
  else if constexpr (G == 2) lane_gather_plain<R, PUB>(d, L, V, pub, acc, cost);
  else if constexpr (G == 3) lane_gather_compact<R, PUB, false>(d, L, V, pub, acc, cost);
  else if constexpr (G == 4) lane_gather_compact<R, PUB, true>(d, L, V, pub, acc, cost);
  else if constexpr (G == 5) tile_gather_bal<R, PUB, false>(d, L, V, pub, acc, cost, smem);
  else if constexpr (G == 6) tile_gather_bal<R, PUB, true>(d, L, V, pub, acc, cost, smem);
  else if constexpr (G == 7) tile_gather_lds<R, PUB, false, KMX_SEG>(d, L, V, pub, acc, cost, smem);
  else if constexpr (G == 8) tile_gather_lds<R, PUB, true, KMX_SEG>(d, L, V, pub, acc, cost, smem);
  else tile_gather<R, PUB>(d, L, V, pub, acc, cost, smem);
}

// LDS footprint of a gather kernel by variant (the reduction scratch follows it).
template <int R, int G>
struct SmemG {
  static constexpr int red_off = Smem<R>::red_off;
  static constexpr int bytes = Smem<R>::bytes;
};
template <int R>
struct SmemG<R, 7> {
  static constexpr int red_off = SmemL<R, KMX_SEG>::red_off;
  static constexpr int bytes = SmemL<R, KMX_SEG>::bytes;
};
template <int R>
struct SmemG<R, 8> : SmemG<R, 7> {};
// G = 9 (k_hess only; k_grad / k_cost run G = 5 / 6): the G = 5 layout here.
template <int R>
struct SmemG<R, 9> : SmemG<R, 5> {};

// Incidence-parallel Hessian gather (G = 9, k_hess). Q's diagonal block D_i
// (k_precond) is applied once per pose, so an incidence only contributes its
// off-diagonal block B_e applied to the other endpoint's row: one lane per
// incidence reads the 96-B record once (not once per row as in G = 5) and the
// whole r x 4 neighbour row, and writes the R contribution rows to LDS; the
// (pose, row) lanes then add their pose's incidences in CSR order
// (deterministic). out_i = D_i v_i + sum_{e at i} B_e v_other(e), with a
// public neighbour's row taken as zero (Hessian of the local problem).
template <int R>
struct SmemH {
  static constexpr int TP = WAVES * (64 / R);
  static constexpr int CH = TP * R;                                       // incidences per chunk (<= BLOCK)
  static constexpr int c_off = 0;                                         // double[CH][R][4]
  static constexpr int ptr_off = CH * R * 32;                             // int[TP + 1]
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + RED_BYTES;
};
// group_symYtG<R, true> scratch: BLOCK x 6 doubles at the start of the LDS
static_assert(WAVES * 64 * 6 * 8 <= SmemH<3>::ptr_off && WAVES * 64 * 6 * 8 <= SmemH<8>::ptr_off, "scratch");
static_assert(WAVES * 64 * 6 * 8 <= Smem<5>::red_off && WAVES * 64 * 6 * 8 <= Smem<8>::red_off, "scratch");
template <int R, int GV>
struct SmemHess : SmemG<R, GV> {};
template <int R>
struct SmemHess<R, 9> : SmemH<R> {};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops but
// not for its outstanding global loads (__syncthreads waits vmcnt(0), which
// would drain the next chunk's prefetched records).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int R>
__device__ __forceinline__ void hinc_gather(const Dev& d, const Lane& L, const double* V, double acc[4],
                                            char* smem) {
  using SM = SmemH<R>;
  constexpr int CH = SM::CH;
  static_assert(CH <= BLOCK, "one incidence per thread per chunk");
  double* Cs = reinterpret_cast<double*>(smem + SM::c_off);
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = d.inc_ptr[p0];
  const int n = d.inc_ptr[p0 + np] - K0;
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  const int pl = L.pose - p0;
  const int lt = min(tid, CH - 1);
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  // clamped, unconditional record loads (hrec holds one zero pad record, so
  // an empty tile at the end of the array still reads inside it)
  auto ld = [&](int c0, double2 q[6]) {
    const int k = max(min(c0 + lt, n - 1), 0);
    const double2* q2 = reinterpret_cast<const double2*>(d.hrec + 12 * (size_t)(K0 + k));
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = q2[i];
  };
  double2 q[6];
  ld(0, q);
  __syncthreads();  // sptr
  for (int c0 = 0; c0 < n; c0 += CH) {
    Edge E;
    edge_from_compact(q, E);
    const int2 in = unpack_int2(q[5].y);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    const double2* b2 = reinterpret_cast<const double2*>(V + (size_t)max(o, 0) * 4 * R);
    double2 vr[2 * R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vr[i] = b2[i];
    if (tid < CH && c0 + tid < n) {
      const double wk = (o >= 0) ? E.wk : 0.0, wt = (o >= 0) ? E.wt : 0.0;
#pragma unroll
      for (int a = 0; a < R; ++a) {
        const double v0 = vr[2 * a].x, v1 = vr[2 * a].y, v2 = vr[2 * a + 1].x, v3 = vr[2 * a + 1].y;
        double h[4];
        if (tail) {  // self = i: row(j) Q_ji = -w [kappa row(j)_Y R^T + tau p_j t^T, tau p_j]
#pragma unroll
          for (int c = 0; c < 3; ++c)
            h[c] = -(wk * (v0 * E.R[c * 3 + 0] + v1 * E.R[c * 3 + 1] + v2 * E.R[c * 3 + 2]) + wt * v3 * E.t[c]);
          h[3] = -(wt * v3);
        } else {  // self = j: row(i) Q_ij = -w [kappa row(i)_Y R, tau (p_i + row(i)_Y t)]
#pragma unroll
          for (int c = 0; c < 3; ++c) h[c] = -(wk * (v0 * E.R[0 * 3 + c] + v1 * E.R[1 * 3 + c] + v2 * E.R[2 * 3 + c]));
          h[3] = -(wt * (v3 + (v0 * E.t[0] + v1 * E.t[1] + v2 * E.t[2])));
        }
        store4(Cs + (tid * R + a) * 4, h);
      }
    }
    // the next chunk's records, issued once this chunk's rows are consumed, stay
    // in flight across the LDS hand-off and the reduction
    asm volatile("" ::: "memory");
    ld(c0 + CH, q);
    lds_barrier();
    if (L.valid) {
      const int j0 = max(sptr[pl], c0) - c0, j1 = min(sptr[pl + 1], c0 + CH) - c0;
      #pragma unroll 4
      for (int j = j0; j < j1; ++j) {
        double h[4];
        load4(Cs + (j * R + L.a) * 4, h);
        acc[0] += h[0]; acc[1] += h[1]; acc[2] += h[2]; acc[3] += h[3];
      }
    }
    lds_barrier();
  }
  if (L.valid) {
    double vs[4];
    load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
    const double* Dp = d.hD + 16 * (size_t)L.pose;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double dr[4];
      load4(Dp + 4 * c, dr);
      acc[c] += vs[0] * dr[0] + vs[1] * dr[1] + vs[2] * dr[2] + vs[3] * dr[3];
    }
  }
}


// Gradient and cost, incidence-parallel (G = 9 k_grad). As hinc_gather, but a
// lane evaluates its whole incidence with incidence_row (diagonal and
// off-diagonal terms, the public neighbour row from the table), so it also
// reads its own pose's row (found by a binary search of the tile CSR), and
// adds the incidence's cost share (1/2 per endpoint; all of it for a shared
// edge). The pose sums run in CSR order.
// k_grad's LDS: a smaller chunk buffer, plus the tile's own rows (every lane
// reads its incidence's own row from LDS instead of L1).
#ifndef KMX_HG_CH
#define KMX_HG_CH 240
#endif
template <int R>
struct SmemHG {
  static constexpr int TP = WAVES * (64 / R);
  static constexpr int CH = KMX_HG_CH;                                    // incidences per chunk
  static constexpr int c_off = 0;                                         // double[CH][R][4]
  static constexpr int x_off = CH * R * 32;                               // double[TP][R][4]
  static constexpr int ptr_off = x_off + TP * R * 32;                     // int[TP + 1]
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + RED_BYTES;
};

template <int R>
__device__ __forceinline__ void hinc_grad(const Dev& d, const Lane& L, const double* V, const double* pub,
                                          double acc[4], double* cost, char* smem) {
  using SM = SmemHG<R>;
  constexpr int CH = SM::CH;
  double* Cs = reinterpret_cast<double*>(smem + SM::c_off);
  double2* xs = reinterpret_cast<double2*>(smem + SM::x_off);
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = d.inc_ptr[p0];
  const int n = d.inc_ptr[p0 + np] - K0;
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  {
    const double2* v2 = reinterpret_cast<const double2*>(V + (size_t)p0 * 4 * R);
    for (int i = tid; i < np * 2 * R; i += BLOCK) xs[i] = v2[i];
  }
  const int pl = L.pose - p0;
  const int lt = min(tid, CH - 1);
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  double csum = 0.0;
  auto ld = [&](int c0, double2 q[6]) {
    const int k = max(min(c0 + lt, n - 1), 0);
    const double2* q2 = reinterpret_cast<const double2*>(d.hrec + 12 * (size_t)(K0 + k));
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = q2[i];
  };
  double2 q[6];
  ld(0, q);
  __syncthreads();  // sptr
  for (int c0 = 0; c0 < n; c0 += CH) {
    const int k = max(min(c0 + lt, n - 1), 0);
    int lo = 0, hi = np;  // owning pose: sptr[lo] <= k < sptr[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sptr[mid] <= k) lo = mid;
      else hi = mid;
    }
    const int2 in = unpack_int2(q[5].y);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    const double2* s2 = xs + lo * 2 * R;
    const double2* o2 = reinterpret_cast<const double2*>((o >= 0) ? V + (size_t)o * 4 * R : pub + (size_t)(-1 - o) * 4 * R);
    double2 vo2[2 * R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vo2[i] = o2[i];
    Edge E;
    edge_from_compact(q, E);
    if (tid < CH && c0 + tid < n) {
#pragma unroll
      for (int a = 0; a < R; ++a) {
        const double2 sa = s2[2 * a], sb = s2[2 * a + 1];  // own row, from LDS
        const double vs[4] = {sa.x, sa.y, sb.x, sb.y};
        const double vo[4] = {vo2[2 * a].x, vo2[2 * a].y, vo2[2 * a + 1].x, vo2[2 * a + 1].y};
        double h[4] = {0.0, 0.0, 0.0, 0.0};
        const double c = incidence_row(E, tail, vs, vo, h);
        csum += (o < 0) ? c : 0.5 * c;
        store4(Cs + (tid * R + a) * 4, h);
      }
    }
    asm volatile("" ::: "memory");
    ld(c0 + CH, q);
    lds_barrier();
    if (L.valid) {
      const int j0 = max(sptr[pl], c0) - c0, j1 = min(sptr[pl + 1], c0 + CH) - c0;
      #pragma unroll 4
      for (int j = j0; j < j1; ++j) {
        double h[4];
        load4(Cs + (j * R + L.a) * 4, h);
        acc[0] += h[0]; acc[1] += h[1]; acc[2] += h[2]; acc[3] += h[3];
      }
    }
    lds_barrier();
  }
  *cost += csum;
}
template <int R, int GV>
struct SmemGrad : SmemG<R, GV> {};
template <int R>
struct SmemGrad<R, 9> : SmemHG<R> {};

// -------------------------------------------- fused per-robot reductions --
// Each tile of robot l publishes its partial sums, then takes a ticket on
// robot l's counter (agent-scope release / acquire, cdna_hip_programming.md
// Guideline 16). The tile that draws the last ticket reduces robot l's
// partials in tile order (deterministic) and runs the RTR / tCG scalar logic
// on thread 0 — no separate reduction launch, robots reduce in parallel.
__device__ void control(const Dev& d, int l, int kind, const double* tot, int R_);

template <int KIND, int NV, int FUSED>
__device__ __forceinline__ void finish_tile(const Dev& d, const Lane& L, const double* vals, char* smem_red,
                                            int R_) {
  double* lds = reinterpret_cast<double*>(smem_red);
  int* flag = reinterpret_cast<int*>(smem_red + 8 * NPART * WAVES);
  static_assert(NV <= NPART && WAVES == 4, "reduction area");
  double tv[NV > 0 ? NV : 1];
  if constexpr (!FUSED) {
    // all NV sums in one LDS round (same wave and wave-order summation as
    // block_sum); only thread 0 needs them. The area is used once per launch,
    // and the barrier is LDS-only, so the caller's row stores keep draining.
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      const double w = wave_sum(vals[s]);
      if ((threadIdx.x & 63) == 0) lds[s * WAVES + (threadIdx.x >> 6)] = w;
    }
    lds_barrier();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int s = 0; s < NV; ++s) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) t += lds[s * WAVES + w];
        d.part[(size_t)L.tile * NPART + s] = t;
      }
    }
    return;
  } else {
#pragma unroll
    for (int s = 0; s < NV; ++s) tv[s] = block_sum(vals[s], lds);
    // Write-through (sc1) partial stores, drained, then one agent-scope
    // ticket per tile; the last arriver reads the partials with sc1 loads
    // (MI355X_MICROARCH.md "Valid forms", table row 1).
    if (threadIdx.x == 0) {
#pragma unroll
      for (int s = 0; s < NV; ++s)
        __hip_atomic_store(d.part + (size_t)L.tile * NPART + s, tv[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned ntl = (unsigned)(d.rtile0[L.l + 1] - d.rtile0[L.l]);
      const unsigned t = __hip_atomic_fetch_add(d.tickets + L.l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (t == ntl - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int NS = (KIND == RED_COST) ? 4 : NV;
    double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
    const int t0 = d.rtile0[L.l], t1 = d.rtile0[L.l + 1];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      double v = 0.0;
      for (int t = t0 + (int)threadIdx.x; t < t1; t += BLOCK)
        v += __hip_atomic_load(d.part + (size_t)t * NPART + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tot[s] = block_sum(v, lds);
    }
    if (threadIdx.x == 0) {
      control(d, L.l, KIND, tot, R_);
      __hip_atomic_store(d.tickets + L.l, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ void control(const Dev& d, int l, int kind, const double* tot, int R_) {
  Ctl& c = d.ctl[l];
  const Params& P = d.p;
  if (kind == RED_GRAD) {
    const double f = tot[0], gn = sqrt(tot[1]);
    if (c.rtr_iter == 0) { c.f_init = f; c.gn_init = gn; }
    c.f_cur = f;
    c.f_final = f;
    c.commit = 0;
    if (gn < P.gn_tol) {
      c.phase = PH_IDLE;
      c.tcg_stop = KMX_TCG_SKIPPED;
      c.tcg_iter = 0;
      c.accepted = 0;
      c.skipped = 1;
    } else {
      c.phase = PH_TCG;
      c.tcg_iter = 0;
      c.norm_r0 = gn;
      c.z_r = tot[2];
      c.d_Pd = tot[2];
      c.e_Pd = 0.0;
      c.e_Pe = 0.0;
      c.beta = 0.0;
      c.tcg_stop = KMX_TCG_MAX_ITER;
      if (c.rtr_iter == 0) {
        atomicAdd(&d.cnt->edges_iters, (unsigned long long)d.m_robot[l]);
        atomicAdd(&d.cnt->block_updates, 1ull);
      }
    }
  } else if (kind == RED_HESS) {
    const double d_Hd = tot[0];
    const double alpha = c.z_r / d_Hd;
    const double e_Pe_new = c.e_Pe + 2.0 * alpha * c.e_Pd + alpha * alpha * c.d_Pd;
    const double D2 = c.Delta * c.Delta;
    c.tcg_iter += 1;
    c.hessvecs += 1;
    atomicAdd(&d.cnt->hessvecs, 1ull);
    atomicAdd(&d.cnt->hess_alg_bytes, 128.0 * (double)d.m_robot[l] + 2.0 * 8.0 * R_ * 4.0 * (double)d.n_robot[l]);
    if (d_Hd <= 0.0 || e_Pe_new >= D2) {
      const double tau = (-c.e_Pd + sqrt(c.e_Pd * c.e_Pd + c.d_Pd * (D2 - c.e_Pe))) / c.d_Pd;
      c.coef = tau;
      c.mode = MODE_BOUNDARY;
      c.tcg_stop = d_Hd <= 0.0 ? KMX_TCG_NEGATIVE_CURVATURE : KMX_TCG_EXCEEDED_TR;
    } else {
      c.alpha = alpha;
      c.coef = alpha;
      c.e_Pe = e_Pe_new;
      c.mode = MODE_INTERIOR;
    }
  } else if (kind == RED_UPDATE) {
    if (c.mode == MODE_BOUNDARY) {
      c.phase = PH_STEP;
      return;
    }
    const double norm_r = sqrt(tot[0]);
    const double zr_new = tot[1];
    const double pw = pow(c.norm_r0, P.theta);
    if (norm_r <= c.norm_r0 * fmin(pw, P.kappa)) {
      c.tcg_stop = (P.kappa < pw) ? KMX_TCG_LINEAR : KMX_TCG_SUPERLINEAR;
      c.phase = PH_STEP;
    } else if (c.tcg_iter >= P.tcg_max) {
      c.tcg_stop = KMX_TCG_MAX_ITER;
      c.phase = PH_STEP;
    } else {
      const double beta = zr_new / c.z_r;
      c.e_Pd = beta * (c.e_Pd + c.alpha * c.d_Pd);
      c.d_Pd = zr_new + beta * beta * c.d_Pd;
      c.z_r = zr_new;
      c.beta = beta;
    }
  } else {  // RED_COST: tot[0] = f(Xt), tot[2] = 2 m(eta), tot[3] = ||Xt - X||^2
    const double ft = tot[0];
    const double model_dec = -0.5 * tot[2];
    const double rho = (model_dec > 0.0) ? (c.f_cur - ft) / model_dec : -1.0;
    const bool boundary = (c.tcg_stop == KMX_TCG_NEGATIVE_CURVATURE || c.tcg_stop == KMX_TCG_EXCEEDED_TR);
    if (!(rho >= 0.25)) c.Delta *= 0.25;
    else if (rho > 0.75 && boundary) c.Delta = fmin(2.0 * c.Delta, P.Delta_max);
    c.rho = rho;
    if (rho > P.accept_rho) {
      c.accepted = 1;
      c.commit = 1;
      c.f_final = ft;
      c.chg_acc += tot[3];
    } else {
      c.accepted = 0;
      c.commit = 0;
      c.f_final = c.f_cur;
    }
    c.rtr_iter += 1;
    c.phase = (c.rtr_iter < P.rtr_iters) ? PH_START : PH_IDLE;
    c.rel_change = sqrt(c.chg_acc / (double)d.n_robot[l]);
  }
}

// Separate-launch reduction (variant F = 0): one workgroup per robot.
__global__ __launch_bounds__(BLOCK) void k_reduce(Dev d, int kind, int R_, HostStatus* hs,
                                                 unsigned long long seq) {
  __shared__ double lds[NPART * WAVES];
  const int l = blockIdx.x;
  const int ph = d.ctl[l].phase;
  bool act = false;
  if (kind == RED_GRAD) act = ph == PH_START;
  if (kind == RED_HESS || kind == RED_UPDATE) act = ph == PH_TCG;
  if (kind == RED_COST) act = ph == PH_STEP;
  if (!act) {
    if (hs && threadIdx.x == 0) post_status(hs, l, seq, false);  // not in tCG after this step
    return;
  }
  const int ns = kind == RED_GRAD ? 3 : kind == RED_HESS ? 1 : kind == RED_UPDATE ? 2 : 4;
  double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
  const int t0 = d.rtile0[l], t1 = d.rtile0[l + 1];
  // all slots in one pass and one LDS round (same per-thread, per-wave and
  // wave-order summation as a block_sum per slot, so the sums are unchanged)
  static_assert(NPART == 4, "two 16-B loads per tile");
  double v[NPART] = {0.0, 0.0, 0.0, 0.0};
  for (int t = t0 + (int)threadIdx.x; t < t1; t += BLOCK) {
    const double2* p2 = reinterpret_cast<const double2*>(d.part + (size_t)t * NPART);
    const double2 a = p2[0], b = p2[1];
    v[0] += a.x; v[1] += a.y; v[2] += b.x; v[3] += b.y;
  }
#pragma unroll
  for (int s = 0; s < NPART; ++s) {
    const double w = wave_sum(v[s]);
    if ((threadIdx.x & 63) == 0) lds[s * WAVES + (threadIdx.x >> 6)] = w;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NPART; ++s) {
    double acc = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) acc += lds[s * WAVES + w];
    tot[s] = s < ns ? acc : 0.0;
  }
  if (threadIdx.x == 0) {
    control(d, l, kind, tot, R_);
    if (hs) post_status(hs, l, seq, d.ctl[l].phase == PH_TCG);
  }
}

#define KMX_SMEM extern __shared__ __attribute__((aligned(16))) char smem[]

// Start of an RTR iteration: egrad (gather X with public neighbours), cost,
// S = sym(Y^T egrad_Y), g = P_Y(egrad), r = g, z = precon(g).
template <int R, int GV, int F>
__global__ __launch_bounds__(BLOCK, (GV == 7 || GV == 9 ? 4 : KMX_LB_GATHER)) void k_grad(Dev d) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  if (d.ctl[L.l].phase != PH_START) return;
  double y[4] = {0, 0, 0, 0}, G[4], cost = 0.0;
  if constexpr (GV == 9) hinc_grad<R>(d, L, d.X, d.pub, G, &cost, smem);
  else gather<R, GV, true>(d, L, d.X, d.pub, G, &cost, smem);
  if (L.valid) load4(d.X + (size_t)L.pose * 4 * R + 4 * L.a, y);
  double S[9], gr[4], zr[4];
  // G = 9: the gather's chunk buffer is free now (its last barrier passed)
  double* scr = reinterpret_cast<double*>(smem + SmemHG<R>::c_off);
  static_assert(WAVES * 64 * 6 * 8 <= SmemHG<R>::x_off, "scratch");
  if (d.dbg & 2) {
    for (int i = 0; i < 9; ++i) S[i] = 0.0;
  } else {
    group_symYtG<R, GV == 9>(y, G, L.base, S, scr);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) gr[c] = G[c] - (y[0] * S[0 * 3 + c] + y[1] * S[1 * 3 + c] + y[2] * S[2 * 3 + c]);
  gr[3] = G[3];
  if (d.dbg & 1) {
    for (int i = 0; i < 4; ++i) zr[i] = gr[i];
  } else {
    group_precon<R, GV == 9>(d, L.pose, L.valid, y, gr, L.base, zr, scr);
  }
  double vals[3] = {0.0, 0.0, 0.0};
  vals[0] = cost;  // the incidence-parallel gather accumulates cost on non-pose lanes too
  if (L.valid) {
    vals[1] = gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2] + gr[3] * gr[3];
    vals[2] = zr[0] * gr[0] + zr[1] * gr[1] + zr[2] * gr[2] + zr[3] * gr[3];
  }
  auto store = [&]() {
    if (L.valid) {
      const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
      store4(d.g + o, gr);  // r = g at the start of tCG: k_update's first step reads g
      store4(d.z + o, zr);
      if (L.a == 0) {
        double* Sp = d.S + 9 * (size_t)L.pose;
#pragma unroll
        for (int i = 0; i < 9; ++i) Sp[i] = S[i];
      }
    }
  };
  // separate reduce launch: store first (frees S, g, z before the block sum);
  // fused reduction: ticket first, so its drain waits only for the partials
  if constexpr (!F) store();
  finish_tile<RED_GRAD, 3, F>(d, L, vals, smem + SmemGrad<R, GV>::red_off, R);
  if constexpr (F) store();
}

// tCG step, part 1 (the dominant kernel): Hz = Hess(z) by gather; then by
// linearity delta = -z + beta delta_old, Hdelta = -Hz + beta Hdelta_old.
template <int R, int GV, int F>
__global__ __launch_bounds__(BLOCK, (GV == 7 || GV == 9 ? 4 : KMX_LB_GATHER)) void k_hess(Dev d) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  const Ctl& c = d.ctl[L.l];
  if (c.phase != PH_TCG) return;
  const bool first = (c.tcg_iter == 0);
  const double beta = c.beta;
  double y[4] = {0, 0, 0, 0}, zs[4] = {0, 0, 0, 0}, H[4], S[9];
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  if constexpr (GV == 9) hinc_gather<R>(d, L, d.z, H, smem);
  else gather<R, GV, false>(d, L, d.z, nullptr, H, nullptr, smem);
  asm volatile("" ::: "memory");  // keep the epilogue loads below the gather loop (VGPR pressure)
  if (L.valid) {
    load4(d.z + o, zs);
    load4(d.X + o, y);
    const double* Sp = d.S + 9 * (size_t)L.pose;
#pragma unroll
    for (int i = 0; i < 9; ++i) S[i] = Sp[i];
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) S[i] = 0.0;
  }
  double hz[4];
  group_rhess<R, GV == 9>(y, zs, H, S, L.base, hz, reinterpret_cast<double*>(smem + SmemH<R>::c_off));
  double v = 0.0;
  double dl[4] = {0, 0, 0, 0}, hdl[4] = {0, 0, 0, 0};
  if (L.valid) {
    if (first) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { dl[k] = -zs[k]; hdl[k] = -hz[k]; }
    } else {
      double dold[4], hold[4];
      load4(d.del + o, dold);
      load4(d.hd + o, hold);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dl[k] = -zs[k] + beta * dold[k];
        hdl[k] = -hz[k] + beta * hold[k];
      }
    }
    v = dl[0] * hdl[0] + dl[1] * hdl[1] + dl[2] * hdl[2] + dl[3] * hdl[3];
  }
  finish_tile<RED_HESS, 1, F>(d, L, &v, smem + SmemHess<R, GV>::red_off, R);
  if (L.valid) {
    store4(d.del + o, dl);
    store4(d.hd + o, hdl);
  }
}

// tCG step, part 2: eta += coef delta, r += coef Hdelta; interior steps also
// z = precon(r) and partial <r,r>, <z,r>.
template <int R, int GV, int F>
__global__ __launch_bounds__(BLOCK) void k_update(Dev d) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  const Ctl& c = d.ctl[L.l];
  if (c.phase != PH_TCG) return;
  const bool first = (c.tcg_iter == 1);
  const double coef = c.coef;
  const bool interior = (c.mode == MODE_INTERIOR);
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double rr[4] = {0, 0, 0, 0}, y[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0};
  if (L.valid) {
    double dl[4], hdl[4];
    load4(d.del + o, dl);
    load4(d.hd + o, hdl);
    load4((first ? d.g : d.r) + o, rr);  // r_0 = g (k_grad does not store r)
    if (!first) load4(d.eta + o, et);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      et[k] += coef * dl[k];
      rr[k] += coef * hdl[k];
    }
    if (interior) load4(d.X + o, y);
  }
  double vals[2] = {0.0, 0.0}, zr[4] = {0, 0, 0, 0};
  if (interior) {  // uniform per robot
    group_precon<R, GV == 9>(d, L.pose, L.valid, y, rr, L.base, zr, reinterpret_cast<double*>(smem));
    if (L.valid) {
      vals[0] = rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2] + rr[3] * rr[3];
      vals[1] = zr[0] * rr[0] + zr[1] * rr[1] + zr[2] * rr[2] + zr[3] * rr[3];
    }
  }
  finish_tile<RED_UPDATE, 2, F>(d, L, vals, smem + Smem<R>::red_off, R);
  if (L.valid) {
    store4(d.eta + o, et);
    store4(d.r + o, rr);
    if (interior) store4(d.z + o, zr);
  }
}

// Trial point Xt = R_X(eta); partials: model m(eta) = 1/2 <eta, g + r> (r = g +
// H eta by the tCG recurrence) and ||Xt - X||^2 (slots 2, 3; k_cost reduces).
template <int R>
__global__ __launch_bounds__(BLOCK) void k_retract(Dev d) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  if (d.ctl[L.l].phase != PH_STEP) return;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double x[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0}, gg[4] = {0, 0, 0, 0}, rr[4] = {0, 0, 0, 0};
  if (L.valid) {  // all four rows in flight before the Gram-Schmidt chain
    load4(d.X + o, x);
    load4(d.eta + o, et);
    load4(d.g + o, gg);
    load4(d.r + o, rr);
  }
  double xt[4];
  group_retract<R>(x, et, L.base, xt);
  double vals[2] = {0.0, 0.0};
  if (L.valid) {
    store4(d.Xt + o, xt);
    double m = 0.0, ch = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m += et[k] * (gg[k] + rr[k]);
      const double dd = xt[k] - x[k];
      ch += dd * dd;
    }
    vals[0] = m;
    vals[1] = ch;
  }
  double* lds = reinterpret_cast<double*>(smem + Smem<R>::red_off);
  for (int s = 0; s < 2; ++s) {
    const double t = block_sum(vals[s], lds);
    if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART + 2 + s] = t;
  }
}

// Trial cost, one lane per owner incidence (G = 9): each local edge is
// visited once by the lane that owns it, which reads the record and both
// endpoint rows and sums the R rows' residual terms; no per-pose reduction.
template <int R>
struct SmemC {
  static constexpr int TP = WAVES * (64 / R);
  static constexpr int x_off = 0;                                    // double[TP][R][4] own rows
  static constexpr int ptr_off = TP * R * 32;                        // int[TP + 1]
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + RED_BYTES;
};
template <int R, int GV>
struct SmemCost : SmemG<R, GV> {};
template <int R>
struct SmemCost<R, 9> : SmemC<R> {};

template <int R>
__device__ __forceinline__ double inc_owner_cost(const Dev& d, const Lane& L, const double* V, const double* pub,
                                                 char* smem) {
  int* sptr = reinterpret_cast<int*>(smem + SmemC<R>::ptr_off);
  double2* xs = reinterpret_cast<double2*>(smem + SmemC<R>::x_off);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = d.optr[p0];
  const int n = d.optr[p0 + np] - K0;
  if (tid <= np) sptr[tid] = d.optr[p0 + tid] - K0;
  {
    const double2* v2 = reinterpret_cast<const double2*>(V + (size_t)p0 * 4 * R);
    for (int i = tid; i < np * 2 * R; i += BLOCK) xs[i] = v2[i];
  }
  __syncthreads();
  double cost = 0.0;
  for (int k = tid; k < n; k += BLOCK) {
    int lo = 0, hi = np;  // owning pose: sptr[lo] <= k < sptr[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sptr[mid] <= k) lo = mid;
      else hi = mid;
    }
    const double2* q2 = reinterpret_cast<const double2*>(d.hocrec + 12 * (size_t)(K0 + k));
    double2 q[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = q2[i];
    const int2 in = unpack_int2(q[5].y);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    const double2* s2 = xs + lo * 2 * R;  // own row, from LDS
    const double2* o2 = reinterpret_cast<const double2*>((o >= 0) ? V + (size_t)o * 4 * R : pub + (size_t)(-1 - o) * 4 * R);
    double2 vs2[2 * R], vo2[2 * R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) { vs2[i] = s2[i]; vo2[i] = o2[i]; }
    Edge E;
    edge_from_compact(q, E);
    double c = 0.0;
#pragma unroll
    for (int a = 0; a < R; ++a) {
      const double vs[4] = {vs2[2 * a].x, vs2[2 * a].y, vs2[2 * a + 1].x, vs2[2 * a + 1].y};
      const double vo[4] = {vo2[2 * a].x, vo2[2 * a].y, vo2[2 * a + 1].x, vo2[2 * a + 1].y};
      double dummy[4] = {0.0, 0.0, 0.0, 0.0};
      c += incidence_row(E, tail, vs, vo, dummy);
    }
    cost += c;
  }
  return cost;
}

template <int R, int GV, int F>
__global__ __launch_bounds__(BLOCK, (GV == 7 || GV == 9 ? 4 : KMX_LB_GATHER)) void k_cost(Dev d) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  if (d.ctl[L.l].phase != PH_STEP) return;
  double acc[4], cost = 0.0;
  if constexpr (GV == 9) cost = inc_owner_cost<R>(d, L, d.Xt, d.pub, smem);
  else gather<R, (GV == 3 ? 4 : GV == 5 ? 6 : GV == 7 ? 8 : GV), true>(d, L, d.Xt, d.pub, acc, &cost, smem);
  finish_tile<RED_COST, 1, F>(d, L, &cost, smem + SmemCost<R, GV>::red_off, R);
}

template <int R>
__global__ __launch_bounds__(BLOCK) void k_commit(Dev d) {
  const Lane L = lane_map<R>(d);
  if (!d.ctl[L.l].commit) return;
  if (!L.valid) return;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double v[4];
  load4(d.Xt + o, v);
  store4(d.X + o, v);
}

__device__ __forceinline__ void begin_robot(const Dev& d, const unsigned char* active, int l) {
  Ctl& c = d.ctl[l];
  const bool a = active ? active[l] != 0 : true;
  const Ctl zero = {};
  c = zero;
  c.phase = a ? PH_START : PH_IDLE;
  c.updated = a ? 1 : 0;
  c.Delta = d.p.Delta0;
}

__global__ void k_round_begin(Dev d, const unsigned char* active) {
  const int l = threadIdx.x;
  if (l >= d.L) return;
  begin_robot(d, active, l);
}

// One 16-B part i of the owned public rows: slot s = i / (ps / 2) (ps = 4r is
// even, rows are 16-B aligned).
__device__ __forceinline__ void publish_part(const double* X, double* pub, const int* src, int nslots, int ps,
                                             long long i) {
  const int ps2 = ps >> 1;
  const long long s = i / ps2;
  if (s >= nslots) return;
  const int q = (int)(i - s * ps2);
  const int p = src[s];
  if (p >= 0)
    reinterpret_cast<double2*>(pub)[s * ps2 + q] = reinterpret_cast<const double2*>(X)[(long long)p * ps2 + q];
}

// Round start fused with k_publish (iterate_async with refresh_local): block 0
// activates the robots, the other blocks copy the owned public rows. The two
// touch disjoint data, so one launch replaces two.
__global__ void k_round_begin_pub(Dev d, const unsigned char* active, const double* X, double* pub, const int* src,
                                  int nslots, int ps) {
  if (blockIdx.x == 0) {
    for (int l = threadIdx.x; l < d.L; l += blockDim.x) begin_robot(d, active, l);
    return;
  }
  publish_part(X, pub, src, nslots, ps, (long long)(blockIdx.x - 1) * blockDim.x + threadIdx.x);
}

__global__ void k_publish(const double* X, double* pub, const int* src, int nslots, int ps) {
  publish_part(X, pub, src, nslots, ps, (long long)blockIdx.x * blockDim.x + threadIdx.x);
}

// Sparse exchange: rows of the given public slots (owned by this handle) from
// the iterate, and rows received from peers written into the table.
// A slot outside the table (or, for gather, not owned here) is skipped
// (gather writes zeros), so a bad index list cannot fault the device.
__global__ void k_gather_slots(const double* X, const int* pub_src, const int* slots, long long n, int npub,
                               double* out, int ps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) return;
  const int q = (int)(i - s * ps);
  const int sl = slots[s];
  const int p = (sl >= 0 && sl < npub) ? pub_src[sl] : -1;
  out[i] = (p >= 0) ? X[(long long)p * ps + q] : 0.0;
}
__global__ void k_scatter_slots(double* pub, const int* slots, long long n, int npub, const double* rows, int ps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) return;
  const int q = (int)(i - s * ps);
  const int sl = slots[s];
  if (sl >= 0 && sl < npub) pub[(long long)sl * ps + q] = rows[i];
}

__global__ void k_pack(const double* X, double* out, const int* src, int first, int count, int ps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= count) return;
  const int q = (int)(i - s * ps);
  out[s * ps + q] = X[(long long)src[first + s] * ps + q];
}

// 4x4 diagonal blocks of Q (+ shift) per pose, Cholesky-inverted. Same
// accumulation order and expressions as oracle build_precond.
__global__ void k_precond(Dev d) {
  const int pose = blockIdx.x * blockDim.x + threadIdx.x;
  if (pose >= d.nloc) return;
  double A[16];
  for (int i = 0; i < 16; ++i) A[i] = 0.0;
  for (int k = d.inc_ptr[pose]; k < d.inc_ptr[pose + 1]; ++k) {
    const int2 in = d.inc[k];
    const bool tail = (in.y >> 31) & 1;
    const double* er = d.irec + 16 * (size_t)k;
    const double wk = er[12], wt = er[13];
    const double* tt = er + 9;
    if (tail) {
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) A[i * 4 + j] += wt * tt[i] * tt[j] + (i == j ? wk : 0.0);
        A[i * 4 + 3] += wt * tt[i];
        A[3 * 4 + i] += wt * tt[i];
      }
      A[15] += wt;
    } else {
      A[0] += wk; A[5] += wk; A[10] += wk; A[15] += wt;
    }
  }
  if (d.hD)
    for (int i = 0; i < 16; ++i) d.hD[16 * (size_t)pose + i] = A[i];
  for (int j = 0; j < 4; ++j) A[j * 5] += d.p.shift;
  double Lm[16], Li[16];
  for (int i = 0; i < 16; ++i) { Lm[i] = 0.0; Li[i] = 0.0; }
  for (int j = 0; j < 4; ++j) {
    double s = A[j * 4 + j];
    for (int k = 0; k < j; ++k) s -= Lm[j * 4 + k] * Lm[j * 4 + k];
    Lm[j * 4 + j] = sqrt(s);
    for (int ii = j + 1; ii < 4; ++ii) {
      double t = A[ii * 4 + j];
      for (int k = 0; k < j; ++k) t -= Lm[ii * 4 + k] * Lm[j * 4 + k];
      Lm[ii * 4 + j] = t / Lm[j * 4 + j];
    }
  }
  for (int c = 0; c < 4; ++c)
    for (int ii = 0; ii < 4; ++ii) {
      double s = (ii == c) ? 1.0 : 0.0;
      for (int k = c; k < ii; ++k) s -= Lm[ii * 4 + k] * Li[k * 4 + c];
      Li[ii * 4 + c] = (ii < c) ? 0.0 : s / Lm[ii * 4 + ii];
    }
  double* Pi = d.Pinv + 16 * (size_t)pose;
  for (int x = 0; x < 4; ++x)
    for (int y = 0; y < 4; ++y) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += Li[k * 4 + x] * Li[k * 4 + y];
      Pi[x * 4 + y] = s;
    }
}

// GNC-TLS weight sweep over owned non-fixed local edges (owner's view of the
// endpoints: its own robot from X, the other robot from the public table).
__global__ void k_gnc(Dev d, const int* gnc_edge, const int2* gnc_ends, int n, int R_, double mu, double barc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = gnc_edge[i];
  const int2 en = gnc_ends[i];
  const int ps = 4 * R_;
  const double* Xi = en.x >= 0 ? d.X + (size_t)en.x * ps : d.pub + (size_t)(-1 - en.x) * ps;
  const double* Xj = en.y >= 0 ? d.X + (size_t)en.y * ps : d.pub + (size_t)(-1 - en.y) * ps;
  const int2 ip = d.eipos[e];
  const double* er = d.irec + 16 * (size_t)(ip.x >= 0 ? ip.x : ip.y);
  const double* Rt = er;
  const double* tt = er + 9;
  double sR = 0.0, sT = 0.0;
  for (int a = 0; a < R_; ++a) {
    const double* yi = Xi + 4 * a;
    const double* yj = Xj + 4 * a;
    for (int c = 0; c < 3; ++c) {
      const double q = yj[c] - (yi[0] * Rt[0 * 3 + c] + yi[1] * Rt[1 * 3 + c] + yi[2] * Rt[2 * 3 + c]);
      sR += q * q;
    }
    const double et = yj[3] - yi[3] - (yi[0] * tt[0] + yi[1] * tt[1] + yi[2] * tt[2]);
    sT += et * et;
  }
  const double rSq = d.ekappa[e] * sR + d.etau[e] * sT;
  const double barcSq = barc * barc;
  const double upper = (mu + 1.0) / mu * barcSq;
  const double lower = mu / (mu + 1.0) * barcSq;
  double w;
  if (rSq >= upper) w = 0.0;
  else if (rSq <= lower) w = 1.0;
  else w = sqrt(barcSq * mu * (mu + 1.0) / rSq) - mu;
  d.ew[e] = w;
}

// Push the per-edge weights into both incidence copies (w*kappa, w*tau).
__global__ void k_apply_weights(Dev d, int mloc) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= mloc) return;
  const double w = d.ew[e];
  const double wk = w * d.ekappa[e], wt = w * d.etau[e];
  const int2 ip = d.eipos[e];
  if (ip.x >= 0) { d.irec[16 * (size_t)ip.x + 12] = wk; d.irec[16 * (size_t)ip.x + 13] = wt; }
  if (ip.y >= 0) { d.irec[16 * (size_t)ip.y + 12] = wk; d.irec[16 * (size_t)ip.y + 13] = wt; }
  if (d.hocrec) {
    const int2 hp = d.heopos[e];
    if (hp.x >= 0) { d.hocrec[12 * (size_t)hp.x + 9] = wk; d.hocrec[12 * (size_t)hp.x + 10] = wt; }
    if (hp.y >= 0) { d.hocrec[12 * (size_t)hp.y + 9] = wk; d.hocrec[12 * (size_t)hp.y + 10] = wt; }
  }
  if (d.hrec) {  // CSR order: the incidence positions
    if (ip.x >= 0) { d.hrec[12 * (size_t)ip.x + 9] = wk; d.hrec[12 * (size_t)ip.x + 10] = wt; }
    if (ip.y >= 0) { d.hrec[12 * (size_t)ip.y + 9] = wk; d.hrec[12 * (size_t)ip.y + 10] = wt; }
  }
  if (d.crec) {
    const int2 cp = d.cipos[e];
    if (cp.x >= 0) { d.crec[12 * (size_t)cp.x + 9] = wk; d.crec[12 * (size_t)cp.x + 10] = wt; }
    if (cp.y >= 0) { d.crec[12 * (size_t)cp.y + 9] = wk; d.crec[12 * (size_t)cp.y + 10] = wt; }
    const int2 op = d.eopos[e];
    if (op.x >= 0) { d.ocrec[12 * (size_t)op.x + 9] = wk; d.ocrec[12 * (size_t)op.x + 10] = wt; }
    if (op.y >= 0) { d.ocrec[12 * (size_t)op.y + 9] = wk; d.ocrec[12 * (size_t)op.y + 10] = wt; }
  }
}

__global__ void k_shared_pack(const double* ew, const int* sh_edge, const int* sh_idx, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[sh_idx[i]] = ew[sh_edge[i]];
}
__global__ void k_shared_unpack(double* ew, const int* sh_edge, const int* sh_idx, int n, const double* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ew[sh_edge[i]] = tab[sh_idx[i]];
}

// --- rounding to SE(3) in the anchor frame (same algorithm as the oracle) --
__device__ void jacobi3(double A[9], double V[9]) {
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        const double apq = A[p * 3 + q];
        if (apq == 0.0) continue;
        const double app = A[p * 3 + p], aqq = A[q * 3 + q];
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

__global__ void k_traj(const double* X, int n, int R_, const double* anchor, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* Xi = X + (size_t)i * 4 * R_;
  double M[9], tv[3];
  for (int x = 0; x < 3; ++x) {
    for (int y = 0; y < 3; ++y) {
      double s = 0.0;
      for (int k = 0; k < R_; ++k) s += anchor[4 * k + x] * Xi[4 * k + y];
      M[x * 3 + y] = s;
    }
    double s = 0.0;
    for (int k = 0; k < R_; ++k) s += anchor[4 * k + x] * (Xi[4 * k + 3] - anchor[4 * k + 3]);
    tv[x] = s;
  }
  double A[9], V[9];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += M[k * 3 + a] * M[k * 3 + b];
      A[a * 3 + b] = s;
    }
  jacobi3(A, V);
  const double det = M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
                     M[2] * (M[3] * M[7] - M[4] * M[6]);
  int kmin = 0;
  for (int k = 1; k < 3; ++k)
    if (A[k * 4] < A[kmin * 4]) kmin = k;
  double Rr[9];
  for (int q = 0; q < 9; ++q) Rr[q] = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double sig = sqrt(fmax(A[k * 4], 0.0));
    double u[3];
    for (int q = 0; q < 3; ++q) u[q] = (M[q * 3 + 0] * V[0 * 3 + k] + M[q * 3 + 1] * V[1 * 3 + k] + M[q * 3 + 2] * V[2 * 3 + k]) / sig;
    const double s = (k == kmin && det < 0.0) ? -1.0 : 1.0;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) Rr[a * 3 + b] += s * u[a] * V[b * 3 + k];
  }
  double* o = out + (size_t)i * 12;
  for (int q = 0; q < 9; ++q) o[q] = Rr[q];
  o[9] = tv[0]; o[10] = tv[1]; o[11] = tv[2];
}

// Primitive evaluation for parity tests (tiles of one robot).
template <int R, int GV>
__global__ __launch_bounds__(BLOCK) void k_eval(Dev d, int robot, int mode, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  if (L.l != robot) return;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double res[4] = {0, 0, 0, 0}, cost = 0.0, v[4] = {0, 0, 0, 0};
  if (mode == KMX_EVAL_COST_EGRAD) {
    gather<R, GV, true>(d, L, V, d.pub, res, &cost, smem);
  } else if (mode == KMX_EVAL_EHESS) {
    gather<R, GV, false>(d, L, V, nullptr, res, nullptr, smem);
    if (L.valid) load4(V + o, v);
  } else {
    double y[4] = {0, 0, 0, 0}, G[4];
    gather<R, GV, true>(d, L, d.X, d.pub, G, nullptr, smem);
    if (L.valid) {
      load4(d.X + o, y);
      load4(V + o, v);
    }
    double S[9];
    group_symYtG<R>(y, G, L.base, S);
    if (mode == KMX_EVAL_RGRAD) {
      for (int c = 0; c < 3; ++c) res[c] = G[c] - (y[0] * S[0 * 3 + c] + y[1] * S[1 * 3 + c] + y[2] * S[2 * 3 + c]);
      res[3] = G[3];
      for (int k = 0; k < 4; ++k) v[k] = res[k];
    } else if (mode == KMX_EVAL_RHESS) {
      double H[4];
      gather<R, GV, false>(d, L, V, nullptr, H, nullptr, smem);
      group_rhess<R>(y, v, H, S, L.base, res);
    } else if (mode == KMX_EVAL_PRECON) {
      group_precon<R>(d, L.pose, L.valid, y, v, L.base, res);
    } else if (mode == KMX_EVAL_RETRACT) {
      group_retract<R>(y, v, L.base, res);
      for (int k = 0; k < 4; ++k) v[k] = 0.0;
    }
  }
  double s = (mode == KMX_EVAL_COST_EGRAD) ? cost : 0.0;
  if (L.valid) {
    store4(out + o, res);
    if (mode != KMX_EVAL_COST_EGRAD) s = v[0] * res[0] + v[1] * res[1] + v[2] * res[2] + v[3] * res[3];
  }
  const double t = block_sum(s, reinterpret_cast<double*>(smem + SmemG<R, GV>::red_off));
  if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
}

// Diagnostic ablation of the plain direct gather: ABL bit0 -> every edge load
// reads record 0 (cache-resident), bit1 -> neighbour row = own row.
template <int R, int ABL>
__global__ __launch_bounds__(BLOCK) void k_gablate(Dev d, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  double acc[4] = {0, 0, 0, 0}, cost = 0.0;
  if (L.valid) {
    double vs[4];
    load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
    const int k0 = d.inc_ptr[L.pose], k1 = d.inc_ptr[L.pose + 1];
    for (int k = k0; k < k1; ++k) {
      int2 in = d.inc[k];
      if (ABL & 2) in.x = L.pose;
      EdgeRaw w;
      double2 b0, b1;
      fetch_incidence<R, true>(d, V, d.pub, L.a, (ABL & 1) ? 0 : k, in, w, b0, b1);
      Edge E;
      edge_from_raw(w, E);
      const double vo[4] = {b0.x, b0.y, b1.x, b1.y};
      cost += incidence_row(E, (in.y >> 31) & 1, vs, vo, acc);
    }
    store4(out + (size_t)L.pose * 4 * R + 4 * L.a, acc);
  }
  const double t = block_sum(cost, reinterpret_cast<double*>(smem + Smem<R>::red_off));
  if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
}

// Diagnostic: the compact gather with each pose's incidence loop capped at CAP
// (wrong results; bounds what a degree-balanced gather could gain).
template <int R, int CAP>
__global__ __launch_bounds__(BLOCK) void k_gcap(Dev d, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  double acc[4] = {0, 0, 0, 0}, cost = 0.0;
  if (L.valid) {
    double vs[4];
    load4(V + (size_t)L.pose * 4 * R + 4 * L.a, vs);
    const int k0 = d.inc_ptr[L.pose], k1 = min(d.inc_ptr[L.pose + 1], k0 + CAP);
    for (int k = k0; k < k1; ++k) {
      const double2* q2 = reinterpret_cast<const double2*>(d.crec + 12 * (size_t)k);
      double2 q[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) q[i] = q2[i];
      const int2 in = unpack_int2(q[5].y);
      const int o = in.x;
      const double* base = (o >= 0) ? V + (size_t)o * 4 * R : d.pub + (size_t)(-1 - o) * 4 * R;
      const double2* b2 = reinterpret_cast<const double2*>(base + 4 * L.a);
      const double2 v0 = b2[0], v1 = b2[1];
      Edge E;
      edge_from_compact(q, E);
      const double vo[4] = {v0.x, v0.y, v1.x, v1.y};
      cost += incidence_row(E, (in.y >> 31) & 1, vs, vo, acc);
    }
    store4(out + (size_t)L.pose * 4 * R + 4 * L.a, acc);
  }
  const double t = block_sum(cost, reinterpret_cast<double*>(smem + Smem<R>::red_off));
  if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
}

// Diagnostic: the gather primitive alone (as in k_cost), for A/B timing of
// gather variants and occupancy bounds (kmx_pgo_debug_gather_bench).
template <int R, int GV, int LBW>
__global__ __launch_bounds__(BLOCK, LBW) void k_gbench(Dev d, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  double acc[4], cost = 0.0;
  gather<R, GV, true>(d, L, V, d.pub, acc, &cost, smem);
  if (L.valid) store4(out + (size_t)L.pose * 4 * R + 4 * L.a, acc);
  const double t = block_sum(cost, reinterpret_cast<double*>(smem + SmemG<R, GV>::red_off));
  if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
}

// 4x4 diagonal blocks D_i of Q per pose (k_precond's accumulation, no shift).
__global__ void k_diag(Dev d, double* D) {
  const int pose = blockIdx.x * blockDim.x + threadIdx.x;
  if (pose >= d.nloc) return;
  double A[16];
  for (int i = 0; i < 16; ++i) A[i] = 0.0;
  for (int k = d.inc_ptr[pose]; k < d.inc_ptr[pose + 1]; ++k) {
    const bool tail = (d.inc[k].y >> 31) & 1;
    const double* er = d.irec + 16 * (size_t)k;
    const double wk = er[12], wt = er[13];
    const double* tt = er + 9;
    if (tail) {
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) A[i * 4 + j] += wt * tt[i] * tt[j] + (i == j ? wk : 0.0);
        A[i * 4 + 3] += wt * tt[i];
        A[3 * 4 + i] += wt * tt[i];
      }
      A[15] += wt;
    } else {
      A[0] += wk; A[5] += wk; A[10] += wk; A[15] += wt;
    }
  }
  for (int i = 0; i < 16; ++i) D[16 * (size_t)pose + i] = A[i];
}

// Prototype (diagnostic, G = 9): lane per incidence. out_i = D_i v_i +
// sum_{e at i} B_e v_other(e): the off-diagonal block of every incidence is
// applied by one lane to all R rows of the other endpoint (no per-row record
// redundancy), the R x 4 results go to LDS, and the (pose, row) lanes add
// their pose's incidences in CSR order. REC 0: 128-B records + inc; REC 1:
// 96-B compact records (CSR order, KMX_RECT=0).
template <int R, int REC, int CH>
__global__ __launch_bounds__(BLOCK, 4) void k_hinc(Dev d, const double* V, const double* Dg, double* out) {
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  double* Cs = hsm;                                    // [CH][R][4]
  int* sptr = reinterpret_cast<int*>(hsm + CH * R * 4);  // [TP + 1]
  const Lane L = lane_map<R>(d);
  const int tid = threadIdx.x;
  const int p0 = d.tile_p0[L.tile], np = d.tile_np[L.tile];
  const int K0 = d.inc_ptr[p0];
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  __syncthreads();
  const int n = sptr[np];
  const int pl = L.pose - p0;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int c0 = 0; c0 < n; c0 += CH) {
    const int k = c0 + tid;
    if (tid < CH && k < n) {
      double Rm[9], t[3], wk, wt;
      int o;
      bool tail;
      if constexpr (REC == 0) {
        const double2* q2 = reinterpret_cast<const double2*>(d.irec + 16 * (size_t)(K0 + k));
        double2 q[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) q[i] = q2[i];
        const int2 in = d.inc[K0 + k];
        Rm[0] = q[0].x; Rm[1] = q[0].y; Rm[2] = q[1].x; Rm[3] = q[1].y; Rm[4] = q[2].x;
        Rm[5] = q[2].y; Rm[6] = q[3].x; Rm[7] = q[3].y; Rm[8] = q[4].x;
        t[0] = q[4].y; t[1] = q[5].x; t[2] = q[5].y;
        wk = q[6].x; wt = q[6].y;
        o = in.x; tail = (in.y >> 31) & 1;
      } else {
        const double2* q2 = reinterpret_cast<const double2*>(d.crec + 12 * (size_t)(K0 + k));
        double2 q[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = q2[i];
        Edge E;
        edge_from_compact(q, E);
        const int2 in = unpack_int2(q[5].y);
#pragma unroll
        for (int i = 0; i < 9; ++i) Rm[i] = E.R[i];
        t[0] = E.t[0]; t[1] = E.t[1]; t[2] = E.t[2];
        wk = E.wk; wt = E.wt;
        o = in.x; tail = (in.y >> 31) & 1;
      }
      const double* base = (o >= 0) ? V + (size_t)o * 4 * R : d.pub + (size_t)(-1 - o) * 4 * R;
      const double2* b2 = reinterpret_cast<const double2*>(base);
      double2 vr[2 * R];
#pragma unroll
      for (int i = 0; i < 2 * R; ++i) vr[i] = b2[i];
#pragma unroll
      for (int a = 0; a < R; ++a) {
        const double v0 = vr[2 * a].x, v1 = vr[2 * a].y, v2 = vr[2 * a + 1].x, v3 = vr[2 * a + 1].y;
        double h[4];
        if (tail) {
#pragma unroll
          for (int c = 0; c < 3; ++c) h[c] = -(wk * (v0 * Rm[c * 3 + 0] + v1 * Rm[c * 3 + 1] + v2 * Rm[c * 3 + 2]) + wt * v3 * t[c]);
          h[3] = -(wt * v3);
        } else {
#pragma unroll
          for (int c = 0; c < 3; ++c) h[c] = -(wk * (v0 * Rm[0 * 3 + c] + v1 * Rm[1 * 3 + c] + v2 * Rm[2 * 3 + c]));
          h[3] = -(wt * (v3 + (v0 * t[0] + v1 * t[1] + v2 * t[2])));
        }
        store4(Cs + (tid * R + a) * 4, h);
      }
    }
    __syncthreads();
    if (L.valid) {
      const int j0 = max(sptr[pl], c0) - c0, j1 = min(sptr[pl + 1], c0 + CH) - c0;
      for (int j = j0; j < j1; ++j) {
        double h[4];
        load4(Cs + (j * R + L.a) * 4, h);
        acc[0] += h[0]; acc[1] += h[1]; acc[2] += h[2]; acc[3] += h[3];
      }
    }
    __syncthreads();
  }
  if (L.valid) {
    const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
    double vs[4];
    load4(V + o, vs);
    const double* Dp = Dg + 16 * (size_t)L.pose;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double dr[4];
      load4(Dp + 4 * c, dr);
      acc[c] += vs[0] * dr[0] + vs[1] * dr[1] + vs[2] * dr[2] + vs[3] * dr[3];
    }
    store4(out + o, acc);
  }
}

// Diagnostic: the product G = 9 Hessian gather alone (needs the handle's
// incidence-parallel records, i.e. KMX_HINC on).
template <int R, bool GRAD>
__global__ __launch_bounds__(BLOCK, 4) void k_gbench_hinc(Dev d, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  double acc[4], cost = 0.0;
  if constexpr (GRAD) hinc_grad<R>(d, L, V, d.pub, acc, &cost, smem);
  else hinc_gather<R>(d, L, V, acc, smem);
  if (L.valid) store4(out + (size_t)L.pose * 4 * R + 4 * L.a, acc);
  if constexpr (GRAD) {
    const double t = block_sum(cost, reinterpret_cast<double*>(smem + SmemHG<R>::red_off));
    if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
  }
}

}  // namespace

// ============================================================== handle ====
struct kmx_pgo {
  kmx_pgo_params P{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool have_graph = false;
  // team
  int n_robots = 0;
  std::vector<int> npose;
  std::vector<int> local_of;  // robot -> local index or -1
  std::vector<int> robots;    // local index -> robot
  std::vector<int> loff;      // local robot -> first local pose
  int nloc = 0;
  int64_t m_global = 0;
  // public table
  int64_t npub = 0, first_owned = 0, n_owned = 0;
  std::vector<int64_t> pub_key;  // sorted (robot<<32 | pose)
  // local edges
  int mloc = 0;
  std::vector<int64_t> loc_edge_gid;
  std::vector<double> ek_h, et_h;  // per local edge kappa / tau
  int ninc = 0;
  int64_t nshared = 0;
  int n_sh_local = 0, n_gnc = 0;
  std::vector<long long> m_robot;
  int ntiles = 0, tile_poses = 0;
  std::vector<int> rt0_h;  // [L + 1] first tile of each local robot
  double mu = 0.0;
  long long round_counter = 0;
  // device
  Dev dv{};
  int *d_tile_robot = nullptr, *d_tile_p0 = nullptr, *d_tile_np = nullptr, *d_rtile0 = nullptr;
  int* d_inc_ptr = nullptr;
  int2* d_inc = nullptr;
  double* d_irec = nullptr;
  double* d_crec = nullptr;  // compact records (gather variant 3), null when not usable
  double* d_ocrec = nullptr;
  bool hinc = false;  // k_hess runs the incidence-parallel gather (G = 9)
  bool publish_in_begin = false;  // the next enqueue_round also publishes the owned rows
  double* d_hrec = nullptr;
  double* d_hD = nullptr;
  double* d_hocrec = nullptr;
  int2* d_heopos = nullptr;
  int* d_optr = nullptr;
  int2* d_eopos = nullptr;
  bool compact_ok = false;
  bool rect = false;                // crec / ocrec in segment-major order (G = 5)
  int* d_trec0 = nullptr;
  int* d_torec0 = nullptr;
  int2* d_cipos = nullptr;
  double *d_ekappa = nullptr, *d_etau = nullptr, *d_ew = nullptr;
  int2* d_eipos = nullptr;
  double* d_vec = nullptr;  // X Xt g r z eta del hd
  double *d_S = nullptr, *d_Pinv = nullptr, *d_pub = nullptr, *d_part = nullptr;
  Ctl* d_ctl = nullptr;
  Counters* d_cnt = nullptr;
  unsigned* d_tickets = nullptr;
  long long* d_m_robot = nullptr;
  int* d_n_robot = nullptr;
  int* d_pub_src = nullptr;  // slot -> local pose (-1 if not local)
  int* d_own_src = nullptr;  // owned slot k -> local pose (index first_owned + k)
  int* d_gnc_edge = nullptr;
  int2* d_gnc_ends = nullptr;
  int *d_sh_edge = nullptr, *d_sh_idx = nullptr;
  int *d_osh_edge = nullptr, *d_osh_idx = nullptr;
  int n_osh = 0;
  unsigned char* d_active = nullptr;
  double* d_scratch = nullptr;  // eval in/out
  // kernel variants (KMX_GATHER: 0 direct / 1 LDS-staged; KMX_FUSED: 0 separate
  // reduce launch / 1 last-arriving-tile reduction)
  int gvar = 2, fvar = 0;
  int gvar_req = -1;  // KMX_GATHER override; default: 3 when compact records are valid, else 2
  HostStatus* hstat = nullptr;  // [L] host-mapped tCG progress per local robot
  int hstat_cap = 0;
  unsigned long long seq = 0;
  bool poll = true;             // KMX_POLL=0 enqueues every tCG step blindly
  bool poll_timeout = false;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
};

namespace {

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * count);
  if (e != hipSuccess) return kmx::fail(KMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return 0;
}

void free_dev(kmx_pgo* h) {
  void* ptrs[] = {h->d_tile_robot, h->d_tile_p0, h->d_tile_np, h->d_rtile0, h->d_inc_ptr, h->d_inc,
                  h->d_irec, h->d_crec, h->d_ocrec, h->d_optr, h->d_eopos, h->d_ekappa, h->d_etau, h->d_ew, h->d_eipos, h->d_vec, h->d_S, h->d_Pinv, h->d_pub, h->d_part, h->d_ctl, h->d_cnt,
                  h->d_m_robot, h->d_n_robot, h->d_pub_src, h->d_own_src, h->d_gnc_edge, h->d_gnc_ends,
                  h->d_sh_edge, h->d_sh_idx, h->d_osh_edge, h->d_osh_idx, h->d_active, h->d_scratch, h->d_tickets,
                  h->d_trec0, h->d_torec0, h->d_cipos, h->d_hrec, h->d_hD, h->d_hocrec, h->d_heopos};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  h->d_tile_robot = h->d_tile_p0 = h->d_tile_np = h->d_rtile0 = h->d_inc_ptr = nullptr;
  h->d_inc = nullptr; h->d_eipos = nullptr; h->d_optr = nullptr; h->d_eopos = nullptr; h->d_irec = h->d_crec = h->d_ocrec = h->d_ekappa = h->d_etau = h->d_ew = nullptr; h->d_vec = h->d_S = h->d_Pinv = h->d_pub = h->d_part = nullptr;
  h->d_ctl = nullptr; h->d_cnt = nullptr; h->d_m_robot = nullptr; h->d_n_robot = nullptr;
  h->d_trec0 = h->d_torec0 = nullptr; h->d_cipos = nullptr; h->d_hrec = h->d_hD = nullptr; h->d_hocrec = nullptr; h->d_heopos = nullptr;
  h->d_pub_src = h->d_own_src = h->d_gnc_edge = nullptr; h->d_gnc_ends = nullptr;
  h->d_sh_edge = h->d_sh_idx = nullptr; h->d_osh_edge = h->d_osh_idx = nullptr; h->d_active = nullptr; h->d_scratch = nullptr; h->d_tickets = nullptr;
}

#define KMX_DISPATCH_R(R_, CALL) \
  switch (R_) {                  \
    case 3: { constexpr int RR = 3; CALL; } break; \
    case 4: { constexpr int RR = 4; CALL; } break; \
    case 5: { constexpr int RR = 5; CALL; } break; \
    case 6: { constexpr int RR = 6; CALL; } break; \
    case 7: { constexpr int RR = 7; CALL; } break; \
    case 8: { constexpr int RR = 8; CALL; } break; \
    default: break;              \
  }

hipEvent_t next_event(kmx_pgo* h) {
  if (h->ev_used == h->ev_pool.size()) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    h->ev_pool.push_back(e);
  }
  return h->ev_pool[h->ev_used++];
}

// Local rows of the public table: this handle's robots own one contiguous
// slot range [first_owned, first_owned + n_owned).
void enqueue_publish(kmx_pgo* h) {
  const int ps = 4 * h->P.r;
  const long long tot = h->n_owned * ps;
  if (tot == 0) return;
  hipLaunchKernelGGL(k_publish, dim3((unsigned)((tot / 2 + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                     h->d_pub + (size_t)h->first_owned * ps, h->d_pub_src + h->first_owned, (int)h->n_owned, ps);
}

void enqueue_precond(kmx_pgo* h) {
  if (h->nloc == 0) return;
  hipLaunchKernelGGL(k_precond, dim3((h->nloc + 127) / 128), dim3(128), 0, h->stream, h->dv);
}

void enqueue_apply_weights(kmx_pgo* h) {
  if (h->mloc > 0)
    hipLaunchKernelGGL(k_apply_weights, dim3((h->mloc + 255) / 256), dim3(256), 0, h->stream, h->dv, h->mloc);
  enqueue_precond(h);
}

void enqueue_gnc(kmx_pgo* h) {
  if (h->n_gnc > 0)
    hipLaunchKernelGGL(k_gnc, dim3((h->n_gnc + 255) / 256), dim3(256), 0, h->stream, h->dv, h->d_gnc_edge,
                       h->d_gnc_ends, h->n_gnc, h->P.r, h->mu, h->P.gnc_barc);
  h->mu *= h->P.gnc_mu_step;
  enqueue_apply_weights(h);
}

template <int R, int G, int F>
void enqueue_round_t(kmx_pgo* h, const unsigned char* d_active) {
  const dim3 grid(h->ntiles), blk(BLOCK);
  const size_t sm = Smem<R>::bytes, smh = SmemHess<R, G>::bytes,
               smc = SmemCost<R, G>::bytes, smr = SmemGrad<R, G>::bytes;
  auto red = [&](int kind, HostStatus* hs = nullptr, unsigned long long seq = 0) {
    if (!F) hipLaunchKernelGGL(k_reduce, dim3(h->dv.L), dim3(BLOCK), 0, h->stream, h->dv, kind, R, hs, seq);
  };
  auto tcg_step = [&]() {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing) {
      e0 = next_event(h);
      e1 = next_event(h);
      (void)hipEventRecord(e0, h->stream);
    }
    hipLaunchKernelGGL((k_hess<R, G, F>), grid, blk, smh, h->stream, h->dv);
    if (h->timing) (void)hipEventRecord(e1, h->stream);
    red(RED_HESS);
    hipLaunchKernelGGL((k_update<R, G, F>), grid, blk, sm, h->stream, h->dv);
    if (h->poll && !F) {  // the per-robot reduction also reports tCG progress
      h->seq += 1;
      red(RED_UPDATE, h->hstat, h->seq);
    } else {
      red(RED_UPDATE);
    }
    return h->seq;
  };
  auto wait_running = [&](unsigned long long seq) -> unsigned long long {
    volatile HostStatus* hs = h->hstat;
    (void)hipStreamQuery(h->stream);  // make sure queued work is submitted
    const auto t0 = std::chrono::steady_clock::now();
    unsigned long long running = 0;
    for (int l = 0; l < h->dv.L; ++l) {
      unsigned long long w;
      while (((w = __atomic_load_n(&hs[l].word, __ATOMIC_ACQUIRE)) >> 1) < seq) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
          h->poll_timeout = true;  // device stalled: stop polling, enqueue blindly
          h->poll = false;
          return 1ull;
        }
      }
      running |= w & 1ull;
    }
    return running;
  };
  const long long npub_el = h->n_owned * 4 * h->P.r;
  if (h->publish_in_begin && npub_el > 0) {
    hipLaunchKernelGGL(k_round_begin_pub, dim3((unsigned)(1 + (npub_el / 2 + 255) / 256)), dim3(256), 0, h->stream,
                       h->dv, d_active, (const double*)h->d_vec, h->d_pub + (size_t)h->first_owned * 4 * h->P.r,
                       (const int*)(h->d_pub_src + h->first_owned), (int)h->n_owned, 4 * h->P.r);
  } else {
    hipLaunchKernelGGL(k_round_begin, dim3(1), dim3(std::max(64, ((h->dv.L + 63) / 64) * 64)), 0, h->stream,
                       h->dv, d_active);
  }
  for (int it = 0; it < h->P.rtr_iterations; ++it) {
    hipLaunchKernelGGL((k_grad<R, G, F>), grid, blk, smr, h->stream, h->dv);
    red(RED_GRAD);
    const int J = h->P.tcg_max_iterations;
    if (!h->poll || F) {  // the fused variant has no per-robot reduce launch to report progress
      for (int j = 0; j < J; ++j) tcg_step();
    } else {
      // Keep exactly one tCG step queued beyond the last one known to be
      // needed; stop enqueuing once every robot has left tCG.
      unsigned long long s_prev = tcg_step();
      int issued = 1;
      while (issued < J) {
        const unsigned long long s_next = tcg_step();
        ++issued;
        if (wait_running(s_prev) == 0) break;
        s_prev = s_next;
      }
    }
    hipLaunchKernelGGL((k_retract<R>), grid, blk, sm, h->stream, h->dv);
    hipLaunchKernelGGL((k_cost<R, G, F>), grid, blk, smc, h->stream, h->dv);
    red(RED_COST);
    hipLaunchKernelGGL((k_commit<R>), grid, blk, 0, h->stream, h->dv);
  }
}

template <int R>
void enqueue_round_r(kmx_pgo* h, const unsigned char* d_active) {
  switch (h->gvar * 2 + h->fvar) {
    case 0: enqueue_round_t<R, 0, 0>(h, d_active); break;
    case 1: enqueue_round_t<R, 0, 1>(h, d_active); break;
    case 2: enqueue_round_t<R, 1, 0>(h, d_active); break;
    case 3: enqueue_round_t<R, 1, 1>(h, d_active); break;
    case 4: enqueue_round_t<R, 2, 0>(h, d_active); break;
    case 5: enqueue_round_t<R, 2, 1>(h, d_active); break;
    case 6: enqueue_round_t<R, 3, 0>(h, d_active); break;
    case 7: enqueue_round_t<R, 3, 1>(h, d_active); break;
    case 10: h->hinc ? enqueue_round_t<R, 9, 0>(h, d_active) : enqueue_round_t<R, 5, 0>(h, d_active); break;
    case 11: h->hinc ? enqueue_round_t<R, 9, 1>(h, d_active) : enqueue_round_t<R, 5, 1>(h, d_active); break;
    case 14: enqueue_round_t<R, 7, 0>(h, d_active); break;
    default: enqueue_round_t<R, 7, 1>(h, d_active); break;
  }
}

// One RBCD round for the robots whose d_active flag is set.
void enqueue_round(kmx_pgo* h, const unsigned char* d_active) {
  switch (h->P.r) {
    case 3: enqueue_round_r<3>(h, d_active); break;
    case 4: enqueue_round_r<4>(h, d_active); break;
    case 5: enqueue_round_r<5>(h, d_active); break;
    case 6: enqueue_round_r<6>(h, d_active); break;
    case 7: enqueue_round_r<7>(h, d_active); break;
    default: enqueue_round_r<8>(h, d_active); break;
  }
}

bool ready(kmx_pgo* h) { return h && h->d_vec != nullptr; }

}  // namespace

// ================================================================ ABI =====
extern "C" int kmx_pgo_create(const kmx_pgo_params* params, int device, kmx_pgo** out) {
  KMX_GUARD_BEGIN
  KMX_CHECK(params && out, KMX_EINVAL, "null argument");
  KMX_CHECK(params->d == 3, KMX_EUNSUP, "only d = 3 is supported");
  KMX_CHECK(params->r >= 3 && params->r <= 8, KMX_EUNSUP, "relaxation rank must be in [3, 8]");
  KMX_CHECK(params->rtr_iterations >= 1 && params->tcg_max_iterations >= 1, KMX_EINVAL,
            "rtr_iterations and tcg_max_iterations must be >= 1");
  int ndev = 0;
  KMX_HIP(hipGetDeviceCount(&ndev));
  KMX_CHECK(device >= 0 && device < ndev, KMX_EINVAL, "bad HIP device ordinal");
  KMX_HIP(hipSetDevice(device));
  kmx_pgo* h = new kmx_pgo();
  h->P = *params;
  h->device = device;
  h->mu = params->gnc_mu_init;
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    return kmx::fail(KMX_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  h->own_stream = true;
  if (const char* v = std::getenv("KMX_GATHER")) h->gvar_req = std::min(7, std::max(0, std::atoi(v)));
  if (const char* v = std::getenv("KMX_FUSED")) h->fvar = std::atoi(v) ? 1 : 0;
  if (const char* v = std::getenv("KMX_POLL")) h->poll = std::atoi(v) != 0;
  *out = h;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_destroy(kmx_pgo* h) {
  if (!h) return KMX_OK;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_dev(h);
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  if (h->hstat) (void)hipHostFree(h->hstat);
  delete h;
  return KMX_OK;
}

extern "C" int kmx_pgo_set_stream(kmx_pgo* h, void* s) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  if (h->own_stream && h->stream) {
    KMX_HIP(hipStreamSynchronize(h->stream));
    KMX_HIP(hipStreamDestroy(h->stream));
  }
  h->own_stream = false;
  h->stream = reinterpret_cast<hipStream_t>(s);
  return KMX_OK;
}

extern "C" int kmx_pgo_set_graph(kmx_pgo* h, int n_robots, const int32_t* n_poses, const uint8_t* local,
                                 int64_t m, const int32_t* r1, const int32_t* p1, const int32_t* r2,
                                 const int32_t* p2, const double* R, const double* t, const double* kappa,
                                 const double* tau, const double* weight, const uint8_t* fixed_weight) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_CHECK(n_robots > 0 && n_poses && local, KMX_EINVAL, "bad robot arrays");
  KMX_CHECK(m >= 0 && m < (1ll << 31) - 1, KMX_EINVAL, "edge count out of range");
  KMX_CHECK(m == 0 || (r1 && p1 && r2 && p2 && R && t && kappa && tau && weight && fixed_weight), KMX_EINVAL,
            "null edge array");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  free_dev(h);
  const int r = h->P.r, ps = 4 * r;
  h->n_robots = n_robots;
  h->npose.assign(n_poses, n_poses + n_robots);
  h->local_of.assign(n_robots, -1);
  h->robots.clear();
  h->loff.clear();
  int nloc = 0;
  for (int a = 0; a < n_robots; ++a) {
    KMX_CHECK(n_poses[a] >= 0, KMX_EINVAL, "negative pose count");
    if (local[a]) {
      h->local_of[a] = (int)h->robots.size();
      h->robots.push_back(a);
      h->loff.push_back(nloc);
      nloc += n_poses[a];
    }
  }
  h->nloc = nloc;
  const int L = (int)h->robots.size();
  KMX_CHECK(L > 0, KMX_EINVAL, "no local robot");
  KMX_CHECK(L <= 1024, KMX_EUNSUP, "at most 1024 local robots per handle");
  h->m_global = m;
  // validate + public table (team-wide, so every handle agrees on slot ids)
  std::vector<int64_t> keys;
  for (int64_t e = 0; e < m; ++e) {
    KMX_CHECK(r1[e] >= 0 && r1[e] < n_robots && r2[e] >= 0 && r2[e] < n_robots, KMX_EINVAL,
              "edge robot id out of range");
    KMX_CHECK(p1[e] >= 0 && p1[e] < n_poses[r1[e]] && p2[e] >= 0 && p2[e] < n_poses[r2[e]], KMX_EINVAL,
              "edge pose id out of range");
    KMX_CHECK(!(r1[e] == r2[e] && p1[e] == p2[e]), KMX_EINVAL, "self-loop edge");
    if (r1[e] != r2[e]) {
      keys.push_back(((int64_t)r1[e] << 32) | (uint32_t)p1[e]);
      keys.push_back(((int64_t)r2[e] << 32) | (uint32_t)p2[e]);
    }
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  h->pub_key = keys;
  h->npub = (int64_t)keys.size();
  auto slot_of = [&](int rb, int pp) -> int64_t {
    const int64_t k = ((int64_t)rb << 32) | (uint32_t)pp;
    auto it = std::lower_bound(h->pub_key.begin(), h->pub_key.end(), k);
    return (it != h->pub_key.end() && *it == k) ? (int64_t)(it - h->pub_key.begin()) : -1;
  };
  std::vector<int> pub_src(std::max<int64_t>(h->npub, 1), -1);
  int64_t first = -1, last = -1;
  for (int64_t s = 0; s < h->npub; ++s) {
    const int rb = (int)(keys[s] >> 32), pp = (int)(keys[s] & 0xffffffff);
    if (h->local_of[rb] >= 0) {
      pub_src[s] = h->loff[h->local_of[rb]] + pp;
      if (first < 0) first = s;
      KMX_CHECK(last < 0 || last == s - 1, KMX_EUNSUP,
                "local robots must own a contiguous range of the public table (assign robot ranges to ranks)");
      last = s;
    }
  }
  h->first_owned = first < 0 ? 0 : first;
  h->n_owned = first < 0 ? 0 : last - first + 1;
  // local edges, incidences
  auto lpose = [&](int rb, int pp) { return h->loff[h->local_of[rb]] + pp; };
  std::vector<int64_t> ledges;
  for (int64_t e = 0; e < m; ++e)
    if (h->local_of[r1[e]] >= 0 || h->local_of[r2[e]] >= 0) ledges.push_back(e);
  h->mloc = (int)ledges.size();
  h->loc_edge_gid = ledges;
  h->ek_h.assign(std::max(h->mloc, 1), 0.0);
  h->et_h.assign(std::max(h->mloc, 1), 0.0);
  std::vector<double> ew_h(std::max(h->mloc, 1), 0.0);
  std::vector<int> deg(nloc + 1, 0);
  h->m_robot.assign(L, 0);
  for (int k = 0; k < h->mloc; ++k) {
    const int64_t e = ledges[k];
    h->ek_h[k] = kappa[e];
    h->et_h[k] = tau[e];
    ew_h[k] = weight[e];
    const int a1 = h->local_of[r1[e]], a2 = h->local_of[r2[e]];
    if (a1 >= 0) { deg[lpose(r1[e], p1[e])]++; h->m_robot[a1]++; }
    if (a2 >= 0) { deg[lpose(r2[e], p2[e])]++; if (r2[e] != r1[e]) h->m_robot[a2]++; }
  }
  std::vector<int> inc_ptr(nloc + 1, 0);
  for (int i = 0; i < nloc; ++i) inc_ptr[i + 1] = inc_ptr[i] + deg[i];
  h->ninc = inc_ptr[nloc];
  std::vector<int2> inc(std::max(inc_ptr[nloc], 1));
  std::vector<double> irec((size_t)std::max(inc_ptr[nloc], 1) * 16, 0.0);
  std::vector<int2> eipos(std::max(h->mloc, 1), make_int2(-1, -1));
  std::vector<int> fill(inc_ptr.begin(), inc_ptr.end() - 1);
  auto put_rec = [&](int pos, int64_t e) {  // per-incidence copy of the edge record
    double* rec = &irec[(size_t)pos * 16];
    for (int q = 0; q < 9; ++q) rec[q] = R[9 * e + q];
    for (int q = 0; q < 3; ++q) rec[9 + q] = t[3 * e + q];
    rec[12] = weight[e] * kappa[e];
    rec[13] = weight[e] * tau[e];
  };
  for (int k = 0; k < h->mloc; ++k) {  // increasing global edge id per pose
    const int64_t e = ledges[k];
    const bool priv = r1[e] == r2[e];
    if (h->local_of[r1[e]] >= 0) {
      const int sp = lpose(r1[e], p1[e]);
      const int other = priv ? lpose(r2[e], p2[e]) : (int)(-1 - slot_of(r2[e], p2[e]));
      eipos[k].x = fill[sp];
      put_rec(fill[sp], e);
      inc[fill[sp]++] = make_int2(other, (int)(k | 0x80000000u));
    }
    if (h->local_of[r2[e]] >= 0) {
      const int sp = lpose(r2[e], p2[e]);
      const int other = priv ? lpose(r1[e], p1[e]) : (int)(-1 - slot_of(r1[e], p1[e]));
      eipos[k].y = fill[sp];
      put_rec(fill[sp], e);
      inc[fill[sp]++] = make_int2(other, k);
    }
  }
  // GNC ownership (owner = lower robot id, drawio:2198) and shared-weight table
  std::vector<int> gnc_edge, sh_edge, sh_idx, osh_edge, osh_idx;
  std::vector<int2> gnc_ends;
  int64_t nsh = 0;
  {
    size_t k = 0;
    for (int64_t e = 0; e < m; ++e) {
      if (r1[e] == r2[e]) continue;
      const int64_t si = nsh++;
      while (k < ledges.size() && ledges[k] < e) ++k;
      if (k < ledges.size() && ledges[k] == e) {
        sh_edge.push_back((int)k);
        sh_idx.push_back((int)si);
        if (h->local_of[std::min(r1[e], r2[e])] >= 0) {
          osh_edge.push_back((int)k);
          osh_idx.push_back((int)si);
        }
      }
    }
  }
  h->nshared = nsh;
  for (int k = 0; k < h->mloc; ++k) {
    const int64_t e = ledges[k];
    if (fixed_weight[e]) continue;
    const int owner = std::min(r1[e], r2[e]);
    if (h->local_of[owner] < 0) continue;
    auto enc = [&](int rb, int pp) -> int {
      if (rb == owner) return lpose(rb, pp);
      return (int)(-1 - slot_of(rb, pp));
    };
    gnc_edge.push_back(k);
    gnc_ends.push_back(make_int2(enc(r1[e], p1[e]), enc(r2[e], p2[e])));
  }
  h->n_gnc = (int)gnc_edge.size();
  h->n_sh_local = (int)sh_edge.size();
  h->n_osh = (int)osh_edge.size();
  // tiles
  const int PPW = 64 / r;
  h->tile_poses = WAVES * PPW;
  std::vector<int> tr, tp0, tnp, rt0(L + 1, 0);
  // Incidence-balanced tiles: a tile holds at most tile_poses poses and about
  // the robot's mean incidences per full tile, so every workgroup's gather
  // walks about the same number of incidences (segments of equal length S =
  // ceil(incidences / groups)); KMX_TILEBAL=0 cuts plain runs of tile_poses.
  bool tilebal = true;
  if (const char* v = std::getenv("KMX_TILEBAL")) tilebal = std::atoi(v) != 0;
  // The incidence-parallel kernels (G = 9) walk a tile in chunks of TP * r
  // incidences, one LDS hand-off each: capping tiles at two chunks takes the
  // Hessian gather from ~3 to 2 hand-offs (32 -> 30 us at configs[3]).
  // KMX_TILECAP overrides (0 = no cap).
  int64_t tilecap = INT64_MAX;
  {
    const char* hv = std::getenv("KMX_HINC");
    const bool g9 = r <= 5 && (h->gvar_req < 0 || h->gvar_req == 5) && !(hv && std::atoi(hv) == 0);
    if (g9) tilecap = 2 * (int64_t)(WAVES * (64 / r) * r);
    if (const char* v = std::getenv("KMX_TILECAP")) tilecap = std::atoi(v) > 0 ? std::atoi(v) : INT64_MAX;
  }
  for (int l = 0; l < L; ++l) {
    const int n = n_poses[h->robots[l]];
    const int base = h->loff[l];
    rt0[l] = (int)tr.size();
    const int64_t inc_l = (int64_t)inc_ptr[base + n] - inc_ptr[base];
    const int64_t full = std::max<int64_t>(1, (n + h->tile_poses - 1) / h->tile_poses);
    const int64_t cap =
        std::min(tilecap, tilebal ? std::max<int64_t>(1, (inc_l * 21 / 20 + full - 1) / full) : INT64_MAX);
    int p0 = 0;
    while (p0 < n) {
      int np = 0;
      int64_t cum = 0;
      while (p0 + np < n && np < h->tile_poses) {
        const int64_t dg = inc_ptr[base + p0 + np + 1] - inc_ptr[base + p0 + np];
        if (np > 0 && cum + dg > cap) break;
        cum += dg;
        ++np;
      }
      tr.push_back(l);
      tp0.push_back(base + p0);
      tnp.push_back(np);
      p0 += np;
    }
  }
  rt0[L] = (int)tr.size();
  h->rt0_h = rt0;
  h->ntiles = (int)tr.size();
  std::vector<int> own_src(std::max<int64_t>(h->n_owned, 1), 0);
  for (int64_t k = 0; k < h->n_owned; ++k) own_src[k] = pub_src[h->first_owned + k];
  std::vector<int> nrob(L);
  for (int l = 0; l < L; ++l) nrob[l] = n_poses[h->robots[l]];
  // device
  int rc;
  const size_t vec = (size_t)std::max(nloc, 1) * ps;
  // Compact records: valid when every local rotation's third row equals row0 x
  // row1 to 1e-12 (measurements in SO(3)); the gathers then rebuild row 2.
  std::vector<double> crec, ocrec;
  std::vector<int> optr;
  std::vector<int2> eopos;
  {
    bool ok = true;
    for (int k = 0; k < h->mloc && ok; ++k) {
      const double* Q = R + 9 * ledges[k];
      const double c0 = Q[1] * Q[5] - Q[2] * Q[4], c1 = Q[2] * Q[3] - Q[0] * Q[5], c2 = Q[0] * Q[4] - Q[1] * Q[3];
      ok = std::fabs(c0 - Q[6]) <= 1e-12 && std::fabs(c1 - Q[7]) <= 1e-12 && std::fabs(c2 - Q[8]) <= 1e-12;
    }
    h->compact_ok = ok;
    const bool want = (h->gvar_req < 0 || h->gvar_req == 3 || h->gvar_req == 5 || h->gvar_req == 7);
    h->gvar = (ok && want) ? (h->gvar_req < 0 ? KMX_GATHER_DEFAULT : h->gvar_req)
                           : (h->gvar_req >= 0 && h->gvar_req < 3 ? h->gvar_req : 2);
    if (h->gvar == 3 || h->gvar == 5 || h->gvar == 7) {
      const size_t ni = (size_t)std::max(h->ninc, 1);
      crec.assign(ni * 12, 0.0);
      for (size_t k = 0; k < (size_t)h->ninc; ++k) {
        const double* a = &irec[k * 16];
        double* c = &crec[k * 12];
        for (int q = 0; q < 6; ++q) c[q] = a[q];
        c[6] = a[9]; c[7] = a[10]; c[8] = a[11];
        c[9] = a[12]; c[10] = a[13];
        const long long bits = (long long)(unsigned)inc[k].x | ((long long)inc[k].y << 32);
        std::memcpy(&c[11], &bits, 8);
      }
      // owner incidences, in CSR order
      optr.assign(nloc + 1, 0);
      eopos.assign(std::max(h->mloc, 1), make_int2(-1, -1));
      for (int p = 0; p < nloc; ++p) {
        optr[p + 1] = optr[p];
        for (int k = inc_ptr[p]; k < inc_ptr[p + 1]; ++k) {
          const bool own = inc[k].x < 0 || (((unsigned)inc[k].y) >> 31);
          if (!own) continue;
          const int pos = optr[p + 1]++;
          ocrec.insert(ocrec.end(), crec.begin() + 12 * (size_t)k, crec.begin() + 12 * (size_t)(k + 1));
          int2& ep = eopos[inc[k].y & 0x7fffffff];
          if (ep.x < 0) ep.x = pos;
          else ep.y = pos;
        }
      }
      if (ocrec.empty()) ocrec.assign(12, 0.0);
    }
  }
  // The incidence-parallel kernels (G = 9: k_hess, k_cost) read the compact
  // records in CSR order; k_grad keeps the degree-balanced gather.
  std::vector<double> hrec, hocrec;
  std::vector<int2> heopos;
  h->hinc = false;
  if (h->gvar == 5 && r <= 5) {  // r >= 6 spills at 128 VGPRs: keep the row gather there
    bool want = true;
    if (const char* v = std::getenv("KMX_HINC")) want = std::atoi(v) != 0;
    if (want) {
      hrec.assign(crec.begin(), crec.begin() + 12 * (size_t)h->ninc);
      hrec.resize(hrec.size() + 12, 0.0);  // pad record (clamped loads of an empty tile)
      hocrec = ocrec;
      hocrec.resize(hocrec.size() + 12, 0.0);
      heopos = eopos;
      h->hinc = true;
    }
  }
  // Segment-major record layout for the degree-balanced gather (G = 5/6): a
  // tile's n incidences form TP lane-group segments of S = ceil(n / TP); the
  // record of (segment g, step j) is stored at tile base + j*TP + g, so at every
  // step the groups of a wave read consecutive records (full cache lines)
  // instead of TP records S apart. KMX_RECT=0 keeps CSR order.
  std::vector<int> trec0, torec0;
  std::vector<int2> cipos;
  h->rect = false;
  {
    bool want = true;
    if (const char* v = std::getenv("KMX_RECT")) want = std::atoi(v) != 0;
    if (want && h->gvar == 5) {
      const int TP = WAVES * (64 / r);
      auto transpose = [&](const std::vector<int>& ptr, std::vector<double>& rec, std::vector<int>& base,
                           std::vector<int64_t>& map) {
        base.assign(h->ntiles + 1, 0);
        int64_t tot = 0;
        for (int t = 0; t < h->ntiles; ++t) {
          const int n = ptr[tp0[t] + tnp[t]] - ptr[tp0[t]];
          base[t] = (int)tot;
          tot += (int64_t)TP * std::max(1, (n + TP - 1) / TP);
        }
        base[h->ntiles] = (int)tot;
        std::vector<double> out((size_t)std::max<int64_t>(tot, 1) * 12, 0.0);
        map.assign(rec.size() / 12, -1);
        for (int t = 0; t < h->ntiles; ++t) {
          const int K0 = ptr[tp0[t]], n = ptr[tp0[t] + tnp[t]] - K0;
          const int S = std::max(1, (n + TP - 1) / TP);
          for (int k = 0; k < n; ++k) {
            const int64_t dst = base[t] + (int64_t)(k % S) * TP + k / S;
            std::memcpy(&out[(size_t)dst * 12], &rec[(size_t)(K0 + k) * 12], 12 * sizeof(double));
            map[K0 + k] = dst;
          }
        }
        rec.swap(out);
      };
      std::vector<int64_t> cmap, omap;
      transpose(inc_ptr, crec, trec0, cmap);
      transpose(optr, ocrec, torec0, omap);
      cipos.assign(std::max(h->mloc, 1), make_int2(-1, -1));
      for (int k = 0; k < h->mloc; ++k) {
        cipos[k].x = eipos[k].x >= 0 ? (int)cmap[eipos[k].x] : -1;
        cipos[k].y = eipos[k].y >= 0 ? (int)cmap[eipos[k].y] : -1;
        int2& ep = eopos[k];
        ep.x = ep.x >= 0 ? (int)omap[ep.x] : -1;
        ep.y = ep.y >= 0 ? (int)omap[ep.y] : -1;
      }
      h->rect = true;
    }
  }
  if ((rc = dalloc(&h->d_tile_robot, h->ntiles)) || (rc = dalloc(&h->d_tile_p0, h->ntiles)) ||
      (rc = dalloc(&h->d_tile_np, h->ntiles)) || (rc = dalloc(&h->d_rtile0, L + 1)) ||
      (rc = dalloc(&h->d_inc_ptr, nloc + 1)) || (rc = dalloc(&h->d_inc, inc.size())) ||
      (rc = dalloc(&h->d_irec, irec.size())) || (rc = dalloc(&h->d_ekappa, h->ek_h.size())) ||
      (rc = dalloc(&h->d_etau, h->et_h.size())) || (rc = dalloc(&h->d_ew, ew_h.size())) ||
      (rc = dalloc(&h->d_eipos, eipos.size())) || (rc = dalloc(&h->d_vec, vec * 8)) ||
      (rc = dalloc(&h->d_S, (size_t)std::max(nloc, 1) * 9)) ||
      (rc = dalloc(&h->d_Pinv, (size_t)std::max(nloc, 1) * 16)) ||
      (rc = dalloc(&h->d_pub, (size_t)std::max<int64_t>(h->npub, 1) * ps)) ||
      (rc = dalloc(&h->d_part, (size_t)std::max(h->ntiles, 1) * NPART)) || (rc = dalloc(&h->d_ctl, L)) ||
      (rc = dalloc(&h->d_cnt, 1)) || (rc = dalloc(&h->d_tickets, L)) || (rc = dalloc(&h->d_m_robot, L)) || (rc = dalloc(&h->d_n_robot, L)) ||
      (rc = dalloc(&h->d_pub_src, pub_src.size())) || (rc = dalloc(&h->d_own_src, own_src.size())) ||
      (rc = dalloc(&h->d_gnc_edge, std::max(h->n_gnc, 1))) ||
      (rc = dalloc(&h->d_gnc_ends, std::max(h->n_gnc, 1))) ||
      (rc = dalloc(&h->d_sh_edge, std::max(h->n_sh_local, 1))) ||
      (rc = dalloc(&h->d_sh_idx, std::max(h->n_sh_local, 1))) || (rc = dalloc(&h->d_active, L)) ||
      (rc = dalloc(&h->d_osh_edge, std::max(h->n_osh, 1))) || (rc = dalloc(&h->d_osh_idx, std::max(h->n_osh, 1))) ||
      (rc = dalloc(&h->d_scratch, vec * 2))) {
    free_dev(h);
    return rc;
  }
  auto up = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream);
  };
  KMX_HIP(up(h->d_tile_robot, tr.data(), sizeof(int) * tr.size()));
  KMX_HIP(up(h->d_tile_p0, tp0.data(), sizeof(int) * tp0.size()));
  KMX_HIP(up(h->d_tile_np, tnp.data(), sizeof(int) * tnp.size()));
  KMX_HIP(up(h->d_rtile0, rt0.data(), sizeof(int) * rt0.size()));
  KMX_HIP(up(h->d_inc_ptr, inc_ptr.data(), sizeof(int) * inc_ptr.size()));
  KMX_HIP(up(h->d_inc, inc.data(), sizeof(int2) * inc.size()));
  KMX_HIP(up(h->d_irec, irec.data(), sizeof(double) * irec.size()));
  if (h->gvar == 3 || h->gvar == 5 || h->gvar == 7) {
    if ((rc = dalloc(&h->d_crec, crec.size())) || (rc = dalloc(&h->d_ocrec, ocrec.size())) ||
        (rc = dalloc(&h->d_optr, optr.size())) || (rc = dalloc(&h->d_eopos, eopos.size()))) {
      free_dev(h);
      return rc;
    }
    KMX_HIP(up(h->d_crec, crec.data(), sizeof(double) * crec.size()));
    KMX_HIP(up(h->d_ocrec, ocrec.data(), sizeof(double) * ocrec.size()));
    KMX_HIP(up(h->d_optr, optr.data(), sizeof(int) * optr.size()));
    KMX_HIP(up(h->d_eopos, eopos.data(), sizeof(int2) * eopos.size()));
  }
  if (h->hinc) {
    if ((rc = dalloc(&h->d_hrec, hrec.size())) || (rc = dalloc(&h->d_hD, (size_t)std::max(nloc, 1) * 16)) ||
        (rc = dalloc(&h->d_hocrec, hocrec.size())) || (rc = dalloc(&h->d_heopos, heopos.size()))) {
      free_dev(h);
      return rc;
    }
    KMX_HIP(up(h->d_hrec, hrec.data(), sizeof(double) * hrec.size()));
    KMX_HIP(up(h->d_hocrec, hocrec.data(), sizeof(double) * hocrec.size()));
    KMX_HIP(up(h->d_heopos, heopos.data(), sizeof(int2) * heopos.size()));
  }
  if (h->rect) {
    if ((rc = dalloc(&h->d_trec0, trec0.size())) || (rc = dalloc(&h->d_torec0, torec0.size())) ||
        (rc = dalloc(&h->d_cipos, cipos.size()))) {
      free_dev(h);
      return rc;
    }
    KMX_HIP(up(h->d_trec0, trec0.data(), sizeof(int) * trec0.size()));
    KMX_HIP(up(h->d_torec0, torec0.data(), sizeof(int) * torec0.size()));
    KMX_HIP(up(h->d_cipos, cipos.data(), sizeof(int2) * cipos.size()));
  }
  KMX_HIP(up(h->d_ekappa, h->ek_h.data(), sizeof(double) * h->ek_h.size()));
  KMX_HIP(up(h->d_etau, h->et_h.data(), sizeof(double) * h->et_h.size()));
  KMX_HIP(up(h->d_ew, ew_h.data(), sizeof(double) * ew_h.size()));
  KMX_HIP(up(h->d_eipos, eipos.data(), sizeof(int2) * eipos.size()));
  KMX_HIP(hipMemsetAsync(h->d_vec, 0, sizeof(double) * vec * 8, h->stream));
  KMX_HIP(hipMemsetAsync(h->d_pub, 0, sizeof(double) * std::max<int64_t>(h->npub, 1) * ps, h->stream));
  KMX_HIP(hipMemsetAsync(h->d_ctl, 0, sizeof(Ctl) * L, h->stream));
  if (L > h->hstat_cap) {  // host-mapped per-robot tCG progress
    if (h->hstat) (void)hipHostFree(h->hstat);
    h->hstat = nullptr;
    h->hstat_cap = 0;
    KMX_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->hstat), sizeof(HostStatus) * L,
                          hipHostMallocMapped | hipHostMallocCoherent));
    h->hstat_cap = L;
  }
  for (int l = 0; l < L; ++l) h->hstat[l].word = 0;
  h->seq = 0;
  KMX_HIP(hipMemsetAsync(h->d_cnt, 0, sizeof(Counters), h->stream));
  KMX_HIP(hipMemsetAsync(h->d_tickets, 0, sizeof(unsigned) * L, h->stream));
  KMX_HIP(up(h->d_m_robot, h->m_robot.data(), sizeof(long long) * L));
  KMX_HIP(up(h->d_n_robot, nrob.data(), sizeof(int) * L));
  KMX_HIP(up(h->d_pub_src, pub_src.data(), sizeof(int) * pub_src.size()));
  KMX_HIP(up(h->d_own_src, own_src.data(), sizeof(int) * own_src.size()));
  if (h->n_gnc) {
    KMX_HIP(up(h->d_gnc_edge, gnc_edge.data(), sizeof(int) * gnc_edge.size()));
    KMX_HIP(up(h->d_gnc_ends, gnc_ends.data(), sizeof(int2) * gnc_ends.size()));
  }
  if (h->n_sh_local) {
    KMX_HIP(up(h->d_sh_edge, sh_edge.data(), sizeof(int) * sh_edge.size()));
    KMX_HIP(up(h->d_sh_idx, sh_idx.data(), sizeof(int) * sh_idx.size()));
  }
  if (h->n_osh) {
    KMX_HIP(up(h->d_osh_edge, osh_edge.data(), sizeof(int) * osh_edge.size()));
    KMX_HIP(up(h->d_osh_idx, osh_idx.data(), sizeof(int) * osh_idx.size()));
  }
  std::vector<unsigned char> ones(L, 1);
  KMX_HIP(up(h->d_active, ones.data(), L));
  // host vectors must outlive the async copies
  KMX_HIP(hipStreamSynchronize(h->stream));
  Dev& d = h->dv;
  d.ntiles = h->ntiles; d.L = L; d.nloc = nloc; d.npub = (int)h->npub;
  d.tile_robot = h->d_tile_robot; d.tile_p0 = h->d_tile_p0; d.tile_np = h->d_tile_np; d.rtile0 = h->d_rtile0;
  d.inc_ptr = h->d_inc_ptr; d.inc = h->d_inc; d.irec = h->d_irec; d.crec = h->d_crec;
  d.ocrec = h->d_ocrec; d.optr = h->d_optr; d.eopos = h->d_eopos;
  d.ekappa = h->d_ekappa; d.etau = h->d_etau; d.ew = h->d_ew; d.eipos = h->d_eipos;
  d.cipos = h->rect ? h->d_cipos : h->d_eipos;
  d.trec0 = h->d_trec0; d.torec0 = h->d_torec0; d.rect = h->rect ? 1 : 0;
  d.hrec = h->hinc ? h->d_hrec : nullptr; d.hD = h->hinc ? h->d_hD : nullptr;
  d.hocrec = h->hinc ? h->d_hocrec : nullptr; d.heopos = h->hinc ? h->d_heopos : nullptr;
  d.dbg = 0;
  if (const char* v = std::getenv("KMX_PGO_DBG")) d.dbg = std::atoi(v);
  d.X = h->d_vec; d.Xt = h->d_vec + vec; d.g = h->d_vec + 2 * vec; d.r = h->d_vec + 3 * vec;
  d.z = h->d_vec + 4 * vec; d.eta = h->d_vec + 5 * vec; d.del = h->d_vec + 6 * vec; d.hd = h->d_vec + 7 * vec;
  d.S = h->d_S; d.Pinv = h->d_Pinv; d.pub = h->d_pub; d.part = h->d_part; d.ctl = h->d_ctl; d.cnt = h->d_cnt; d.tickets = h->d_tickets;
  d.m_robot = h->d_m_robot; d.n_robot = h->d_n_robot;
  d.p.tcg_max = h->P.tcg_max_iterations; d.p.rtr_iters = h->P.rtr_iterations;
  d.p.use_precond = h->P.use_preconditioner; d.p.robust = h->P.robust_cost;
  d.p.kappa = h->P.tcg_kappa; d.p.theta = h->P.tcg_theta; d.p.Delta0 = h->P.rtr_initial_radius;
  d.p.Delta_max = h->P.rtr_max_radius; d.p.accept_rho = h->P.rtr_accept_rho; d.p.gn_tol = h->P.gradnorm_tol;
  d.p.shift = h->P.precond_shift; d.p.barc = h->P.gnc_barc;
  enqueue_precond(h);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
  h->round_counter = 0;
  return KMX_OK;
  KMX_GUARD_END
}

static int check_robot(kmx_pgo* h, int robot) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(robot >= 0 && robot < h->n_robots && h->local_of[robot] >= 0, KMX_EINVAL, "robot is not local");
  return 0;
}

extern "C" int kmx_pgo_set_iterate(kmx_pgo* h, int robot, const double* X) {
  if (int rc = check_robot(h, robot)) return rc;
  KMX_CHECK(X, KMX_EINVAL, "null X");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r, l = h->local_of[robot];
  KMX_HIP(hipMemcpyAsync(h->d_vec + (size_t)h->loff[l] * ps, X, sizeof(double) * h->npose[robot] * ps,
                         hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_get_iterate(kmx_pgo* h, int robot, double* X) {
  if (int rc = check_robot(h, robot)) return rc;
  KMX_CHECK(X, KMX_EINVAL, "null X");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r, l = h->local_of[robot];
  KMX_HIP(hipMemcpyAsync(X, h->d_vec + (size_t)h->loff[l] * ps, sizeof(double) * h->npose[robot] * ps,
                         hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_public_count(kmx_pgo* h, int64_t* n_public, int64_t* first_owned, int64_t* n_owned) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  if (n_public) *n_public = h->npub;
  if (first_owned) *first_owned = h->first_owned;
  if (n_owned) *n_owned = h->n_owned;
  return KMX_OK;
}

extern "C" int kmx_pgo_pack_public(kmx_pgo* h, void* dev_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(dev_out || h->n_owned == 0, KMX_EINVAL, "null device buffer");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r;
  const long long tot = h->n_owned * ps;
  if (tot)
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                       (double*)dev_out, h->d_own_src, 0, (int)h->n_owned, ps);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_unpack_public(kmx_pgo* h, const void* dev_table) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(dev_table || h->npub == 0, KMX_EINVAL, "null device buffer");
  KMX_HIP(hipSetDevice(h->device));
  if (h->npub)
    KMX_HIP(hipMemcpyAsync(h->d_pub, dev_table, sizeof(double) * h->npub * 4 * h->P.r, hipMemcpyDeviceToDevice,
                           h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_gather_public_rows(kmx_pgo* h, const int32_t* dev_slots, int64_t n, void* dev_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(n >= 0 && (n == 0 || (dev_slots && dev_out)), KMX_EINVAL, "bad argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r;
  const long long tot = (long long)n * ps;
  if (tot)
    hipLaunchKernelGGL(k_gather_slots, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                       h->d_pub_src, (const int*)dev_slots, (long long)n, (int)h->npub, (double*)dev_out, ps);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_scatter_public_rows(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const void* dev_rows) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(n >= 0 && (n == 0 || (dev_slots && dev_rows)), KMX_EINVAL, "bad argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r;
  const long long tot = (long long)n * ps;
  if (tot)
    hipLaunchKernelGGL(k_scatter_slots, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->d_pub,
                       (const int*)dev_slots, (long long)n, (int)h->npub, (const double*)dev_rows, ps);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_refresh_local(kmx_pgo* h) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_HIP(hipSetDevice(h->device));
  enqueue_publish(h);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_set_neighbor_poses(kmx_pgo* h, int64_t count, const int32_t* robot, const int32_t* pose,
                                          const double* X) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(count == 0 || (robot && pose && X), KMX_EINVAL, "null argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r;
  std::vector<double> tab((size_t)std::max<int64_t>(h->npub, 1) * ps);
  KMX_HIP(hipMemcpyAsync(tab.data(), h->d_pub, sizeof(double) * h->npub * ps, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  for (int64_t i = 0; i < count; ++i) {
    const int64_t k = ((int64_t)robot[i] << 32) | (uint32_t)pose[i];
    auto it = std::lower_bound(h->pub_key.begin(), h->pub_key.end(), k);
    KMX_CHECK(it != h->pub_key.end() && *it == k, KMX_EINVAL, "pose is not public (no shared edge)");
    std::memcpy(&tab[(size_t)(it - h->pub_key.begin()) * ps], X + (size_t)i * ps, sizeof(double) * ps);
  }
  KMX_HIP(hipMemcpyAsync(h->d_pub, tab.data(), sizeof(double) * h->npub * ps, hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_iterate(kmx_pgo* h, const uint8_t* active, kmx_iter_stats* stats) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(active, KMX_EINVAL, "null active mask");
  KMX_HIP(hipSetDevice(h->device));
  const int L = (int)h->robots.size();
  std::vector<unsigned char> act(L);
  for (int l = 0; l < L; ++l) act[l] = active[h->robots[l]] ? 1 : 0;
  KMX_HIP(hipMemcpyAsync(h->d_active, act.data(), L, hipMemcpyHostToDevice, h->stream));
  enqueue_round(h, h->d_active);
  KMX_HIP(hipGetLastError());
  std::vector<Ctl> ctl(L);
  KMX_HIP(hipMemcpyAsync(ctl.data(), h->d_ctl, sizeof(Ctl) * L, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  // restore the all-active mask used by iterate_async
  std::vector<unsigned char> ones(L, 1);
  KMX_HIP(hipMemcpyAsync(h->d_active, ones.data(), L, hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  if (stats) {
    for (int a = 0; a < h->n_robots; ++a) std::memset(&stats[a], 0, sizeof(kmx_iter_stats));
    for (int l = 0; l < L; ++l) {
      const Ctl& c = ctl[l];
      kmx_iter_stats& s = stats[h->robots[l]];
      s.updated = c.updated;
      s.tcg_iterations = c.tcg_iter;
      s.tcg_stop = c.tcg_stop;
      s.accepted = c.accepted;
      s.f_init = c.f_init;
      s.gradnorm_init = c.gn_init;
      s.f_final = c.f_final;
      s.rho = c.rho;
      s.radius = c.Delta;
      s.rel_change = c.rel_change;
      s.edges = h->m_robot[l];
      s.hessvecs = c.hessvecs;
    }
  }
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_iterate_async(kmx_pgo* h, int rounds, int refresh_local, int gnc_every) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(rounds >= 0, KMX_EINVAL, "negative rounds");
  KMX_HIP(hipSetDevice(h->device));
  for (int i = 0; i < rounds; ++i) {
    h->publish_in_begin = refresh_local != 0;  // k_publish folded into the round's first launch
    enqueue_round(h, h->d_active);
    h->publish_in_begin = false;
    h->round_counter++;
    if (gnc_every > 0 && h->P.robust_cost == KMX_COST_GNC_TLS && h->round_counter % gnc_every == 0) {
      if (refresh_local) enqueue_publish(h);
      enqueue_gnc(h);
    }
  }
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_sync(kmx_pgo* h) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_update_weights(kmx_pgo* h, double* mu_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_HIP(hipSetDevice(h->device));
  if (mu_out) *mu_out = h->mu;
  if (h->P.robust_cost != KMX_COST_GNC_TLS) return KMX_OK;
  enqueue_gnc(h);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_get_mu(kmx_pgo* h, double* mu) {
  KMX_CHECK(h && mu, KMX_EINVAL, "null argument");
  *mu = h->mu;
  return KMX_OK;
}
extern "C" int kmx_pgo_set_mu(kmx_pgo* h, double mu) {
  KMX_CHECK(h && mu > 0.0, KMX_EINVAL, "mu must be positive");
  h->mu = mu;
  return KMX_OK;
}

extern "C" int kmx_pgo_get_weights(kmx_pgo* h, double* w) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h) && w, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  std::vector<double> ew(std::max(h->mloc, 1));
  KMX_HIP(hipMemcpyAsync(ew.data(), h->d_ew, sizeof(double) * h->mloc, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  for (int k = 0; k < h->mloc; ++k) w[h->loc_edge_gid[k]] = ew[k];
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_set_weights(kmx_pgo* h, const double* w) {
  KMX_CHECK(ready(h) && w, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  std::vector<double> ew(std::max(h->mloc, 1));
  for (int k = 0; k < h->mloc; ++k) ew[k] = w[h->loc_edge_gid[k]];
  KMX_HIP(hipMemcpyAsync(h->d_ew, ew.data(), sizeof(double) * h->mloc, hipMemcpyHostToDevice, h->stream));
  enqueue_apply_weights(h);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_shared_count(kmx_pgo* h, int64_t* n_shared) {
  KMX_CHECK(ready(h) && n_shared, KMX_EINVAL, "null argument / no graph");
  *n_shared = h->nshared;
  return KMX_OK;
}

extern "C" int kmx_pgo_pack_shared_weights(kmx_pgo* h, void* dev_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(dev_out || h->nshared == 0, KMX_EINVAL, "null device buffer");
  KMX_HIP(hipSetDevice(h->device));
  if (h->nshared == 0) return KMX_OK;
  KMX_HIP(hipMemsetAsync(dev_out, 0, sizeof(double) * h->nshared, h->stream));
  if (h->n_osh)
    hipLaunchKernelGGL(k_shared_pack, dim3((h->n_osh + 255) / 256), dim3(256), 0, h->stream,
                       (const double*)h->d_ew, h->d_osh_edge, h->d_osh_idx, h->n_osh, (double*)dev_out);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_unpack_shared_weights(kmx_pgo* h, const void* dev_table) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(dev_table || h->nshared == 0, KMX_EINVAL, "null device buffer");
  KMX_HIP(hipSetDevice(h->device));
  if (h->n_sh_local)
    hipLaunchKernelGGL(k_shared_unpack, dim3((h->n_sh_local + 255) / 256), dim3(256), 0, h->stream, h->d_ew,
                       h->d_sh_edge, h->d_sh_idx, h->n_sh_local, (const double*)dev_table);
  enqueue_apply_weights(h);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_get_trajectory(kmx_pgo* h, int robot, const double* anchor, double* out) {
  KMX_GUARD_BEGIN
  if (int rc = check_robot(h, robot)) return rc;
  KMX_CHECK(anchor && out, KMX_EINVAL, "null argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r, l = h->local_of[robot], n = h->npose[robot];
  double* d_anchor = h->d_scratch;
  double* d_out = h->d_scratch + ps;
  KMX_CHECK((size_t)ps + (size_t)n * 12 <= (size_t)std::max(h->nloc, 1) * ps * 2, KMX_EINVAL, "scratch too small");
  KMX_HIP(hipMemcpyAsync(d_anchor, anchor, sizeof(double) * ps, hipMemcpyHostToDevice, h->stream));
  if (n)
    hipLaunchKernelGGL(k_traj, dim3((n + 127) / 128), dim3(128), 0, h->stream,
                       (const double*)(h->d_vec + (size_t)h->loff[l] * ps), n, h->P.r, (const double*)d_anchor, d_out);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipMemcpyAsync(out, d_out, sizeof(double) * n * 12, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_eval(kmx_pgo* h, int robot, int mode, const double* V, double* out, double* scalar) {
  KMX_GUARD_BEGIN
  if (int rc = check_robot(h, robot)) return rc;
  KMX_CHECK(mode >= KMX_EVAL_COST_EGRAD && mode <= KMX_EVAL_RETRACT, KMX_EINVAL, "bad eval mode");
  KMX_CHECK(out && (V || mode == KMX_EVAL_RGRAD), KMX_EINVAL, "null argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r, l = h->local_of[robot], n = h->npose[robot];
  const size_t vec = (size_t)std::max(h->nloc, 1) * ps;
  double* dV = h->d_scratch;
  double* dO = h->d_scratch + vec;
  const size_t o = (size_t)h->loff[l] * ps;
  KMX_HIP(hipMemsetAsync(h->d_scratch, 0, sizeof(double) * vec * 2, h->stream));
  if (V) KMX_HIP(hipMemcpyAsync(dV + o, V, sizeof(double) * n * ps, hipMemcpyHostToDevice, h->stream));
  const int R_ = h->P.r;
  if (h->gvar == 1) {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 1>), dim3(h->ntiles), dim3(BLOCK), Smem<RR>::bytes, h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  } else if (h->gvar == 2) {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 2>), dim3(h->ntiles), dim3(BLOCK), Smem<RR>::bytes, h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  } else if (h->gvar == 3) {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 3>), dim3(h->ntiles), dim3(BLOCK), Smem<RR>::bytes, h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  } else if (h->gvar == 5) {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 5>), dim3(h->ntiles), dim3(BLOCK), Smem<RR>::bytes, h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  } else if (h->gvar == 7) {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 7>), dim3(h->ntiles), dim3(BLOCK), (SmemG<RR, 7>::bytes), h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  } else {
    KMX_DISPATCH_R(R_, hipLaunchKernelGGL((k_eval<RR, 0>), dim3(h->ntiles), dim3(BLOCK), Smem<RR>::bytes, h->stream,
                                          h->dv, l, mode, (const double*)dV, dO));
  }
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipMemcpyAsync(out, dO + o, sizeof(double) * n * ps, hipMemcpyDeviceToHost, h->stream));
  std::vector<int> rt0(2);
  std::vector<double> part((size_t)h->ntiles * NPART);
  KMX_HIP(hipMemcpyAsync(part.data(), h->d_part, sizeof(double) * part.size(), hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  // tiles of robot l are contiguous
  const int t0 = h->rt0_h[l], nt = h->rt0_h[l + 1] - h->rt0_h[l];
  double s = 0.0;
  for (int tt = t0; tt < t0 + nt; ++tt) s += part[(size_t)tt * NPART];
  if (scalar) *scalar = s;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_local_edges(kmx_pgo* h, int robot, int64_t* m_local) {
  if (int rc = check_robot(h, robot)) return rc;
  KMX_CHECK(m_local, KMX_EINVAL, "null argument");
  *m_local = h->m_robot[h->local_of[robot]];
  return KMX_OK;
}

extern "C" int kmx_pgo_enable_timing(kmx_pgo* h, int enable) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  h->timing = enable != 0;
  return KMX_OK;
}

extern "C" int kmx_pgo_read_counters(kmx_pgo* h, kmx_pgo_counters* out) {
  KMX_CHECK(ready(h) && out, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  Counters c;
  KMX_HIP(hipMemcpy(&c, h->d_cnt, sizeof(Counters), hipMemcpyDeviceToHost));
  double ms_total = 0.0;
  for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
    float ms = 0.f;
    KMX_HIP(hipEventElapsedTime(&ms, h->ev_pool[i], h->ev_pool[i + 1]));
    ms_total += ms;
  }
  out->hessvec_ms_total = ms_total;
  out->hessvec_launches = (int64_t)(h->ev_used / 2);
  out->hessvec_alg_bytes = c.hess_alg_bytes;
  out->edges_iters = (int64_t)c.edges_iters;
  out->block_updates = (int64_t)c.block_updates;
  out->hessvecs = (int64_t)c.hessvecs;
  h->ev_used = 0;
  KMX_HIP(hipMemset(h->d_cnt, 0, sizeof(Counters)));
  return KMX_OK;
}

// Diagnostic launcher shared by the gather bench / compare entry points.
static bool gbench_launch(kmx_pgo* h, int variant, double* out, const double* Dg) {
  const dim3 grid(h->ntiles), blk(BLOCK);
  const size_t sm = Smem<5>::bytes;
  constexpr int HCH = 240;
  const size_t smh = sizeof(double) * HCH * 5 * 4 + sizeof(int) * (Smem<5>::TP + 1);
  switch (variant) {
#define KMX_GB(V, G, W) case V: hipLaunchKernelGGL((k_gbench<5, G, W>), grid, blk, sm, h->stream, h->dv, (const double*)h->dv.X, out); return true;
    KMX_GB(0, 0, 1) KMX_GB(1, 0, 4) KMX_GB(2, 0, 6) KMX_GB(3, 0, 8)
    KMX_GB(10, 1, 1) KMX_GB(11, 1, 4) KMX_GB(12, 1, 6)
    KMX_GB(20, 2, 1) KMX_GB(21, 2, 4) KMX_GB(22, 2, 6) KMX_GB(23, 2, 8)
    KMX_GB(40, 3, 1) KMX_GB(41, 3, 4) KMX_GB(42, 3, 6) KMX_GB(45, 4, 1)
    KMX_GB(60, 5, 1) KMX_GB(61, 5, 4) KMX_GB(62, 5, 6) KMX_GB(65, 6, 1)
#undef KMX_GB
#define KMX_GB(V, G, W) case V: hipLaunchKernelGGL((k_gbench<5, G, W>), grid, blk, (SmemG<5, G>::bytes), h->stream, h->dv, (const double*)h->dv.X, out); return true;
    KMX_GB(70, 7, 1) KMX_GB(71, 7, 4) KMX_GB(72, 7, 5) KMX_GB(75, 8, 1)
#define KMX_GC(V, C) case V: hipLaunchKernelGGL((k_gcap<5, C>), grid, blk, sm, h->stream, h->dv, (const double*)h->dv.X, out); return true;
    KMX_GC(50, 1000) KMX_GC(51, 12) KMX_GC(52, 10) KMX_GC(53, 8) KMX_GC(54, 4)
#undef KMX_GC
#undef KMX_GB
#define KMX_GA(V, A) case V: hipLaunchKernelGGL((k_gablate<5, A>), grid, blk, sm, h->stream, h->dv, (const double*)h->dv.X, out); return true;
    KMX_GA(30, 0) KMX_GA(31, 1) KMX_GA(32, 2) KMX_GA(33, 3)
#undef KMX_GA
    case 90: hipLaunchKernelGGL((k_hinc<5, 0, HCH>), grid, blk, smh, h->stream, h->dv, (const double*)h->dv.X, Dg, out); return true;
    case 91: hipLaunchKernelGGL((k_hinc<5, 1, HCH>), grid, blk, smh, h->stream, h->dv, (const double*)h->dv.X, Dg, out); return true;
    case 92:
      if (!h->hinc) return false;
      hipLaunchKernelGGL((k_gbench_hinc<5, false>), grid, blk, SmemH<5>::bytes, h->stream, h->dv, (const double*)h->dv.X, out);
      return true;
    case 93:
      if (!h->hinc) return false;
      hipLaunchKernelGGL((k_gbench_hinc<5, true>), grid, blk, SmemHG<5>::bytes, h->stream, h->dv, (const double*)h->dv.X, out);
      return true;
    default: return false;
  }
}

static int gbench_check(kmx_pgo* h, int variant) {
  KMX_CHECK(variant < 40 || variant == 90 || h->d_crec, KMX_EINVAL, "compact records not built (KMX_GATHER / non-SO(3) input)");
  KMX_CHECK(variant != 91 || !h->rect, KMX_EINVAL, "variant 91 reads CSR-order compact records (KMX_RECT=0)");
  return KMX_OK;
}

// D_i blocks for the lane-per-incidence prototype (caller frees).
static int gbench_diag(kmx_pgo* h, double** D) {
  KMX_HIP(hipMalloc(D, sizeof(double) * 16 * (size_t)std::max(h->nloc, 1)));
  hipLaunchKernelGGL(k_diag, dim3((h->nloc + 255) / 256), dim3(256), 0, h->stream, h->dv, *D);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

// Diagnostic entry point (not used by the product path): time `reps` launches
// of the gather primitive variant (GV, LBW) = (variant / 10, variant % 10 ->
// min waves per SIMD {0: none, 1: 4, 2: 6, 3: 8}) over the current iterate;
// 90 / 91: the lane-per-incidence prototype (k_hinc).
extern "C" int kmx_pgo_debug_gather_bench(kmx_pgo* h, int variant, int reps, double* ms_out) {
  KMX_CHECK(ready(h) && ms_out && reps > 0, KMX_EINVAL, "bad argument");
  KMX_CHECK(h->P.r == 5, KMX_EUNSUP, "gather bench is built for r = 5");
  KMX_HIP(hipSetDevice(h->device));
  int rc = gbench_check(h, variant);
  if (rc) return rc;
  const size_t vec = (size_t)std::max(h->nloc, 1) * 4 * h->P.r;
  double* out = h->d_scratch + vec;
  double* Dg = nullptr;
  if ((rc = gbench_diag(h, &Dg))) return rc;
  hipEvent_t e0, e1;
  KMX_HIP(hipEventCreate(&e0));
  KMX_HIP(hipEventCreate(&e1));
  if (!gbench_launch(h, variant, out, Dg)) { (void)hipFree(Dg); return kmx::fail(KMX_EINVAL, "unknown gather variant"); }
  KMX_HIP(hipEventRecord(e0, h->stream));
  for (int i = 0; i < reps; ++i) gbench_launch(h, variant, out, Dg);
  KMX_HIP(hipEventRecord(e1, h->stream));
  KMX_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  KMX_HIP(hipEventElapsedTime(&ms, e0, e1));
  *ms_out = (double)ms / reps;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  KMX_HIP(hipFree(Dg));
  return KMX_OK;
}

// Diagnostic: run gather variants va and vb over the current iterate and
// report max |out_a - out_b| and max |out_a| (valid pose rows only).
extern "C" int kmx_pgo_debug_gather_cmp(kmx_pgo* h, int va, int vb, double* maxdiff, double* maxabs) {
  KMX_CHECK(ready(h) && maxdiff && maxabs, KMX_EINVAL, "bad argument");
  KMX_CHECK(h->P.r == 5, KMX_EUNSUP, "gather bench is built for r = 5");
  KMX_HIP(hipSetDevice(h->device));
  int rc;
  if ((rc = gbench_check(h, va)) || (rc = gbench_check(h, vb))) return rc;
  const size_t vec = (size_t)std::max(h->nloc, 1) * 4 * h->P.r;
  double* out = h->d_scratch + vec;
  double* Dg = nullptr;
  if ((rc = gbench_diag(h, &Dg))) return rc;
  std::vector<double> A(vec), B(vec);
  bool ok = gbench_launch(h, va, out, Dg);
  KMX_HIP(hipMemcpyAsync(A.data(), out, sizeof(double) * vec, hipMemcpyDeviceToHost, h->stream));
  ok = ok && gbench_launch(h, vb, out, Dg);
  KMX_HIP(hipMemcpyAsync(B.data(), out, sizeof(double) * vec, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  KMX_HIP(hipFree(Dg));
  if (!ok) return kmx::fail(KMX_EINVAL, "unknown gather variant");
  double md = 0.0, ma = 0.0;
  for (size_t i = 0; i < vec; ++i) {
    md = std::max(md, std::fabs(A[i] - B[i]));
    ma = std::max(ma, std::fabs(A[i]));
  }
  *maxdiff = md;
  *maxabs = ma;
  return KMX_OK;
}
