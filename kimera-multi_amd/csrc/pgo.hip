// pgo.hip — MI355X (gfx950) RBCD block updates on lifted SE(3) with GNC-TLS.
//
// Replaces dpgo's PGOAgent::iterate / updateMeasurementWeights hot path
// (drawio:2058-2066, 2215, 2466-2469, 2513).
// Design:
//   * Every local robot block lives in HBM and all blocks are updated by the
//     same launches (batched RBCD). Workgroup tiles never straddle robots, so
//     every reduction is per robot and its RTR / tCG scalars live on the device
//     in one Ctl record per robot.
//   * No scalar reaches the host inside a round. Each tile publishes its
//     partial sums; a robot's partials are reduced in tile order
//     (deterministic) either by a one-workgroup-per-robot k_reduce launch
//     (large problems) or by every workgroup of the next kernel, which needs
//     the decision anyway (the consumer form, small problems: no reduction
//     launch at all). The host only reads one progress word per robot to stop
//     enqueueing tCG steps (polled, blind or adaptive, kmx_pgo_set_tcg_poll).
//   * tCG in the linearity form: Hz by gather, delta = -z + beta delta_old,
//     Hdelta = -Hz + beta Hdelta_old; eta = sum coef_k delta_k is folded from
//     two kept directions every second step and finished in k_retract.
//   * Edge data: one 72-B compact record per incidence in CSR order (unit
//     quaternion of R, t, w kappa, +-w tau — the sign bit is the tail flag)
//     plus its other endpoint in a 4-B array (Dev::rec_o), 76 B per incidence
//     (struct Rec<10>); or a 128-B record with the full rotation when some
//     measurement is not a rotation to 1e-12 (Rec<16>). The gathers are
//     incidence-parallel:
//     one lane per incidence evaluates its block against the neighbour's whole
//     r x 4 row and parks the r contribution rows in LDS; the (pose, row) lanes
//     then add their pose's contributions in CSR (= increasing edge id) order.
//     No atomics: every sum has a fixed order, so results are deterministic and
//     independent of rank placement.
//   * GNC-TLS on the device: the round-begin launch decides
//     shouldUpdateMeasurementWeights (drawio:2466-2469: inner iterations >
//     robustOptInnerIters, or every agent converged; capped at
//     robustOptNumWeightUpdates) from device state and re-weights the loop
//     closures in the same launch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <string>
#include <vector>

#include "common.h"

// KMX_HESS_PROBE (diagnostic builds only, scripts/gpu_hess_probe.sh): bits
// remove one k_hess stream each so its PMC traffic can be attributed; the
// results of such a build are wrong by design. 0 in the product build.
#ifndef KMX_HESS_PROBE
#define KMX_HESS_PROBE 0
#endif

namespace {

constexpr int WAVES = 4;
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
  int hessvecs, skipped, retracted, pad1;  // retracted: the consumer k_update formed the trial point
  double Delta, f_init, gn_init, f_cur;
  double f_final, norm_r0, z_r, e_Pe;
  double e_Pd, d_Pd, alpha, beta;
  double coef, rho, chg_acc, rel_change;
  double r_stop;    // tCG residual stop: ||r_0|| min(||r_0||^theta, kappa), formed once per tCG
  int lin_stop, pad3;  // kappa < ||r_0||^theta: a stop at r_stop is KMX_TCG_LINEAR
  double pad2[8];   // 256 B: one robot's record never shares a line with the next
};
static_assert(sizeof(Ctl) == 256, "Ctl is 256 B");

struct Counters {
  unsigned long long edges_iters;
  unsigned long long block_updates;
  unsigned long long hessvecs;
  unsigned long long gnc_updates;
  double hess_alg_bytes;
  double pad2[3];
};

// GNC schedule state (dpgo PGOAgent: mRobustOptInnerIter, mWeightUpdateCount, mu).
struct Gnc {
  int inner;    // rounds since the last weight update
  int updates;  // weight updates so far
  int fired;    // the last round-begin launch updated the weights
  int rounds;   // rounds completed
  double mu;
  double pad[3];
};

// Field-wise copies of the schedule state (a struct assignment between global
// pointers is lowered through a scratch temporary).
__device__ __forceinline__ Gnc load_gnc(const Gnc* p) {
  Gnc s;
  s.inner = p->inner; s.updates = p->updates; s.fired = p->fired; s.rounds = p->rounds;
  s.mu = p->mu; s.pad[0] = s.pad[1] = s.pad[2] = 0.0;
  return s;
}
__device__ __forceinline__ void store_gnc(Gnc* p, const Gnc& s) {
  p->inner = s.inner; p->updates = s.updates; p->fired = s.fired; p->rounds = s.rounds; p->mu = s.mu;
}

// Host-visible tCG progress of one robot, written after every tCG step by the
// robot's update reduction (k_reduce, or the robot's first tile of the
// consumer-form k_hess) into host-mapped memory as ONE 64-bit word (seq << 1 |
// still-in-tCG): a single relaxed system-scope store, no release fence, so no
// L2 writeback. The host keeps one tCG step queued beyond the last one known
// to be needed and stops enqueueing once no robot is in tCG.
struct HostStatus {
  unsigned long long word;
};
__device__ __forceinline__ void post_status(HostStatus* hs, int l, unsigned long long seq, bool running) {
  __hip_atomic_store(&hs[l].word, (seq << 1) | (running ? 1ull : 0ull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Params {
  int tcg_max, rtr_iters, use_precond, robust;
  double kappa, theta, Delta0, Delta_max, accept_rho, gn_tol, shift, barc, mu_step, rel_tol;
  int gnc_on, inner_iters, max_updates, n_ext;
  int rgd;          // KMX_METHOD_RGD: one preconditioned gradient step per block update
  double rgd_step;
  int early_stop;   // RM_CONSUMER k_hess: the stop decision before the gather (else after)
};

// One tile's description, read by a single 32-B scalar load at the start of
// every tile kernel: its robot, its first pose, its incidence range start
// inc_ptr[p0] and, packed, its pose count np (< 256) and incidence count
// n = inc_ptr[p0 + np] - inc_ptr[p0] (np | n << 8), so the record loads do not
// wait for an inc_ptr lookup; and its robot's tile range, so the consumer
// kernels' robot sums do not wait for an rtile0 lookup.
struct alignas(16) TileDesc {
  int robot, p0, k0, np_n;
  int rt0, rt1;  // the robot's tile range: the consumer kernels' robot sums start from it
  int pad0, pad1;
};

struct Dev {
  int ntiles, L, nloc, npub;
  const TileDesc* tile;
  const int* rtile0;   // [L+1]
  const int* inc_ptr;  // [nloc+1]
  double* rec;         // [ninc + 1][Rec<RW>::GS] incidence records in CSR order (+ one zero pad record)
  const int* rec_o;    // [ninc + 1] compact records: the other endpoint of each incidence
  double* ekappa;      // [mloc] per local edge
  double* etau;
  double* ew;          // GNC weight
  const int2* eipos;   // [mloc] record positions (tail, head) of each local edge, -1 if not local
  double *X, *Xt, *g, *r, *z, *hd, *S, *Pinv, *hD, *pub;
  // D_i - S_i (S embedded in the rotation block; SYM4 per pose), written by
  // k_grad: k_hess applies it in place of D_i and S (48 B per pose per launch)
  double* hDS;
  // tCG search directions: delta_k lives in dh + (k % dhn) * vec, so eta =
  // sum_k coef_k delta_k is not updated at every Hess-vec: k_hess folds the
  // dhn oldest directions into eta before their buffer is reused (every dhn
  // steps) and k_retract adds the rest, in step order (the additions of the
  // serial eta += coef delta, same bits).
  double* dh;          // [dhn][vec]
  double* eta;         // [vec] folded directions (tcg_max > dhn only)
  double* coefh;       // [L][tcg_max] the eta coefficient (alpha or tau) of each step
  long long vec;       // doubles per vector
  int dhn;
  double* part;        // [ntiles][NPART]
  double* part_h;      // [ntiles][2] k_hess partials (RM_CONSUMER: read by k_update)
  double* part_u;      // [ntiles][2] k_update partials (RM_CONSUMER: read by the next k_hess)
  Ctl* ctl;
  Ctl* ctl2;           // [L] RM_CONSUMER: the state between k_hess and k_update of a tCG step
  Counters* cnt;
  const long long* m_robot;   // [L] local-problem edges per robot
  const int* n_robot;         // [L] poses per robot
  const int* pose_slot;       // [nloc] owned public-table slot of a pose, or -1
  double* relc;               // [L] relative change of each robot's last block update (inf: none yet)
  Gnc* gnc;                   // schedule state
  Gnc* gnc_next;              // state after the current round-begin launch (k_precond commits it)
  const double* ext;          // [n_ext] peers' largest relative change (multi-process team status)
  const int* gnc_edge;        // [n_gnc] local edges re-weighted here (non-fixed, >= 1 local endpoint)
  const int2* gnc_ends;       // [n_gnc] endpoints: >= 0 local pose, < 0 public slot -1-x
  int n_gnc;
  int* hv_launch;             // [HV_SLOTS] robots that ran a Hess-vec in timed launch k
  Params p;
  // one-sync tCG (P.tcg_form, body_step): H z_k, and w_k = precon(H delta_k)
  // double-buffered by step parity (the gathered vector), and the step's
  // 8-wide partials
  double *hz, *w0, *w1;
  double* part_f;             // [2][ntiles][8], by step parity (a launch reads step k's
                              // partials of every tile of its robot while its own tile writes step k+1's)
};

constexpr int HV_SLOTS = 1 << 16;
// tCG directions kept (Dev::dh). Same-box A/B at configs[3] (profiles/r03/dhist/):
// all ten (eta formed only in k_retract) gives the fastest k_hess (38.2 vs
// 40.5 us) but k_retract then reads up to ten vectors, and the round is 1.7 %
// slower; two (eta folded at every second step) keeps the round at the
// one-buffer form's time or better with half its eta traffic in k_hess.
#ifndef KMX_DHMAX
#define KMX_DHMAX 2
#endif
constexpr int DHMAX = KMX_DHMAX;

// Wave sum by DPP lane moves inside each row of 16 (xor 1, xor 2 by
// quad_perm, then the half-row and row mirrors: every lane of a row holds the
// row's sum, bitwise alike since each step adds the same two values), then
// the four row sums read out as scalars and added in a fixed order: the same
// value in every lane. (A shuffle butterfly costs 12 LDS permutes per sum: the
// one-sync k_step's 15 sums took ~4 us of its decision and epilogue.)
template <int CTRL>
__device__ __forceinline__ double dpp_row(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double read_lane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_row<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_row<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_row<0x141>(v);  // row_half_mirror
  v += dpp_row<0x140>(v);  // row_mirror
  return (read_lane(v, 0) + read_lane(v, 16)) + (read_lane(v, 32) + read_lane(v, 48));
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

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops but
// not for its outstanding global loads (__syncthreads waits vmcnt(0), which
// would drain the next chunk's prefetched records).
// Symmetric 4x4 blocks (Q's diagonal blocks, the preconditioner) are stored
// as their upper triangle, row by row: 10 doubles, five 16-B loads.
constexpr int SYM4 = 10;
__device__ __forceinline__ void load_sym4(const double* p, double M[16]) {
  const double2* p2 = reinterpret_cast<const double2*>(p);
  const double2 a = p2[0], b = p2[1], c = p2[2], e = p2[3], f = p2[4];
  M[0] = a.x; M[1] = M[4] = a.y; M[2] = M[8] = b.x; M[3] = M[12] = b.y;
  M[5] = c.x; M[6] = M[9] = c.y; M[7] = M[13] = e.x;
  M[10] = e.y; M[11] = M[14] = f.x;
  M[15] = f.y;
}
// S = sym(Y^T G_Y) stored as its 6 upper entries
__device__ __forceinline__ void load_sym3(const double* p, double S[9]) {
  S[0] = p[0]; S[1] = S[3] = p[1]; S[2] = S[6] = p[2];
  S[4] = p[3]; S[5] = S[7] = p[4];
  S[8] = p[5];
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ------------------------------------------------------------ edge records --
struct Edge {
  double R[9], t[3], wk, wt;
};

__device__ __forceinline__ int2 unpack_int2(double v) {
  const long long b = __double_as_longlong(v);
  return make_int2((int)(b & 0xffffffffll), (int)(b >> 32));
}

// RW = 10: compact record — 64 B in HBM (GS = 8 doubles, four 16-B parts):
// three components of the unit quaternion of R (all but its largest, which is
// made >= 0 and rebuilt as sqrt(1 - the others' squares): well conditioned,
// since it is >= 1/2), t, w kappa, +-w tau (the sign bit is the tail flag; w
// tau >= 0, a zero weight is +-0.0); Dev::rec_o (4 B) holds the other endpoint
// in its low 29 bits (two's complement) and the rebuilt component's index in
// bits 29-31: 68 B per incidence (round 5: the whole quaternion, 76 B). In
// registers it is the 10-word form (w, x, y, z, t, w kappa, w tau, {other,
// tail << 31}), five 16-B parts; the gathers rebuild R from the quaternion
// (R R^T = I to rounding, as the preconditioner assumes).
// RW = 16: full record (R, t, w kappa, w tau, {other, edge|tail}, pad), for
// measurement rotations off SO(3).
template <int RW>
struct Rec {
  static constexpr int Q = RW / 2;        // 16-B parts in registers
  static constexpr int GS = RW == 10 ? 8 : 16;  // doubles per record in HBM
  static constexpr int WK = RW == 10 ? 6 : 12;  // index of w kappa (w tau follows)
  __device__ static __forceinline__ void load(const Dev& d, size_t k, double2 q[Q]) {
    if constexpr (RW == 10) {
      const double2* p2 = reinterpret_cast<const double2*>(d.rec + (size_t)GS * k);
      const double2 a0 = p2[0], a1 = p2[1], a2 = p2[2], a3 = p2[3];  // (qa, qb) (qc, t0) (t1, t2) (wk, +-wt)
      const unsigned raw = (unsigned)d.rec_o[k];
      const int other = (int)(raw << 3) >> 3;
      const unsigned big = raw >> 29;
      const double qa = a0.x, qb = a0.y, qc = a1.x;
      const double ql = sqrt(1.0 - (qa * qa + qb * qb + qc * qc));
      const double w = big == 0 ? ql : qa, x = big == 0 ? qa : (big == 1 ? ql : qb);
      const double y = big <= 1 ? qb : (big == 2 ? ql : qc), z = big == 3 ? ql : qc;
      q[0] = make_double2(w, x);
      q[1] = make_double2(y, z);
      q[2] = make_double2(a1.y, a2.x);
      q[3] = make_double2(a2.y, a3.x);
      const double wt = a3.y;
      const long long bits = (long long)(unsigned)other | (std::signbit(wt) ? (1ll << 63) : 0ll);
      q[4] = make_double2(std::fabs(wt), __longlong_as_double(bits));
    } else {
      const double2* q2 = reinterpret_cast<const double2*>(d.rec + (size_t)GS * k);
#pragma unroll
      for (int i = 0; i < Q; ++i) q[i] = q2[i];
    }
  }
  // the stored w tau of an incidence (compact: its sign is the tail flag)
  __device__ static __forceinline__ double wt_word(double wt, bool tail) {
    return (RW == 10 && tail) ? -wt : wt;
  }
  __device__ static __forceinline__ void edge(const double2 q[Q], Edge& E) {
    if constexpr (RW == 10) {
      const double w = q[0].x, x = q[0].y, y = q[1].x, z = q[1].y;
      const double xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
      const double wx = w * x, wy = w * y, wz = w * z;
      E.R[0] = 1.0 - 2.0 * (yy + zz); E.R[1] = 2.0 * (xy - wz); E.R[2] = 2.0 * (xz + wy);
      E.R[3] = 2.0 * (xy + wz); E.R[4] = 1.0 - 2.0 * (xx + zz); E.R[5] = 2.0 * (yz - wx);
      E.R[6] = 2.0 * (xz - wy); E.R[7] = 2.0 * (yz + wx); E.R[8] = 1.0 - 2.0 * (xx + yy);
      E.t[0] = q[2].x; E.t[1] = q[2].y; E.t[2] = q[3].x;
      E.wk = q[3].y;
      E.wt = q[4].x;
    } else {
      E.R[0] = q[0].x; E.R[1] = q[0].y; E.R[2] = q[1].x; E.R[3] = q[1].y; E.R[4] = q[2].x;
      E.R[5] = q[2].y; E.R[6] = q[3].x; E.R[7] = q[3].y; E.R[8] = q[4].x;
      E.t[0] = q[4].y; E.t[1] = q[5].x; E.t[2] = q[5].y;
      E.wk = q[6].x;
      E.wt = q[6].y;
    }
  }
  __device__ static __forceinline__ int2 inc(const double2 q[Q]) {
    return unpack_int2(RW == 10 ? q[4].y : q[7].x);
  }
};

// Contribution of one incidence to row a of pose `self`. vs = self row, vo =
// other endpoint row. Expressions mirror oracle/dpgo_oracle.c edge_eval
// exactly. Returns the row's share of 1/2 w (kappa |E_R|^2 + tau E_t^2).
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

// ------------------------------------------------------ Stiefel group ops --
// S = sym(Y^T G_Y) for the pose group (9 entries, identical in all R lanes).
// LDS = true (kernels with a free BLOCK x 6-double LDS scratch `scr`): every
// lane writes its 6 products, then reads its group's R x 6 back and adds them
// in lane order: one LDS round trip instead of 6 chained shuffle chains. Only
// lanes of one wave exchange data (in-order LDS queue; no workgroup barrier).
// LDS = false: 6 shuffle sums, each chained to the previous one (empty asm) so
// only one sum's R shuffles are in flight (VGPR pressure).
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

// Preconditioner: P_Y(V Pinv_i) (block-Jacobi on Q's 4x4 diagonal blocks).
// Pre (LDS form only, has_pre): the pose's block, already loaded by the caller.
template <int R, bool LDS = false>
__device__ __forceinline__ void group_precon(const Dev& d, int pose, bool valid, const double y[4],
                                             const double V[4], int base, double out[4], double* scr = nullptr,
                                             const double* Pre = nullptr, bool has_pre = false) {
  if (!d.p.use_precond) {
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = V[k];
    return;
  }
  double buf[4] = {0.0, 0.0, 0.0, 0.0};
  static_assert(LDS, "the LDS form only");
  double P[16];
  if (has_pre) {
#pragma unroll
    for (int i = 0; i < 16; ++i) P[i] = Pre[i];
  } else {
    load_sym4(d.Pinv + SYM4 * (size_t)pose, P);  // pose is valid on every lane
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) buf[k] = (i == 0) ? V[0] * P[k] : buf[k] + V[i] * P[4 * i + k];
  group_proj<R, LDS>(y, buf, base, out, scr);
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

// ------------------------------------------------------------- lane map ----
struct Lane {
  int tile, l, w, ln, pw, a, base, pose;
  int p0, np, k0, n;  // the tile's poses and incidences (TileDesc)
  int rt0, rt1;       // the robot's tiles
  bool valid;
};
template <int R>
__device__ __forceinline__ Lane lane_map(const Dev& d) {
  constexpr int PPW = 64 / R;
  Lane L;
  // XCD-aware, bijective block -> tile remap (cdna_hip_programming.md T1):
  // blocks b and b + 8 share an XCD, so each XCD gets one contiguous range of
  // tiles — about one robot block, whose rows then stay in that XCD's L2.
  {
    const int nwg = d.ntiles, b = blockIdx.x;
    const int q = nwg >> 3, rr = nwg & 7, x = b & 7;
    L.tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  const TileDesc t = d.tile[L.tile];
  L.l = t.robot;
  L.p0 = t.p0;
  L.np = t.np_n & 0xff;
  L.k0 = t.k0;
  L.n = t.np_n >> 8;
  L.rt0 = t.rt0;
  L.rt1 = t.rt1;
  L.w = threadIdx.x >> 6;
  L.ln = threadIdx.x & 63;
  L.pw = L.ln / R;
  L.a = L.ln - L.pw * R;
  L.base = L.pw * R;
  const int local = L.w * PPW + L.pw;
  L.valid = (L.pw < PPW) && (local < L.np);
  L.pose = L.p0 + (L.valid ? local : 0);
  if (L.base + R > 64) L.base = 64 - R;  // idle tail lanes shuffle within range
  return L;
}

// --------------------------------------------------------------- gathers ---
// LDS layouts. A tile holds TP = W * (64 / R) poses (W = WAVES waves per
// workgroup); its
// incidences are one contiguous CSR range walked in chunks of CH incidences
// (one lane each).
template <int R, int W = WAVES>
struct SmemH {  // Hessian gather (k_hess, eval EHESS)
  static constexpr int TP = W * (64 / R);
  static constexpr int CH = TP * R;                                       // <= 64 W
  static constexpr int c_off = 0;                                         // double[CH][R][4]
  static constexpr int ptr_off = CH * R * 32;                             // int[TP + 1]
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + 8 * NPART * W + 16;
};
template <int R, int W = WAVES>
struct SmemHG {  // gradient / cost gathers: a chunk buffer plus the tile's own rows
  static constexpr int TP = W * (64 / R);
  static constexpr int CH = 240;                                          // incidences per chunk
  static constexpr int c_off = 0;                                         // double[CH][R][4]
  static constexpr int x_off = CH * R * 32;                               // double[TP][R][4]
  static constexpr int ptr_off = x_off + TP * R * 32;                     // int[TP + 1]
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + 8 * NPART * W + 16;
};
template <int R, int W = WAVES>
struct SmemC {  // trial cost: own rows + CSR pointers only
  static constexpr int TP = W * (64 / R);
  static constexpr int x_off = 0;
  static constexpr int ptr_off = TP * R * 32;
  static constexpr int red_off = ptr_off + ((TP + 1) * 4 + 15) / 16 * 16;
  static constexpr int bytes = red_off + 8 * NPART * W + 16;
};
constexpr int SCR_BYTES = BLOCK * 6 * 8;  // group_symYtG<R, true> scratch
struct SmemU {                            // element-wise kernels: scratch + reduction
  static constexpr int red_off = SCR_BYTES;
  static constexpr int bytes = red_off + RED_BYTES;
};
static_assert(SCR_BYTES <= SmemH<3>::ptr_off && SCR_BYTES <= SmemH<8>::ptr_off, "scratch");
static_assert(SCR_BYTES <= SmemHG<3>::x_off, "scratch");

// Euclidean Hessian-vector product Q V of the tile's poses (the local problem:
// a public neighbour's row counts as zero). Q's diagonal block D_i (k_precond)
// is applied once per pose; an incidence contributes only its off-diagonal
// block applied to the other endpoint's whole r x 4 row.
struct NoPre {
  __device__ bool operator()() const { return true; }
};
// `pre` runs once the first chunk's records are in flight, before any row is
// gathered (workgroup-uniform; false: leave without gathering).
// REC_FIRST: the first chunk's records are issued before the tile's CSR
// offsets, so the two loads overlap (the consumer form keeps the offsets
// first: its decision in `pre` is a call, and the records live across it
// would spill)
// DIAG = false: the caller applies the diagonal block itself (k_step, whose
// epilogue loads the own row and D_i with the rest of its rows in one batch).
template <int R, int RW, bool REC_FIRST, typename Src, typename Pre, bool DIAG = true, int W = WAVES>
__device__ __forceinline__ bool hinc_gather_src(const Dev& d, const Lane& L, Src& src, double acc[4], char* smem,
                                                Pre&& pre) {
  using SM = SmemH<R, W>;
  using RC = Rec<RW>;
  constexpr int CH = SM::CH;
  double* Cs = reinterpret_cast<double*>(smem + SM::c_off);
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  const int tid = threadIdx.x;
  const int p0 = L.p0, np = L.np, K0 = L.k0, n = L.n;
  const int pl = L.pose - p0;
  const int lt = min(tid, CH - 1);
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  // clamped, unconditional record loads (the pad record keeps an empty tile
  // at the end of the array inside it)
  auto ld = [&](int c0, double2* q) { RC::load(d, (size_t)(K0 + max(min(c0 + lt, n - 1), 0)), q); };
  double2 q[RC::Q];
  if constexpr (REC_FIRST) ld(0, q);
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  if constexpr (!REC_FIRST) ld(0, q);
  __syncthreads();  // sptr
  if (!pre()) return false;
  for (int c0 = 0; c0 < n; c0 += CH) {
    Edge E;
    RC::edge(q, E);
    const int2 in = RC::inc(q);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    double2 vr[2 * R];
    src.nbr(o, vr);
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
    // in flight across the LDS hand-off and the pose sums
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
  if (DIAG && L.valid) {
    double vs[4];
    double D[16];
    src.own(L.pose, L.a, vs);
#if KMX_HESS_PROBE & 2  // traffic attribution build: no diagonal-block loads
    for (int c = 0; c < 16; ++c) D[c] = (c % 5 == 0) ? 1.0 : 0.0;
#else
    load_sym4(d.hD + SYM4 * (size_t)L.pose, D);
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c)
      acc[c] += vs[0] * D[4 * c] + vs[1] * D[4 * c + 1] + vs[2] * D[4 * c + 2] + vs[3] * D[4 * c + 3];
  }
  return true;
}

// Where the gathered rows come from: a stored vector (the rows of the
// traffic-attribution builds replaced by constants).
template <int R>
struct PlainRows {
  const double* V;
  // the other endpoint's whole r x 4 row (o < 0, a public neighbour: any row; its weight is zeroed)
  __device__ __forceinline__ void nbr(int o, double2 vr[2 * R]) const {
    const double2* b2 = reinterpret_cast<const double2*>(V + (size_t)max(o, 0) * 4 * R);
#if KMX_HESS_PROBE & 1  // traffic attribution build: no neighbour rows
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vr[i] = make_double2(1e-3 * i, 1e-3);
    (void)b2;
#else
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vr[i] = b2[i];
#endif
  }
  // row a of the lane's own pose
  __device__ __forceinline__ void own(int pose, int a, double vs[4]) {
#if KMX_HESS_PROBE & 2  // traffic attribution build: no own-row loads
    for (int c = 0; c < 4; ++c) vs[c] = 1e-3 * c;
#else
    load4(V + (size_t)pose * 4 * R + 4 * a, vs);
#endif
  }
};
template <int R, int RW, bool REC_FIRST = false, bool DIAG = true, typename Pre = NoPre>
__device__ __forceinline__ bool hinc_gather(const Dev& d, const Lane& L, const double* V, double acc[4],
                                            char* smem, Pre&& pre = Pre{}) {
  PlainRows<R> src{V};
  return hinc_gather_src<R, RW, REC_FIRST, PlainRows<R>, Pre&, DIAG, WAVES>(d, L, src, acc, smem, pre);
}

// Gradient and cost, incidence-parallel. A lane evaluates its whole incidence
// with incidence_row (diagonal and off-diagonal terms; a public neighbour's row
// from the table), reading its own pose's row from an LDS copy of the tile's
// rows (owning pose found by a binary search of the tile CSR), and adds the
// incidence's cost share (1/2 per endpoint of a local edge; all of a shared
// edge). The pose sums run in CSR order.
template <int R, int RW, int W = WAVES>
__device__ __forceinline__ void hinc_grad(const Dev& d, const Lane& L, const double* V, const double* pub,
                                          double acc[4], double* cost, char* smem) {
  using SM = SmemHG<R, W>;
  using RC = Rec<RW>;
  constexpr int CH = SM::CH;
  double* Cs = reinterpret_cast<double*>(smem + SM::c_off);
  double2* xs = reinterpret_cast<double2*>(smem + SM::x_off);
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  const int tid = threadIdx.x;
  const int p0 = L.p0, np = L.np, K0 = L.k0, n = L.n;
  const int pl = L.pose - p0;
  const int lt = min(tid, CH - 1);
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
  double csum = 0.0;
  auto ld = [&](int c0, double2* q) { RC::load(d, (size_t)(K0 + max(min(c0 + lt, n - 1), 0)), q); };
  double2 q[RC::Q];
  ld(0, q);  // in flight with the CSR offsets and the tile's rows
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  {
    const double2* v2 = reinterpret_cast<const double2*>(V + (size_t)p0 * 4 * R);
    for (int i = tid; i < np * 2 * R; i += 64 * W) xs[i] = v2[i];
  }
  __syncthreads();  // sptr, xs
  for (int c0 = 0; c0 < n; c0 += CH) {
    const int k = max(min(c0 + lt, n - 1), 0);
    // the other endpoint's row first (it needs only the record), so its
    // latency runs under the owning pose's search
    const int2 in = RC::inc(q);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    const double2* o2 =
        reinterpret_cast<const double2*>((o >= 0) ? V + (size_t)o * 4 * R : pub + (size_t)(-1 - o) * 4 * R);
    double2 vo2[2 * R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vo2[i] = o2[i];
    int lo = 0, hi = np;  // owning pose: sptr[lo] <= k < sptr[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sptr[mid] <= k) lo = mid;
      else hi = mid;
    }
    const double2* s2 = xs + lo * 2 * R;
    Edge E;
    RC::edge(q, E);
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

// Trial cost f(Xt), one lane per incidence of the tile; only the owner
// incidence of an edge contributes (the tail of a local edge, the local end of
// a shared one), so each edge of the local problem counts once. The owner lane
// reads its own row from LDS and the other endpoint's row, and sums the r
// rows' residual terms: no per-pose reduction.
template <int R, int RW>
__device__ __forceinline__ double inc_owner_cost(const Dev& d, const Lane& L, const double* V, const double* pub,
                                                 char* smem) {
  using SM = SmemC<R>;
  using RC = Rec<RW>;
  int* sptr = reinterpret_cast<int*>(smem + SM::ptr_off);
  double2* xs = reinterpret_cast<double2*>(smem + SM::x_off);
  const int tid = threadIdx.x;
  const int p0 = L.p0, np = L.np, K0 = L.k0, n = L.n;
  if (tid <= np) sptr[tid] = d.inc_ptr[p0 + tid] - K0;
  {
    const double2* v2 = reinterpret_cast<const double2*>(V + (size_t)p0 * 4 * R);
    for (int i = tid; i < np * 2 * R; i += BLOCK) xs[i] = v2[i];
  }
  __syncthreads();
  double cost = 0.0;
  for (int k = tid; k < n; k += BLOCK) {
    double2 q[RC::Q];
    RC::load(d, (size_t)(K0 + k), q);
    const int2 in = RC::inc(q);
    const int o = in.x;
    const bool tail = (in.y >> 31) & 1;
    if (o >= 0 && !tail) continue;  // the head of a local edge: its tail counts it
    // the other endpoint's row first: its latency runs under the owning pose's search
    const double2* o2 =
        reinterpret_cast<const double2*>((o >= 0) ? V + (size_t)o * 4 * R : pub + (size_t)(-1 - o) * 4 * R);
    double2 vs2[2 * R], vo2[2 * R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vo2[i] = o2[i];
    int lo = 0, hi = np;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sptr[mid] <= k) lo = mid;
      else hi = mid;
    }
    const double2* s2 = xs + lo * 2 * R;
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) vs2[i] = s2[i];
    Edge E;
    RC::edge(q, E);
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

// -------------------------------------------------- per-robot reductions --
// Each tile reduces its NV values over the workgroup (wave sums, then the 4
// waves in order) and stores them as the tile's partials; the robot's sums are
// taken in tile order by whoever consumes them (robot_sum's fixed order):
// RM_LAUNCH: k_reduce, a one-workgroup-per-robot launch after the producing
// kernel, which then runs the RTR / tCG control logic; RM_CONSUMER: no
// reduction launch inside tCG — every workgroup of k_update reduces its robot's
// k_hess partials itself (and every workgroup of the next k_hess the k_update
// partials) in the same order and runs the control step on a private copy of
// the robot's state; the robot's first tile writes the state out,
// double-buffered (k_hess: ctl -> ctl2, k_update: ctl2 -> ctl), so no
// workgroup reads a state another one of the same launch writes. The round's
// other reductions are folded too (gradient -> first k_hess, last update ->
// k_retract, trial cost -> k_commit), so a consumer-form round has no k_reduce
// launch (12.5k poses 167.7 -> 161.4 us per round, profiles/r02/small_round/3_*).
// Measured on configs[3] (profiles/r02/ab_red): at 100k poses the consumer
// form loses (k_hess 41.2 us and k_update 22.7 us against 32.4 + 19.8 us plus
// two 4.6 us k_reduce launches: each workgroup of the latency-bound gather
// waits for its robot's sums), so RM_LAUNCH stays the form above 80k poses per
// GPU. Two more forms were measured and removed in round 3: agent-scope
// tickets in the producing launch (k_hess 47.5 vs 39.9 us: the ticket keeps
// each workgroup resident for microseconds after its work) and a half form
// with only the update's k_reduce kept (0.814 / 0.839 vs 0.817 / 0.839 ms per
// round: no gain).
enum RedMode { RM_LAUNCH = 0, RM_CONSUMER = 2 };

template <int KIND, int NV, int RM, typename Store>
__device__ __forceinline__ void finish_tile(const Dev& d, const Lane& L, const double* vals, char* smem_red,
                                            Store&& store) {
  double* lds = reinterpret_cast<double*>(smem_red);
  static_assert(NV <= NPART && WAVES == 4, "reduction area");
#pragma unroll
  for (int s = 0; s < NV; ++s) {
    const double w = wave_sum(vals[s]);
    if ((threadIdx.x & 63) == 0) lds[s * WAVES + (threadIdx.x >> 6)] = w;
  }
  __syncthreads();
  constexpr bool two = RM == RM_CONSUMER && (KIND == RED_HESS || KIND == RED_UPDATE);
  static_assert(!two || NV <= 2, "consumer partials");
  if (threadIdx.x == 0) {  // 2-wide partials for the consumer launch, else NPART-wide for k_reduce
    double* dst = two ? (KIND == RED_HESS ? d.part_h : d.part_u) + (size_t)L.tile * 2 : d.part + (size_t)L.tile * NPART;
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) t += lds[s * WAVES + w];
      dst[s] = t;
    }
  }
  store();
}

// The tCG decisions after the Hess-vec and after the update, shared by
// control_on and by RM_CONSUMER's workgroups (which evaluate them from the
// robot's state without a copy of it); contraction off so every call site
// rounds alike.
struct HessStep {
  double alpha, e_Pe_new, coef;
  int boundary, stop;
};
__device__ __forceinline__ HessStep hess_step(double z_r, double e_Pe, double e_Pd, double d_Pd, double Delta,
                                              double d_Hd) {
#pragma clang fp contract(off)
  HessStep h;
  h.alpha = z_r / d_Hd;
  h.e_Pe_new = e_Pe + 2.0 * h.alpha * e_Pd + h.alpha * h.alpha * d_Pd;
  const double D2 = Delta * Delta;
  h.boundary = (d_Hd <= 0.0 || h.e_Pe_new >= D2) ? 1 : 0;
  h.stop = d_Hd <= 0.0 ? KMX_TCG_NEGATIVE_CURVATURE : KMX_TCG_EXCEEDED_TR;
  h.coef = h.boundary ? (-e_Pd + sqrt(e_Pd * e_Pd + d_Pd * (D2 - e_Pe))) / d_Pd : h.alpha;
  return h;
}
struct UpdStep {
  int done, stop;
  double beta;
};
__device__ __forceinline__ UpdStep upd_step(int mode, double r_stop, int lin_stop, double z_r, int tcg_iter, double rr,
                                            double zr_new, const Params& P) {
#pragma clang fp contract(off)
  UpdStep u;
  u.done = 0;
  u.stop = KMX_TCG_MAX_ITER;
  u.beta = 0.0;
  if (mode == MODE_BOUNDARY) {
    u.done = 1;
    u.stop = -1;  // keep the boundary reason
    return u;
  }
  const double norm_r = sqrt(rr);
  if (norm_r <= r_stop) {
    u.done = 1;
    u.stop = lin_stop ? KMX_TCG_LINEAR : KMX_TCG_SUPERLINEAR;
  } else if (tcg_iter >= P.tcg_max) {
    u.done = 1;
    u.stop = KMX_TCG_MAX_ITER;
  } else {
    u.beta = zr_new / z_r;
  }
  return u;
}

// The RTR / tCG scalar logic of robot l after a reduction of `kind`, applied
// to c. `side`: perform the side effects (team status, counters) — exactly one
// caller per robot and reduction does.
__device__ __forceinline__ void control_core(Ctl& c, const Dev& d, int l, int kind, const double* tot, int R_,
                                             bool side) {
  const Params& P = d.p;
  if (kind == RED_GRAD) {
    const double f = tot[0], gn = sqrt(tot[1]);
    if (c.rtr_iter == 0) { c.f_init = f; c.gn_init = gn; }
    c.f_cur = f;
    c.f_final = f;
    c.commit = 0;
    if (gn < P.gn_tol) {  // no step: the iterate does not change
      c.phase = PH_IDLE;
      c.tcg_stop = KMX_TCG_SKIPPED;
      c.tcg_iter = 0;
      c.accepted = 0;
      c.skipped = 1;
      if (side) d.relc[l] = (c.rtr_iter == 0) ? 0.0 : c.rel_change;
    } else if (P.rgd) {  // RGD: eta = -s z (z = precon(g), from k_grad), straight to the step
      c.phase = PH_STEP;
      c.tcg_iter = 0;
      c.tcg_stop = KMX_TCG_NONE;
      c.coef = -P.rgd_step;
      if (side && c.rtr_iter == 0) {
        atomicAdd(&d.cnt->edges_iters, (unsigned long long)d.m_robot[l]);
        atomicAdd(&d.cnt->block_updates, 1ull);
      }
    } else {
      c.phase = PH_TCG;
      c.tcg_iter = 0;
      c.norm_r0 = gn;
      {  // the residual stop of this tCG (upd_step), formed once instead of at every step
        const double pw = pow(gn, P.theta);
        c.r_stop = gn * fmin(pw, P.kappa);
        c.lin_stop = (P.kappa < pw) ? 1 : 0;
      }
      c.z_r = tot[2];
      c.d_Pd = tot[2];
      c.e_Pd = 0.0;
      c.e_Pe = 0.0;
      c.beta = 0.0;
      c.tcg_stop = KMX_TCG_MAX_ITER;
      if (side && c.rtr_iter == 0) {
        atomicAdd(&d.cnt->edges_iters, (unsigned long long)d.m_robot[l]);
        atomicAdd(&d.cnt->block_updates, 1ull);
      }
    }
  } else if (kind == RED_HESS) {
    const double d_Hd = tot[0];
    const HessStep hs = hess_step(c.z_r, c.e_Pe, c.e_Pd, c.d_Pd, c.Delta, d_Hd);
    if (side) d.coefh[(size_t)l * P.tcg_max + min(c.tcg_iter, P.tcg_max - 1)] = hs.coef;  // delta_k's eta coefficient
    c.tcg_iter += 1;
    c.hessvecs += 1;
    if (side) {
      atomicAdd(&d.cnt->hessvecs, 1ull);
      atomicAdd(&d.cnt->hess_alg_bytes, 128.0 * (double)d.m_robot[l] + 2.0 * 8.0 * R_ * 4.0 * (double)d.n_robot[l]);
    }
    if (hs.boundary) {
      c.coef = hs.coef;
      c.mode = MODE_BOUNDARY;
      c.tcg_stop = hs.stop;
    } else {
      c.alpha = hs.alpha;
      c.coef = hs.coef;
      c.e_Pe = hs.e_Pe_new;
      c.mode = MODE_INTERIOR;
    }
  } else if (kind == RED_UPDATE) {
    const double zr_new = tot[1];
    const UpdStep u = upd_step(c.mode, c.r_stop, c.lin_stop, c.z_r, c.tcg_iter, tot[0], zr_new, P);
    if (u.done) {
      if (u.stop >= 0) c.tcg_stop = u.stop;
      c.phase = PH_STEP;
    } else {
      const double beta = u.beta;
      c.e_Pd = beta * (c.e_Pd + c.alpha * c.d_Pd);
      c.d_Pd = zr_new + beta * beta * c.d_Pd;
      c.z_r = zr_new;
      c.beta = beta;
    }
  } else if (P.rgd) {  // RED_COST after an RGD step: always accepted, one step per block update
    c.rho = 0.0;
    c.accepted = 1;
    c.commit = 1;
    c.f_final = tot[0];
    c.chg_acc += tot[3];
    c.rtr_iter += 1;
    c.phase = PH_IDLE;
    c.rel_change = sqrt(c.chg_acc / (double)d.n_robot[l]);
    if (side) d.relc[l] = c.rel_change;
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
    c.retracted = 0;
    c.rel_change = sqrt(c.chg_acc / (double)d.n_robot[l]);
    if (side && c.phase == PH_IDLE) d.relc[l] = c.rel_change;  // the team status of dpgo's getStatus
  }
}
// Out of line: inlined, it costs the 128-VGPR gather kernels spills.
__device__ void control_on(Ctl& c, const Dev& d, int l, int kind, const double* tot, int R_, bool side) {
  control_core(c, d, l, kind, tot, R_, side);
}

// RM_LAUNCH: one workgroup per robot reduces the robot's tile partials in
// tile order and runs the control logic (after k_update it also reports the
// robot's tCG progress to the host).
constexpr int TILES_TARGET = 736;  // tile count the cut of small problems aims at (set_graph)
constexpr int RBLOCK = 256;  // k_reduce: one workgroup per robot (1024 threads measured slower: 6.3 vs 4.6 us)
static_assert(RBLOCK == BLOCK, "robot_sum runs in k_reduce and in the tCG kernels");
// Sum of NS partials (row stride `stride`) over tiles [t0, t1) of a robot by
// the whole workgroup: two tiles per thread in flight (512 tiles, ~24k poses
// per robot, in one round trip), tile order within a thread, then the wave
// sums and the 4 waves in order; every thread gets the totals. The one order
// used by k_reduce and by RM_CONSUMER's tCG kernels. lds: >= NS * 4 doubles.
template <int NS>
__device__ __forceinline__ void robot_sum(const double* part, int stride, int t0, int t1, double* lds,
                                          double tot[NPART]) {
  constexpr int RW_ = RBLOCK / 64;
  double v[NPART] = {0.0, 0.0, 0.0, 0.0};
  for (int tb = t0; tb < t1; tb += 2 * RBLOCK) {
    double a[2][NS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = min(tb + (int)threadIdx.x + u * RBLOCK, t1 - 1);
      if constexpr (NS == 4) {
        const double2* p2 = reinterpret_cast<const double2*>(part + (size_t)t * stride);
        const double2 x = p2[0], y = p2[1];
        a[u][0] = x.x; a[u][1] = x.y; a[u][NS - 2] = y.x; a[u][NS - 1] = y.y;
      } else {
        const double2 x = *reinterpret_cast<const double2*>(part + (size_t)t * stride);
        a[u][0] = x.x;
        if constexpr (NS > 1) a[u][NS - 1] = x.y;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (tb + (int)threadIdx.x + u * RBLOCK < t1) {
#pragma unroll
        for (int k = 0; k < NS; ++k) v[k] += a[u][k];
      }
  }
  __syncthreads();  // lds may still be read by an earlier user
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const double w = wave_sum(v[k]);
    if ((threadIdx.x & 63) == 0) lds[k * RW_ + (threadIdx.x >> 6)] = w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NPART; ++k) {
    double acc = 0.0;
    if (k < NS) {
#pragma unroll
      for (int w = 0; w < RW_; ++w) acc += lds[k * RW_ + w];
    }
    tot[k] = acc;
  }
}

// robot_sum in two halves, so the partial loads can be in flight during other
// work: issue() loads a robot's <= U * RBLOCK tiles into registers (larger
// robots fall back to robot_sum in finish()); finish() adds them in
// robot_sum's order (a thread's tiles in tile order, then the wave sums and
// the waves in order: the same sums for any U).
// NS <= 2: 2-wide partials (part_h / part_u); NS = 3, 4: d.part (stride NPART).
// A tile partial pair part[i], part[i + 1] (i even): one 16-B load.
__device__ __forceinline__ double2 ldpart(const double* part, size_t i) {
  return *reinterpret_cast<const double2*>(part + i);
}

template <int NS, int U = 2>
struct RobotSum {
  double a[U][NS];
  int t0, t1;
  __device__ __forceinline__ void issue(const double* part, int stride, int t0_, int t1_) {
    t0 = t0_;
    t1 = t1_;
    if (t1 - t0 > U * RBLOCK) return;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(t0 + (int)threadIdx.x + u * RBLOCK, t1 - 1);
      const size_t pt = (size_t)t * stride;
      const double2 x = ldpart(part, pt);
      if constexpr (NS > 2) {
        const double2 y = ldpart(part, pt + 2);
        a[u][2] = y.x;
        if constexpr (NS > 3) a[u][3] = y.y;
      }
      a[u][0] = x.x;
      if constexpr (NS > 1) a[u][1] = x.y;
    }
  }
  __device__ __forceinline__ void finish(const double* part, int stride, double* lds, double tot[NPART]) {
    static_assert(NS <= NPART, "partials");
    if (t1 - t0 > U * RBLOCK) {
      robot_sum<(NS > 2 ? NPART : NS)>(part, stride, t0, t1, lds, tot);
      if constexpr (NS == 3) tot[3] = 0.0;
      return;
    }
    constexpr int RW_ = RBLOCK / 64;
    double v[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) v[k] = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (t0 + (int)threadIdx.x + u * RBLOCK < t1 && threadIdx.x < RBLOCK) {
#pragma unroll
        for (int k = 0; k < NS; ++k) v[k] += a[u][k];
      }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const double w = wave_sum(v[k]);
      if ((threadIdx.x & 63) == 0 && threadIdx.x < RBLOCK) lds[k * RW_ + (threadIdx.x >> 6)] = w;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPART; ++k) {
      double acc = 0.0;
      if (k < NS) {
#pragma unroll
        for (int w = 0; w < RW_; ++w) acc += lds[k * RW_ + w];
      }
      tot[k] = acc;
    }
  }
};

// The robot's state (256 B, into LDS) and its tile partials are loaded
// together at the start, the control logic runs on the LDS copy and 32 lanes
// write it back: no global round trip is serialised behind another.
__global__ __launch_bounds__(RBLOCK) void k_reduce(Dev d, int kind, int R_, HostStatus* hs, unsigned long long seq,
                                                  int slot, const double* src) {
  constexpr int RW_ = RBLOCK / 64;
  constexpr int CW = sizeof(Ctl) / 8;
  static_assert(CW <= RBLOCK, "Ctl copy");
  __shared__ double lds[NPART * RW_];
  __shared__ Ctl cs;
  const int l = blockIdx.x;
  if (threadIdx.x < CW)
    reinterpret_cast<double*>(&cs)[threadIdx.x] = reinterpret_cast<const double*>(d.ctl + l)[threadIdx.x];
  const int t0 = d.rtile0[l], t1 = d.rtile0[l + 1];
  double tot[NPART];
  if (src) {  // RM_CONSUMER's 2-wide partials
    RobotSum<2> rs;
    rs.issue(src, 2, t0, t1);
    rs.finish(src, 2, lds, tot);  // (its barriers also publish cs)
  } else {
    RobotSum<NPART> rs;
    rs.issue(d.part, NPART, t0, t1);
    rs.finish(d.part, NPART, lds, tot);
  }
  const int ph = cs.phase;
  bool act = false;
  if (kind == RED_GRAD) act = ph == PH_START;
  if (kind == RED_HESS || kind == RED_UPDATE) act = ph == PH_TCG;
  if (kind == RED_COST) act = ph == PH_STEP;
  if (threadIdx.x == 0) {
    if (act) {
      const int ns = kind == RED_GRAD ? 3 : kind == RED_HESS ? 1 : kind == RED_UPDATE ? 2 : 4;
#pragma unroll
      for (int s = 0; s < NPART; ++s) tot[s] = s < ns ? tot[s] : 0.0;
      control_on(cs, d, l, kind, tot, R_, true);
      if (kind == RED_HESS && slot >= 0) atomicAdd(d.hv_launch + slot, 1);
    }
    if (hs) post_status(hs, l, seq, act && cs.phase == PH_TCG);
  }
  if (!act) return;
  __syncthreads();
  if (threadIdx.x < CW)
    reinterpret_cast<double*>(d.ctl + l)[threadIdx.x] = reinterpret_cast<const double*>(&cs)[threadIdx.x];
}

#define KMX_SMEM extern __shared__ __attribute__((aligned(16))) char smem[]

// Minimum waves per SIMD of the gather kernels: 4 at r <= 5 (128 VGPRs); the
// r >= 6 rows need more registers.
template <int R>
struct LB {
  static constexpr int w = R <= 5 ? 4 : 2;
};

// Start of an RTR iteration: egrad (gather X with public neighbours), cost,
// S = sym(Y^T egrad_Y), g = P_Y(egrad), z = precon(g); partials f, |g|^2, <z,g>.
// The per-pose 4x4 blocks D_i and the preconditioner (k_precond's work, same
// expressions and order), also used by k_grad's gated prologue.
template <int RW>
__device__ __forceinline__ void pose_precond(const Dev& d, int pose) {
  // A: the preconditioner's blocks (kappa I for the rotation part, as in the
  // oracle); Dq: Q's exact diagonal block for the Hessian gather, which with
  // the full records (measurements off SO(3)) carries w kappa R R^T instead
  double A[16], Dq[16];
  for (int i = 0; i < 16; ++i) A[i] = Dq[i] = 0.0;
  for (int k = d.inc_ptr[pose]; k < d.inc_ptr[pose + 1]; ++k) {
    double2 q[Rec<RW>::Q];
    Rec<RW>::load(d, (size_t)k, q);
    Edge E;
    Rec<RW>::edge(q, E);
    const bool tail = (Rec<RW>::inc(q).y >> 31) & 1;
    const double wk = E.wk, wt = E.wt;
    const double* tt = E.t;
    if (tail) {
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
          A[i * 4 + j] += wt * tt[i] * tt[j] + (i == j ? wk : 0.0);
          const double rr = (RW == 10) ? (i == j ? 1.0 : 0.0)
                                       : E.R[i * 3 + 0] * E.R[j * 3 + 0] + E.R[i * 3 + 1] * E.R[j * 3 + 1] +
                                             E.R[i * 3 + 2] * E.R[j * 3 + 2];
          Dq[i * 4 + j] += wt * tt[i] * tt[j] + wk * rr;
        }
        A[i * 4 + 3] += wt * tt[i];
        A[3 * 4 + i] += wt * tt[i];
        Dq[i * 4 + 3] += wt * tt[i];
        Dq[3 * 4 + i] += wt * tt[i];
      }
      A[15] += wt;
      Dq[15] += wt;
    } else {
      A[0] += wk; A[5] += wk; A[10] += wk; A[15] += wt;
      Dq[0] += wk; Dq[5] += wk; Dq[10] += wk; Dq[15] += wt;
    }
  }
  {
    double* Dp = d.hD + SYM4 * (size_t)pose;
    int j = 0;
    for (int a = 0; a < 4; ++a)
      for (int b = a; b < 4; ++b) Dp[j++] = Dq[a * 4 + b];
  }
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
  double* Pi = d.Pinv + SYM4 * (size_t)pose;  // Li^T Li: symmetric (upper triangle)
  int j = 0;
  for (int x = 0; x < 4; ++x)
    for (int y = x; y < 4; ++y) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += Li[k * 4 + x] * Li[k * 4 + y];
      Pi[j++] = s;
    }
}

// gated: the first gradient of a round whose begin launch may have re-weighted
// (the k_precond launch folded in): block 0 commits the GNC state and, when
// the begin fired, every tile rebuilds D_i and the preconditioner of its own
// poses (only its own incidence records are read) before the phase test, so
// idle robots are rebuilt too. The writes are read back by the tile's own
// lanes after the workgroup barrier (one CU: workgroup-scope visibility).
template <int R, int RW, int RM>
__device__ __forceinline__ void body_grad(const Dev& d, int gated, char* smem) {
  const Lane L = lane_map<R>(d);
  if (gated) {
    if (blockIdx.x == 0 && threadIdx.x == 0) store_gnc(d.gnc, load_gnc(d.gnc_next));
    if (d.gnc_next->fired) {
      const int np = L.np, p0 = L.p0;
      for (int t = threadIdx.x; t < np; t += blockDim.x) pose_precond<RW>(d, p0 + t);
      __syncthreads();
    }
  }
  if (d.ctl[L.l].phase != PH_START) return;
  double y[4] = {0, 0, 0, 0}, G[4], cost = 0.0;
  hinc_grad<R, RW>(d, L, d.X, d.pub, G, &cost, smem);
  if (L.valid) load4(d.X + (size_t)L.pose * 4 * R + 4 * L.a, y);
  // D_i - S_i for k_hess: the pose's D_i (five 16-B parts; a gated re-weight's
  // rebuild above is this workgroup's own writes) is loaded here, spread over its
  // lanes (parts a and a + r), so its latency runs under the group operations
  constexpr int NDP = R >= 5 ? 1 : 2;
  double2 dpart[NDP];
  {
    const double2* Dp2 = reinterpret_cast<const double2*>(d.hD + SYM4 * (size_t)L.pose);
#pragma unroll
    for (int u = 0; u < NDP; ++u) {
      const int i = L.a + u * R;
      dpart[u] = (L.valid && i < 5) ? Dp2[i] : make_double2(0.0, 0.0);
    }
  }
  double S[9], gr[4], zr[4];
  double* scr = reinterpret_cast<double*>(smem);  // the chunk buffer is free after the gather's last barrier
  group_symYtG<R, true>(y, G, L.base, S, scr);
#pragma unroll
  for (int c = 0; c < 3; ++c) gr[c] = G[c] - (y[0] * S[0 * 3 + c] + y[1] * S[1 * 3 + c] + y[2] * S[2 * 3 + c]);
  gr[3] = G[3];
  group_precon<R, true>(d, L.pose, L.valid, y, gr, L.base, zr, scr);
  double vals[3] = {cost, 0.0, 0.0};  // cost is accumulated on every incidence lane
  if (L.valid) {
    vals[1] = gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2] + gr[3] * gr[3];
    vals[2] = zr[0] * gr[0] + zr[1] * gr[1] + zr[2] * gr[2] + zr[3] * gr[3];
  }
  finish_tile<RED_GRAD, 3, RM>(d, L, vals, smem + SmemHG<R>::red_off, [&]() {
    if (!L.valid) return;
    const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
    store4(d.g + o, gr);  // r = g at the start of tCG: k_update's first step reads g
    store4(d.z + o, zr);
    if (L.a == 0) {
      double* Sp = d.S + 6 * (size_t)L.pose;
      Sp[0] = S[0]; Sp[1] = S[1]; Sp[2] = S[2]; Sp[3] = S[4]; Sp[4] = S[5]; Sp[5] = S[8];
    }
    // part i holds SYM4 entries 2i, 2i + 1: (00, 01), (02, 03), (11, 12), (13, 22), (23, 33)
    double2* Fp2 = reinterpret_cast<double2*>(d.hDS + SYM4 * (size_t)L.pose);
#pragma unroll
    for (int u = 0; u < NDP; ++u) {
      const int i = L.a + u * R;
      if (i < 5) {
        const double sx = i == 0 ? S[0] : i == 1 ? S[2] : i == 2 ? S[4] : 0.0;
        const double sy = i == 0 ? S[1] : i == 2 ? S[5] : i == 3 ? S[8] : 0.0;
        Fp2[i] = make_double2(dpart[u].x - sx, dpart[u].y - sy);
      }
    }
  });
}

// eta = sum_k coef_k delta_k over a tCG's T directions, in step order (the
// first F were folded into d.eta by the Hess-vec launches), added to et. LAST:
// the coefficient of direction T - 1 is clast (a k_step that ends the tCG
// decided it in the same launch whose writer stores it to coefh).
template <bool LAST>
__device__ __forceinline__ void eta_rows(const Dev& d, int l, size_t o, int T, double clast, double et[4]) {
  const int dhn = d.dhn;
  const int F = T > 0 ? (T - 1) / dhn * dhn : 0;
  if (F > 0) load4(d.eta + o, et);
  double dd[DHMAX][4];
#pragma unroll
  for (int i = 0; i < DHMAX; ++i)
    if (F + i < T) load4(d.dh + (size_t)i * d.vec + o, dd[i]);
  const double* ch = d.coefh + (size_t)l * d.p.tcg_max;
#pragma unroll
  for (int i = 0; i < DHMAX; ++i)
    if (F + i < T) {
      const double cj = (LAST && F + i == T - 1) ? clast : ch[F + i];
#pragma unroll
      for (int k = 0; k < 4; ++k) et[k] += cj * dd[i][k];
    }
}

// The trial point Xt = R_X(eta) of the lane's row, and the tile's partials
// m(eta) = 1/2 <eta, g + r> (as 2 m) and ||Xt - X||^2 into d.part slots 2, 3
// (k_cost adds the cost in slot 0). Every lane of the workgroup calls it.
template <int R>
__device__ __forceinline__ void trial_rows(const Dev& d, const Lane& L, size_t o, const double x[4],
                                           const double gg[4], const double rr[4], const double et[4], char* smem) {
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
  double* lds = reinterpret_cast<double*>(smem);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double w = wave_sum(vals[s]);
    if ((threadIdx.x & 63) == 0) lds[s * WAVES + (threadIdx.x >> 6)] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) t += lds[s * WAVES + w];
      d.part[(size_t)L.tile * NPART + 2 + s] = t;
    }
  }
}

// tCG step, part 1 (the dominant kernel): Hz = Hess(z) by gather; then by
// linearity delta = -z + beta delta_old, Hdelta = -Hz + beta Hdelta_old;
// partial <delta, Hdelta>. delta_k is kept for k_retract's eta (Dev::dh).
// Hz and Hdelta are kept BEFORE the tangent projection (Hz^ = H z - z S;
// the Riemannian H delta = P_Y(H delta^)): projection is linear, so the
// recurrence holds for the unprojected rows, and <delta, Hdelta^> equals
// <delta, P_Y(Hdelta^)> for a tangent delta (Y^T delta skew, Y sym(.) S
// symmetric). k_update, which loads Y anyway, projects; this kernel then
// reads no X row (16 MB per launch at configs[3]: VERDICT r4 item 2).
template <int R, int RW, int RM>
__device__ __forceinline__ void body_hess(const Dev& d, int first_launch, int slot, HostStatus* hs,
                                          unsigned long long seq, char* smem) {
  const Lane L = lane_map<R>(d);
  int tcg_iter;
  double beta;
  double y[4] = {0, 0, 0, 0}, zs[4] = {0, 0, 0, 0}, H[4];
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  if constexpr (RM == RM_CONSUMER) {
    // the previous step's k_update partials give this robot's control step
    // after the update (stop test, beta); the partial loads are in flight with
    // the gather's first records, and the decision comes before the rows are
    // gathered (a stopped robot's tiles leave without the gather). The robot's
    // first tile writes the state to ctl2 for k_update and reports tCG
    // progress to the host.
    __shared__ Ctl cs;
    __shared__ double rl[NPART * WAVES];
    const Ctl& c0 = d.ctl[L.l];
    const bool writer = L.tile == L.rt0;
    // the writer's working copy of the state, loaded by wave 0 at the start
    // (its lane 0 reads it after these in-order LDS writes of its own wave)
    if (writer && threadIdx.x < (int)(sizeof(Ctl) / 8))
      reinterpret_cast<double*>(&cs)[threadIdx.x] = reinterpret_cast<const double*>(&c0)[threadIdx.x];
    // first (the host's launch 0 of a tCG loop): a robot in it is at
    // PH_START, the first step of the tCG, whose gradient reduction (k_grad's
    // partials) this launch also consumes in place of a k_reduce launch; later
    // launches find it in PH_TCG. The robot sums' loads go out before the
    // state arrives.
    const bool grad = (first_launch & 1) != 0;
    const bool upd = !grad;
    RobotSum<2> rs;  // (four tiles per thread here: spills at 128 VGPRs)
    RobotSum<3> rg;
    if (upd) rs.issue(d.part_u, 2, L.rt0, L.rt1);
    if (grad) rg.issue(d.part, NPART, L.rt0, L.rt1);
    const int ph0 = c0.phase;  // written by an earlier launch: uniform
    const bool active = ph0 == (grad ? PH_START : PH_TCG);  // uniform: a tile never straddles robots
    auto idle = [&]() {
      if (writer && threadIdx.x == 0) {
        d.ctl2[L.l] = c0;
        if (hs) post_status(hs, L.l, seq, false);
      }
    };
    // early (below): the phase test waits in the decision, so the first
    // records load with the state instead of after it
    // gated (first_launch & 2, a launch the host expects to find robots
    // stopped): the phase test before the first records are issued, so a
    // launch with nothing to do reads its control words and leaves
    if (!active && (!d.p.early_stop || (first_launch & 2))) {
      idle();
      return;
    }
    UpdStep u{0, 0, 0.0};
    // the decision runs while the first chunk's records are in flight and
    // before any row is gathered: a robot whose tCG stops here (or whose
    // gradient is below tolerance) skips the gather, and the host sees the
    // stop at the start of the launch
    auto decide = [&]() {
      if (!active) {
        idle();
        return false;
      }
      double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
      if (upd) rs.finish(d.part_u, 2, rl, tot);
      if (grad) rg.finish(d.part, NPART, rl, tot);
      // every thread evaluates the decision; the first tile's thread 0 also
      // updates the robot's state (on an LDS copy: a private one would live in
      // scratch) and publishes it
      if (upd) u = upd_step(c0.mode, c0.r_stop, c0.lin_stop, c0.z_r, c0.tcg_iter, tot[0], tot[1], d.p);
      if (grad) u.done = sqrt(tot[1]) < d.p.gn_tol ? 1 : 0;  // control_on's RED_GRAD test
      if (writer && threadIdx.x == 0) {
        if (upd || grad) control_on(cs, d, L.l, grad ? RED_GRAD : RED_UPDATE, tot, R, true);
        d.ctl2[L.l] = cs;
        if (hs) post_status(hs, L.l, seq, cs.phase == PH_TCG);
      }
      return !u.done;
    };
    // early (small problems): decide before the gather; otherwise after it,
    // speculatively, so the robot sums' latency hides behind the gather
    bool go;
    if (d.p.early_stop) {
      go = hinc_gather<R, RW, false, false>(d, L, d.z, H, smem, decide);
    } else {
      hinc_gather<R, RW, false, false>(d, L, d.z, H, smem);
      go = decide();
    }
    if (!go) return;
    tcg_iter = grad ? 0 : c0.tcg_iter;
    beta = u.beta;
  } else {
    // the phase test runs once the first chunk's records are in flight (a
    // robot out of tCG leaves before any row is gathered); the robot's state
    // (written by an earlier launch) loads with those records, not after the
    // gather's first barrier
    const Ctl& c = d.ctl[L.l];
    const int ph = c.phase;
    tcg_iter = c.tcg_iter;
    beta = c.beta;
    // gated (first_launch & 2, see the consumer form): no record is fetched
    // before the phase test
    if ((first_launch & 2) && ph != PH_TCG) return;
    if (!hinc_gather<R, RW, true, false>(d, L, d.z, H, smem, [&]() { return ph == PH_TCG; })) return;
  }
  const bool first = (tcg_iter == 0) || (KMX_HESS_PROBE & 4);  // (probe 4: no delta_old / Hdelta_old traffic)
  asm volatile("" ::: "memory");  // keep the epilogue loads below the gather loop (VGPR pressure)
  // every row the epilogue needs in one batch, one round trip after the gather:
  // the own z row, D_i - S_i (the diagonal block with the tangent correction
  // -z S folded in), delta_old and H delta_old
  const int dhn = d.dhn;
  double dold[4] = {0, 0, 0, 0}, hold[4] = {0, 0, 0, 0};
  if (L.valid) {
    double Dg[16];
#if KMX_HESS_PROBE & 2  // traffic attribution build: no own-row / diagonal-block loads
    for (int k = 0; k < 4; ++k) zs[k] = 1e-3 * k;
    for (int c = 0; c < 16; ++c) Dg[c] = (c % 5 == 0) ? 1.0 : 0.0;
#else
    load4(d.z + o, zs);
    load_sym4(d.hDS + SYM4 * (size_t)L.pose, Dg);
#endif
    if (!first) {
      load4(d.dh + (size_t)((tcg_iter - 1) % dhn) * d.vec + o, dold);
      load4(d.hd + o, hold);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)  // (hinc_gather_src's DIAG term, same expression)
      H[c] += zs[0] * Dg[4 * c] + zs[1] * Dg[4 * c + 1] + zs[2] * Dg[4 * c + 2] + zs[3] * Dg[4 * c + 3];
  }
  double hz[4];  // H z - z S (group_rhess before its projection)
#pragma unroll
  for (int k = 0; k < 4; ++k) hz[k] = H[k];
  (void)y;
  double v = 0.0;
  double dl[4] = {0, 0, 0, 0}, hdl[4] = {0, 0, 0, 0};
  if (L.valid) {
    if (first) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { dl[k] = -zs[k]; hdl[k] = -hz[k]; }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dl[k] = -zs[k] + beta * dold[k];
        hdl[k] = -hz[k] + beta * hold[k];
      }
      if (tcg_iter >= dhn && tcg_iter % dhn == 0) {
        // tcg_max > dhn only: delta_k goes into the oldest direction's buffer,
        // so the dhn directions k - dhn .. k - 1 join eta first, in step order
        double et[4] = {0, 0, 0, 0};
        if (tcg_iter > dhn) load4(d.eta + o, et);
        const double* ch = d.coefh + (size_t)L.l * d.p.tcg_max;
        for (int j = tcg_iter - dhn; j < tcg_iter; ++j) {
          double dj[4];
          if (j + 1 < tcg_iter) {
            load4(d.dh + (size_t)(j % dhn) * d.vec + o, dj);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) dj[k] = dold[k];
          }
          const double cj = ch[j];
#pragma unroll
          for (int k = 0; k < 4; ++k) et[k] += cj * dj[k];
        }
        store4(d.eta + o, et);
      }
    }
    v = dl[0] * hdl[0] + dl[1] * hdl[1] + dl[2] * hdl[2] + dl[3] * hdl[3];
  }
  finish_tile<RED_HESS, 1, RM>(d, L, &v, smem + SmemH<R>::red_off, [&]() {
    if (L.valid && !(KMX_HESS_PROBE & 8)) {  // (probe 8: no stores)
      store4(d.dh + (size_t)(tcg_iter % dhn) * d.vec + o, dl);
      store4(d.hd + o, hdl);
    }
  });
}

// tCG step, part 2: r += coef Hdelta (eta = sum coef_k delta_k is formed in
// k_retract); interior steps also z = precon(r) and partials <r,r>, <z,r>.
template <int R, int RM>
__device__ __forceinline__ void body_update(const Dev& d, HostStatus* hs, unsigned long long seq, int slot,
                                            char* smem) {
  const Lane L = lane_map<R>(d);
  int tcg_iter, mode;
  double coef;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double rr[4] = {0, 0, 0, 0}, y[4] = {0, 0, 0, 0}, hdl[4] = {0, 0, 0, 0};
  double Pm[16];
  bool pre = false;
  if constexpr (RM == RM_CONSUMER) {
    // this step's k_hess partials: the control step after the Hess-vec (alpha
    // or the boundary tau) on a private copy, with the step's vector loads in
    // flight; the first tile writes the robot's state (ctl2 -> ctl)
    __shared__ Ctl cs;
    __shared__ double rl[NPART * WAVES];
    Ctl* const cin = d.ctl2;
    Ctl* const cout = d.ctl;
    const Ctl& cq = cin[L.l];
    const bool writer = L.tile == L.rt0;
    if (writer && threadIdx.x < (int)(sizeof(Ctl) / 8))  // as in k_hess
      reinterpret_cast<double*>(&cs)[threadIdx.x] = reinterpret_cast<const double*>(&cq)[threadIdx.x];
    if (cq.phase != PH_TCG) {
      if (cq.phase == PH_STEP && !cq.retracted) {
        // this step's k_hess ended the robot's tCG at its stop test: the trial
        // point and the model partials here (k_retract's arithmetic; every
        // coefficient was decided by an earlier launch), so a round whose
        // robots all stop this way needs no k_retract (the host skips it, or
        // launches it with fold = 2 for the robots still in tCG at the cap)
        const size_t o2 = (size_t)L.pose * 4 * R + 4 * L.a;
        double x[4] = {0, 0, 0, 0}, gg[4] = {0, 0, 0, 0}, rr2[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0};
        if (L.valid) {
          load4(d.X + o2, x);
          load4(d.g + o2, gg);
          load4(d.r + o2, rr2);
          eta_rows<false>(d, L.l, o2, cq.tcg_iter, 0.0, et);
        }
        trial_rows<R>(d, L, o2, x, gg, rr2, et, smem);
        if (writer && threadIdx.x == 0) {
          cout[L.l] = cq;
          cout[L.l].retracted = 1;
        }
        return;
      }
      if (writer && threadIdx.x == 0) cout[L.l] = cq;
      return;
    }
    const bool first0 = cq.tcg_iter == 0;  // the control step makes it 1
    RobotSum<1, 4> rs;
    rs.issue(d.part_h, 2, L.rt0, L.rt1);
    if (L.valid) {
      load4(d.hd + o, hdl);
      load4((first0 ? d.g : d.r) + o, rr);
      load4(d.X + o, y);  // the projection of H delta, and the precon of interior steps
      if (d.p.use_precond) {  // the preconditioner block too: no load after the decision
        load_sym4(d.Pinv + SYM4 * (size_t)L.pose, Pm);
      }
    }
    double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
    rs.finish(d.part_h, 2, rl, tot);
    const HessStep hsx = hess_step(cq.z_r, cq.e_Pe, cq.e_Pd, cq.d_Pd, cq.Delta, tot[0]);
    if (writer && threadIdx.x == 0) {  // the state update, on an LDS copy
      control_on(cs, d, L.l, RED_HESS, tot, R, true);
      cout[L.l] = cs;
      if (slot >= 0) atomicAdd(d.hv_launch + slot, 1);
    }
    tcg_iter = cq.tcg_iter + 1;
    mode = hsx.boundary ? MODE_BOUNDARY : MODE_INTERIOR;
    coef = hsx.coef;
    pre = L.valid;
  } else {
    const Ctl& c = d.ctl[L.l];
    if (c.phase != PH_TCG) {  // not in tCG: the robot's first tile reports it
      if (hs && threadIdx.x == 0 && L.tile == L.rt0) post_status(hs, L.l, seq, false);
      return;
    }
    tcg_iter = c.tcg_iter;
    mode = c.mode;
    coef = c.coef;
    if (L.valid) {
      load4(d.hd + o, hdl);
      load4((tcg_iter == 1 ? d.g : d.r) + o, rr);  // r_0 = g (k_grad does not store r)
      load4(d.X + o, y);  // the projection of H delta (and the precon of interior steps)
    }
  }
  const bool interior = (mode == MODE_INTERIOR);
  (void)tcg_iter;
  {  // H delta = P_Y(H delta^) (k_hess keeps it unprojected); every lane of the group takes part
    double hp[4];
    group_proj<R, true>(y, hdl, L.base, hp, reinterpret_cast<double*>(smem));
    if (L.valid) {
#pragma unroll
      for (int k = 0; k < 4; ++k) rr[k] += coef * hp[k];
    }
  }
  double vals[2] = {0.0, 0.0}, zr[4] = {0, 0, 0, 0};
  if (interior) {  // uniform per robot
    group_precon<R, true>(d, L.pose, L.valid, y, rr, L.base, zr, reinterpret_cast<double*>(smem),
                          Pm, pre);
    if (L.valid) {
      vals[0] = rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2] + rr[3] * rr[3];
      vals[1] = zr[0] * rr[0] + zr[1] * rr[1] + zr[2] * rr[2] + zr[3] * rr[3];
    }
  }
  finish_tile<RED_UPDATE, 2, RM>(d, L, vals, smem + SmemU::red_off, [&]() {
    if (L.valid) {
      store4(d.r + o, rr);
      if (interior) store4(d.z + o, zr);
    }
  });
}

// ------------------------------------------------ one-sync tCG (opt-in) ---
// P.tcg_form = KMX_TCG_FORM_ONESYNC: one kernel per tCG step (k_step), so a
// step has one grid-wide dependency instead of two (k_hess -> k_update ->
// k_hess). Launch j applies step j-1's decision and forms step j:
//  1. every workgroup reduces the robot's 8-wide partials of launch j-1
//     (RobotSum8, tile order) and evaluates the decisions on them:
//     alpha (or the boundary tau) from <delta,H delta> and <r,z>, then the
//     stop test and beta from <r',r'> and <r',z'> formed by the recurrences
//       <r',r'> = <r,r> + 2 alpha <r,Hd> + alpha^2 <Hd,Hd>
//       <r',z'> = <r,z> + alpha (<r,w> + <Hd,z>) + alpha^2 <Hd,w>
//     (w = precon(H delta), precon linear); <r,z> and <r,r> are reduced from
//     the recurred vectors at every step, so the scalar recurrences are one
//     step deep. The robot's first tile writes the state (cin -> cout,
//     alternating buffers) and the host status;
//  2. the gather applies the Hessian to w (step 0: to z_0) — one row per
//     incidence, as k_hess — and the owner forms, by linearity,
//       z' = z + alpha w,        Hz' = Hz + alpha Hw,
//       delta' = -z' + beta delta,  H delta' = -Hz' + beta H delta,
//       r' = r + coef H delta,   w' = precon(H delta')
//     (fused multiply-adds, as the restatement), and the 7 partials.
// A robot whose tCG stops in step 1 only updates r (k_retract's model). What
// a launch reads across tiles — w and the robot's 8-wide partials — is
// double-buffered by step parity (launch j reads step j-1's and writes step
// j's); the kept directions are d.dh as in the standard form.
// Restated by oracle/dpgo_oracle.c tcg_onesync (same recurrences); parity
// with the standard form at convergence only.
__device__ __forceinline__ void onesync_scalars(double al, const double* tot, double* rrn, double* zrn) {
#pragma clang fp contract(off)
  *rrn = fmax(tot[2] + 2.0 * al * tot[5] + al * al * tot[6], 0.0);
  *zrn = tot[1] + al * tot[3] + al * al * tot[4];
}

// RobotSum for the one-sync step's 8-wide partials (d.part_f), same order as
// robot_sum: U tiles per thread in one round trip (1024 tiles, the 736-tile
// cut of a 12.5k-pose block included), tile order within a thread, then the
// wave sums and the waves in order; larger robots loop.
template <int U>
struct RobotSum8 {
  double a[U][8];
  int t0, t1;
  __device__ __forceinline__ void load(const double* part, int tb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(tb + (int)threadIdx.x + u * RBLOCK, t1 - 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double2 x = ldpart(part, (size_t)t * 8 + 2 * k);
        a[u][2 * k] = x.x;
        a[u][2 * k + 1] = x.y;
      }
    }
  }
  __device__ __forceinline__ void issue(const double* part, int t0_, int t1_) {
    t0 = t0_;
    t1 = t1_;
    if (t1 - t0 <= U * RBLOCK) load(part, t0);
  }
  __device__ __forceinline__ void finish(const double* part, double* lds, double tot[8]) {
    constexpr int RW_ = RBLOCK / 64;
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.0;
    for (int tb = t0; tb < t1; tb += U * RBLOCK) {
      if (t1 - t0 > U * RBLOCK) load(part, tb);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (tb + (int)threadIdx.x + u * RBLOCK < t1 && threadIdx.x < RBLOCK) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += a[u][k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double w = wave_sum(v[k]);
      if ((threadIdx.x & 63) == 0 && threadIdx.x < RBLOCK) lds[k * RW_ + (threadIdx.x >> 6)] = w;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      double acc = 0.0;
#pragma unroll
      for (int w = 0; w < RW_; ++w) acc += lds[k * RW_ + w];
      tot[k] = acc;
    }
  }
};

template <int R, int W = WAVES>
struct SmemF {  // k_step: the Hessian gather's layout with an 8-wide reduction area
  static constexpr int red_off = SmemH<R, W>::red_off;
  static constexpr int bytes = red_off + 8 * 8 * W + 16;
};

__device__ __forceinline__ double dot4(const double a[4], const double b[4]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}

// KMX_STEP_STAMPS builds (diagnostic, `make stamps`): thread 0 of every
// workgroup of the k_step launches that form step 2 records the wall clock
// (100 MHz) at entry, once the robot sums' loads are issued, once they (and
// the first records) have landed, after the decision, after the gather loop,
// after the Hessian's own-row part and at exit (kmx_pgo_debug_step_stamps;
// scripts/step_stamps.py).
#ifdef KMX_STEP_STAMPS
constexpr int STEP_STAMP_TILES = 8192;
__device__ unsigned long long g_step_stamp[16 * STEP_STAMP_TILES];
#define KMX_SS(i) \
  do { if (threadIdx.x == 0) ss_[i] = wall_clock64(); } while (0)
#else
#define KMX_SS(i) do {} while (0)
#endif

template <int R, int RW>
__device__ __forceinline__ void body_step(const Dev& d, const Ctl* cin, Ctl* cout, int jl, int slot,
                                          HostStatus* hs, unsigned long long seq, char* smem) {
#ifdef KMX_STEP_STAMPS
  unsigned long long ss_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  KMX_SS(0);
  const Lane L = lane_map<R>(d);
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  __shared__ Ctl cs;
  __shared__ double rl[8 * WAVES];
  const Ctl& c0 = cin[L.l];
  const bool writer = L.tile == L.rt0;
  if (writer && threadIdx.x < (int)(sizeof(Ctl) / 8))  // as in k_hess
    reinterpret_cast<double*>(&cs)[threadIdx.x] = reinterpret_cast<const double*>(&c0)[threadIdx.x];
  // first (the host's launch 0 of a tCG loop): a robot in it is at PH_START
  // and the launch consumes k_grad's partials, else it is in PH_TCG; the
  // robot sums' loads go out before the state arrives
  const bool grad = jl == 0;
  const int t0 = L.rt0, t1 = L.rt1;
  RobotSum<3> rg;
  RobotSum8<4> rf;
  if (grad) rg.issue(d.part, NPART, t0, t1);
  // launch jl consumes step jl - 1's partials (buffer (jl - 1) & 1) and
  // writes step jl's into the other buffer, so no tile of the robot can
  // overwrite a partial another tile of the same launch has yet to read (a
  // robot in tCG at launch jl is at tcg_iter jl - 1)
  const double* pf_in = d.part_f + (size_t)(((jl + 1) & 1) * d.ntiles) * 8;
  if (!grad) rf.issue(pf_in, t0, t1);
  const int ph0 = c0.phase;
  if (ph0 != (grad ? PH_START : PH_TCG)) {
    if (writer && threadIdx.x == 0) {
      cout[L.l] = c0;
      if (hs) post_status(hs, L.l, seq, false);
    }
    return;
  }
  const int k = grad ? -1 : c0.tcg_iter;  // the step whose partials this launch consumes
  double coef = 0.0, al = 0.0, be = 0.0;
  KMX_SS(1);
  auto decide = [&]() -> bool {
    bool go;
    KMX_SS(2);
    if (grad) {
      double tot[NPART];
      rg.finish(d.part, NPART, rl, tot);
      go = !(sqrt(tot[1]) < d.p.gn_tol);  // control_on's RED_GRAD test
      if (writer && threadIdx.x == 0) control_on(cs, d, L.l, RED_GRAD, tot, R, true);
    } else {
      double tot[8];
      rf.finish(pf_in, rl, tot);
      const double zr = tot[1];
      const HessStep hx = hess_step(zr, c0.e_Pe, c0.e_Pd, c0.d_Pd, c0.Delta, tot[0]);
      double rrn, zrn;
      onesync_scalars(hx.alpha, tot, &rrn, &zrn);
      const UpdStep u = upd_step(hx.boundary ? MODE_BOUNDARY : MODE_INTERIOR, c0.r_stop, c0.lin_stop, zr, k + 1,
                                 rrn, zrn, d.p);
      coef = hx.coef;
      al = hx.alpha;
      be = u.beta;
      go = !u.done;
      if (writer && threadIdx.x == 0) {  // the standard form's two control steps, on the LDS copy
        cs.z_r = zr;
        double th[NPART] = {tot[0], 0.0, 0.0, 0.0};
        control_on(cs, d, L.l, RED_HESS, th, R, true);
        double tu[NPART] = {rrn, zrn, 0.0, 0.0};
        control_on(cs, d, L.l, RED_UPDATE, tu, R, true);
      }
    }
    if (writer && threadIdx.x == 0) {
      cout[L.l] = cs;
      if (hs) post_status(hs, L.l, seq, cs.phase == PH_TCG);
      if (go && slot >= 0) atomicAdd(d.hv_launch + slot, 1);
    }
    KMX_SS(3);
    return go;
  };
  const int dhn = d.dhn;
  const double* V = grad ? d.z : ((k & 1) ? d.w1 : d.w0);  // the vector the Hessian is applied to
  double H[4];
  PlainRows<R> src{V};
  const bool go = hinc_gather_src<R, RW, false, PlainRows<R>, decltype(decide)&, false>(d, L, src, H, smem, decide);
  if (!grad && !go) {
    // the robot's tCG ends here: the last step's residual, then (no k_retract
    // in this form) the trial point of its rows and the model partials, with
    // this launch's coefficient for the last direction
    double x[4] = {0, 0, 0, 0}, gg[4] = {0, 0, 0, 0}, rr[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0};
    if (L.valid) {
      double hd[4];
      load4(d.r + o, rr);
      load4(d.hd + o, hd);
      load4(d.X + o, x);
      load4(d.g + o, gg);
#pragma unroll
      for (int c = 0; c < 4; ++c) rr[c] = fma(coef, hd[c], rr[c]);
      store4(d.r + o, rr);
      eta_rows<true>(d, L.l, o, k + 1, coef, et);
    }
    trial_rows<R>(d, L, o, x, gg, rr, et, smem);
    return;
  }
  if (!go) return;
  const int kn = k + 1;  // the step this launch forms
  KMX_SS(4);
  asm volatile("" ::: "memory");  // keep the epilogue loads below the gather loop (VGPR pressure)
  // every row the epilogue needs, in one batch (one round trip after the gather)
  // delta_kn goes into the oldest direction's buffer: directions kn - dhn ..
  // kn - 1 join eta first, in step order (the standard form's fold; the
  // newest coefficient is this launch's own decision). dhn = 2 (the
  // default): the older direction and eta load with the rest
  const bool fold = !grad && kn >= dhn && kn % dhn == 0;
  const bool fold2 = fold && dhn == 2;
  double dprev[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0};
  const double cprev = fold2 ? d.coefh[(size_t)L.l * d.p.tcg_max + kn - 2] : 0.0;
  double y[4] = {0, 0, 0, 0}, S[9], v[4] = {0, 0, 0, 0}, D[16], Pm[16];
  double rn[4] = {0, 0, 0, 0}, hold[4] = {0, 0, 0, 0}, zo[4] = {0, 0, 0, 0}, hzo[4] = {0, 0, 0, 0},
         dold[4] = {0, 0, 0, 0};
  if (L.valid) {
    load4(V + o, v);
    load_sym4(d.hD + SYM4 * (size_t)L.pose, D);
    load4(d.X + o, y);
    load_sym3(d.S + 6 * (size_t)L.pose, S);
    if (d.p.use_precond) load_sym4(d.Pinv + SYM4 * (size_t)L.pose, Pm);
    if (grad) {
      load4(d.g + o, rn);  // r_0 = g
    } else {
      load4(d.r + o, rn);
      load4(d.hd + o, hold);
      load4(d.z + o, zo);
      load4(d.hz + o, hzo);
      load4(d.dh + (size_t)(k % dhn) * d.vec + o, dold);
      if (fold2) {  // the direction folded with dold (below), and eta
        load4(d.dh + (size_t)(kn % dhn) * d.vec + o, dprev);
        if (kn > dhn) load4(d.eta + o, et);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)  // the diagonal block (hinc_gather's DIAG term, same expression)
      H[c] += v[0] * D[4 * c] + v[1] * D[4 * c + 1] + v[2] * D[4 * c + 2] + v[3] * D[4 * c + 3];
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) S[i] = 0.0;
  }
  double* scr = reinterpret_cast<double*>(smem);  // the chunk buffer is free after the gather
  double hv[4];
  group_rhess<R, true>(y, v, H, S, L.base, hv, scr);  // Riemannian Hess of z_0 or w_k
  KMX_SS(5);
  double zn[4], hzn[4], dl[4], hdl[4];
  if (grad) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      zn[c] = v[c];
      hzn[c] = hv[c];
      dl[c] = -v[c];
      hdl[c] = -hv[c];
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      rn[c] = fma(coef, hold[c], rn[c]);
      zn[c] = fma(al, v[c], zo[c]);
      hzn[c] = fma(al, hv[c], hzo[c]);
      dl[c] = fma(be, dold[c], -zn[c]);
      hdl[c] = fma(be, hold[c], -hzn[c]);
    }
  }
  double wn[4];
  group_precon<R, true>(d, L.pose, L.valid, y, hdl, L.base, wn, scr, Pm, L.valid);
  if (fold2 && L.valid) {
#pragma unroll
    for (int c = 0; c < 4; ++c) et[c] += cprev * dprev[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) et[c] += coef * dold[c];
    store4(d.eta + o, et);
  } else if (fold && L.valid) {  // other KMX_DHMAX builds
    if (kn > dhn) load4(d.eta + o, et);
    const double* ch = d.coefh + (size_t)L.l * d.p.tcg_max;
    for (int j = kn - dhn; j < kn; ++j) {
      double dj[4];
      load4(d.dh + (size_t)(j % dhn) * d.vec + o, dj);
      const double cj = (j == kn - 1) ? coef : ch[j];
#pragma unroll
      for (int c = 0; c < 4; ++c) et[c] += cj * dj[c];
    }
    store4(d.eta + o, et);
  }
  double pv[7] = {0, 0, 0, 0, 0, 0, 0};
  if (L.valid) {
    pv[0] = dot4(dl, hdl);
    pv[1] = dot4(rn, zn);
    pv[2] = dot4(rn, rn);
    pv[3] = dot4(rn, wn) + dot4(hdl, zn);
    pv[4] = dot4(hdl, wn);
    pv[5] = dot4(rn, hdl);
    pv[6] = dot4(hdl, hdl);
  }
  double* lds = reinterpret_cast<double*>(smem + SmemF<R>::red_off);
#pragma unroll
  for (int s2 = 0; s2 < 7; ++s2) {
    const double w = wave_sum(pv[s2]);
    if ((threadIdx.x & 63) == 0) lds[s2 * WAVES + (threadIdx.x >> 6)] = w;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    double t = 0.0;
    if (threadIdx.x < 7) {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) t += lds[threadIdx.x * WAVES + w];
    }
    d.part_f[((size_t)(kn & 1) * d.ntiles + L.tile) * 8 + threadIdx.x] = t;
  }
  if (L.valid) {
    store4(d.dh + (size_t)(kn % dhn) * d.vec + o, dl);
    store4(d.hd + o, hdl);
    store4(d.hz + o, hzn);
    if (!grad) store4(d.z + o, zn);
    store4(((kn & 1) ? d.w1 : d.w0) + o, wn);
    store4(d.r + o, rn);
  }
#ifdef KMX_STEP_STAMPS
  KMX_SS(6);
  if (kn == 2 && threadIdx.x == 0 && L.tile < STEP_STAMP_TILES) {
    for (int i = 0; i < 7; ++i) g_step_stamp[(size_t)L.tile * 16 + i] = ss_[i];
    g_step_stamp[(size_t)L.tile * 16 + 8] = (unsigned long long)L.np;
    g_step_stamp[(size_t)L.tile * 16 + 9] = (unsigned long long)L.n;
    g_step_stamp[(size_t)L.tile * 16 + 10] = (unsigned long long)blockIdx.x;
    g_step_stamp[(size_t)L.tile * 16 + 11] = (unsigned long long)(L.tile == L.rt0);
  }
#endif
}

// Trial point Xt = R_X(eta); partials: model m(eta) = 1/2 <eta, g + r> (r = g +
// H eta by the tCG recurrence) and ||Xt - X||^2 (slots 2, 3; k_cost reduces).
// fold (RM_CONSUMER): a robot still in tCG ran its last step's update with no
// k_hess after it; its reduction (the 2-wide part_u) and stop decision run
// here, in place of a k_reduce launch. The robot's first tile writes the
// decision into ctl in place: it changes only phase and tcg_stop, and a tile
// that reads the new phase goes straight to the retraction, as the decision
// says, so every tile acts alike.
// src: where the tCG left the robot's state — d.ctl, or d.ctl2 after an odd
// number of one-sync steps; the robot's first tile copies it to d.ctl, which
// the launches after this one read.
template <int R>
__device__ __forceinline__ void body_retract(const Dev& d, int fold, const Ctl* src, char* smem) {
  const Lane L = lane_map<R>(d);
  const Ctl& c = src[L.l];
  __shared__ int sph;
  __shared__ double rl[NPART * WAVES];
  if (threadIdx.x == 0) {
    sph = c.phase;
    if (src != d.ctl && L.tile == L.rt0) d.ctl[L.l] = c;
  }
  __syncthreads();
  const int ph = sph;  // one read per workgroup
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double x[4] = {0, 0, 0, 0}, et[4] = {0, 0, 0, 0}, gg[4] = {0, 0, 0, 0}, rr[4] = {0, 0, 0, 0}, dl[4];
  if (fold && ph == PH_TCG) {  // fold 2: a robot at PH_STEP may already be retracted (k_update)
    RobotSum<2> rs;
    rs.issue(d.part_u, 2, L.rt0, L.rt1);
    double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
    rs.finish(d.part_u, 2, rl, tot);
    const UpdStep u = upd_step(c.mode, c.r_stop, c.lin_stop, c.z_r, c.tcg_iter, tot[0], tot[1], d.p);
    if (!u.done) return;  // (cannot happen: the host stops enqueueing only when no robot is in tCG or at tcg_max)
    if (threadIdx.x == 0 && L.tile == L.rt0) {  // (fold: src is d.ctl)
      if (u.stop >= 0) d.ctl[L.l].tcg_stop = u.stop;
      d.ctl[L.l].phase = PH_STEP;
    }
  } else if (ph != PH_STEP || (fold == 2 && c.retracted)) {
    return;
  }
  if (L.valid) {  // all rows in flight before the Gram-Schmidt chain
    load4(d.X + o, x);
    load4(d.g + o, gg);
    load4(d.r + o, rr);
    if (d.p.rgd) {  // RGD: eta = -s z
      load4(d.z + o, dl);
      const double coef = c.coef;
#pragma unroll
      for (int k = 0; k < 4; ++k) et[k] += coef * dl[k];
    } else {
      eta_rows<false>(d, L.l, o, c.tcg_iter, 0.0, et);
    }
  }
  trial_rows<R>(d, L, o, x, gg, rr, et, smem);
}

// src: as k_retract's (the one-sync form has no k_retract: its k_step
// retracts a robot's rows in the launch that ends its tCG, so k_cost carries
// the state over to d.ctl).
template <int R, int RW, int RM>
__device__ __forceinline__ void body_cost(const Dev& d, const Ctl* src, char* smem) {
  const Lane L = lane_map<R>(d);
  const Ctl& c = src[L.l];
  if (src != d.ctl && threadIdx.x == 0 && L.tile == L.rt0) d.ctl[L.l] = c;
  if (c.phase != PH_STEP) return;
  double cost = inc_owner_cost<R, RW>(d, L, d.Xt, d.pub, smem);
  finish_tile<RED_COST, 1, RM>(d, L, &cost, smem + SmemC<R>::red_off, []() {});
}

// End of a round: X <- Xt where the step was accepted, and the owned public
// rows of the committed poses are published (the single-device exchange), so
// the next round — and a GNC weight update before it — sees the new poses.
// Tile 0 also counts the round for the GNC schedule.
// fold (RM_CONSUMER, one RTR iteration): the trial-cost reduction and the
// accept decision run here in place of a k_reduce launch; every tile decides
// from the robot's totals and f_cur, which the decision does not change. The
// robot's first tile writes the RTR state, except the phase, which stays
// PH_STEP (the next round's k_begin resets it), so tiles that read the state
// after that write still see a robot with a step to decide.
// final = 0: between two RTR iterations of one block update — the accepted
// trial point becomes the iterate the next iteration starts from, but the
// public rows (the neighbours' snapshot of this round) and the round counters
// wait for the block update's end.
template <int R>
__device__ __forceinline__ void body_commit(const Dev& d, int fold, int final) {
  const Lane L = lane_map<R>(d);
  if (final && L.tile == 0 && threadIdx.x == 0) {
    d.gnc->inner += 1;
    d.gnc->rounds += 1;
  }
  bool commit;
  if (fold) {
    __shared__ int sph;
    __shared__ Ctl cs;
    __shared__ double rl[NPART * WAVES];
    const Ctl& c = d.ctl[L.l];
    const bool writer = L.tile == L.rt0;
    if (writer && threadIdx.x < (int)(sizeof(Ctl) / 8))  // as in k_hess
      reinterpret_cast<double*>(&cs)[threadIdx.x] = reinterpret_cast<const double*>(&c)[threadIdx.x];
    if (threadIdx.x == 0) sph = c.phase;
    __syncthreads();
    if (sph != PH_STEP) return;
    RobotSum<NPART> rs;
    rs.issue(d.part, NPART, L.rt0, L.rt1);
    double tot[NPART] = {0.0, 0.0, 0.0, 0.0};
    rs.finish(d.part, NPART, rl, tot);
    if (d.p.rgd) {
      commit = true;
    } else {  // control_on's RED_COST acceptance test
      const double model_dec = -0.5 * tot[2];
      const double rho = (model_dec > 0.0) ? (c.f_cur - tot[0]) / model_dec : -1.0;
      commit = rho > d.p.accept_rho;
    }
    if (threadIdx.x == 0 && writer) {
      control_on(cs, d, L.l, RED_COST, tot, R, true);
      cs.phase = PH_STEP;
      d.ctl[L.l] = cs;
    }
  } else {
    commit = d.ctl[L.l].commit != 0;
  }
  if (!commit || !L.valid) return;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double v[4];
  load4(d.Xt + o, v);
  store4(d.X + o, v);
  if (!final) return;
  const int s = d.pose_slot[L.pose];
  if (s >= 0) store4(d.pub + (size_t)s * 4 * R + 4 * L.a, v);
}

// One kernel per phase of the round.
template <int R, int RW, int RM>
__global__ __launch_bounds__(BLOCK, LB<R>::w) void k_grad(Dev d, int gated) {
  KMX_SMEM;
  body_grad<R, RW, RM>(d, gated, smem);
}
template <int R, int RW, int RM>
__global__ __launch_bounds__(BLOCK, LB<R>::w) void k_hess(Dev d, int first, int slot, HostStatus* hs,
                                                          unsigned long long seq) {
  KMX_SMEM;
  body_hess<R, RW, RM>(d, first, slot, hs, seq, smem);
}
template <int R, int RM>
__global__ __launch_bounds__(BLOCK) void k_update(Dev d, HostStatus* hs, unsigned long long seq, int slot) {
  KMX_SMEM;
  body_update<R, RM>(d, hs, seq, slot, smem);
}
// 3 waves per SIMD at r <= 5: the 736-tile cut of a small shard is resident
// in one generation (256 CUs x 3), without the spills of a 128-VGPR bound
template <int R, int RW>
__global__ __launch_bounds__(BLOCK, (R <= 5 ? 3 : 2)) void k_step(Dev d, const Ctl* cin, Ctl* cout, int jl, int slot,
                                                                  HostStatus* hs, unsigned long long seq) {
  KMX_SMEM;
  body_step<R, RW>(d, cin, cout, jl, slot, hs, seq, smem);
}
template <int R>
__global__ __launch_bounds__(BLOCK) void k_retract(Dev d, int fold, const Ctl* src) {
  KMX_SMEM;
  body_retract<R>(d, fold, src, smem);
}
template <int R, int RW, int RM>
__global__ __launch_bounds__(BLOCK, LB<R>::w) void k_cost(Dev d, const Ctl* src) {
  KMX_SMEM;
  body_cost<R, RW, RM>(d, src, smem);
}
template <int R>
__global__ __launch_bounds__(BLOCK) void k_commit(Dev d, int fold, int final) {
  body_commit<R>(d, fold, final);
}

// ------------------------------------------------- round begin + GNC-TLS ---
// shouldUpdateMeasurementWeights (drawio:2466-2469): never for L2 or once
// robustOptNumWeightUpdates updates were made; otherwise when more than
// robustOptInnerIters rounds ran since the last update, or when every agent of
// the team has converged (relative change of its last block update <=
// relChangeTol; this handle's robots plus the peers' statuses in `ext`).
__device__ __forceinline__ bool gnc_should_update(const Dev& d) {
  const Params& P = d.p;
  if (!P.robust || !P.gnc_on) return false;
  const Gnc& s = *d.gnc;
  if (s.updates >= P.max_updates) return false;
  if (s.inner > P.inner_iters) return true;
  for (int l = 0; l < d.L; ++l)
    if (!(d.relc[l] <= P.rel_tol)) return false;
  for (int k = 0; k < P.n_ext; ++k)
    if (!(d.ext[k] <= P.rel_tol)) return false;
  return true;
}

// TLS weight of one loop closure on the lifted poses (oracle residual_sq and
// gnc_tls_weight): the owner's and the peer's handles both evaluate a shared
// loop closure from the same two rows, so both get the owner's value bit for
// bit without the measurement_weights message (drawio:2195-2198).
template <int RW>
__device__ __forceinline__ void gnc_edge(const Dev& d, int i, int R_, double mu) {
  const int e = d.gnc_edge[i];
  const int2 en = d.gnc_ends[i];
  const int ps = 4 * R_;
  const double* Xi = en.x >= 0 ? d.X + (size_t)en.x * ps : d.pub + (size_t)(-1 - en.x) * ps;
  const double* Xj = en.y >= 0 ? d.X + (size_t)en.y * ps : d.pub + (size_t)(-1 - en.y) * ps;
  const int2 ip = d.eipos[e];
  double2 q[Rec<RW>::Q];
  Rec<RW>::load(d, (size_t)(ip.x >= 0 ? ip.x : ip.y), q);
  Edge E;
  Rec<RW>::edge(q, E);
  double sR = 0.0, sT = 0.0;
  for (int a = 0; a < R_; ++a) {
    const double* yi = Xi + 4 * a;
    const double* yj = Xj + 4 * a;
    for (int c = 0; c < 3; ++c) {
      const double r = yj[c] - (yi[0] * E.R[0 * 3 + c] + yi[1] * E.R[1 * 3 + c] + yi[2] * E.R[2 * 3 + c]);
      sR += r * r;
    }
    const double et = yj[3] - yi[3] - (yi[0] * E.t[0] + yi[1] * E.t[1] + yi[2] * E.t[2]);
    sT += et * et;
  }
  const double rSq = d.ekappa[e] * sR + d.etau[e] * sT;
  const double barcSq = d.p.barc * d.p.barc;
  const double upper = (mu + 1.0) / mu * barcSq;
  const double lower = mu / (mu + 1.0) * barcSq;
  double w;
  if (rSq >= upper) w = 0.0;
  else if (rSq <= lower) w = 1.0;
  else w = sqrt(barcSq * mu * (mu + 1.0) / rSq) - mu;
  d.ew[e] = w;
  const double wk = w * d.ekappa[e], wt = w * d.etau[e];
  constexpr int WK = Rec<RW>::WK;
  constexpr int GS = Rec<RW>::GS;  // ip.x: the tail's record, ip.y: the head's
  if (ip.x >= 0) { d.rec[(size_t)GS * ip.x + WK] = wk; d.rec[(size_t)GS * ip.x + WK + 1] = Rec<RW>::wt_word(wt, true); }
  if (ip.y >= 0) { d.rec[(size_t)GS * ip.y + WK] = wk; d.rec[(size_t)GS * ip.y + WK + 1] = Rec<RW>::wt_word(wt, false); }
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

enum BeginMode { BEGIN_ROUND = 1, BEGIN_FORCE_GNC = 2, BEGIN_SOLO = 4 };

// Round begin (BEGIN_ROUND: reset the robots' Ctl) and/or a GNC weight update:
// scheduled (gnc_should_update) or forced (BEGIN_FORCE_GNC, the explicit
// updateMeasurementWeights). Every block takes the same decision from the
// same state; block 0 writes the next state to gnc_next (k_precond commits
// it), the other blocks re-weight their loop closures and rewrite both
// incidence records of each.
template <int RW>
__global__ void k_begin(Dev d, const unsigned char* active, int mode, int R_) {
  const bool fire = d.p.robust && ((mode & BEGIN_FORCE_GNC) ? true : gnc_should_update(d));
  const double mu = d.gnc->mu;
  if (blockIdx.x == 0) {
    if (mode & BEGIN_ROUND)
      for (int l = threadIdx.x; l < d.L; l += blockDim.x) begin_robot(d, active, l);
    if (threadIdx.x == 0) {
      Gnc s = load_gnc(d.gnc);
      s.fired = fire ? 1 : 0;
      if (fire) {
        s.inner = 0;
        s.updates += 1;
        s.mu = mu * d.p.mu_step;
      }
      store_gnc(d.gnc_next, s);
      if (mode & BEGIN_SOLO) store_gnc(d.gnc, s);  // one-block launch: no reader of the state is left
      if (fire) atomicAdd(&d.cnt->gnc_updates, 1ull);
    }
    return;
  }
  if (!fire) return;
  for (int i = (blockIdx.x - 1) * blockDim.x + threadIdx.x; i < d.n_gnc; i += (gridDim.x - 1) * blockDim.x)
    gnc_edge<RW>(d, i, R_, mu);
}

// 4x4 diagonal blocks D_i of Q per pose (hD, for the Hessian gather) and the
// inverse preconditioner blocks (D_i + shift I)^-1 by Cholesky; same
// accumulation order and expressions as oracle build_precond. `gated`: only
// after a round-begin launch that re-weighted (then block 0 commits gnc_next).
template <int RW>
__global__ void k_precond(Dev d, int gated) {
  if (gated) {
    if (blockIdx.x == 0 && threadIdx.x == 0) store_gnc(d.gnc, load_gnc(d.gnc_next));
    if (!d.gnc_next->fired) return;
  }
  for (int pose = blockIdx.x * blockDim.x + threadIdx.x; pose < d.nloc; pose += gridDim.x * blockDim.x)
    pose_precond<RW>(d, pose);
}

// setMeasurementWeight in bulk: push the per-edge weights into both incidence
// records (w kappa, w tau).
template <int RW>
__global__ void k_apply_weights(Dev d, int mloc) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= mloc) return;
  const double w = d.ew[e];
  const double wk = w * d.ekappa[e], wt = w * d.etau[e];
  const int2 ip = d.eipos[e];
  constexpr int WK = Rec<RW>::WK;
  constexpr int GS = Rec<RW>::GS;  // ip.x: the tail's record, ip.y: the head's
  if (ip.x >= 0) { d.rec[(size_t)GS * ip.x + WK] = wk; d.rec[(size_t)GS * ip.x + WK + 1] = Rec<RW>::wt_word(wt, true); }
  if (ip.y >= 0) { d.rec[(size_t)GS * ip.y + WK] = wk; d.rec[(size_t)GS * ip.y + WK + 1] = Rec<RW>::wt_word(wt, false); }
}

// ------------------------------------------------------- public exchange ---
// One 16-B part i of the owned public rows: slot s = i / (ps / 2) (ps = 4r is
// even, rows are 16-B aligned).
__global__ void k_publish(const double* X, double* pub, const int* src, int nslots, int ps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int ps2 = ps >> 1;
  const long long s = i / ps2;
  if (s >= nslots) return;
  const int q = (int)(i - s * ps2);
  const int p = src[s];
  if (p >= 0)
    reinterpret_cast<double2*>(pub)[s * ps2 + q] = reinterpret_cast<const double2*>(X)[(long long)p * ps2 + q];
}

// Sparse exchange: rows of the given public slots (owned by this handle) from
// the iterate, and rows received from peers written into the table. With
// per-peer segments (nseg > 0, seg[k] = first row of peer k's segment), every
// segment is followed by one status double (this handle's largest relative
// change, dpgo's Status message, drawio:2375): segment k starts at row
// seg[k] * ps + k. A slot outside the table (or, for gather, not owned here)
// is skipped (gather writes zeros), so a bad index list cannot fault the device.
__device__ __forceinline__ long long seg_offset(const int* seg, int nseg, long long s) {
  int k = 0;
  while (k + 1 < nseg && seg[k + 1] <= s) ++k;
  return nseg > 0 ? k : 0;
}
// The status words ride in the same launch: threads n*ps .. n*ps + nseg - 1
// write this handle's max relative change after every segment (gather) /
// read the peers' into ext (scatter). One launch per side of the exchange.
__global__ void k_gather_slots(const double* X, const int* pub_src, const int* slots, long long n, int npub,
                               double* out, int ps, const int* seg, int nseg, const double* relc, int L) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) {
    const long long k = i - n * ps;
    if (k >= nseg) return;
    double m = 0.0;
    for (int l = 0; l < L; ++l) m = (relc[l] > m || relc[l] != relc[l]) ? relc[l] : m;
    out[(long long)seg[k + 1] * ps + k] = m;
    return;
  }
  const int q = (int)(i - s * ps);
  const int sl = slots[s];
  const int p = (sl >= 0 && sl < npub) ? pub_src[sl] : -1;
  out[i + seg_offset(seg, nseg, s)] = (p >= 0) ? X[(long long)p * ps + q] : 0.0;
}
__global__ void k_scatter_slots(double* pub, const int* slots, long long n, int npub, const double* rows, int ps,
                                const int* seg, int nseg, double* ext) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) {
    const long long k = i - n * ps;
    if (k < nseg) ext[k] = rows[(long long)seg[k + 1] * ps + k];
    return;
  }
  const int q = (int)(i - s * ps);
  const int sl = slots[s];
  if (sl >= 0 && sl < npub) pub[(long long)sl * ps + q] = rows[i + seg_offset(seg, nseg, s)];
}

// The native exchange's gather / scatter (enqueue_exchange): the segment of
// every row is precomputed (rseg[s], set_exchange), so a thread reads one int
// instead of walking the segment table; status words as above.
__global__ void k_xgather(const double* X, const int* pub_src, const int* slots, const int* rseg, long long n,
                          double* out, int ps, const int* seg, int nseg, const double* relc, int L) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) {
    const long long k = i - n * ps;
    if (k >= nseg) return;
    double m = 0.0;
    for (int l = 0; l < L; ++l) m = (relc[l] > m || relc[l] != relc[l]) ? relc[l] : m;
    out[(long long)seg[k + 1] * ps + k] = m;
    return;
  }
  const int q = (int)(i - s * ps);
  const int p = pub_src[slots[s]];
  out[i + rseg[s]] = (p >= 0) ? X[(long long)p * ps + q] : 0.0;
}
__global__ void k_xscatter(double* pub, const int* slots, const int* rseg, long long n, const double* rows, int ps,
                           const int* seg, int nseg, double* ext) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= n) {
    const long long k = i - n * ps;
    if (k < nseg) ext[k] = rows[(long long)seg[k + 1] * ps + k];
    return;
  }
  const int q = (int)(i - s * ps);
  pub[(long long)slots[s] * ps + q] = rows[i + rseg[s]];
}

__global__ void k_pack(const double* X, double* out, const int* src, int first, int count, int ps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long s = i / ps;
  if (s >= count) return;
  const int q = (int)(i - s * ps);
  out[s * ps + q] = X[(long long)src[first + s] * ps + q];
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
    for (int q = 0; q < 3; ++q)
      u[q] = (M[q * 3 + 0] * V[0 * 3 + k] + M[q * 3 + 1] * V[1 * 3 + k] + M[q * 3 + 2] * V[2 * 3 + k]) / sig;
    const double s = (k == kmin && det < 0.0) ? -1.0 : 1.0;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) Rr[a * 3 + b] += s * u[a] * V[b * 3 + k];
  }
  double* o = out + (size_t)i * 12;
  for (int q = 0; q < 9; ++q) o[q] = Rr[q];
  o[9] = tv[0]; o[10] = tv[1]; o[11] = tv[2];
}

// Nesterov acceleration (oracle orc_pgo_accel_pre / _post; RBCD++):
//   mode 0: Y = Proj((1 - c) X + c V) -> Yb, X and the owned public rows
//   mode 1: V = Proj(V + c (X - Yb))
//   mode 2: V = X (restart)
// Proj: polar factor of the pose's r x 3 rotation block, M (M^T M)^(-1/2) from
// the group's 3 x 3 Gram matrix (gsum in row order) and jacobi3; translation
// unchanged. One lane per (pose, row), as k_retract.
template <int R>
__global__ __launch_bounds__(BLOCK) void k_accel(Dev d, double* V, double* Yb, double c, int mode) {
  const Lane L = lane_map<R>(d);
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double x[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0}, y[4] = {0, 0, 0, 0};
  if (L.valid) {
    load4(d.X + o, x);
    if (mode != 2) load4(V + o, v);
    if (mode == 1) load4(Yb + o, y);
  }
  if (mode == 2) {
    if (L.valid) store4(V + o, x);
    return;
  }
  double m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = (mode == 0) ? (1.0 - c) * x[k] + c * v[k] : v[k] + c * (x[k] - y[k]);
  double G[9], W[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) {
      const double g = gsum<R>(m[i] * m[j], L.base);
      G[i * 3 + j] = g;
      G[j * 3 + i] = g;
    }
  jacobi3(G, W);
  double isq[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) isq[k] = 1.0 / sqrt(G[k * 4]);
  double cc[3], out[4];
#pragma unroll
  for (int k = 0; k < 3; ++k) cc[k] = (m[0] * W[0 * 3 + k] + m[1] * W[1 * 3 + k] + m[2] * W[2 * 3 + k]) * isq[k];
#pragma unroll
  for (int j = 0; j < 3; ++j) out[j] = cc[0] * W[j * 3 + 0] + cc[1] * W[j * 3 + 1] + cc[2] * W[j * 3 + 2];
  out[3] = m[3];
  if (!L.valid) return;
  if (mode == 0) {
    store4(Yb + o, out);
    store4(d.X + o, out);
    const int s = d.pose_slot[L.pose];
    if (s >= 0) store4(d.pub + (size_t)s * 4 * R + 4 * L.a, out);
  } else {
    store4(V + o, out);
  }
}

// Primitive evaluation for parity tests (tiles of one robot), through the same
// gathers as the round kernels.
template <int R>
struct SmemE {
  static constexpr int g = SmemHG<R>::red_off > SmemH<R>::red_off ? SmemHG<R>::red_off : SmemH<R>::red_off;
  static constexpr int red_off = g;
  static constexpr int bytes = red_off + RED_BYTES;
};
template <int R, int RW>
__global__ __launch_bounds__(BLOCK, LB<R>::w) void k_eval(Dev d, int robot, int mode, const double* V, double* out) {
  KMX_SMEM;
  const Lane L = lane_map<R>(d);
  if (L.l != robot) return;
  const size_t o = (size_t)L.pose * 4 * R + 4 * L.a;
  double res[4] = {0, 0, 0, 0}, cost = 0.0, v[4] = {0, 0, 0, 0};
  double* scr = reinterpret_cast<double*>(smem);
  if (mode == KMX_EVAL_COST_EGRAD) {
    hinc_grad<R, RW>(d, L, V, d.pub, res, &cost, smem);
  } else if (mode == KMX_EVAL_EHESS) {
    hinc_gather<R, RW>(d, L, V, res, smem);
    if (L.valid) load4(V + o, v);
  } else {
    double y[4] = {0, 0, 0, 0}, G[4], c0 = 0.0;
    hinc_grad<R, RW>(d, L, d.X, d.pub, G, &c0, smem);
    if (L.valid) {
      load4(d.X + o, y);
      load4(V + o, v);
    }
    double S[9];
    group_symYtG<R, true>(y, G, L.base, S, scr);
    if (mode == KMX_EVAL_RGRAD) {
      for (int c = 0; c < 3; ++c) res[c] = G[c] - (y[0] * S[0 * 3 + c] + y[1] * S[1 * 3 + c] + y[2] * S[2 * 3 + c]);
      res[3] = G[3];
      for (int k = 0; k < 4; ++k) v[k] = res[k];
    } else if (mode == KMX_EVAL_RHESS) {
      __syncthreads();  // the scratch reads are done before the next gather reuses the LDS
      double H[4];
      hinc_gather<R, RW>(d, L, V, H, smem);
      group_rhess<R, true>(y, v, H, S, L.base, res, scr);
    } else if (mode == KMX_EVAL_PRECON) {
      group_precon<R, true>(d, L.pose, L.valid, y, v, L.base, res, scr);
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
  const double t = block_sum(s, reinterpret_cast<double*>(smem + SmemE<R>::red_off));
  if (threadIdx.x == 0) d.part[(size_t)L.tile * NPART] = t;
}

}  // namespace

// ============================================================ handle =====
struct kmx_pgo {
  kmx_pgo_params P{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
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
  int ninc = 0;
  int rw = 10;  // record width in doubles (10 compact quaternion / 16 full)
  int64_t nshared = 0;
  int n_sh_local = 0, n_gnc = 0, n_osh = 0;
  std::vector<long long> m_robot;
  int ntiles = 0;
  std::vector<int> rt0_h;  // [L + 1] first tile of each local robot
  // GNC schedule (host copy of the parameters)
  int gnc_on = 0, gnc_inner_iters = 20, gnc_max_updates = 0x7fffffff, n_ext = 0;
  double gnc_rel_tol = 1e-3;
  // device
  Dev dv{};
  TileDesc* d_tile = nullptr;
  int* d_rtile0 = nullptr;
  int* d_inc_ptr = nullptr;
  double* d_rec = nullptr;
  int* d_rec_o = nullptr;
  double *d_ekappa = nullptr, *d_etau = nullptr, *d_ew = nullptr;
  int2* d_eipos = nullptr;
  double* d_vec = nullptr;  // X Xt g r z hd eta, then the dhn tCG directions (nvec())
  double* d_coefh = nullptr;  // [L][tcg_max]
  double* d_part_f = nullptr;  // [ntiles][8] one-sync tCG partials (P.tcg_form)
  int ctl_par = 0;             // one-sync tCG: the state after the last tCG loop is in ctl2 (odd step count)
  bool tcg_stopped = false;    // consumer tCG loop saw every robot stop (each was retracted by its k_update)
  double *d_S = nullptr, *d_Pinv = nullptr, *d_hD = nullptr, *d_hDS = nullptr, *d_pub = nullptr, *d_part = nullptr;
  Ctl* d_ctl = nullptr;
  Ctl* d_ctl2 = nullptr;
  double *d_part_h = nullptr, *d_part_u = nullptr;
  Counters* d_cnt = nullptr;
  long long* d_m_robot = nullptr;
  int* d_n_robot = nullptr;
  int* d_pub_src = nullptr;    // slot -> local pose (-1 if not local)
  int* d_own_src = nullptr;    // owned slot k -> local pose (index first_owned + k)
  int* d_pose_slot = nullptr;  // local pose -> owned slot or -1
  int* d_gnc_edge = nullptr;
  int2* d_gnc_ends = nullptr;
  int *d_sh_edge = nullptr, *d_sh_idx = nullptr;
  int *d_osh_edge = nullptr, *d_osh_idx = nullptr;
  double* d_relc = nullptr;
  Gnc* d_gnc = nullptr;  // [2]: state, next
  double* d_ext = nullptr;
  int ext_cap = 0;
  unsigned char* d_active = nullptr;
  double* d_scratch = nullptr;  // eval / trajectory in-out, allocated on first use
  size_t scratch_cap = 0;
  // tCG progress polling (see HostStatus)
  HostStatus* hstat = nullptr;
  int hstat_cap = 0;
  unsigned long long seq = 0;
  bool poll = true;          // kmx_pgo_set_tcg_poll(0): enqueue every tCG step (finished robots exit at once)
  // kmx_pgo_set_tcg_poll(-1) (the default): adaptive. A polled tCG loop
  // that ran to within BLIND_SLACK steps of the cap sends the next
  // BLIND_WINDOW loops blind (no host wait: at most BLIND_SLACK empty step
  // pairs of ~1.5 us each, against the host round trip of every polled step
  // and the host seam of a multi-rank round); then one polled loop measures
  // again. Measured on configs[3] (scripts/host_seam.py, round_sizes.py):
  // blind wins at 100k poses (728 vs 740 us), on the N = 4 / 8 rank handles
  // (274 vs 284, 197 vs 217 us), loses on a 12.5k block needing ~5 steps
  // (163 vs 150 us), where the adaptive rule keeps polling.
  bool poll_auto = true;
  // native exchange (kmx_pgo_comm_init + kmx_pgo_set_exchange): every round
  // of iterate / iterate_async starts with gather -> RCCL send/recv with each
  // peer -> scatter, all on the handle's stream (no cross-stream event, no
  // host round trip between the exchange and the round)
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  bool xchg = false, xchg_self_p2p = false;
  // KMX_XCHG_LAG=1 (a measurement mode, off by default):
  // the exchange of the rows published after round i-1 runs on xstream while
  // round i computes, and round i+1 installs them — a one-round-stale public
  // table (round k >= 2 reads the peers' rows of X^(k-2)). It changes the
  // iterate sequence and lets the ranks' GNC decisions drift apart (a peer's
  // status word is a round older too), so it is a timing instrument only.
  int xchg_lag = 0;
  bool x_inflight = false;
  hipStream_t xstream = nullptr;
  hipEvent_t ev_xg = nullptr, ev_xd = nullptr;
  int *d_xs_slots = nullptr, *d_xr_slots = nullptr, *d_xs_seg = nullptr, *d_xr_seg = nullptr;
  int *d_xs_rseg = nullptr, *d_xr_rseg = nullptr;  // segment index of every row
  double *d_xsbuf = nullptr, *d_xrbuf = nullptr;
  long long xn_send = 0, xn_recv = 0;
  std::vector<long long> xs_cnt, xr_cnt, xs_off, xr_off;  // per peer, in doubles (rows * 4r + 1 status)
  int blind_left = 0;
  static constexpr int BLIND_SLACK = 2, BLIND_WINDOW = 8;
  // Gated k_hess launches (KMX_HESS_GATE=0: off): every k_hess launch after a
  // tCG's first tests its robot's phase before its first record chunk is
  // fetched. Ungated, a launch enqueued before the host knows whether any robot
  // is still in tCG fetched that chunk before the test (the records' round
  // trip overlapping the state's), so a launch every robot skips still read
  // ~42 MB at configs[3]. Measured (profiles/r06/hess_gate/, two runs each):
  // gating every launch after the first 0.685 / 0.683 ms per round, ungated
  // 0.692 / 0.691, gating only the steps at or past where the last polled loop
  // stopped 0.691 / 0.691 — the state's round trip costs a gated launch less
  // than a skipped launch's record fetch costs the round.
  bool hess_gate = true;
  // (measured and removed: a hipStreamQuery before the status spin put a ~5 us
  // bubble before the next tCG step's first kernel, profiles/r02/ab_query)
  // reduction mode: set per graph (below) unless KMX_RED forces one (0 launch,
  // 2 consumer). Measured at the end of round 2
  // (profiles/r02/small_round/16_*): the consumer form (no reduction launch,
  // the stop decision before the gather) wins per round at 25k poses (244 vs
  // 280 us), 37.5k (318 vs 357), 62.5k (530 vs 543) and 75k (583 vs 591), ties
  // at 50k and 87.5k, and loses at 100k (773 vs 731-738: two and a bit
  // generations of workgroups, each waiting for its robot's sums)
  int rm = RM_LAUNCH;
  int rm_forced = -1;
  int early_stop = 1;
  static constexpr int RM_CONSUMER_MAX_POSES = 80000;
  bool poll_timeout = false;
  // timing
  bool timing = false;
  int* d_hv_launch = nullptr;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  // Nesterov acceleration (P.acceleration): momentum V and this round's Y
  // (allocated only when enabled), gamma and the restart counter on the host
  double *d_accV = nullptr, *d_accY = nullptr;
  double acc_gamma = 0.0;
  int acc_k = 0;
  bool acc_ready = false, acc_started = false;
};

namespace {

// Unit quaternion (w, x, y, z) of a rotation matrix (row-major), by the
// largest of the four diagonal combinations (Shepperd), and back.
void rot_to_quat(const double* R, double* q) {
  const double tr = R[0] + R[4] + R[8];
  double w, x, y, z;
  if (tr > 0.0) {
    const double s = 2.0 * std::sqrt(tr + 1.0);
    w = 0.25 * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const double s = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
    w = (R[7] - R[5]) / s; x = 0.25 * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    const double s = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
    w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25 * s; z = (R[5] + R[7]) / s;
  } else {
    const double s = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
    w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25 * s;
  }
  const double n = std::sqrt(w * w + x * x + y * y + z * z);
  q[0] = w / n; q[1] = x / n; q[2] = y / n; q[3] = z / n;
}
// Rec<10>'s three stored components: all but the largest (made >= 0 by
// negating the quaternion, which leaves R unchanged), whose index goes to
// rec_o's bits 29-31; and the device's rebuild of the fourth (Rec<10>::load).
int quat_pack(const double* q, double* q3) {
  int big = 0;
  for (int i = 1; i < 4; ++i)
    if (std::fabs(q[i]) > std::fabs(q[big])) big = i;
  const double sg = q[big] < 0.0 ? -1.0 : 1.0;
  for (int i = 0, j = 0; i < 4; ++i)
    if (i != big) q3[j++] = sg * q[i];
  return big;
}
void quat_unpack(const double* q3, int big, double* q) {
  const double ql = std::sqrt(1.0 - (q3[0] * q3[0] + q3[1] * q3[1] + q3[2] * q3[2]));
  for (int i = 0, j = 0; i < 4; ++i) q[i] = i == big ? ql : q3[j++];
}
// the device's Rec<10>::edge expressions
void quat_to_rot(const double* q, double* R) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
  const double wx = w * x, wy = w * y, wz = w * z;
  R[0] = 1.0 - 2.0 * (yy + zz); R[1] = 2.0 * (xy - wz); R[2] = 2.0 * (xz + wy);
  R[3] = 2.0 * (xy + wz); R[4] = 1.0 - 2.0 * (xx + zz); R[5] = 2.0 * (yz - wx);
  R[6] = 2.0 * (xz - wy); R[7] = 2.0 * (yz + wx); R[8] = 1.0 - 2.0 * (xx + yy);
}

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * count);
  if (e != hipSuccess) return kmx::fail(KMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return 0;
}

void free_xchg(kmx_pgo* h) {
  if (h->xstream) (void)hipStreamSynchronize(h->xstream);
  h->x_inflight = false;
  void* ptrs[] = {h->d_xs_slots, h->d_xr_slots, h->d_xs_seg, h->d_xr_seg, h->d_xs_rseg, h->d_xr_rseg,
                  h->d_xsbuf, h->d_xrbuf};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  h->d_xs_slots = h->d_xr_slots = h->d_xs_seg = h->d_xr_seg = h->d_xs_rseg = h->d_xr_rseg = nullptr;
  h->d_xsbuf = h->d_xrbuf = nullptr;
  h->xchg = false;
}

void free_dev(kmx_pgo* h) {
  void* ptrs[] = {h->d_tile, h->d_rtile0, h->d_inc_ptr, h->d_rec, h->d_rec_o, h->d_ekappa,
                  h->d_etau, h->d_ew, h->d_eipos, h->d_vec, h->d_S, h->d_Pinv, h->d_hD, h->d_hDS, h->d_pub, h->d_part,
                  h->d_ctl, h->d_cnt, h->d_m_robot, h->d_n_robot, h->d_pub_src, h->d_own_src,
                  h->d_pose_slot, h->d_gnc_edge, h->d_gnc_ends, h->d_sh_edge, h->d_sh_idx, h->d_osh_edge,
                  h->d_osh_idx, h->d_relc, h->d_gnc, h->d_ext, h->d_active, h->d_scratch, h->d_hv_launch,
                  h->d_accV, h->d_accY, h->d_ctl2, h->d_part_h,
                  h->d_part_u, h->d_coefh, h->d_part_f};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  h->d_tile = nullptr;
  h->d_rtile0 = h->d_inc_ptr = nullptr;
  h->d_rec = h->d_ekappa = h->d_etau = h->d_ew = nullptr;
  h->d_rec_o = nullptr;
  h->d_eipos = nullptr;
  h->d_vec = h->d_S = h->d_Pinv = h->d_hD = h->d_hDS = h->d_pub = h->d_part = nullptr;
  h->d_ctl = nullptr;
  h->d_cnt = nullptr;
  h->d_m_robot = nullptr;
  h->d_n_robot = h->d_pub_src = h->d_own_src = h->d_pose_slot = h->d_gnc_edge = nullptr;
  h->d_gnc_ends = nullptr;
  h->d_sh_edge = h->d_sh_idx = h->d_osh_edge = h->d_osh_idx = nullptr;
  h->d_relc = nullptr;
  h->d_gnc = nullptr;
  h->d_ext = nullptr;
  h->ext_cap = 0;
  h->d_active = nullptr;
  h->d_scratch = nullptr;
  h->scratch_cap = 0;
  h->d_hv_launch = nullptr;
  h->d_accV = h->d_accY = nullptr;
  h->d_ctl2 = nullptr;
  h->d_coefh = nullptr;
  h->d_part_h = h->d_part_u = nullptr;
  h->d_part_f = nullptr;
}

hipEvent_t next_event(kmx_pgo* h) {
  if (h->ev_used == h->ev_pool.size()) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    h->ev_pool.push_back(e);
  }
  return h->ev_pool[h->ev_used++];
}

bool ready(kmx_pgo* h) { return h && h->d_vec != nullptr; }

// Vectors of d_vec: X Xt g r z hd eta + the tCG directions kept for k_retract
// (+ Hz, w_0, w_1 for the one-sync tCG, which needs two directions).
bool onesync(const kmx_pgo* h) {
  return h->P.tcg_form == KMX_TCG_FORM_ONESYNC && h->P.method == KMX_METHOD_RTR;
}
int dh_count(const kmx_pgo* h) {
  return std::max(onesync(h) ? 2 : 1, std::min(h->P.tcg_max_iterations, DHMAX));
}
size_t nvec(const kmx_pgo* h) { return 7 + (size_t)dh_count(h) + (onesync(h) ? 3 : 0); }

// Scratch of the diagnostic / output entry points (not resident with the graph).
int ensure_scratch(kmx_pgo* h, size_t doubles) {
  if (doubles <= h->scratch_cap) return 0;
  if (h->d_scratch) {
    KMX_HIP(hipStreamSynchronize(h->stream));
    (void)hipFree(h->d_scratch);
  }
  h->d_scratch = nullptr;
  h->scratch_cap = 0;
  if (int rc = dalloc(&h->d_scratch, doubles)) return rc;
  h->scratch_cap = doubles;
  return 0;
}

void sync_params(kmx_pgo* h) {
  Params& p = h->dv.p;
  p.tcg_max = h->P.tcg_max_iterations;
  p.rtr_iters = h->P.rtr_iterations;
  p.use_precond = h->P.use_preconditioner;
  p.robust = h->P.robust_cost == KMX_COST_GNC_TLS ? 1 : 0;
  p.kappa = h->P.tcg_kappa;
  p.theta = h->P.tcg_theta;
  p.Delta0 = h->P.rtr_initial_radius;
  p.Delta_max = h->P.rtr_max_radius;
  p.accept_rho = h->P.rtr_accept_rho;
  p.gn_tol = h->P.gradnorm_tol;
  p.shift = h->P.precond_shift;
  p.barc = h->P.gnc_barc;
  p.mu_step = h->P.gnc_mu_step;
  p.rel_tol = h->gnc_rel_tol;
  p.gnc_on = h->gnc_on;
  p.inner_iters = h->gnc_inner_iters;
  p.max_updates = h->gnc_max_updates;
  p.n_ext = h->n_ext;
  p.rgd = h->P.method == KMX_METHOD_RGD ? 1 : 0;
  p.rgd_step = h->P.rgd_stepsize;
  p.early_stop = h->early_stop;
  h->dv.ext = h->d_ext;
}

// Owned public rows into the table (the single-device exchange).
void enqueue_publish(kmx_pgo* h) {
  const int ps = 4 * h->P.r;
  const long long tot = h->n_owned * ps;
  if (tot == 0) return;
  hipLaunchKernelGGL(k_publish, dim3((unsigned)((tot / 2 + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                     h->d_pub + (size_t)h->first_owned * ps, h->d_pub_src + h->first_owned, (int)h->n_owned, ps);
}

template <int RW>
void enqueue_precond_t(kmx_pgo* h, int gated) {
  const int blocks = std::max(1, std::min(gated ? 256 : 1024, (h->nloc + 127) / 128));
  hipLaunchKernelGGL(k_precond<RW>, dim3(blocks), dim3(128), 0, h->stream, h->dv, gated);
}
void enqueue_precond(kmx_pgo* h, int gated) {
  if (h->rw == 10) enqueue_precond_t<10>(h, gated);
  else enqueue_precond_t<16>(h, gated);
}

// Round begin (mode BEGIN_ROUND) and/or GNC update, then the gated
// preconditioner rebuild that commits the GNC state.
// Returns whether the gated preconditioner rebuild is left to the next k_grad
// (defer: the round's first gradient follows this launch directly).
bool enqueue_begin(kmx_pgo* h, const unsigned char* d_active, int mode, bool defer = false) {
  const bool may_fire = h->P.robust_cost == KMX_COST_GNC_TLS && (h->gnc_on || (mode & BEGIN_FORCE_GNC));
  if (!may_fire) mode |= BEGIN_SOLO;  // no weight update possible: one block, no preconditioner rebuild
  // a capped grid: when the schedule does not fire, the launch costs its dispatch
  const unsigned grid = may_fire ? 1 + (unsigned)std::min(256, std::max(1, (h->n_gnc + 255) / 256)) : 1;
  if (h->rw == 10)
    hipLaunchKernelGGL(k_begin<10>, dim3(grid), dim3(256), 0, h->stream, h->dv, d_active, mode, h->P.r);
  else
    hipLaunchKernelGGL(k_begin<16>, dim3(grid), dim3(256), 0, h->stream, h->dv, d_active, mode, h->P.r);
  if (may_fire && !defer) enqueue_precond(h, 1);
  return may_fire && defer;
}

// Wait until every robot with tiles reported tCG step `seq`; returns whether
// any robot is still in tCG. A device that stops reporting for 30 s switches
// the handle to blind enqueueing (every tCG step launched).
bool wait_running(kmx_pgo* h, unsigned long long seq) {
  volatile HostStatus* hs = h->hstat;
  const auto t0 = std::chrono::steady_clock::now();
  bool running = false;
  for (int l = 0; l < h->dv.L; ++l) {
    if (h->rt0_h[l + 1] == h->rt0_h[l]) continue;  // no tiles: never in tCG
    unsigned long long w;
    while (((w = __atomic_load_n(&hs[l].word, __ATOMIC_ACQUIRE)) >> 1) < seq) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
        h->poll_timeout = true;
        h->poll = false;
        return true;
      }
    }
    running |= (w & 1ull) != 0;
  }
  return running;
}

template <int R, int RM>
void red_t(kmx_pgo* h, int kind, HostStatus* hs = nullptr, unsigned long long seq = 0, int slot = -1,
           const double* src = nullptr) {
  hipLaunchKernelGGL(k_reduce, dim3(h->dv.L), dim3(RBLOCK), 0, h->stream, h->dv, kind, R, hs, seq, slot, src);
}

// The parts of a round: gradient, tCG (host-polled steps), trial point and
// cost; round begin before and commit after. Replaying the launches between
// two tCG loops from a hipGraph was measured on one 12.5k-pose block (170.1
// vs 167.7 us per round eager: the graph launch moves the host latency to the
// first tCG step after it; profiles/r02/small_round/2_*) and not kept.
// RM_CONSUMER folds the round's other reductions into the kernel after them
// (no k_reduce launch in a round): the gradient's into the first k_hess, the
// last tCG update's into k_retract, the trial cost's into k_commit (one RTR
// iteration). RGD keeps the gradient's launch (no k_hess follows).
template <int RM>
bool fold_grad(const kmx_pgo* h) {
  return RM == RM_CONSUMER && h->P.method != KMX_METHOD_RGD && h->P.tcg_max_iterations > 0;
}
template <int RM>
bool fold_cost(const kmx_pgo* h) {
  return RM == RM_CONSUMER && (h->P.rtr_iterations == 1 || h->P.method == KMX_METHOD_RGD);
}

template <int R, int RW, int RM>
void enqueue_grad_t(kmx_pgo* h, int gated = 0) {
  hipLaunchKernelGGL((k_grad<R, RW, RM>), dim3(h->ntiles), dim3(BLOCK), SmemHG<R>::bytes, h->stream, h->dv, gated);
  if (!fold_grad<RM>(h)) red_t<R, RM>(h, RED_GRAD);
}

template <int R, int RW, int RM>
void enqueue_tcg_t(kmx_pgo* h) {
  const dim3 grid(h->ntiles), blk(BLOCK);
  // tCG: each step is (k_hess, k_update); with polling, exactly one step
  // stays queued beyond the last one known to be needed
  unsigned long long prev = 0;
  // this loop polled or blind (see kmx_pgo::poll_auto)
  bool poll = h->poll && h->hstat;
  if (poll && h->poll_auto && h->blind_left > 0) {
    --h->blind_left;
    poll = false;
  }
  const int tmax = h->P.tcg_max_iterations;
  int steps = tmax;  // steps enqueued by a polled loop
  h->tcg_stopped = false;
  if constexpr (RM == RM_CONSUMER) {
    if (onesync(h)) {
      // one k_step per step: launch j applies step j-1's decision (which it
      // reports at its start) and runs Hess-vec j; launch tmax only decides.
      // A polled loop waits for launch j's report while launch j still
      // gathers, so the next launch is queued before the GPU runs dry.
      int J = tmax + 1;
      for (int j = 0; j <= tmax; ++j) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        int slot = -1;
        if (h->timing && h->ev_used / 2 < (size_t)HV_SLOTS) {
          slot = (int)(h->ev_used / 2);
          e0 = next_event(h);
          e1 = next_event(h);
        }
        poll = poll && h->poll;
        const unsigned long long seq = poll ? ++h->seq : 0;
        HostStatus* hs = poll ? h->hstat : nullptr;
        const Ctl* cin = (j & 1) ? h->d_ctl2 : h->d_ctl;
        Ctl* cout = (j & 1) ? h->d_ctl : h->d_ctl2;
        if (slot >= 0)  // the events take the dispatch's own start / end timestamps
          hipExtLaunchKernelGGL((k_step<R, RW>), grid, blk, SmemF<R>::bytes, h->stream, e0, e1, 0u, h->dv, cin,
                                cout, j, slot, hs, seq);
        else
          hipLaunchKernelGGL((k_step<R, RW>), grid, blk, SmemF<R>::bytes, h->stream, h->dv, cin, cout, j,
                             slot, hs, seq);
        if (poll && j > 0 && !wait_running(h, seq)) {
          J = j + 1;
          break;
        }
      }
      h->ctl_par = J & 1;
      steps = J - 1;
      if (poll && h->poll_auto && steps + kmx_pgo::BLIND_SLACK >= tmax) h->blind_left = kmx_pgo::BLIND_WINDOW;
      return;
    }
  }
  for (int j = 0; j < tmax; ++j) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int slot = -1;
    if (h->timing && h->ev_used / 2 < (size_t)HV_SLOTS) {
      slot = (int)(h->ev_used / 2);
      e0 = next_event(h);
      e1 = next_event(h);
    }
    poll = poll && h->poll;  // a poll timeout inside wait_running switches to blind
    const unsigned long long seq = poll ? ++h->seq : 0;
    HostStatus* hs = poll ? h->hstat : nullptr;
    const bool gate = j > 0 && h->hess_gate;
    const int fl = (j == 0 ? 1 : 0) | (gate ? 2 : 0);
    if constexpr (RM == RM_CONSUMER) {
      // k_hess reports the stop test of the previous step's update
      if (slot >= 0)  // the events take the dispatch's own start / end timestamps
        hipExtLaunchKernelGGL((k_hess<R, RW, RM>), grid, blk, SmemH<R>::bytes, h->stream, e0, e1, 0u, h->dv,
                              fl, slot, hs, seq);
      else
        hipLaunchKernelGGL((k_hess<R, RW, RM>), grid, blk, SmemH<R>::bytes, h->stream, h->dv, fl, slot,
                           hs, seq);
      hipLaunchKernelGGL((k_update<R, RM>), grid, blk, SmemU::bytes, h->stream, h->dv, nullptr, 0ull, slot);
      if (poll && j > 0 && !wait_running(h, seq)) {
        steps = j + 1;
        h->tcg_stopped = true;
        break;
      }
      continue;
    }
    if (slot >= 0)
      hipExtLaunchKernelGGL((k_hess<R, RW, RM>), grid, blk, SmemH<R>::bytes, h->stream, e0, e1, 0u, h->dv, fl, slot,
                            (HostStatus*)nullptr, 0ull);
    else
      hipLaunchKernelGGL((k_hess<R, RW, RM>), grid, blk, SmemH<R>::bytes, h->stream, h->dv, fl, slot, nullptr, 0ull);
    red_t<R, RM>(h, RED_HESS, nullptr, 0, slot);
    hipLaunchKernelGGL((k_update<R, RM>), grid, blk, SmemU::bytes, h->stream, h->dv, nullptr, seq, -1);
    red_t<R, RM>(h, RED_UPDATE, hs, seq, -1, nullptr);
    if (poll) {
      if (j > 0 && !wait_running(h, prev)) {
        steps = j + 1;
        break;
      }
      prev = seq;
    }
  }
  if (poll && h->poll_auto && steps + kmx_pgo::BLIND_SLACK >= tmax) h->blind_left = kmx_pgo::BLIND_WINDOW;
}

// after the tCG loop (or the RGD step): trial point and its cost
template <int R, int RW, int RM>
void enqueue_trial_t(kmx_pgo* h, bool rgd) {
  const dim3 grid(h->ntiles), blk(BLOCK);
  // RM_CONSUMER: the last step's update has no k_hess after it; k_retract
  // reduces it
  // one-sync form: each k_step that ended a robot's tCG also formed its trial
  // point, so there is no k_retract; k_cost takes the state from where the
  // tCG left it
  const bool os = RM == RM_CONSUMER && !rgd && onesync(h);
  const Ctl* src = os && h->ctl_par ? h->d_ctl2 : h->d_ctl;
  // consumer form: the k_update after the k_hess that stopped a robot formed
  // its trial point; k_retract (fold 2) decides and retracts the robots still
  // in tCG at the cap, and is not needed when the polled loop saw every robot
  // stop
  const bool cons = RM == RM_CONSUMER && !rgd;
  if (!os && !(cons && h->tcg_stopped))
    hipLaunchKernelGGL((k_retract<R>), grid, blk, SmemU::bytes, h->stream, h->dv, cons ? 2 : 0, (const Ctl*)h->d_ctl);
  hipLaunchKernelGGL((k_cost<R, RW, RM>), grid, blk, SmemC<R>::bytes, h->stream, h->dv, src);
  if (!fold_cost<RM>(h)) red_t<R, RM>(h, RED_COST);
}

template <int R, int RW, int RM>
void enqueue_round_t(kmx_pgo* h, const unsigned char* d_active) {
  // no tiles: nothing would run the deferred rebuild
  const bool pend = enqueue_begin(h, d_active, BEGIN_ROUND, h->ntiles > 0);
  const bool rgd = h->P.method == KMX_METHOD_RGD;
  const int iters = rgd ? 1 : h->P.rtr_iterations;
  for (int it = 0; it < iters; ++it) {
    enqueue_grad_t<R, RW, RM>(h, it == 0 && pend ? 1 : 0);
    if (!rgd) enqueue_tcg_t<R, RW, RM>(h);
    enqueue_trial_t<R, RW, RM>(h, rgd);
    if (it + 1 < iters)  // the next RTR iteration starts from the accepted point
      hipLaunchKernelGGL((k_commit<R>), dim3(h->ntiles), dim3(BLOCK), 0, h->stream, h->dv, 0, 0);
  }
  hipLaunchKernelGGL((k_commit<R>), dim3(h->ntiles), dim3(BLOCK), 0, h->stream, h->dv, fold_cost<RM>(h) ? 1 : 0, 1);
}

template <int R>
void enqueue_round_r(kmx_pgo* h, const unsigned char* d_active) {
  if (h->rm == RM_CONSUMER) {
    if (h->rw == 10) enqueue_round_t<R, 10, RM_CONSUMER>(h, d_active);
    else enqueue_round_t<R, 16, RM_CONSUMER>(h, d_active);
  } else {
    if (h->rw == 10) enqueue_round_t<R, 10, RM_LAUNCH>(h, d_active);
    else enqueue_round_t<R, 16, RM_LAUNCH>(h, d_active);
  }
}

// One RBCD round for the robots whose d_active flag is set; it starts with
// the scheduled GNC decision when the handle's schedule is enabled.
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

// Acceleration (oracle orc_pgo_accel_pre / _post): gamma' = (1 + sqrt(1 +
// 4 N^2 gamma^2)) / (2 N), alpha = 1 / (gamma' N), N = team size.
double accel_gamma_next(const kmx_pgo* h) {
  const double N = (double)h->n_robots;
  return (1.0 + std::sqrt(1.0 + 4.0 * N * N * h->acc_gamma * h->acc_gamma)) / (2.0 * N);
}
void launch_accel(kmx_pgo* h, double c, int mode) {
  const dim3 grid(h->ntiles), blk(BLOCK);
  switch (h->P.r) {
#define KMX_ACC(RR) \
  case RR: hipLaunchKernelGGL(k_accel<RR>, grid, blk, 0, h->stream, h->dv, h->d_accV, h->d_accY, c, mode); break;
    KMX_ACC(3) KMX_ACC(4) KMX_ACC(5) KMX_ACC(6) KMX_ACC(7)
    default: hipLaunchKernelGGL(k_accel<8>, grid, blk, 0, h->stream, h->dv, h->d_accV, h->d_accY, c, mode); break;
#undef KMX_ACC
  }
}
// Y for the upcoming round (X := Y, owned public rows := Y); once per round.
void enqueue_accel_pre(kmx_pgo* h) {
  if (!h->P.acceleration || h->acc_ready || h->ntiles == 0) return;
  if (!h->acc_started) {
    launch_accel(h, 0.0, 2);  // V = X
    h->acc_started = true;
  }
  const double g = accel_gamma_next(h);
  launch_accel(h, 1.0 / (g * (double)h->n_robots), 0);
  h->acc_ready = true;
}
void enqueue_accel_post(kmx_pgo* h) {
  if (!h->P.acceleration || !h->acc_ready || h->ntiles == 0) return;
  const double g = accel_gamma_next(h);
  const bool restart = h->P.restart_interval > 0 && (h->acc_k + 1) % h->P.restart_interval == 0;
  launch_accel(h, g, restart ? 2 : 1);
  h->acc_gamma = restart ? 0.0 : g;
  h->acc_k = restart ? 0 : h->acc_k + 1;
  h->acc_ready = false;
}
void accel_reset(kmx_pgo* h) {
  h->acc_gamma = 0.0;
  h->acc_k = 0;
  h->acc_ready = h->acc_started = false;
}

template <int RW>
void enqueue_apply_weights_t(kmx_pgo* h) {
  if (h->mloc > 0)
    hipLaunchKernelGGL(k_apply_weights<RW>, dim3((h->mloc + 255) / 256), dim3(256), 0, h->stream, h->dv, h->mloc);
}
void enqueue_apply_weights(kmx_pgo* h) {
  if (h->rw == 10) enqueue_apply_weights_t<10>(h);
  else enqueue_apply_weights_t<16>(h);
  enqueue_precond(h, 0);
}

}  // namespace

// ================================================================ ABI =====
extern "C" int kmx_pgo_create(const kmx_pgo_params* params, int device, kmx_pgo** out) {
  KMX_GUARD_BEGIN
  KMX_CHECK(params && out, KMX_EINVAL, "null argument");
  KMX_CHECK(params->d == 3, KMX_EUNSUP, "only d = 3 is supported");
  KMX_CHECK(params->r >= 3 && params->r <= 8, KMX_EUNSUP, "relaxation rank must be in [3, 8]");
  KMX_CHECK(params->rtr_iterations >= 1 && params->tcg_max_iterations >= 1, KMX_EINVAL,
            "rtr_iterations and tcg_max_iterations must be >= 1");
  KMX_CHECK(params->robust_cost == KMX_COST_L2 || params->robust_cost == KMX_COST_GNC_TLS, KMX_EUNSUP,
            "robust cost must be L2 or GNC_TLS");
  KMX_CHECK((params->acceleration == 0 || params->acceleration == 1) && params->restart_interval >= 0, KMX_EINVAL,
            "acceleration is 0 or 1, restart_interval >= 0");
  KMX_CHECK(params->method == KMX_METHOD_RTR || params->method == KMX_METHOD_RGD, KMX_EUNSUP,
            "method must be KMX_METHOD_RTR or KMX_METHOD_RGD");
  // (tcg_form 2, the resident round of ABI 7, was removed in ABI 8: DESIGN.md section 10)
  KMX_CHECK(params->tcg_form == KMX_TCG_FORM_STANDARD || params->tcg_form == KMX_TCG_FORM_ONESYNC, KMX_EINVAL,
            "tcg_form must be KMX_TCG_FORM_STANDARD or KMX_TCG_FORM_ONESYNC");
  KMX_CHECK(params->method != KMX_METHOD_RGD || params->rgd_stepsize > 0.0, KMX_EINVAL, "rgd_stepsize must be > 0");
  KMX_CHECK(params->tile_incidences >= 0, KMX_EINVAL, "tile_incidences must be >= 0 (0: automatic)");
  int ndev = 0;
  KMX_HIP(hipGetDeviceCount(&ndev));
  KMX_CHECK(device >= 0 && device < ndev, KMX_EINVAL, "bad HIP device ordinal");
  KMX_HIP(hipSetDevice(device));
  kmx_pgo* h = new kmx_pgo();
  h->P = *params;
  h->device = device;
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    return kmx::fail(KMX_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  h->own_stream = true;
  if (const char* v = std::getenv("KMX_RED")) {
    const int m = std::atoi(v);
    h->rm_forced = m == 0 ? RM_LAUNCH : m == 2 ? RM_CONSUMER : -1;  // 1 and 3 (tickets, half) were removed
  }
  if (const char* v = std::getenv("KMX_HESS_GATE")) h->hess_gate = std::atoi(v) != 0;
  *out = h;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_destroy(kmx_pgo* h) {
  if (!h) return KMX_OK;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_dev(h);
  free_xchg(h);
  if (h->comm) (void)ncclCommAbort(h->comm);  // non-blocking communicator: no finalize handshake at teardown
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  if (h->hstat) (void)hipHostFree(h->hstat);
  if (h->xstream) {
    (void)hipStreamDestroy(h->xstream);
    (void)hipEventDestroy(h->ev_xg);
    (void)hipEventDestroy(h->ev_xd);
  }
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

extern "C" int kmx_pgo_set_tcg_poll(kmx_pgo* h, int mode) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_CHECK(mode >= -1 && mode <= 1, KMX_EINVAL, "mode is -1 (adaptive), 0 (blind) or 1 (polled)");
  h->poll = mode != 0;
  h->poll_auto = mode == -1;
  h->blind_left = 0;
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
  free_xchg(h);  // the exchange slot lists index this graph's public table
  accel_reset(h);
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
  h->rm = h->rm_forced >= 0 ? h->rm_forced : (nloc <= kmx_pgo::RM_CONSUMER_MAX_POSES ? RM_CONSUMER : RM_LAUNCH);
  if (onesync(h)) h->rm = RM_CONSUMER;  // its decisions are taken by every workgroup
  h->early_stop = nloc <= kmx_pgo::RM_CONSUMER_MAX_POSES ? 1 : 0;  // decide before the gather on small problems
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
  std::vector<int> pose_slot(std::max(nloc, 1), -1);
  int64_t first = -1, last = -1;
  for (int64_t s = 0; s < h->npub; ++s) {
    const int rb = (int)(keys[s] >> 32), pp = (int)(keys[s] & 0xffffffff);
    if (h->local_of[rb] >= 0) {
      pub_src[s] = h->loff[h->local_of[rb]] + pp;
      pose_slot[pub_src[s]] = (int)s;
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
  std::vector<double> ek_h(std::max(h->mloc, 1), 0.0), et_h(std::max(h->mloc, 1), 0.0);
  std::vector<double> ew_h(std::max(h->mloc, 1), 0.0);
  std::vector<int> deg(nloc + 1, 0);
  h->m_robot.assign(L, 0);
  for (int k = 0; k < h->mloc; ++k) {
    const int64_t e = ledges[k];
    ek_h[k] = kappa[e];
    et_h[k] = tau[e];
    ew_h[k] = weight[e];
    const int a1 = h->local_of[r1[e]], a2 = h->local_of[r2[e]];
    if (a1 >= 0) { deg[lpose(r1[e], p1[e])]++; h->m_robot[a1]++; }
    if (a2 >= 0) { deg[lpose(r2[e], p2[e])]++; if (r2[e] != r1[e]) h->m_robot[a2]++; }
  }
  // record width: compact (quaternion) when every local measurement rotation
  // is rebuilt from its unit quaternion to 1e-12 (a rotation), full otherwise
  // (the three stored components per edge, and the rebuilt one's index)
  std::vector<double> quat((size_t)std::max(h->mloc, 1) * 3);
  std::vector<int> qbig(std::max(h->mloc, 1), 0);
  {
    // (the other endpoint takes rec_o's low 29 bits: local poses and public
    // slots below 2^28, far above any single GPU's share)
    bool ok = nloc < (1 << 28) && h->npub < (1 << 28);
    for (int k = 0; k < h->mloc && ok; ++k) {
      const double* Q = R + 9 * ledges[k];
      double q4[4], qr[4], Rq[9];
      rot_to_quat(Q, q4);
      qbig[k] = quat_pack(q4, &quat[3 * (size_t)k]);
      quat_unpack(&quat[3 * (size_t)k], qbig[k], qr);
      quat_to_rot(qr, Rq);
      for (int i = 0; i < 9 && ok; ++i) ok = std::fabs(Rq[i] - Q[i]) <= 1e-12;
    }
    h->rw = ok ? 10 : 16;
  }
  const int RW = h->rw;
  std::vector<int> inc_ptr(nloc + 1, 0);
  for (int i = 0; i < nloc; ++i) inc_ptr[i + 1] = inc_ptr[i] + deg[i];
  h->ninc = inc_ptr[nloc];
  const int GS = RW == 10 ? 8 : 16;  // Rec<RW>::GS
  std::vector<double> rec((size_t)(h->ninc + 1) * GS, 0.0);  // + one zero pad record
  std::vector<int> rec_o(RW == 10 ? h->ninc + 1 : 1, 0);
  std::vector<int2> eipos(std::max(h->mloc, 1), make_int2(-1, -1));
  std::vector<int> fill(inc_ptr.begin(), inc_ptr.end() - 1);
  auto put_rec = [&](int pos, int k, int64_t e, int other, int code) {
    double* c = &rec[(size_t)pos * GS];
    const double* Q = RW == 10 ? &quat[3 * (size_t)k] : R + 9 * e;
    int j = 0;
    for (int q = 0; q < (RW == 10 ? 3 : 9); ++q) c[j++] = Q[q];
    for (int q = 0; q < 3; ++q) c[j++] = t[3 * e + q];
    c[j++] = weight[e] * kappa[e];
    const double wt = weight[e] * tau[e];
    if (RW == 10) {  // compact: the tail flag in w tau's sign bit, the other endpoint apart
      c[j++] = (code & 0x80000000) ? -wt : wt;
      rec_o[pos] = (int)(((unsigned)other & 0x1fffffffu) | ((unsigned)qbig[k] << 29));
    } else {
      c[j++] = wt;
      const long long bits = (long long)(unsigned)other | ((long long)code << 32);
      std::memcpy(&c[j], &bits, 8);
    }
  };
  for (int k = 0; k < h->mloc; ++k) {  // increasing global edge id per pose
    const int64_t e = ledges[k];
    const bool priv = r1[e] == r2[e];
    if (h->local_of[r1[e]] >= 0) {
      const int sp = lpose(r1[e], p1[e]);
      const int other = priv ? lpose(r2[e], p2[e]) : (int)(-1 - slot_of(r2[e], p2[e]));
      eipos[k].x = fill[sp];
      put_rec(fill[sp]++, k, e, other, (int)(k | 0x80000000u));
    }
    if (h->local_of[r2[e]] >= 0) {
      const int sp = lpose(r2[e], p2[e]);
      const int other = priv ? lpose(r1[e], p1[e]) : (int)(-1 - slot_of(r1[e], p1[e]));
      eipos[k].y = fill[sp];
      put_rec(fill[sp]++, k, e, other, k);
    }
  }
  // GNC: every non-fixed local edge is re-weighted here (a shared loop closure
  // on both handles of its robots, identically); the owner-packed shared-weight
  // table (owner = lower robot id, drawio:2198) is kept for the explicit exchange.
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
    // a local endpoint is read from the iterate, a foreign one from the public
    // table (after the exchange they hold the same row)
    auto enc = [&](int rb, int pp) -> int {
      return h->local_of[rb] >= 0 ? lpose(rb, pp) : (int)(-1 - slot_of(rb, pp));
    };
    gnc_edge.push_back(k);
    gnc_ends.push_back(make_int2(enc(r1[e], p1[e]), enc(r2[e], p2[e])));
  }
  h->n_gnc = (int)gnc_edge.size();
  h->n_sh_local = (int)sh_edge.size();
  h->n_osh = (int)osh_edge.size();
  // tiles: at most TP poses of one robot, cut by incidence count so every
  // workgroup's gather walks about the same number of incidences (a tile closes
  // when the next pose would take it past 1.05 x the robot's mean per full tile)
  // and capped at two chunks of TP * r incidences (two LDS hand-offs in k_hess)
  std::vector<int> tr, tp0, tnp, rt0(L + 1, 0);
  // incidences per tile: at most two gather chunks; small problems are cut
  // finer, to about TILES_TARGET tiles (3 workgroups per CU, one generation),
  // but not below 180 (3/4 of a chunk). Measured on one 12.5k-pose block
  // (125k incidences): 160.0 / 156.5 / 154.9 / 152.6 us per round at caps
  // 480 / 360 / 240 / 180, 207 at 120 (> 1024 tiles: a second generation);
  // 25k poses: 254.7 at 480, 245.6 at 360, 301 at 240
  // (profiles/r02/small_round/5_tile_cap.log). kmx_pgo_params.tile_incidences
  // overrides it (the multi-rank driver sets it from the team; bench.py
  // --tile-incidences for sweeps).
  int64_t inc_all = (int64_t)inc_ptr[nloc] - inc_ptr[0];
  auto cut = [&](int TP, int64_t tilecap) {
    tr.clear(); tp0.clear(); tnp.clear();
    for (int l = 0; l < L; ++l) {
      const int n = n_poses[h->robots[l]];
      const int base = h->loff[l];
      rt0[l] = (int)tr.size();
      const int64_t inc_l = (int64_t)inc_ptr[base + n] - inc_ptr[base];
      const int64_t full = std::max<int64_t>(1, (n + TP - 1) / TP);
      const int64_t cap = std::min(tilecap, std::max<int64_t>(1, (inc_l * 21 / 20 + full - 1) / full));
      int p0 = 0;
      while (p0 < n) {
        int np = 0;
        int64_t cum = 0;
        while (p0 + np < n && np < TP) {
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
  };
  {
    const int TP = WAVES * (64 / r);
    int64_t tilecap = std::min<int64_t>(2 * (int64_t)TP * r,
                                        std::max<int64_t>(180, (inc_all + TILES_TARGET - 1) / TILES_TARGET));
    if (h->P.tile_incidences > 0) tilecap = std::max(16, h->P.tile_incidences);
    cut(TP, tilecap);
  }
  rt0[L] = (int)tr.size();
  h->rt0_h = rt0;
  h->ntiles = (int)tr.size();
  KMX_CHECK(h->ntiles > 0, KMX_EINVAL, "no local poses");
  std::vector<int> own_src(std::max<int64_t>(h->n_owned, 1), 0);
  for (int64_t k = 0; k < h->n_owned; ++k) own_src[k] = pub_src[h->first_owned + k];
  std::vector<int> nrob(L);
  for (int l = 0; l < L; ++l) nrob[l] = n_poses[h->robots[l]];
  // tile descriptors: validated before any device allocation, so a rejected
  // graph leaves the handle without buffers (ready() false)
  std::vector<TileDesc> tdesc(h->ntiles);
  for (int t = 0; t < h->ntiles; ++t) {
    TileDesc& td = tdesc[t];
    td.robot = tr[t];
    td.p0 = tp0[t];
    td.k0 = inc_ptr[tp0[t]];
    const int ninc = inc_ptr[tp0[t] + tnp[t]] - td.k0;
    KMX_CHECK(tnp[t] < 256 && ninc < (1 << 23), KMX_EINVAL, "tile too large");
    td.np_n = tnp[t] | (ninc << 8);
    td.rt0 = rt0[tr[t]];
    td.rt1 = rt0[tr[t] + 1];
    td.pad0 = td.pad1 = 0;
  }
  // device
  int rc;
  const size_t vec = (size_t)std::max(nloc, 1) * ps;
  if ((rc = dalloc(&h->d_tile, h->ntiles)) || (rc = dalloc(&h->d_rtile0, L + 1)) ||
      (rc = dalloc(&h->d_inc_ptr, nloc + 1)) || (rc = dalloc(&h->d_rec, rec.size())) || (rc = dalloc(&h->d_rec_o, rec_o.size())) ||
      (rc = dalloc(&h->d_ekappa, ek_h.size())) || (rc = dalloc(&h->d_etau, et_h.size())) ||
      (rc = dalloc(&h->d_ew, ew_h.size())) || (rc = dalloc(&h->d_eipos, eipos.size())) ||
      (rc = dalloc(&h->d_vec, vec * nvec(h))) || (rc = dalloc(&h->d_S, (size_t)std::max(nloc, 1) * 6)) ||
      (rc = dalloc(&h->d_Pinv, (size_t)std::max(nloc, 1) * SYM4)) ||
      (rc = dalloc(&h->d_hD, (size_t)std::max(nloc, 1) * SYM4)) ||
      (rc = dalloc(&h->d_hDS, (size_t)std::max(nloc, 1) * SYM4)) ||
      (rc = dalloc(&h->d_pub, (size_t)std::max<int64_t>(h->npub, 1) * ps)) ||
      (h->P.acceleration && ((rc = dalloc(&h->d_accV, vec)) || (rc = dalloc(&h->d_accY, vec)))) ||
      (rc = dalloc(&h->d_part, (size_t)h->ntiles * NPART)) || (rc = dalloc(&h->d_ctl, L)) ||
      (rc = dalloc(&h->d_ctl2, L)) || (rc = dalloc(&h->d_part_h, (size_t)h->ntiles * 2)) ||
      (rc = dalloc(&h->d_part_u, (size_t)h->ntiles * 2)) ||
      (rc = dalloc(&h->d_cnt, 1)) || (rc = dalloc(&h->d_m_robot, L)) ||
      (rc = dalloc(&h->d_n_robot, L)) || (rc = dalloc(&h->d_pub_src, pub_src.size())) ||
      (rc = dalloc(&h->d_own_src, own_src.size())) || (rc = dalloc(&h->d_pose_slot, pose_slot.size())) ||
      (rc = dalloc(&h->d_gnc_edge, std::max(h->n_gnc, 1))) || (rc = dalloc(&h->d_gnc_ends, std::max(h->n_gnc, 1))) ||
      (rc = dalloc(&h->d_sh_edge, std::max(h->n_sh_local, 1))) ||
      (rc = dalloc(&h->d_sh_idx, std::max(h->n_sh_local, 1))) || (rc = dalloc(&h->d_active, L)) ||
      (rc = dalloc(&h->d_osh_edge, std::max(h->n_osh, 1))) || (rc = dalloc(&h->d_osh_idx, std::max(h->n_osh, 1))) ||
      (rc = dalloc(&h->d_relc, L)) || (rc = dalloc(&h->d_gnc, 2)) || (rc = dalloc(&h->d_ext, 64)) ||
      (rc = dalloc(&h->d_hv_launch, HV_SLOTS)) ||
      (rc = dalloc(&h->d_coefh, (size_t)L * std::max(h->P.tcg_max_iterations, 1))) ||
      (onesync(h) && (rc = dalloc(&h->d_part_f, (size_t)h->ntiles * 16)))) {
    free_dev(h);
    return rc;
  }
  h->ext_cap = 64;
  auto up = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream);
  };
  KMX_HIP(up(h->d_tile, tdesc.data(), sizeof(TileDesc) * tdesc.size()));
  KMX_HIP(up(h->d_rtile0, rt0.data(), sizeof(int) * rt0.size()));
  KMX_HIP(up(h->d_inc_ptr, inc_ptr.data(), sizeof(int) * inc_ptr.size()));
  KMX_HIP(up(h->d_rec, rec.data(), sizeof(double) * rec.size()));
  KMX_HIP(up(h->d_rec_o, rec_o.data(), sizeof(int) * rec_o.size()));
  KMX_HIP(up(h->d_ekappa, ek_h.data(), sizeof(double) * ek_h.size()));
  KMX_HIP(up(h->d_etau, et_h.data(), sizeof(double) * et_h.size()));
  KMX_HIP(up(h->d_ew, ew_h.data(), sizeof(double) * ew_h.size()));
  KMX_HIP(up(h->d_eipos, eipos.data(), sizeof(int2) * eipos.size()));
  KMX_HIP(hipMemsetAsync(h->d_vec, 0, sizeof(double) * vec * nvec(h), h->stream));
  KMX_HIP(hipMemsetAsync(h->d_coefh, 0, sizeof(double) * L * std::max(h->P.tcg_max_iterations, 1), h->stream));
  KMX_HIP(hipMemsetAsync(h->d_pub, 0, sizeof(double) * std::max<int64_t>(h->npub, 1) * ps, h->stream));
  KMX_HIP(hipMemsetAsync(h->d_ctl, 0, sizeof(Ctl) * L, h->stream));
  KMX_HIP(hipMemsetAsync(h->d_cnt, 0, sizeof(Counters), h->stream));
  KMX_HIP(hipMemsetAsync(h->d_ext, 0, sizeof(double) * 64, h->stream));
  KMX_HIP(hipMemsetAsync(h->d_hv_launch, 0, sizeof(int) * HV_SLOTS, h->stream));
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
  {
    std::vector<double> relc(L);  // no block update yet: not converged (an empty block is)
    for (int l = 0; l < L; ++l) relc[l] = nrob[l] > 0 ? std::numeric_limits<double>::infinity() : 0.0;
    KMX_HIP(up(h->d_relc, relc.data(), sizeof(double) * L));
    Gnc g0[2] = {};
    g0[0].mu = g0[1].mu = h->P.gnc_mu_init;
    KMX_HIP(up(h->d_gnc, g0, sizeof(g0)));
  }
  KMX_HIP(up(h->d_m_robot, h->m_robot.data(), sizeof(long long) * L));
  KMX_HIP(up(h->d_n_robot, nrob.data(), sizeof(int) * L));
  KMX_HIP(up(h->d_pub_src, pub_src.data(), sizeof(int) * pub_src.size()));
  KMX_HIP(up(h->d_own_src, own_src.data(), sizeof(int) * own_src.size()));
  KMX_HIP(up(h->d_pose_slot, pose_slot.data(), sizeof(int) * pose_slot.size()));
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
  d = Dev{};
  d.ntiles = h->ntiles; d.L = L; d.nloc = nloc; d.npub = (int)h->npub;
  d.tile = h->d_tile; d.rtile0 = h->d_rtile0;
  d.inc_ptr = h->d_inc_ptr; d.rec = h->d_rec; d.rec_o = h->d_rec_o;
  d.ekappa = h->d_ekappa; d.etau = h->d_etau; d.ew = h->d_ew; d.eipos = h->d_eipos;
  d.X = h->d_vec; d.Xt = h->d_vec + vec; d.g = h->d_vec + 2 * vec; d.r = h->d_vec + 3 * vec;
  d.z = h->d_vec + 4 * vec; d.hd = h->d_vec + 5 * vec; d.eta = h->d_vec + 6 * vec; d.dh = h->d_vec + 7 * vec;
  d.coefh = h->d_coefh; d.vec = (long long)vec; d.dhn = dh_count(h);
  d.S = h->d_S; d.Pinv = h->d_Pinv; d.hD = h->d_hD; d.hDS = h->d_hDS; d.pub = h->d_pub; d.part = h->d_part;
  d.ctl = h->d_ctl; d.cnt = h->d_cnt;
  d.ctl2 = h->d_ctl2; d.part_h = h->d_part_h; d.part_u = h->d_part_u;
  d.m_robot = h->d_m_robot; d.n_robot = h->d_n_robot; d.pose_slot = h->d_pose_slot;
  d.relc = h->d_relc; d.gnc = h->d_gnc; d.gnc_next = h->d_gnc + 1;
  d.gnc_edge = h->d_gnc_edge; d.gnc_ends = h->d_gnc_ends; d.n_gnc = h->n_gnc;
  d.hv_launch = h->d_hv_launch;
  if (onesync(h)) {
    const size_t v0 = 7 + (size_t)dh_count(h);
    d.hz = h->d_vec + v0 * vec; d.w0 = h->d_vec + (v0 + 1) * vec; d.w1 = h->d_vec + (v0 + 2) * vec;
    d.part_f = h->d_part_f;
  }
  h->n_ext = 0;
  sync_params(h);
  enqueue_precond(h, 0);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
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
  accel_reset(h);  // a new initial iterate restarts the acceleration (V = X at the next round)
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
  return kmx_pgo_exchange_pack(h, dev_slots, n, nullptr, 0, dev_out);
}

extern "C" int kmx_pgo_scatter_public_rows(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const void* dev_rows) {
  return kmx_pgo_exchange_unpack(h, dev_slots, n, nullptr, 0, dev_rows);
}

extern "C" int kmx_pgo_exchange_pack(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const int32_t* dev_seg,
                                     int n_seg, void* dev_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(n >= 0 && n_seg >= 0 && n_seg <= 1024 && (n == 0 || (dev_slots && dev_out)) &&
                (n_seg == 0 || (dev_seg && dev_out)),
            KMX_EINVAL, "bad argument");
  KMX_HIP(hipSetDevice(h->device));
  enqueue_accel_pre(h);  // accelerated rounds exchange Y
  const int ps = 4 * h->P.r;
  const long long tot = (long long)n * ps + n_seg;  // rows, then the status words
  if (tot)
    hipLaunchKernelGGL(k_gather_slots, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                       h->d_pub_src, (const int*)dev_slots, (long long)n, (int)h->npub, (double*)dev_out, ps,
                       (const int*)dev_seg, n_seg, (const double*)h->d_relc, h->dv.L);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_exchange_unpack(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const int32_t* dev_seg,
                                       int n_seg, const void* dev_in) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(n >= 0 && n_seg >= 0 && n_seg <= 1024 && (n == 0 || (dev_slots && dev_in)) &&
                (n_seg == 0 || (dev_seg && dev_in)),
            KMX_EINVAL, "bad argument");
  KMX_HIP(hipSetDevice(h->device));
  const int ps = 4 * h->P.r;
  if (n_seg > h->ext_cap) {
    KMX_HIP(hipStreamSynchronize(h->stream));
    if (h->d_ext) (void)hipFree(h->d_ext);
    h->d_ext = nullptr;
    h->ext_cap = 0;
    if (int rc = dalloc(&h->d_ext, n_seg)) return rc;
    h->ext_cap = n_seg;
  }
  const long long tot = (long long)n * ps + n_seg;  // rows, then the status words
  if (tot)
    hipLaunchKernelGGL(k_scatter_slots, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->d_pub,
                       (const int*)dev_slots, (long long)n, (int)h->npub, (const double*)dev_in, ps,
                       (const int*)dev_seg, n_seg, h->d_ext);
  h->n_ext = n_seg;
  sync_params(h);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

#define KMX_NCCL(call)                                                                      \
  do {                                                                                      \
    const ncclResult_t r_ = (call);                                                         \
    if (r_ != ncclSuccess) return kmx::fail(KMX_EHIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// A call on a non-blocking communicator may return ncclInProgress: wait for
// it to settle (bounded), then report its final status.
int nccl_settle(kmx_pgo* h, ncclResult_t r, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
      return kmx::fail(KMX_EHIP, std::string(what) + ": still in progress after 60 s");
    std::this_thread::yield();
    if (ncclCommGetAsyncError(h->comm, &r) != ncclSuccess) r = ncclSystemError;
  }
  if (r != ncclSuccess) return kmx::fail(KMX_EHIP, std::string(what) + ": " + ncclGetErrorString(r));
  return KMX_OK;
}

// publishPublicPoses -> updateNeighborPoses + publishStatus of one round
// (drawio:2340-2375) over RCCL: the rows every peer needs (+ this handle's
// status word) are gathered, each peer's segment goes by ncclSend / ncclRecv in
// one group on the handle's stream, then the received rows land in the public
// table and the peers' status words in ext. Segment layout as
// kmx_pgo_exchange_pack / _unpack.
int enqueue_exchange_lag(kmx_pgo* h);
int enqueue_exchange(kmx_pgo* h) {
  if (!h->xchg) return KMX_OK;
  if (h->xchg_lag) return enqueue_exchange_lag(h);
  const int ps = 4 * h->P.r, W = h->world;
  const long long ts = h->xn_send * ps + W, tr = h->xn_recv * ps + W;
  hipLaunchKernelGGL(k_xgather, dim3((unsigned)((ts + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                     h->d_pub_src, h->d_xs_slots, h->d_xs_rseg, h->xn_send, h->d_xsbuf, ps, h->d_xs_seg, W,
                     (const double*)h->d_relc, h->dv.L);
  KMX_NCCL(ncclGroupStart());
  for (int q = 0; q < W; ++q) {
    if (q == h->rank && !h->xchg_self_p2p) continue;
    KMX_NCCL(ncclSend(h->d_xsbuf + h->xs_off[q], (size_t)h->xs_cnt[q], ncclDouble, q, h->comm, h->stream));
    KMX_NCCL(ncclRecv(h->d_xrbuf + h->xr_off[q], (size_t)h->xr_cnt[q], ncclDouble, q, h->comm, h->stream));
  }
  // the communicator is non-blocking (kmx_pgo_comm_init): the group may still
  // be enqueueing when ncclGroupEnd returns
  if (int rc = nccl_settle(h, ncclGroupEnd(), "ncclGroupEnd")) return rc;
  if (!h->xchg_self_p2p)  // this handle's own segment (its status word)
    KMX_HIP(hipMemcpyAsync(h->d_xrbuf + h->xr_off[h->rank], h->d_xsbuf + h->xs_off[h->rank],
                           sizeof(double) * h->xs_cnt[h->rank], hipMemcpyDeviceToDevice, h->stream));
  hipLaunchKernelGGL(k_xscatter, dim3((unsigned)((tr + 255) / 256)), dim3(256), 0, h->stream, h->d_pub,
                     h->d_xr_slots, h->d_xr_rseg, h->xn_recv, (const double*)h->d_xrbuf, ps, h->d_xr_seg, W, h->d_ext);
  if (h->n_ext != W) {
    h->n_ext = W;
    sync_params(h);
  }
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

// KMX_XCHG_LAG: the previous round's exchange (done on xstream while that
// round computed) is installed, then this round's rows are gathered and sent
// on xstream behind an event, and the round runs without waiting for them.
// The first round of a sequence waits (round 1 reads X^0 as in the in-round
// form). The send / receive buffers need no second copy: the scatter of
// exchange i-1 and the gather of exchange i both wait for exchange i-1 to
// finish, and exchange i starts after both.
int enqueue_exchange_lag(kmx_pgo* h) {
  const int ps = 4 * h->P.r, W = h->world;
  const long long ts = h->xn_send * ps + W, tr = h->xn_recv * ps + W;
  if (!h->xstream) {
    KMX_HIP(hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking));
    KMX_HIP(hipEventCreateWithFlags(&h->ev_xg, hipEventDisableTiming));
    KMX_HIP(hipEventCreateWithFlags(&h->ev_xd, hipEventDisableTiming));
  }
  auto scatter = [&]() {
    hipLaunchKernelGGL(k_xscatter, dim3((unsigned)((tr + 255) / 256)), dim3(256), 0, h->stream, h->d_pub,
                       h->d_xr_slots, h->d_xr_rseg, h->xn_recv, (const double*)h->d_xrbuf, ps, h->d_xr_seg, W,
                       h->d_ext);
  };
  if (h->x_inflight) {
    KMX_HIP(hipStreamWaitEvent(h->stream, h->ev_xd, 0));
    scatter();
  }
  hipLaunchKernelGGL(k_xgather, dim3((unsigned)((ts + 255) / 256)), dim3(256), 0, h->stream, h->d_vec,
                     h->d_pub_src, h->d_xs_slots, h->d_xs_rseg, h->xn_send, h->d_xsbuf, ps, h->d_xs_seg, W,
                     (const double*)h->d_relc, h->dv.L);
  KMX_HIP(hipEventRecord(h->ev_xg, h->stream));
  KMX_HIP(hipStreamWaitEvent(h->xstream, h->ev_xg, 0));
  KMX_NCCL(ncclGroupStart());
  for (int q = 0; q < W; ++q) {
    if (q == h->rank && !h->xchg_self_p2p) continue;
    KMX_NCCL(ncclSend(h->d_xsbuf + h->xs_off[q], (size_t)h->xs_cnt[q], ncclDouble, q, h->comm, h->xstream));
    KMX_NCCL(ncclRecv(h->d_xrbuf + h->xr_off[q], (size_t)h->xr_cnt[q], ncclDouble, q, h->comm, h->xstream));
  }
  if (int rc = nccl_settle(h, ncclGroupEnd(), "ncclGroupEnd")) return rc;
  if (!h->xchg_self_p2p)
    KMX_HIP(hipMemcpyAsync(h->d_xrbuf + h->xr_off[h->rank], h->d_xsbuf + h->xs_off[h->rank],
                           sizeof(double) * h->xs_cnt[h->rank], hipMemcpyDeviceToDevice, h->xstream));
  KMX_HIP(hipEventRecord(h->ev_xd, h->xstream));
  if (!h->x_inflight) {  // the first round: its own exchange's rows
    KMX_HIP(hipStreamWaitEvent(h->stream, h->ev_xd, 0));
    scatter();
  }
  h->x_inflight = true;
  if (h->n_ext != W) {
    h->n_ext = W;
    sync_params(h);
  }
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

// Which RCCL / HIP runtime libkmx's own calls resolve to in this process
// (torch bundles a librccl.so.1 of the same SONAME: whichever was loaded first
// serves both), their versions and the RCCL headers kmx was built against.
extern "C" int kmx_runtime_info(char* out, int64_t nbytes) {
  KMX_GUARD_BEGIN
  KMX_CHECK(out && nbytes > 0, KMX_EINVAL, "null buffer");
  Dl_info di{}, dh{};
  const char* rp = dladdr(reinterpret_cast<void*>(&ncclSend), &di) && di.dli_fname ? di.dli_fname : "?";
  const char* hp = dladdr(reinterpret_cast<void*>(static_cast<hipError_t (*)(void**, size_t)>(&hipMalloc)), &dh) && dh.dli_fname ? dh.dli_fname : "?";
  int rv = 0, hv = 0, dv = 0;
  (void)ncclGetVersion(&rv);
  (void)hipRuntimeGetVersion(&hv);
  (void)hipDriverGetVersion(&dv);
  const std::string js = std::string("{\"rccl_path\": \"") + rp + "\", \"rccl_version\": " + std::to_string(rv) +
                         ", \"rccl_header_version\": " + std::to_string(NCCL_VERSION_CODE) + ", \"hip_path\": \"" + hp +
                         "\", \"hip_runtime_version\": " + std::to_string(hv) + ", \"hip_driver_version\": " +
                         std::to_string(dv) + "}";
  KMX_CHECK((int64_t)js.size() < nbytes, KMX_EINVAL, "buffer too small");
  std::memcpy(out, js.c_str(), js.size() + 1);
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_comm_unique_id(void* out, int64_t nbytes) {
  KMX_GUARD_BEGIN
  KMX_CHECK(out && nbytes >= (int64_t)sizeof(ncclUniqueId), KMX_EINVAL, "need a buffer of KMX_COMM_ID_BYTES");
  ncclUniqueId id;
  KMX_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return KMX_OK;
  KMX_GUARD_END
}

// Non-blocking communicator creation with a deadline: a rank whose peers never
// arrive (one of them failed before ncclCommInitRank) aborts its half-built
// communicator and returns an error instead of blocking in the rendezvous.
extern "C" int kmx_pgo_comm_init(kmx_pgo* h, const void* unique_id, int world, int rank, double timeout_s) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h && unique_id, KMX_EINVAL, "null argument");
  KMX_CHECK(world >= 1 && world <= 1024 && rank >= 0 && rank < world, KMX_EINVAL, "bad world / rank");
  KMX_CHECK(timeout_s > 0.0, KMX_EINVAL, "timeout_s must be > 0");
  KMX_CHECK(!h->comm, KMX_ESTATE, "communicator already initialised");
  KMX_HIP(hipSetDevice(h->device));
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  ncclComm_t c = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
      if (c) (void)ncclCommAbort(c);
      return kmx::fail(KMX_EHIP, "ncclCommInitRankConfig: no rendezvous within the timeout (a peer failed?)");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
    if (ncclCommGetAsyncError(c, &r) != ncclSuccess) r = ncclSystemError;
  }
  if (r != ncclSuccess) {
    if (c) (void)ncclCommAbort(c);
    return kmx::fail(KMX_EHIP, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  h->comm = c;
  h->world = world;
  h->rank = rank;
  if (const char* v = std::getenv("KMX_XCHG_SELF_P2P")) h->xchg_self_p2p = std::atoi(v) != 0;
  if (const char* v = std::getenv("KMX_XCHG_LAG")) h->xchg_lag = std::atoi(v) != 0;
  return KMX_OK;
  KMX_GUARD_END
}

// Abort first: a round whose exchange waits on a peer that never posts its
// half (the peer failed) only leaves the stream once the communicator is
// aborted; then the stream drains and the exchange buffers can go.
extern "C" int kmx_pgo_comm_destroy(kmx_pgo* h) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  if (h->comm) (void)ncclCommAbort(h->comm);
  h->comm = nullptr;
  KMX_HIP(hipStreamSynchronize(h->stream));
  free_xchg(h);
  h->world = 1;
  h->rank = 0;
  if (h->n_ext) {  // the peers' statuses came with the exchange
    h->n_ext = 0;
    sync_params(h);
  }
  return KMX_OK;
  KMX_GUARD_END
}

// The handle's stream drained within timeout_s (polled), or KMX_ETIMEOUT: a
// bounded wait for a round whose exchange depends on peers.
extern "C" int kmx_pgo_sync_timeout(kmx_pgo* h, double timeout_s) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_CHECK(timeout_s > 0.0, KMX_EINVAL, "timeout_s must be > 0");
  KMX_HIP(hipSetDevice(h->device));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    hipError_t e = hipStreamQuery(h->stream);
    if (e == hipSuccess && h->xstream) e = hipStreamQuery(h->xstream);  // a lagged exchange in flight
    if (e == hipSuccess) return KMX_OK;
    if (e != hipErrorNotReady) return kmx::fail(KMX_EHIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return kmx::fail(KMX_ETIMEOUT, "the stream did not drain within the timeout (an exchange peer is missing?)");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

extern "C" int kmx_pgo_get_public(kmx_pgo* h, double* table, double* ext) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(table || h->npub == 0, KMX_EINVAL, "null table");
  KMX_HIP(hipSetDevice(h->device));
  if (h->npub)
    KMX_HIP(hipMemcpyAsync(table, h->d_pub, sizeof(double) * h->npub * 4 * h->P.r, hipMemcpyDeviceToHost, h->stream));
  if (ext && h->n_ext)
    KMX_HIP(hipMemcpyAsync(ext, h->d_ext, sizeof(double) * h->n_ext, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_set_exchange(kmx_pgo* h, const int32_t* send_slots, const int64_t* send_counts,
                                    const int32_t* recv_slots, const int64_t* recv_counts) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(h->comm, KMX_ESTATE, "kmx_pgo_comm_init first");
  KMX_CHECK(send_counts && recv_counts, KMX_EINVAL, "null counts");
  const int W = h->world, ps = 4 * h->P.r;
  long long ns = 0, nr = 0;
  for (int q = 0; q < W; ++q) {
    KMX_CHECK(send_counts[q] >= 0 && recv_counts[q] >= 0, KMX_EINVAL, "negative count");
    ns += send_counts[q];
    nr += recv_counts[q];
  }
  KMX_CHECK(send_counts[h->rank] == recv_counts[h->rank], KMX_EINVAL, "own segment: send and receive counts differ");
  KMX_CHECK((ns == 0 || send_slots) && (nr == 0 || recv_slots), KMX_EINVAL, "null slot list");
  for (long long i = 0; i < ns; ++i) KMX_CHECK(send_slots[i] >= 0 && send_slots[i] < h->npub, KMX_EINVAL, "send slot out of range");
  for (long long i = 0; i < nr; ++i) KMX_CHECK(recv_slots[i] >= 0 && recv_slots[i] < h->npub, KMX_EINVAL, "recv slot out of range");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  free_xchg(h);
  std::vector<int> sseg(W + 1, 0), rseg(W + 1, 0);
  h->xs_cnt.assign(W, 0); h->xr_cnt.assign(W, 0); h->xs_off.assign(W, 0); h->xr_off.assign(W, 0);
  for (int q = 0; q < W; ++q) {
    sseg[q + 1] = sseg[q] + (int)send_counts[q];
    rseg[q + 1] = rseg[q] + (int)recv_counts[q];
    h->xs_cnt[q] = send_counts[q] * ps + 1;
    h->xr_cnt[q] = recv_counts[q] * ps + 1;
    h->xs_off[q] = (long long)sseg[q] * ps + q;
    h->xr_off[q] = (long long)rseg[q] * ps + q;
  }
  int rc = 0;
  if ((rc = dalloc(&h->d_xs_slots, ns)) || (rc = dalloc(&h->d_xr_slots, nr)) || (rc = dalloc(&h->d_xs_seg, W + 1)) ||
      (rc = dalloc(&h->d_xs_rseg, ns)) || (rc = dalloc(&h->d_xr_rseg, nr)) ||
      (rc = dalloc(&h->d_xr_seg, W + 1)) || (rc = dalloc(&h->d_xsbuf, ns * ps + W)) ||
      (rc = dalloc(&h->d_xrbuf, nr * ps + W))) {
    free_xchg(h);
    return rc;
  }
  if (W > h->ext_cap) {
    if (h->d_ext) (void)hipFree(h->d_ext);
    h->d_ext = nullptr;
    h->ext_cap = 0;
    if ((rc = dalloc(&h->d_ext, W))) return rc;
    h->ext_cap = W;
  }
  if (ns) KMX_HIP(hipMemcpy(h->d_xs_slots, send_slots, sizeof(int) * ns, hipMemcpyHostToDevice));
  if (nr) KMX_HIP(hipMemcpy(h->d_xr_slots, recv_slots, sizeof(int) * nr, hipMemcpyHostToDevice));
  {
    std::vector<int> srs(std::max<long long>(ns, 1)), rrs(std::max<long long>(nr, 1));
    for (int q = 0; q < W; ++q) {
      for (int k = sseg[q]; k < sseg[q + 1]; ++k) srs[k] = q;
      for (int k = rseg[q]; k < rseg[q + 1]; ++k) rrs[k] = q;
    }
    if (ns) KMX_HIP(hipMemcpy(h->d_xs_rseg, srs.data(), sizeof(int) * ns, hipMemcpyHostToDevice));
    if (nr) KMX_HIP(hipMemcpy(h->d_xr_rseg, rrs.data(), sizeof(int) * nr, hipMemcpyHostToDevice));
  }
  KMX_HIP(hipMemcpy(h->d_xs_seg, sseg.data(), sizeof(int) * (W + 1), hipMemcpyHostToDevice));
  KMX_HIP(hipMemcpy(h->d_xr_seg, rseg.data(), sizeof(int) * (W + 1), hipMemcpyHostToDevice));
  h->xn_send = ns;
  h->xn_recv = nr;
  h->xchg = true;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_exchange(kmx_pgo* h) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(h->xchg, KMX_ESTATE, "kmx_pgo_set_exchange first");
  KMX_HIP(hipSetDevice(h->device));
  enqueue_accel_pre(h);
  return enqueue_exchange(h);
  KMX_GUARD_END
}

extern "C" int kmx_pgo_refresh_local(kmx_pgo* h) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_HIP(hipSetDevice(h->device));
  enqueue_accel_pre(h);  // accelerated rounds publish Y
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
  if (h->P.acceleration)
    for (int l = 0; l < L; ++l)
      KMX_CHECK(act[l], KMX_EUNSUP, "acceleration needs every local robot active (concurrent schedule)");
  KMX_HIP(hipMemcpyAsync(h->d_active, act.data(), L, hipMemcpyHostToDevice, h->stream));
  enqueue_accel_pre(h);
  if (int rc = enqueue_exchange(h)) return rc;
  enqueue_round(h, h->d_active);
  enqueue_accel_post(h);
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

extern "C" int kmx_pgo_iterate_async(kmx_pgo* h, int rounds, int refresh_local) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(rounds >= 0, KMX_EINVAL, "negative rounds");
  KMX_HIP(hipSetDevice(h->device));
  // every round's k_commit republishes the committed owned rows, so the
  // single-device exchange needs one publish per call
  if (refresh_local && rounds > 0) enqueue_publish(h);
  for (int i = 0; i < rounds; ++i) {
    enqueue_accel_pre(h);  // publishes Y itself
    if (int rc = enqueue_exchange(h)) return rc;
    enqueue_round(h, h->d_active);
    enqueue_accel_post(h);
  }
  KMX_HIP(hipGetLastError());
  return KMX_OK;
}

extern "C" int kmx_pgo_sync(kmx_pgo* h) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  if (h->xstream) KMX_HIP(hipStreamSynchronize(h->xstream));
  return KMX_OK;
}

extern "C" int kmx_pgo_set_gnc_schedule(kmx_pgo* h, int enabled, int inner_iters, int max_updates,
                                        double rel_change_tol) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_CHECK(inner_iters >= 0 && max_updates >= 0, KMX_EINVAL, "negative schedule parameter");
  h->gnc_on = enabled ? 1 : 0;
  h->gnc_inner_iters = inner_iters;
  h->gnc_max_updates = max_updates;
  h->gnc_rel_tol = rel_change_tol;
  sync_params(h);
  return KMX_OK;
}

extern "C" int kmx_pgo_get_gnc_state(kmx_pgo* h, kmx_gnc_state* out) {
  KMX_CHECK(ready(h) && out, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  Gnc g;
  KMX_HIP(hipMemcpyAsync(&g, h->d_gnc, sizeof(Gnc), hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  std::memset(out, 0, sizeof(*out));
  out->inner_iter = g.inner;
  out->updates = g.updates;
  out->last_fired = g.fired;
  out->rounds = g.rounds;
  out->mu = g.mu;
  return KMX_OK;
}

extern "C" int kmx_pgo_set_gnc_state(kmx_pgo* h, const kmx_gnc_state* in) {
  KMX_CHECK(ready(h) && in && in->mu > 0.0, KMX_EINVAL, "null argument / no graph / mu <= 0");
  KMX_HIP(hipSetDevice(h->device));
  Gnc g[2] = {};
  g[0].inner = in->inner_iter;
  g[0].updates = in->updates;
  g[0].fired = in->last_fired;
  g[0].rounds = in->rounds;
  g[0].mu = in->mu;
  g[1] = g[0];
  KMX_HIP(hipMemcpyAsync(h->d_gnc, g, sizeof(g), hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_get_status(kmx_pgo* h, double* rel_change) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h) && rel_change, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  std::vector<double> v(h->robots.size());
  KMX_HIP(hipMemcpyAsync(v.data(), h->d_relc, sizeof(double) * v.size(), hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  for (size_t l = 0; l < v.size(); ++l) rel_change[h->robots[l]] = v[l];
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_set_status(kmx_pgo* h, const double* rel_change) {
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h) && rel_change, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  std::vector<double> v(h->robots.size());
  for (size_t l = 0; l < v.size(); ++l) v[l] = rel_change[h->robots[l]];
  KMX_HIP(hipMemcpyAsync(h->d_relc, v.data(), sizeof(double) * v.size(), hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_pgo_update_weights(kmx_pgo* h, double* mu_out) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  KMX_HIP(hipSetDevice(h->device));
  Gnc g;
  KMX_HIP(hipMemcpyAsync(&g, h->d_gnc, sizeof(Gnc), hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  if (mu_out) *mu_out = g.mu;
  if (h->P.robust_cost != KMX_COST_GNC_TLS) return KMX_OK;
  enqueue_begin(h, h->d_active, BEGIN_FORCE_GNC);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_pgo_get_mu(kmx_pgo* h, double* mu) {
  KMX_CHECK(ready(h) && mu, KMX_EINVAL, "null argument / no graph");
  kmx_gnc_state s;
  if (int rc = kmx_pgo_get_gnc_state(h, &s)) return rc;
  *mu = s.mu;
  return KMX_OK;
}
extern "C" int kmx_pgo_set_mu(kmx_pgo* h, double mu) {
  KMX_CHECK(ready(h) && mu > 0.0, KMX_EINVAL, "mu must be positive / no graph");
  kmx_gnc_state s;
  if (int rc = kmx_pgo_get_gnc_state(h, &s)) return rc;
  s.mu = mu;
  return kmx_pgo_set_gnc_state(h, &s);
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
  KMX_GUARD_BEGIN
  KMX_CHECK(ready(h) && w, KMX_EINVAL, "null argument / no graph");
  KMX_HIP(hipSetDevice(h->device));
  std::vector<double> ew(std::max(h->mloc, 1));
  for (int k = 0; k < h->mloc; ++k) ew[k] = w[h->loc_edge_gid[k]];
  KMX_HIP(hipMemcpyAsync(h->d_ew, ew.data(), sizeof(double) * h->mloc, hipMemcpyHostToDevice, h->stream));
  enqueue_apply_weights(h);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
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
  if (int rc = ensure_scratch(h, (size_t)ps + (size_t)std::max(n, 1) * 12)) return rc;
  double* d_anchor = h->d_scratch;
  double* d_out = h->d_scratch + ps;
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
  if (int rc = ensure_scratch(h, vec * 2)) return rc;
  double* dV = h->d_scratch;
  double* dO = h->d_scratch + vec;
  const size_t o = (size_t)h->loff[l] * ps;
  KMX_HIP(hipMemsetAsync(h->d_scratch, 0, sizeof(double) * vec * 2, h->stream));
  if (V) KMX_HIP(hipMemcpyAsync(dV + o, V, sizeof(double) * n * ps, hipMemcpyHostToDevice, h->stream));
#define KMX_EVAL_LAUNCH(RR)                                                                                      \
  if (h->rw == 10)                                                                                               \
    hipLaunchKernelGGL((k_eval<RR, 10>), dim3(h->ntiles), dim3(BLOCK), SmemE<RR>::bytes, h->stream, h->dv, l, mode, \
                       (const double*)dV, dO);                                                                   \
  else                                                                                                           \
    hipLaunchKernelGGL((k_eval<RR, 16>), dim3(h->ntiles), dim3(BLOCK), SmemE<RR>::bytes, h->stream, h->dv, l, mode, \
                       (const double*)dV, dO);
  switch (h->P.r) {
    case 3: KMX_EVAL_LAUNCH(3) break;
    case 4: KMX_EVAL_LAUNCH(4) break;
    case 5: KMX_EVAL_LAUNCH(5) break;
    case 6: KMX_EVAL_LAUNCH(6) break;
    case 7: KMX_EVAL_LAUNCH(7) break;
    default: KMX_EVAL_LAUNCH(8) break;
  }
#undef KMX_EVAL_LAUNCH
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipMemcpyAsync(out, dO + o, sizeof(double) * n * ps, hipMemcpyDeviceToHost, h->stream));
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

extern "C" int kmx_pgo_memory(kmx_pgo* h, int64_t* device_bytes, int* record_bytes) {
  KMX_CHECK(ready(h), KMX_ESTATE, "set_graph first");
  const int64_t L = (int64_t)h->robots.size(), n = std::max(h->nloc, 1), ps = 4 * h->P.r;
  int64_t b = 0;
  const int rb = h->rw == 10 ? 8 * 8 + 4 : 128;  // bytes per incidence record (compact: 64 + the 4-B other endpoint)
  b += (int64_t)(h->ninc + 1) * rb + (int64_t)(h->nloc + 1) * 4;         // records, CSR
  b += (int64_t)std::max(h->mloc, 1) * (3 * 8 + 8);                      // kappa, tau, w, positions
  b += n * ps * 8 * (int64_t)nvec(h) + n * (6 + 3 * SYM4) * 8;         // vectors, S, Pinv, D, D - S
  b += L * 8 * (int64_t)std::max(h->P.tcg_max_iterations, 1);            // tCG coefficients
  b += std::max<int64_t>(h->npub, 1) * (ps * 8 + 4) + n * 4;             // public table + maps
  b += (int64_t)h->ntiles * (NPART * 8 + 12 + (onesync(h) ? 64 : 0)) + L * (int64_t)(sizeof(Ctl) + 32);
  b += (int64_t)std::max(h->n_gnc, 1) * 12 + (int64_t)h->scratch_cap * 8;  // GNC lists, scratch in use
  if (h->P.acceleration) b += 2 * n * ps * 8;                              // V, Y
  if (device_bytes) *device_bytes = b;
  if (record_bytes) *record_bytes = rb;
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
  // event pairs of k_hess launches in which at least one robot ran a Hess-vec
  const size_t nl = std::min(h->ev_used / 2, (size_t)HV_SLOTS);
  std::vector<int> hv(std::max<size_t>(nl, 1), 0);
  if (nl) KMX_HIP(hipMemcpy(hv.data(), h->d_hv_launch, sizeof(int) * nl, hipMemcpyDeviceToHost));
  double ms_total = 0.0;
  int64_t launches = 0;
  for (size_t i = 0; i < nl; ++i) {
    if (hv[i] == 0) continue;
    float ms = 0.f;
    KMX_HIP(hipEventElapsedTime(&ms, h->ev_pool[2 * i], h->ev_pool[2 * i + 1]));
    ms_total += ms;
    ++launches;
  }
  if (nl) KMX_HIP(hipMemset(h->d_hv_launch, 0, sizeof(int) * nl));
  std::memset(out, 0, sizeof(*out));
  out->hessvec_ms_total = ms_total;
  out->hessvec_launches = launches;
  out->hessvec_alg_bytes = c.hess_alg_bytes;
  out->edges_iters = (int64_t)c.edges_iters;
  out->block_updates = (int64_t)c.block_updates;
  out->hessvecs = (int64_t)c.hessvecs;
  out->gnc_updates = (int64_t)c.gnc_updates;
  h->ev_used = 0;
  KMX_HIP(hipMemset(h->d_cnt, 0, sizeof(Counters)));
  return KMX_OK;
}

// Diagnostic: the k_step phase stamps of a KMX_STEP_STAMPS build (16 words per
// tile: 7 wall-clock stamps, -, poses, incidences, block index, writer);
// KMX_EUNSUP in the product build.
extern "C" int kmx_pgo_debug_step_stamps(uint64_t* out, int64_t n) {
  KMX_GUARD_BEGIN
#ifdef KMX_STEP_STAMPS
  KMX_CHECK(out && n >= 0, KMX_EINVAL, "null buffer");
  const int64_t m = std::min<int64_t>(n, 16 * (int64_t)STEP_STAMP_TILES);
  KMX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_stamp), sizeof(uint64_t) * m, 0, hipMemcpyDeviceToHost));
  return KMX_OK;
#else
  (void)out;
  (void)n;
  return kmx::fail(KMX_EUNSUP, "not a KMX_STEP_STAMPS build");
#endif
  KMX_GUARD_END
}
