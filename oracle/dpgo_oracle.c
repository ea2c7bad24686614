/*
 * oracle/dpgo_oracle.c — CPU restatement of dpgo's RBCD block update with
 * GNC-TLS weights. TEST INFRASTRUCTURE ONLY: it is the parity checker for the
 * HIP path and the timed CPU baseline of bench.py (cpu_baseline.kind = "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it; the product path (kimera-multi_amd/kmx) never does.
 *
 * PARITY STATUS: the dpgo / ROPTLIB sources are not vendored in
 * /root/reference (SURVEY.md §0 finding 1, §8c) and the reference ships no
 * golden vectors or tests for this path. This restatement is
 * therefore "parity unpinned" against upstream dpgo; it is pinned instead by
 * analytic known answers (noise-free graphs converge to ground truth up to
 * gauge; gradient/Hessian vs finite differences; an independent numpy
 * restatement) — see tests/test_oracle_dpgo.py.
 *
 * What it restates (SURVEY.md §8a rows, §9.1 formulas):
 *   D1  edge classification / storage ......... PoseGraph::addMeasurement (drawio:2779-2826)
 *   D2/D3 cost, Euclidean gradient, Hess-vec .. QuadraticProblem inside PGOAgent::iterate (drawio:2513)
 *         f(X) = 1/2 sum_e w_e (kappa_e ||Y_j - Y_i R_e||^2 + tau_e ||p_j - p_i - Y_i t_e||^2)
 *         over the robot's private and shared edges; neighbour poses fixed.
 *   D4  Stiefel projection, Riemannian Hessian (Weingarten term), QF retraction
 *   D5  RTR outer step + preconditioned Steihaug-Toint tCG (ROPTLIB RTRNewton),
 *       optional Nesterov acceleration with periodic restart (orc_pgo_accel_*)
 *   D6  GNC_TLS weights + mu schedule ......... updateMeasurementWeights (drawio:2215, 2466-2469)
 *   D8  rounding to SE(3) in the anchor frame . getTrajectoryInGlobalFrame / publishTrajectory (drawio:2148)
 *   D9  concurrent / sequential round ......... runOnceSynchronous (drawio:2071, 2478-2481)
 * Edge-centric (scatter to both endpoints), deliberately unlike the GPU's
 * node-centric gather, so the two implementations are independent.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#include "../include/kmx_abi.h"

#define D 3

typedef struct {
  kmx_pgo_params P;
  int R;          /* robots */
  int* npose;     /* [R] */
  int64_t* poff;  /* [R+1] global pose offsets */
  int64_t ntot;
  int64_t m;
  int32_t *r1, *p1, *r2, *p2;
  double *Rm, *tv, *kappa, *tau, *w;
  uint8_t* fixed;
  int64_t** redges; /* per robot: edge ids touching it */
  int64_t* nredges;
  double* X;    /* ntot * 4r current iterate */
  double* nbr;  /* ntot * 4r neighbour snapshot (public poses) */
  double mu;
  /* Nesterov acceleration (P.acceleration): momentum V, the extrapolated
   * point Y of the current round, gamma, rounds since the last restart, and
   * whether Y has been formed for the upcoming round */
  double *V, *Yb;
  double gamma;
  int acc_k, acc_ready, acc_started;
  /* all-cores timing variant (orc_pgo_round_mt2): per robot, each local pose's
   * incidences (edge id << 1 | is_head), built on first use */
  int64_t** inc_ptr;
  int64_t** inc_e;
  /* per robot: the block update's work vectors, kept between rounds (12 of
   * n*4r doubles + S, Pinv), so a round does not page in fresh allocations */
  double** work;
} orc_pgo;

static int PS(const orc_pgo* h) { return 4 * h->P.r; } /* doubles per pose */

/* ---------------------------------------------------------------- setup -- */
void* orc_pgo_create(const kmx_pgo_params* p) {
  orc_pgo* h = (orc_pgo*)calloc(1, sizeof(orc_pgo));
  h->P = *p;
  h->mu = p->gnc_mu_init;
  return h;
}

static void free_graph(orc_pgo* h) {
  free(h->npose); free(h->poff);
  free(h->r1); free(h->p1); free(h->r2); free(h->p2);
  free(h->Rm); free(h->tv); free(h->kappa); free(h->tau); free(h->w); free(h->fixed);
  if (h->redges) for (int a = 0; a < h->R; ++a) free(h->redges[a]);
  free(h->redges); free(h->nredges); free(h->X); free(h->nbr); free(h->V); free(h->Yb);
  h->V = h->Yb = NULL;
  if (h->inc_ptr)
    for (int a = 0; a < h->R; ++a) { free(h->inc_ptr[a]); free(h->inc_e[a]); }
  free(h->inc_ptr); free(h->inc_e);
  h->inc_ptr = h->inc_e = NULL;
  if (h->work)
    for (int a = 0; a < h->R; ++a) free(h->work[a]);
  free(h->work);
  h->work = NULL;
}

void orc_pgo_destroy(void* vh) {
  orc_pgo* h = (orc_pgo*)vh;
  if (!h) return;
  free_graph(h);
  free(h);
}

int orc_pgo_set_graph(void* vh, int n_robots, const int32_t* n_poses, int64_t m,
                      const int32_t* r1, const int32_t* p1, const int32_t* r2,
                      const int32_t* p2, const double* R, const double* t,
                      const double* kappa, const double* tau, const double* w,
                      const uint8_t* fixed) {
  orc_pgo* h = (orc_pgo*)vh;
  free_graph(h);
  h->R = n_robots;
  h->npose = (int*)malloc(sizeof(int) * n_robots);
  h->poff = (int64_t*)malloc(sizeof(int64_t) * (n_robots + 1));
  h->poff[0] = 0;
  for (int a = 0; a < n_robots; ++a) {
    h->npose[a] = n_poses[a];
    h->poff[a + 1] = h->poff[a] + n_poses[a];
  }
  h->ntot = h->poff[n_robots];
  h->m = m;
#define DUP(dst, src, T, k) do { dst = (T*)malloc(sizeof(T) * (size_t)(k) + 1); memcpy(dst, src, sizeof(T) * (size_t)(k)); } while (0)
  DUP(h->r1, r1, int32_t, m); DUP(h->p1, p1, int32_t, m);
  DUP(h->r2, r2, int32_t, m); DUP(h->p2, p2, int32_t, m);
  DUP(h->Rm, R, double, 9 * m); DUP(h->tv, t, double, 3 * m);
  DUP(h->kappa, kappa, double, m); DUP(h->tau, tau, double, m);
  DUP(h->w, w, double, m); DUP(h->fixed, fixed, uint8_t, m);
#undef DUP
  for (int64_t e = 0; e < m; ++e) {
    if (r1[e] < 0 || r1[e] >= n_robots || r2[e] < 0 || r2[e] >= n_robots) return KMX_EINVAL;
    if (p1[e] < 0 || p1[e] >= n_poses[r1[e]] || p2[e] < 0 || p2[e] >= n_poses[r2[e]]) return KMX_EINVAL;
  }
  h->nredges = (int64_t*)calloc(n_robots, sizeof(int64_t));
  h->redges = (int64_t**)calloc(n_robots, sizeof(int64_t*));
  for (int64_t e = 0; e < m; ++e) {
    h->nredges[r1[e]]++;
    if (r2[e] != r1[e]) h->nredges[r2[e]]++;
  }
  for (int a = 0; a < n_robots; ++a) h->redges[a] = (int64_t*)malloc(sizeof(int64_t) * (h->nredges[a] + 1));
  int64_t* fill = (int64_t*)calloc(n_robots, sizeof(int64_t));
  for (int64_t e = 0; e < m; ++e) {
    h->redges[r1[e]][fill[r1[e]]++] = e;
    if (r2[e] != r1[e]) h->redges[r2[e]][fill[r2[e]]++] = e;
  }
  free(fill);
  h->X = (double*)calloc((size_t)h->ntot * PS(h) + 1, sizeof(double));
  h->nbr = (double*)calloc((size_t)h->ntot * PS(h) + 1, sizeof(double));
  if (h->P.acceleration) {
    h->V = (double*)calloc((size_t)h->ntot * PS(h) + 1, sizeof(double));
    h->Yb = (double*)calloc((size_t)h->ntot * PS(h) + 1, sizeof(double));
  }
  h->gamma = 0.0;
  h->acc_k = h->acc_ready = h->acc_started = 0;
  h->work = (double**)calloc(n_robots, sizeof(double*));
  return 0;
}

int orc_pgo_set_iterate(void* vh, int a, const double* X) {
  orc_pgo* h = (orc_pgo*)vh;
  memcpy(h->X + h->poff[a] * PS(h), X, sizeof(double) * (size_t)h->npose[a] * PS(h));
  h->gamma = 0.0; /* a new initial iterate restarts the acceleration */
  h->acc_k = h->acc_ready = h->acc_started = 0;
  return 0;
}
int orc_pgo_get_iterate(void* vh, int a, double* X) {
  orc_pgo* h = (orc_pgo*)vh;
  memcpy(X, h->X + h->poff[a] * PS(h), sizeof(double) * (size_t)h->npose[a] * PS(h));
  return 0;
}
/* neighbour table := current iterate of every robot (publishPublicPoses of all) */
int orc_pgo_refresh(void* vh) {
  orc_pgo* h = (orc_pgo*)vh;
  memcpy(h->nbr, h->X, sizeof(double) * (size_t)h->ntot * PS(h));
  return 0;
}
/* updateNeighborPoses: overwrite neighbour-table rows (robot, pose) with X rows */
int orc_pgo_set_nbr_rows(void* vh, int64_t n, const int32_t* robot, const int32_t* pose, const double* X) {
  orc_pgo* h = (orc_pgo*)vh;
  for (int64_t i = 0; i < n; ++i)
    memcpy(h->nbr + (h->poff[robot[i]] + pose[i]) * PS(h), X + i * PS(h), sizeof(double) * PS(h));
  return 0;
}
int orc_pgo_get_x_rows(void* vh, int64_t n, const int32_t* robot, const int32_t* pose, double* X) {
  orc_pgo* h = (orc_pgo*)vh;
  for (int64_t i = 0; i < n; ++i)
    memcpy(X + i * PS(h), h->X + (h->poff[robot[i]] + pose[i]) * PS(h), sizeof(double) * PS(h));
  return 0;
}
int orc_pgo_get_weights(void* vh, double* w) {
  orc_pgo* h = (orc_pgo*)vh;
  memcpy(w, h->w, sizeof(double) * h->m);
  return 0;
}
int orc_pgo_set_weights(void* vh, const double* w) {
  orc_pgo* h = (orc_pgo*)vh;
  memcpy(h->w, w, sizeof(double) * h->m);
  return 0;
}
double orc_pgo_get_mu(void* vh) { return ((orc_pgo*)vh)->mu; }
void orc_pgo_set_mu(void* vh, double mu) { ((orc_pgo*)vh)->mu = mu; }
int64_t orc_pgo_local_edges(void* vh, int a) { return ((orc_pgo*)vh)->nredges[a]; }

/* ------------------------------------------------------- block algebra -- */
typedef struct {
  orc_pgo* h;
  int a;       /* robot */
  int n;       /* poses in block */
  int r;
  int ps;      /* 4r */
  int64_t off; /* global offset */
  int inner;   /* threads inside the block update (1: the serial restatement) */
} blk;

static double dot(const double* x, const double* y, int64_t k) {
  double s = 0.0;
  for (int64_t i = 0; i < k; ++i) s += x[i] * y[i];
  return s;
}

/* Edge-centric evaluation of the block's quadratic model.
 * V: block vector (n*4r). If use_nbr, non-local endpoints take the neighbour
 * snapshot (cost / gradient); else they are 0 (Hessian-vector: the linear term
 * G of shared edges drops out). out = d/dV of 1/2 sum_e w(kappa|E_R|^2 + tau|E_t|^2). */
static double edge_eval(const blk* b, const double* V, int use_nbr, double* out) {
  orc_pgo* h = b->h;
  const int r = b->r, ps = b->ps;
  memset(out, 0, sizeof(double) * (size_t)b->n * ps);
  double cost = 0.0;
  double zero[4 * 8];
  memset(zero, 0, sizeof(zero));
  for (int64_t k = 0; k < h->nredges[b->a]; ++k) {
    const int64_t e = h->redges[b->a][k];
    const int ti = (h->r1[e] == b->a), hi = (h->r2[e] == b->a);
    const double* Vi;
    const double* Vj;
    if (ti) Vi = V + (int64_t)h->p1[e] * ps;
    else Vi = use_nbr ? h->nbr + (h->poff[h->r1[e]] + h->p1[e]) * ps : zero;
    if (hi) Vj = V + (int64_t)h->p2[e] * ps;
    else Vj = use_nbr ? h->nbr + (h->poff[h->r2[e]] + h->p2[e]) * ps : zero;
    const double* Rt = h->Rm + 9 * e;
    const double* tt = h->tv + 3 * e;
    const double wk = h->w[e] * h->kappa[e];
    const double wt = h->w[e] * h->tau[e];
    for (int a = 0; a < r; ++a) {
      const double* yi = Vi + 4 * a;
      const double* yj = Vj + 4 * a;
      double ER[3], Et;
      for (int c = 0; c < 3; ++c)
        ER[c] = yj[c] - (yi[0] * Rt[0 * 3 + c] + yi[1] * Rt[1 * 3 + c] + yi[2] * Rt[2 * 3 + c]);
      Et = yj[3] - yi[3] - (yi[0] * tt[0] + yi[1] * tt[1] + yi[2] * tt[2]);
      cost += 0.5 * (wk * (ER[0] * ER[0] + ER[1] * ER[1] + ER[2] * ER[2]) + wt * Et * Et);
      if (hi) {
        double* oj = out + (int64_t)h->p2[e] * ps + 4 * a;
        oj[0] += wk * ER[0]; oj[1] += wk * ER[1]; oj[2] += wk * ER[2];
        oj[3] += wt * Et;
      }
      if (ti) {
        double* oi = out + (int64_t)h->p1[e] * ps + 4 * a;
        for (int c = 0; c < 3; ++c)
          oi[c] -= wk * (ER[0] * Rt[c * 3 + 0] + ER[1] * Rt[c * 3 + 1] + ER[2] * Rt[c * 3 + 2]) + wt * Et * tt[c];
        oi[3] -= wt * Et;
      }
    }
  }
  return cost;
}

/* ---- all-cores timing variant (orc_pgo_round_mt2, bench.py's cpu_baseline
 * "all_cores"): the same block update with its O(m) and O(n) loops spread over
 * b->inner threads — edge_eval in gather form (each pose sums its incidences),
 * per-pose loops split, dot products by OpenMP reductions. The summation
 * order differs from the serial restatement (results agree to rounding), so it
 * is a timing leg only: parity is always checked against the serial form. */
static void build_incidences(orc_pgo* h) {
  if (h->inc_ptr) return;
  h->inc_ptr = (int64_t**)calloc(h->R, sizeof(int64_t*));
  h->inc_e = (int64_t**)calloc(h->R, sizeof(int64_t*));
  for (int a = 0; a < h->R; ++a) {
    const int n = h->npose[a];
    int64_t* ip = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t k = 0; k < h->nredges[a]; ++k) {
      const int64_t e = h->redges[a][k];
      if (h->r1[e] == a) ip[h->p1[e] + 1]++;
      if (h->r2[e] == a) ip[h->p2[e] + 1]++;
    }
    for (int i = 0; i < n; ++i) ip[i + 1] += ip[i];
    int64_t* ie = (int64_t*)malloc(sizeof(int64_t) * ((size_t)ip[n] + 1));
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * ((size_t)n + 1));
    memcpy(fill, ip, sizeof(int64_t) * (size_t)n);
    for (int64_t k = 0; k < h->nredges[a]; ++k) {
      const int64_t e = h->redges[a][k];
      if (h->r1[e] == a) ie[fill[h->p1[e]]++] = e << 1;
      if (h->r2[e] == a) ie[fill[h->p2[e]]++] = (e << 1) | 1;
    }
    free(fill);
    h->inc_ptr[a] = ip;
    h->inc_e[a] = ie;
  }
}

static double edge_eval_par(const blk* b, const double* V, int use_nbr, double* out) {
  orc_pgo* h = b->h;
  const int r = b->r, ps = b->ps, ra = b->a;
  const int64_t* ip = h->inc_ptr[ra];
  const int64_t* ie = h->inc_e[ra];
  double cost = 0.0;
#pragma omp parallel for num_threads(b->inner) schedule(static) reduction(+ : cost)
  for (int i = 0; i < b->n; ++i) {
    double acc[4 * 8];
    const double zero[4 * 8] = {0};
    memset(acc, 0, sizeof(acc));
    for (int64_t q = ip[i]; q < ip[i + 1]; ++q) {
      const int64_t e = ie[q] >> 1;
      const int head = (int)(ie[q] & 1);
      const int ti = (h->r1[e] == ra), hi = (h->r2[e] == ra);
      const double* Vi = ti ? V + (int64_t)h->p1[e] * ps
                            : (use_nbr ? h->nbr + (h->poff[h->r1[e]] + h->p1[e]) * ps : zero);
      const double* Vj = hi ? V + (int64_t)h->p2[e] * ps
                            : (use_nbr ? h->nbr + (h->poff[h->r2[e]] + h->p2[e]) * ps : zero);
      const double* Rt = h->Rm + 9 * e;
      const double* tt = h->tv + 3 * e;
      const double wk = h->w[e] * h->kappa[e], wt = h->w[e] * h->tau[e];
      const int owner = head ? !ti : 1;  /* each edge's cost once: at its tail if local, else its head */
      for (int a = 0; a < r; ++a) {
        const double* yi = Vi + 4 * a;
        const double* yj = Vj + 4 * a;
        double ER[3], Et;
        for (int c = 0; c < 3; ++c)
          ER[c] = yj[c] - (yi[0] * Rt[0 * 3 + c] + yi[1] * Rt[1 * 3 + c] + yi[2] * Rt[2 * 3 + c]);
        Et = yj[3] - yi[3] - (yi[0] * tt[0] + yi[1] * tt[1] + yi[2] * tt[2]);
        if (owner) cost += 0.5 * (wk * (ER[0] * ER[0] + ER[1] * ER[1] + ER[2] * ER[2]) + wt * Et * Et);
        double* o = acc + 4 * a;
        if (head) {
          o[0] += wk * ER[0]; o[1] += wk * ER[1]; o[2] += wk * ER[2];
          o[3] += wt * Et;
        } else {
          for (int c = 0; c < 3; ++c)
            o[c] -= wk * (ER[0] * Rt[c * 3 + 0] + ER[1] * Rt[c * 3 + 1] + ER[2] * Rt[c * 3 + 2]) + wt * Et * tt[c];
          o[3] -= wt * Et;
        }
      }
    }
    memcpy(out + (int64_t)i * ps, acc, sizeof(double) * (size_t)ps);
  }
  return cost;
}

static double EVAL(const blk* b, const double* V, int use_nbr, double* out) {
  return b->inner > 1 ? edge_eval_par(b, V, use_nbr, out) : edge_eval(b, V, use_nbr, out);
}

static double pdot(const blk* b, const double* x, const double* y, int64_t k) {
  if (b->inner <= 1) return dot(x, y, k);
  double s = 0.0;
#pragma omp parallel for num_threads(b->inner) schedule(static) reduction(+ : s)
  for (int64_t i = 0; i < k; ++i) s += x[i] * y[i];
  return s;
}

/* per pose: S = sym(Y^T G_Y) (3x3) */
static void sym_YtG(int r, const double* X, const double* G, double* S) {
  double M[9];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 3; ++k) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += X[4 * a + c] * G[4 * a + k];
      M[c * 3 + k] = s;
    }
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 3; ++k) S[c * 3 + k] = 0.5 * (M[c * 3 + k] + M[k * 3 + c]);
}

/* tangent projection at X of V (in place on out): out_Y = V_Y - Y sym(Y^T V_Y) */
static void proj_pose(int r, const double* X, const double* V, double* out) {
  double S[9];
  sym_YtG(r, X, V, S);
  for (int a = 0; a < r; ++a) {
    for (int c = 0; c < 3; ++c)
      out[4 * a + c] = V[4 * a + c] - (X[4 * a + 0] * S[0 * 3 + c] + X[4 * a + 1] * S[1 * 3 + c] + X[4 * a + 2] * S[2 * 3 + c]);
    out[4 * a + 3] = V[4 * a + 3];
  }
}

/* 4x4 diagonal block of Q for each pose of the block + shift, inverted. */
static void build_precond(const blk* b, double* Pinv /* n*16 */) {
  orc_pgo* h = b->h;
  double* Dm = (double*)calloc((size_t)b->n * 16, sizeof(double));
  if (b->inner > 1) {  /* gather: each pose sums its incidences in redges order, as the scatter does */
    const int64_t* ip = h->inc_ptr[b->a];
    const int64_t* ie = h->inc_e[b->a];
#pragma omp parallel for num_threads(b->inner) schedule(static)
    for (int i = 0; i < b->n; ++i) {
      double* M = Dm + (int64_t)i * 16;
      for (int64_t q = ip[i]; q < ip[i + 1]; ++q) {
        const int64_t e = ie[q] >> 1;
        const double wk = h->w[e] * h->kappa[e], wt = h->w[e] * h->tau[e];
        const double* tt = h->tv + 3 * e;
        if (!(ie[q] & 1)) {
          for (int ii = 0; ii < 3; ++ii) {
            for (int j = 0; j < 3; ++j) M[ii * 4 + j] += wt * tt[ii] * tt[j] + (ii == j ? wk : 0.0);
            M[ii * 4 + 3] += wt * tt[ii];
            M[3 * 4 + ii] += wt * tt[ii];
          }
          M[15] += wt;
        } else {
          M[0] += wk; M[5] += wk; M[10] += wk; M[15] += wt;
        }
      }
    }
  }
  for (int64_t k = 0; k < (b->inner > 1 ? 0 : h->nredges[b->a]); ++k) {
    const int64_t e = h->redges[b->a][k];
    const double wk = h->w[e] * h->kappa[e], wt = h->w[e] * h->tau[e];
    const double* tt = h->tv + 3 * e;
    if (h->r1[e] == b->a) { /* tail: w[[kI + tau t t^T, tau t],[tau t^T, tau]] */
      double* M = Dm + (int64_t)h->p1[e] * 16;
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) M[i * 4 + j] += wt * tt[i] * tt[j] + (i == j ? wk : 0.0);
        M[i * 4 + 3] += wt * tt[i];
        M[3 * 4 + i] += wt * tt[i];
      }
      M[15] += wt;
    }
    if (h->r2[e] == b->a) { /* head: w diag(kappa I, tau) */
      double* M = Dm + (int64_t)h->p2[e] * 16;
      M[0] += wk; M[5] += wk; M[10] += wk; M[15] += wt;
    }
  }
#pragma omp parallel for num_threads(b->inner) schedule(static) if (b->inner > 1)
  for (int i = 0; i < b->n; ++i) {
    double A[16], L[16] = {0}, Li[16] = {0};
    memcpy(A, Dm + (int64_t)i * 16, sizeof(A));
    for (int j = 0; j < 4; ++j) A[j * 5] += h->P.precond_shift;
    /* Cholesky A = L L^T */
    for (int j = 0; j < 4; ++j) {
      double s = A[j * 4 + j];
      for (int k = 0; k < j; ++k) s -= L[j * 4 + k] * L[j * 4 + k];
      L[j * 4 + j] = sqrt(s);
      for (int ii = j + 1; ii < 4; ++ii) {
        double t = A[ii * 4 + j];
        for (int k = 0; k < j; ++k) t -= L[ii * 4 + k] * L[j * 4 + k];
        L[ii * 4 + j] = t / L[j * 4 + j];
      }
    }
    /* L^{-1} by forward substitution */
    for (int c = 0; c < 4; ++c) {
      for (int ii = 0; ii < 4; ++ii) {
        double s = (ii == c) ? 1.0 : 0.0;
        for (int k = c; k < ii; ++k) s -= L[ii * 4 + k] * Li[k * 4 + c];
        Li[ii * 4 + c] = (ii < c) ? 0.0 : s / L[ii * 4 + ii];
      }
    }
    /* A^{-1} = L^{-T} L^{-1} */
    double* Pi = Pinv + (int64_t)i * 16;
    for (int x = 0; x < 4; ++x)
      for (int y = 0; y < 4; ++y) {
        double s = 0.0;
        for (int k = 0; k < 4; ++k) s += Li[k * 4 + x] * Li[k * 4 + y];
        Pi[x * 4 + y] = s;
      }
  }
  free(Dm);
}

typedef struct {
  double* Xb;   /* block iterate (points into h->X) */
  double* eg;   /* Euclidean gradient */
  double* g;    /* Riemannian gradient */
  double* S;    /* n*9 curvature sym(Y^T egrad_Y) */
  double* Pinv; /* n*16 */
  double* tmp;
} ctx;

static void rhess(const blk* b, const ctx* c, const double* V, double* out) {
  EVAL(b, V, 0, c->tmp); /* Euclidean Hess-vec Q V */
  const int r = b->r, ps = b->ps;
#pragma omp parallel for num_threads(b->inner) schedule(static) if (b->inner > 1)
  for (int i = 0; i < b->n; ++i) {
    double buf[32];
    const double* Xi = c->Xb + (int64_t)i * ps;
    const double* Vi = V + (int64_t)i * ps;
    const double* Hi = c->tmp + (int64_t)i * ps;
    const double* Si = c->S + (int64_t)i * 9;
    for (int a = 0; a < r; ++a) {
      for (int k = 0; k < 3; ++k)
        buf[4 * a + k] = Hi[4 * a + k] - (Vi[4 * a + 0] * Si[0 * 3 + k] + Vi[4 * a + 1] * Si[1 * 3 + k] + Vi[4 * a + 2] * Si[2 * 3 + k]);
      buf[4 * a + 3] = Hi[4 * a + 3];
    }
    proj_pose(r, Xi, buf, out + (int64_t)i * ps);
  }
}

static void precon(const blk* b, const ctx* c, const double* V, double* out) {
  const int r = b->r, ps = b->ps;
  if (!b->h->P.use_preconditioner) {
    memcpy(out, V, sizeof(double) * (size_t)b->n * ps);
    return;
  }
#pragma omp parallel for num_threads(b->inner) schedule(static) if (b->inner > 1)
  for (int i = 0; i < b->n; ++i) {
    double buf[32];
    const double* Vi = V + (int64_t)i * ps;
    const double* P = c->Pinv + (int64_t)i * 16;
    for (int a = 0; a < r; ++a)
      for (int k = 0; k < 4; ++k)
        buf[4 * a + k] = Vi[4 * a + 0] * P[0 * 4 + k] + Vi[4 * a + 1] * P[1 * 4 + k] + Vi[4 * a + 2] * P[2 * 4 + k] + Vi[4 * a + 3] * P[3 * 4 + k];
    proj_pose(r, c->Xb + (int64_t)i * ps, buf, out + (int64_t)i * ps);
  }
}

/* QF retraction per pose: Y' = qf(Y + V_Y) (modified Gram-Schmidt, positive
 * diagonal), p' = p + V_p. */
static void retract_pose(int r, const double* X, const double* V, double* out) {
  double A[8 * 3];
  for (int a = 0; a < r; ++a)
    for (int c = 0; c < 3; ++c) A[a * 3 + c] = X[4 * a + c] + V[4 * a + c];
  for (int c = 0; c < 3; ++c) {
    for (int k = 0; k < c; ++k) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += A[a * 3 + k] * A[a * 3 + c];
      for (int a = 0; a < r; ++a) A[a * 3 + c] -= s * A[a * 3 + k];
    }
    double nn = 0.0;
    for (int a = 0; a < r; ++a) nn += A[a * 3 + c] * A[a * 3 + c];
    const double inv = 1.0 / sqrt(nn);
    for (int a = 0; a < r; ++a) A[a * 3 + c] *= inv;
  }
  for (int a = 0; a < r; ++a) {
    for (int c = 0; c < 3; ++c) out[4 * a + c] = A[a * 3 + c];
    out[4 * a + 3] = X[4 * a + 3] + V[4 * a + 3];
  }
}

/* ------------------------------------------------- one-sync tCG (opt-in) -- */
/* KMX_TCG_FORM_ONESYNC: the same Steihaug-Toint iteration with every scalar of
 * step k+1 formed from ONE reduction after step k, so the GPU runs one kernel
 * (one grid-wide dependency) per step (pgo.hip body_step, DESIGN.md §5
 * "one-sync tCG"). With w = precon(H delta) (precon and H linear):
 *   r' = r + alpha H delta,   z' = z + alpha w,   Hz' = Hz + alpha Hw,
 *   delta' = -z' + beta delta,   H delta' = -Hz' + beta H delta
 *   <r',r'> = <r,r> + 2 alpha <r,H delta> + alpha^2 <H delta,H delta>
 *   <r',z'> = <r,z> + alpha (<r,w> + <H delta,z>) + alpha^2 <H delta,w>
 * so the Hessian is applied to w (step 0: to z_0; one gathered row per
 * incidence, as in the standard form's linearity H delta = -Hz + beta H
 * delta_old), and the reduction after step k carries <delta,H delta>, <r,z>,
 * <r,r>, <r,w> + <H delta,z>, <H delta,w>, <r,H delta>, <H delta,H delta>;
 * <r,z> and <r,r> are taken from the recurred vectors at every step (residual
 * replacement for the scalars), so the scalar recurrences are one step deep.
 * Pipelined CG in the sense of Ghysels & Vanroose (Parallel Computing 40,
 * 2014) and Chronopoulos & Gear (J. Comput. Appl. Math. 25, 1989), inside the
 * trust-region tests of ROPTLIB's tCG (the standard loop in block_update).
 * The vector recurrences are fused multiply-adds, as on the GPU. Parity with
 * the standard form is at convergence only; against the GPU's
 * same form, per round within rounding.
 * Hz and Hw use the work vectors the tCG does not touch (the trial point's
 * and the Euclidean gradient's). */
static int tcg_onesync(const blk* b, const ctx* c, double Delta, double norm_r0, double d_Pd, double* rr, double* z,
                       double* del, double* Hd, double* w, double* Hz, double* Hw, double* eta, double* Heta,
                       kmx_iter_stats* st, int* stop_out) {
  const orc_pgo* h = b->h;
  const int64_t N = (int64_t)b->n * b->ps;
  const double r_stop = norm_r0 * fmin(pow(norm_r0, h->P.tcg_theta), h->P.tcg_kappa);
  const int lin = (h->P.tcg_kappa < pow(norm_r0, h->P.tcg_theta)) ? 1 : 0;
  double e_Pe = 0.0, e_Pd = 0.0;
  int stop = KMX_TCG_MAX_ITER, j;
  rhess(b, c, z, Hz); /* step 0: delta_0 = -z_0, H delta_0 = -H z_0 */
  for (int64_t k = 0; k < N; ++k) Hd[k] = -Hz[k];
  precon(b, c, Hd, w);
  for (j = 1; j <= h->P.tcg_max_iterations; ++j) {
    st->hessvecs++;
    /* the step's one reduction */
    const double d_Hd = pdot(b, del, Hd, N), zr = pdot(b, rr, z, N), rr2 = pdot(b, rr, rr, N);
    const double s1 = pdot(b, rr, w, N) + pdot(b, Hd, z, N), s2 = pdot(b, Hd, w, N);
    const double s3 = pdot(b, rr, Hd, N), s4 = pdot(b, Hd, Hd, N);
    const double alpha = zr / d_Hd;
    const double e_Pe_new = e_Pe + 2.0 * alpha * e_Pd + alpha * alpha * d_Pd;
    if (d_Hd <= 0.0 || e_Pe_new >= Delta * Delta) {
      const double tau = (-e_Pd + sqrt(e_Pd * e_Pd + d_Pd * (Delta * Delta - e_Pe))) / d_Pd;
      for (int64_t k = 0; k < N; ++k) { eta[k] += tau * del[k]; Heta[k] += tau * Hd[k]; rr[k] = fma(tau, Hd[k], rr[k]); }
      stop = d_Hd <= 0.0 ? KMX_TCG_NEGATIVE_CURVATURE : KMX_TCG_EXCEEDED_TR;
      break;
    }
    e_Pe = e_Pe_new;
    for (int64_t k = 0; k < N; ++k) {
      eta[k] += alpha * del[k];
      Heta[k] += alpha * Hd[k];
    }
    const double rr_new = fmax(rr2 + 2.0 * alpha * s3 + alpha * alpha * s4, 0.0);
    const double zr_new = zr + alpha * s1 + alpha * alpha * s2;
    if (sqrt(rr_new) <= r_stop) {
      for (int64_t k = 0; k < N; ++k) rr[k] = fma(alpha, Hd[k], rr[k]);
      stop = lin ? KMX_TCG_LINEAR : KMX_TCG_SUPERLINEAR;
      break;
    }
    if (j == h->P.tcg_max_iterations) {
      for (int64_t k = 0; k < N; ++k) rr[k] = fma(alpha, Hd[k], rr[k]);
      break;
    }
    const double beta = zr_new / zr;
    rhess(b, c, w, Hw);
    for (int64_t k = 0; k < N; ++k) {
      rr[k] = fma(alpha, Hd[k], rr[k]);
      z[k] = fma(alpha, w[k], z[k]);
      Hz[k] = fma(alpha, Hw[k], Hz[k]);
      del[k] = fma(beta, del[k], -z[k]);
      Hd[k] = fma(beta, Hd[k], -Hz[k]);
    }
    precon(b, c, Hd, w);
    e_Pd = beta * (e_Pd + alpha * d_Pd);
    d_Pd = zr_new + beta * beta * d_Pd;
  }
  *stop_out = stop;
  return j;
}

/* --------------------------------------------------------- block update -- */
static void block_update(orc_pgo* h, int a, kmx_iter_stats* st, int inner) {
  blk b = {h, a, h->npose[a], h->P.r, PS(h), h->poff[a], inner};
  const int64_t N = (int64_t)b.n * b.ps;
  ctx c;
  c.Xb = h->X + b.off * b.ps;
  /* work vectors: 12 of N doubles, S (n*9) and Pinv (n*16), one allocation per
   * robot kept across rounds (h->work; robots write only their own) */
  const int64_t NP = N + 1;
  double* wk_ = h->work[a];
  if (!wk_) wk_ = h->work[a] = (double*)malloc(sizeof(double) * (size_t)(12 * NP + (int64_t)b.n * 25 + 2));
  c.eg = wk_;
  c.g = wk_ + NP;
  c.tmp = wk_ + 2 * NP;
  double* eta = wk_ + 3 * NP;
  double* Heta = wk_ + 4 * NP;
  double* rr = wk_ + 5 * NP;
  double* z = wk_ + 6 * NP;
  double* del = wk_ + 7 * NP;
  double* Hd = wk_ + 8 * NP;
  double* Xt = wk_ + 9 * NP;
  double* X0 = wk_ + 10 * NP;
  c.S = wk_ + 12 * NP;
  c.Pinv = c.S + (int64_t)b.n * 9 + 1;
  memcpy(X0, c.Xb, sizeof(double) * N);
  build_precond(&b, c.Pinv);

  memset(st, 0, sizeof(*st));
  st->updated = 1;
  st->edges = h->nredges[a];
  double Delta = h->P.rtr_initial_radius;
  if (h->P.method == KMX_METHOD_RGD) {
    /* dpgo QuadraticOptimizer::gradientDescent (ROptMethod RGD) [U: dpgo not vendored]:
     * X <- Retr_X(-s * precon(rgrad)), always accepted; the same gradient-norm skip as RTR */
    const double f = EVAL(&b, c.Xb, 1, c.eg);
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
    for (int i = 0; i < b.n; ++i) {
      sym_YtG(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.S + (int64_t)i * 9);
      proj_pose(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.g + (int64_t)i * b.ps);
    }
    const double gn = sqrt(pdot(&b, c.g, c.g, N));
    st->f_init = f;
    st->gradnorm_init = gn;
    st->f_final = f;
    if (gn < h->P.gradnorm_tol) {
      st->tcg_stop = KMX_TCG_SKIPPED;
    } else {
      precon(&b, &c, c.g, z);
      const double s = h->P.rgd_stepsize;
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
      for (int64_t k = 0; k < N; ++k) eta[k] = -s * z[k];
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
      for (int i = 0; i < b.n; ++i)
        retract_pose(b.r, c.Xb + (int64_t)i * b.ps, eta + (int64_t)i * b.ps, Xt + (int64_t)i * b.ps);
      st->f_final = EVAL(&b, Xt, 1, c.tmp);
      memcpy(c.Xb, Xt, sizeof(double) * N);
      st->accepted = 1;
    }
  }
  for (int it = 0; it < (h->P.method == KMX_METHOD_RGD ? 0 : h->P.rtr_iterations); ++it) {
    double f = EVAL(&b, c.Xb, 1, c.eg);
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
    for (int i = 0; i < b.n; ++i) {
      sym_YtG(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.S + (int64_t)i * 9);
      proj_pose(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.g + (int64_t)i * b.ps);
    }
    const double gn = sqrt(pdot(&b, c.g, c.g, N));
    if (it == 0) { st->f_init = f; st->gradnorm_init = gn; }
    st->f_final = f;
    if (gn < h->P.gradnorm_tol) {
      st->tcg_stop = KMX_TCG_SKIPPED;
      st->tcg_iterations = 0;
      st->accepted = 0;
      break;
    }
    /* ---- preconditioned Steihaug-Toint truncated CG ---- */
    memset(eta, 0, sizeof(double) * N);
    memset(Heta, 0, sizeof(double) * N);
    memcpy(rr, c.g, sizeof(double) * N);
    double e_Pe = 0.0, e_Pd = 0.0;
    const double norm_r0 = sqrt(pdot(&b, rr, rr, N));
    precon(&b, &c, rr, z);
    double z_r = pdot(&b, z, rr, N);
    double d_Pd = z_r;
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
    for (int64_t k = 0; k < N; ++k) del[k] = -z[k];
    int stop = KMX_TCG_MAX_ITER, j;
    if (h->P.tcg_form != KMX_TCG_FORM_STANDARD) { /* ONESYNC, and RESIDENT (same arithmetic) */
      j = tcg_onesync(&b, &c, Delta, norm_r0, d_Pd, rr, z, del, Hd, wk_ + 11 * NP, Xt, c.eg, eta, Heta, st, &stop);
    } else
    for (j = 1; j <= h->P.tcg_max_iterations; ++j) {
      rhess(&b, &c, del, Hd);
      st->hessvecs++;
      const double d_Hd = pdot(&b, del, Hd, N);
      const double alpha = z_r / d_Hd;
      const double e_Pe_new = e_Pe + 2.0 * alpha * e_Pd + alpha * alpha * d_Pd;
      if (d_Hd <= 0.0 || e_Pe_new >= Delta * Delta) {
        const double tau = (-e_Pd + sqrt(e_Pd * e_Pd + d_Pd * (Delta * Delta - e_Pe))) / d_Pd;
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
        for (int64_t k = 0; k < N; ++k) { eta[k] += tau * del[k]; Heta[k] += tau * Hd[k]; }
        stop = d_Hd <= 0.0 ? KMX_TCG_NEGATIVE_CURVATURE : KMX_TCG_EXCEEDED_TR;
        break;
      }
      e_Pe = e_Pe_new;
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
      for (int64_t k = 0; k < N; ++k) {
        eta[k] += alpha * del[k];
        Heta[k] += alpha * Hd[k];
        rr[k] += alpha * Hd[k];
      }
      const double norm_r = sqrt(pdot(&b, rr, rr, N));
      if (norm_r <= norm_r0 * fmin(pow(norm_r0, h->P.tcg_theta), h->P.tcg_kappa)) {
        stop = (h->P.tcg_kappa < pow(norm_r0, h->P.tcg_theta)) ? KMX_TCG_LINEAR : KMX_TCG_SUPERLINEAR;
        break;
      }
      if (j == h->P.tcg_max_iterations) break;
      precon(&b, &c, rr, z);
      const double zold_rold = z_r;
      z_r = pdot(&b, z, rr, N);
      const double beta = z_r / zold_rold;
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
      for (int64_t k = 0; k < N; ++k) del[k] = -z[k] + beta * del[k];
      e_Pd = beta * (e_Pd + alpha * d_Pd);
      d_Pd = z_r + beta * beta * d_Pd;
    }
    st->tcg_iterations = j > h->P.tcg_max_iterations ? h->P.tcg_max_iterations : j;
    st->tcg_stop = stop;
    /* ---- trial point, model decrease, acceptance ---- */
#pragma omp parallel for num_threads(b.inner) schedule(static) if (b.inner > 1)
    for (int i = 0; i < b.n; ++i)
      retract_pose(b.r, c.Xb + (int64_t)i * b.ps, eta + (int64_t)i * b.ps, Xt + (int64_t)i * b.ps);
    const double ft = EVAL(&b, Xt, 1, c.tmp);
    const double model_dec = -(pdot(&b, eta, c.g, N) + 0.5 * pdot(&b, eta, Heta, N));
    const double rho = (model_dec > 0.0) ? (f - ft) / model_dec : -1.0;
    const int boundary = (stop == KMX_TCG_NEGATIVE_CURVATURE || stop == KMX_TCG_EXCEEDED_TR);
    if (!(rho >= 0.25)) Delta *= 0.25;
    else if (rho > 0.75 && boundary) Delta = fmin(2.0 * Delta, h->P.rtr_max_radius);
    st->rho = rho;
    st->radius = Delta;
    if (rho > h->P.rtr_accept_rho) {
      memcpy(c.Xb, Xt, sizeof(double) * N);
      st->accepted = 1;
      st->f_final = ft;
    } else {
      st->accepted = 0;
      st->f_final = f;
    }
  }
  double ch = 0.0;
  for (int64_t k = 0; k < N; ++k) { const double dd = c.Xb[k] - X0[k]; ch += dd * dd; }
  st->rel_change = sqrt(ch / (double)b.n);
}

/* ------------------------------------------------ Nesterov acceleration -- */
/* dpgo's accelerated RBCD (RBCD++, Tian et al. T-RO 2021 Alg. 3/4; PGOAgent
 * updateGamma / updateAlpha / updateY / updateV / restartNesterovAcceleration
 * [U: dpgo source not vendored]) for the concurrent schedule, N = team size:
 *   gamma' = (1 + sqrt(1 + 4 N^2 gamma^2)) / (2 N),  alpha = 1 / (gamma' N)
 *   Y      = Proj((1 - alpha) X + alpha V)        (before the round: the
 *            public poses and the block update start from Y)
 *   X'     = block update from Y
 *   V      = Proj(V + gamma' (X' - Y))
 * and every restart_interval rounds V = X', gamma = 0 (else gamma = gamma').
 * Proj: the rotation block to the Stiefel manifold by its polar factor
 * M (M^T M)^(-1/2) (the SVD's U V^T), translation unchanged. */
static void jacobi3(double A[9], double V[9]);
static void proj_stiefel(int r, const double* M, double* out) {
  double G[9], W[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += M[4 * a + i] * M[4 * a + j];
      G[i * 3 + j] = s;
    }
  jacobi3(G, W);
  double isq[3];
  for (int k = 0; k < 3; ++k) isq[k] = 1.0 / sqrt(G[k * 4]);
  for (int a = 0; a < r; ++a) {
    double c[3];
    for (int k = 0; k < 3; ++k)
      c[k] = (M[4 * a + 0] * W[0 * 3 + k] + M[4 * a + 1] * W[1 * 3 + k] + M[4 * a + 2] * W[2 * 3 + k]) * isq[k];
    for (int j = 0; j < 3; ++j) out[4 * a + j] = c[0] * W[j * 3 + 0] + c[1] * W[j * 3 + 1] + c[2] * W[j * 3 + 2];
    out[4 * a + 3] = M[4 * a + 3];
  }
}

static double accel_gamma_next(const orc_pgo* h) {
  const double N = (double)h->R;
  return (1.0 + sqrt(1.0 + 4.0 * N * N * h->gamma * h->gamma)) / (2.0 * N);
}

/* updateGamma / updateAlpha / updateY for the robots in `mask` (NULL: all);
 * X := Y. A no-op when Y is already formed for this round. */
int orc_pgo_accel_pre(void* vh, const uint8_t* mask) {
  orc_pgo* h = (orc_pgo*)vh;
  if (!h->P.acceleration || h->acc_ready) return 0;
  const int ps = PS(h), r = h->P.r;
  if (!h->acc_started) {
    memcpy(h->V, h->X, sizeof(double) * (size_t)h->ntot * ps);
    h->acc_started = 1;
  }
  const double g = accel_gamma_next(h), alpha = 1.0 / (g * (double)h->R);
  double M[4 * 8];
  for (int a = 0; a < h->R; ++a) {
    if (mask && !mask[a]) continue;
    for (int64_t i = h->poff[a]; i < h->poff[a + 1]; ++i) {
      const double* x = h->X + i * ps;
      const double* v = h->V + i * ps;
      for (int k = 0; k < ps; ++k) M[k] = (1.0 - alpha) * x[k] + alpha * v[k];
      proj_stiefel(r, M, h->Yb + i * ps);
      memcpy(h->X + i * ps, h->Yb + i * ps, sizeof(double) * ps);
    }
  }
  h->acc_ready = 1;
  return 0;
}

/* updateV after the block updates, then the periodic restart. */
int orc_pgo_accel_post(void* vh, const uint8_t* mask) {
  orc_pgo* h = (orc_pgo*)vh;
  if (!h->P.acceleration || !h->acc_ready) return 0;
  const int ps = PS(h), r = h->P.r;
  const double g = accel_gamma_next(h);
  const int restart = h->P.restart_interval > 0 && (h->acc_k + 1) % h->P.restart_interval == 0;
  double M[4 * 8];
  for (int a = 0; a < h->R; ++a) {
    if (mask && !mask[a]) continue;
    for (int64_t i = h->poff[a]; i < h->poff[a + 1]; ++i) {
      double* v = h->V + i * ps;
      const double* x = h->X + i * ps;
      if (restart) {
        memcpy(v, x, sizeof(double) * ps);
        continue;
      }
      const double* y = h->Yb + i * ps;
      for (int k = 0; k < ps; ++k) M[k] = v[k] + g * (x[k] - y[k]);
      proj_stiefel(r, M, v);
    }
  }
  h->gamma = restart ? 0.0 : g;
  h->acc_k = restart ? 0 : h->acc_k + 1;
  h->acc_ready = 0;
  return 0;
}

double orc_pgo_accel_gamma(void* vh) { return ((orc_pgo*)vh)->gamma; }

/* One RBCD round: neighbour table = iterate at round start (every robot
 * published after its previous iterate), then every active robot updates its
 * block against that table. */
int orc_pgo_round(void* vh, const uint8_t* active, kmx_iter_stats* stats) {
  orc_pgo* h = (orc_pgo*)vh;
  orc_pgo_accel_pre(h, active);
  orc_pgo_refresh(h);
  for (int a = 0; a < h->R; ++a) {
    kmx_iter_stats st;
    memset(&st, 0, sizeof(st));
    if (active[a]) block_update(h, a, &st, 1);
    if (stats) stats[a] = st;
  }
  orc_pgo_accel_post(h, active);
  return 0;
}

/* Round against the neighbour table as last installed (no refresh): the
 * multi-process form, where neighbour rows arrive by exchange. */
int orc_pgo_round_nbr(void* vh, const uint8_t* active, kmx_iter_stats* stats) {
  orc_pgo* h = (orc_pgo*)vh;
  orc_pgo_accel_pre(h, active); /* normally already formed before the exchange */
  for (int a = 0; a < h->R; ++a) {
    kmx_iter_stats st;
    memset(&st, 0, sizeof(st));
    if (active[a]) block_update(h, a, &st, 1);
    if (stats) stats[a] = st;
  }
  orc_pgo_accel_post(h, active);
  return 0;
}

/* Same round with the robot blocks spread over `threads` OpenMP threads (one
 * block per thread at a time; blocks write disjoint iterate slices). This is
 * the all-cores CPU baseline of BASELINE.md §2.4. */
int orc_pgo_round_mt(void* vh, const uint8_t* active, kmx_iter_stats* stats, int threads) {
  orc_pgo* h = (orc_pgo*)vh;
  if (h->P.acceleration) return KMX_EUNSUP;
  orc_pgo_refresh(h);
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
  for (int a = 0; a < h->R; ++a) {
    kmx_iter_stats st;
    memset(&st, 0, sizeof(st));
    if (active[a]) block_update(h, a, &st, 1);
    if (stats) stats[a] = st;
  }
  return 0;
}

/* The all-cores timing variant: blocks over `outer` threads, each block update
 * over `inner` more (nested), e.g. 8 blocks x 2 on a 16-core share. Results
 * agree with orc_pgo_round to rounding, not bit for bit (see edge_eval_par). */
int orc_pgo_round_mt2(void* vh, const uint8_t* active, kmx_iter_stats* stats, int outer, int inner) {
  orc_pgo* h = (orc_pgo*)vh;
  if (h->P.acceleration) return KMX_EUNSUP;
  build_incidences(h);
  omp_set_max_active_levels(2);
  orc_pgo_refresh(h);
#pragma omp parallel for schedule(dynamic, 1) num_threads(outer) if (outer > 1)
  for (int a = 0; a < h->R; ++a) {
    kmx_iter_stats st;
    memset(&st, 0, sizeof(st));
    if (active[a]) block_update(h, a, &st, inner);
    if (stats) stats[a] = st;
  }
  return 0;
}

/* ------------------------------------------------------------- GNC-TLS -- */
/* RobustCost::weight for GNC_TLS (Yang et al. 2020 eq. 14), on squared residual. */
static double gnc_tls_weight(double rSq, double mu, double barc) {
  const double barcSq = barc * barc;
  const double upper = (mu + 1.0) / mu * barcSq;
  const double lower = mu / (mu + 1.0) * barcSq;
  if (rSq >= upper) return 0.0;
  if (rSq <= lower) return 1.0;
  return sqrt(barcSq * mu * (mu + 1.0) / rSq) - mu;
}

/* r^2 = kappa ||Y_j - Y_i R||^2 + tau ||p_j - p_i - Y_i t||^2 on lifted poses */
static double residual_sq(const orc_pgo* h, int64_t e, const double* Xi, const double* Xj) {
  const double* Rt = h->Rm + 9 * e;
  const double* tt = h->tv + 3 * e;
  double sR = 0.0, sT = 0.0;
  for (int a = 0; a < h->P.r; ++a) {
    const double* yi = Xi + 4 * a;
    const double* yj = Xj + 4 * a;
    for (int c = 0; c < 3; ++c) {
      const double er = yj[c] - (yi[0] * Rt[0 * 3 + c] + yi[1] * Rt[1 * 3 + c] + yi[2] * Rt[2 * 3 + c]);
      sR += er * er;
    }
    const double et = yj[3] - yi[3] - (yi[0] * tt[0] + yi[1] * tt[1] + yi[2] * tt[2]);
    sT += et * et;
  }
  return h->kappa[e] * sR + h->tau[e] * sT;
}

int orc_pgo_update_weights(void* vh, double* mu_used) {
  orc_pgo* h = (orc_pgo*)vh;
  if (mu_used) *mu_used = h->mu;
  if (h->P.robust_cost != KMX_COST_GNC_TLS) return 0;
  const int ps = PS(h);
  for (int64_t e = 0; e < h->m; ++e) {
    if (h->fixed[e]) continue;
    const double* Xi = h->X + (h->poff[h->r1[e]] + h->p1[e]) * ps;
    const double* Xj = h->X + (h->poff[h->r2[e]] + h->p2[e]) * ps;
    h->w[e] = gnc_tls_weight(residual_sq(h, e, Xi, Xj), h->mu, h->P.gnc_barc);
  }
  h->mu *= h->P.gnc_mu_step;
  return 0;
}

/* Owner's-view sweep for a process that holds only the robots in `local`:
 * edges owned by a local robot (owner = min(r1, r2), drawio:2198); the owner's
 * endpoint from its iterate, the other robot's from the neighbour table. */
int orc_pgo_update_weights_owned(void* vh, const uint8_t* local, double* mu_used) {
  orc_pgo* h = (orc_pgo*)vh;
  if (mu_used) *mu_used = h->mu;
  if (h->P.robust_cost != KMX_COST_GNC_TLS) return 0;
  const int ps = PS(h);
  for (int64_t e = 0; e < h->m; ++e) {
    if (h->fixed[e]) continue;
    const int owner = h->r1[e] < h->r2[e] ? h->r1[e] : h->r2[e];
    if (!local[owner]) continue;
    const double* Xi = (h->r1[e] == owner ? h->X : h->nbr) + (h->poff[h->r1[e]] + h->p1[e]) * ps;
    const double* Xj = (h->r2[e] == owner ? h->X : h->nbr) + (h->poff[h->r2[e]] + h->p2[e]) * ps;
    h->w[e] = gnc_tls_weight(residual_sq(h, e, Xi, Xj), h->mu, h->P.gnc_barc);
  }
  h->mu *= h->P.gnc_mu_step;
  return 0;
}

/* Sweep of a process that holds only the robots in `local`, as the HIP
 * handle does: every non-fixed edge with a local endpoint, local endpoints
 * from the iterate, foreign ones from the neighbour table. A shared loop
 * closure is evaluated on both robots' processes from the same two rows, so
 * both get the owner's weight (owner = min(r1, r2), drawio:2195-2198). */
int orc_pgo_update_weights_local(void* vh, const uint8_t* local, double* mu_used) {
  orc_pgo* h = (orc_pgo*)vh;
  if (mu_used) *mu_used = h->mu;
  if (h->P.robust_cost != KMX_COST_GNC_TLS) return 0;
  const int ps = PS(h);
  for (int64_t e = 0; e < h->m; ++e) {
    if (h->fixed[e]) continue;
    if (!local[h->r1[e]] && !local[h->r2[e]]) continue;
    const double* Xi = (local[h->r1[e]] ? h->X : h->nbr) + (h->poff[h->r1[e]] + h->p1[e]) * ps;
    const double* Xj = (local[h->r2[e]] ? h->X : h->nbr) + (h->poff[h->r2[e]] + h->p2[e]) * ps;
    h->w[e] = gnc_tls_weight(residual_sq(h, e, Xi, Xj), h->mu, h->P.gnc_barc);
  }
  h->mu *= h->P.gnc_mu_step;
  return 0;
}

/* ------------------------------------------------------------ rounding -- */
/* symmetric 3x3 Jacobi eigen-decomposition (cyclic, fixed sweeps) */
static void jacobi3(double A[9], double V[9]) {
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
        for (int k = 0; k < 3; ++k) { /* A = J^T A J */
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

/* nearest rotation: R = U diag(1,1,sign det M) V^T via M^T M = V L V^T */
static void proj_so3(const double M[9], double Rout[9]) {
  double A[9], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += M[k * 3 + i] * M[k * 3 + j];
      A[i * 3 + j] = s;
    }
  jacobi3(A, V);
  const double det = M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
  int kmin = 0;
  for (int k = 1; k < 3; ++k) if (A[k * 4] < A[kmin * 4]) kmin = k;
  for (int i = 0; i < 9; ++i) Rout[i] = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double sig = sqrt(fmax(A[k * 4], 0.0));
    double u[3];
    for (int i = 0; i < 3; ++i) u[i] = (M[i * 3 + 0] * V[0 * 3 + k] + M[i * 3 + 1] * V[1 * 3 + k] + M[i * 3 + 2] * V[2 * 3 + k]) / sig;
    const double s = (k == kmin && det < 0.0) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rout[i * 3 + j] += s * u[i] * V[j * 3 + k];
  }
}

int orc_pgo_get_trajectory(void* vh, int a, const double* anchor, double* out) {
  orc_pgo* h = (orc_pgo*)vh;
  const int r = h->P.r, ps = PS(h);
  for (int i = 0; i < h->npose[a]; ++i) {
    const double* Xi = h->X + (h->poff[a] + i) * ps;
    double M[9];
    for (int x = 0; x < 3; ++x) {
      for (int y = 0; y < 3; ++y) {
        double s = 0.0;
        for (int k = 0; k < r; ++k) s += anchor[4 * k + x] * Xi[4 * k + y];
        M[x * 3 + y] = s;
      }
      double s = 0.0;
      for (int k = 0; k < r; ++k) s += anchor[4 * k + x] * (Xi[4 * k + 3] - anchor[4 * k + 3]);
      out[(int64_t)i * 12 + 9 + x] = s;
    }
    proj_so3(M, out + (int64_t)i * 12);
  }
  return 0;
}

/* ------------------------------------------------ primitive evaluation -- */
int orc_pgo_eval(void* vh, int a, int mode, const double* V, double* out, double* scalar) {
  orc_pgo* h = (orc_pgo*)vh;
  blk b = {h, a, h->npose[a], h->P.r, PS(h), h->poff[a], 1};
  const int64_t N = (int64_t)b.n * b.ps;
  ctx c;
  c.Xb = h->X + b.off * b.ps;
  c.eg = (double*)malloc(sizeof(double) * N + 8);
  c.g = (double*)malloc(sizeof(double) * N + 8);
  c.S = (double*)malloc(sizeof(double) * (size_t)b.n * 9 + 8);
  c.Pinv = (double*)malloc(sizeof(double) * (size_t)b.n * 16 + 8);
  c.tmp = (double*)malloc(sizeof(double) * N + 8);
  double s = 0.0;
  if (mode == KMX_EVAL_COST_EGRAD) {
    s = edge_eval(&b, V, 1, out);
  } else if (mode == KMX_EVAL_EHESS) {
    edge_eval(&b, V, 0, out);
    s = dot(V, out, N);
  } else {
    edge_eval(&b, c.Xb, 1, c.eg);
    for (int i = 0; i < b.n; ++i) {
      sym_YtG(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.S + (int64_t)i * 9);
      proj_pose(b.r, c.Xb + (int64_t)i * b.ps, c.eg + (int64_t)i * b.ps, c.g + (int64_t)i * b.ps);
    }
    build_precond(&b, c.Pinv);
    if (mode == KMX_EVAL_RGRAD) {
      memcpy(out, c.g, sizeof(double) * N);
      s = dot(out, out, N);
    } else if (mode == KMX_EVAL_RHESS) {
      rhess(&b, &c, V, out);
      s = dot(V, out, N);
    } else if (mode == KMX_EVAL_PRECON) {
      precon(&b, &c, V, out);
      s = dot(V, out, N);
    } else if (mode == KMX_EVAL_RETRACT) {
      for (int i = 0; i < b.n; ++i)
        retract_pose(b.r, c.Xb + (int64_t)i * b.ps, V + (int64_t)i * b.ps, out + (int64_t)i * b.ps);
    }
  }
  if (scalar) *scalar = s;
  free(c.eg); free(c.g); free(c.S); free(c.Pinv); free(c.tmp);
  return 0;
}
