/*
 * kmx_abi.h — the C ABI of the MI355X-native dpgo / Kimera-Multi-LCD hot path.
 *
 * This is the drop-in boundary. Every entry point replaces the
 * bottom of one reference interface. The reference sources are NOT vendored in
 * /root/reference (SURVEY.md §0 finding 1); the interfaces are cited from the
 * fork author's call-flow diagram `images/kimera-multi.drawio` (drawio:N) and the
 * in-tree parameter files.
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no C++/torch types.
 *   - Every function returns int: 0 = ok, < 0 = error (KMX_E*). kmx_last_error()
 *     returns a thread-local message for the last failing call.
 *   - Host arrays are owned by the caller and only read/written during the call.
 *     Device buffers are owned by the handle, except the exchange buffers of
 *     kmx_pgo_pack_public / kmx_pgo_unpack_public, which are caller-owned device
 *     pointers (e.g. torch tensors used with RCCL).
 *   - A handle is not thread-safe. All of its device work is enqueued on one HIP
 *     stream (its own, or the caller's via kmx_pgo_set_stream); calls that return
 *     host data synchronise that stream.
 *   - Lifted pose layout: pose i of a robot block is X_i = [Y_i p_i] in
 *     R^{r x (d+1)}, stored row-major: X[i*4r + a*4 + c], a < r, c < 4 (c = 3 is p).
 *     d = 3 is fixed.
 */
#ifndef KMX_ABI_H
#define KMX_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMX_ABI_VERSION 8

/* error codes */
#define KMX_OK 0
#define KMX_EINVAL (-1)   /* bad argument / shape */
#define KMX_EHIP (-2)     /* HIP runtime error */
#define KMX_ESTATE (-3)   /* call out of order (e.g. iterate before set_graph) */
#define KMX_ENOMEM (-4)
#define KMX_EUNSUP (-5)   /* unsupported parameter value (e.g. relaxation rank) */
#define KMX_ETIMEOUT (-6) /* a bounded wait expired (kmx_pgo_sync_timeout)       */

const char* kmx_last_error(void);
int kmx_abi_version(void);
/* number of visible HIP devices (0 when no GPU). Does not create a context. */
int kmx_device_count(int* out);

/* ------------------------------------------------------------------------- */
/* dpgo: distributed pose-graph optimisation (RBCD on lifted SE(3) with GNC)  */
/* ------------------------------------------------------------------------- */

/* Robust cost selector. Reference: dpgo RobustCostType, selector `GNC_TLS`
 * (drawio:2175). Only L2 and GNC_TLS are on the hot path. */
#define KMX_COST_L2 0
#define KMX_COST_GNC_TLS 1

/* Local solver of a block update (dpgo ROptParameters::ROptMethod). */
#define KMX_METHOD_RTR 0 /* Riemannian trust region + truncated CG (the default) */
#define KMX_METHOD_RGD 1 /* one preconditioned Riemannian gradient step, fixed step size */

/* Block-update schedule across robots (SURVEY.md §0 finding 6). */
#define KMX_SCHEDULE_SEQUENTIAL 0 /* one executing robot per round (dpgo_ros sync) */
#define KMX_SCHEDULE_CONCURRENT 1 /* every active robot per round (Jacobi)        */

/* Mirrors dpgo PGOAgentParameters + ROptParameters + RobustCostParameters
 * (drawio:2457-2513). Values in comments are the defaults kmx.dpgo uses. */
typedef struct kmx_pgo_params {
  int d;                    /* 3 (only 3 is supported)                        */
  int r;                    /* relaxation rank, 3..8 (5)                      */
  int rtr_iterations;       /* RTR outer iterations per block update (1)      */
  int tcg_max_iterations;   /* truncated-CG inner iterations (10)             */
  double tcg_kappa;         /* tCG linear-convergence target (0.1)            */
  double tcg_theta;         /* tCG superlinear exponent (1.0)                 */
  double rtr_initial_radius;/* trust radius at the start of a block update (100) */
  double rtr_max_radius;    /* (1e4)                                          */
  double rtr_accept_rho;    /* accept the step if rho > this (0.1)            */
  double gradnorm_tol;      /* skip the block update if ||grad|| < tol (1e-2) */
  int use_preconditioner;   /* block-Jacobi preconditioner on/off (1)         */
  double precond_shift;     /* lambda added to each 4x4 diagonal block (1e-1) */
  int robust_cost;          /* KMX_COST_* (GNC_TLS)                           */
  double gnc_barc;          /* TLS error threshold c-bar (5.0)                */
  double gnc_mu_init;       /* GNC initial mu (1e-5)                          */
  double gnc_mu_step;       /* mu <- mu * step after each weight update (1.4) */
  int acceleration;         /* Nesterov-accelerated RBCD (RBCD++) on/off (0); concurrent
                               schedule only: every local robot updates every round      */
  int restart_interval;     /* acceleration restart period in rounds (30)               */
  int method;               /* KMX_METHOD_RTR (0) or KMX_METHOD_RGD (1)                  */
  int tcg_form;             /* KMX_TCG_FORM_STANDARD (0): ROPTLIB's tCG, two dependent
                               reductions per step; KMX_TCG_FORM_ONESYNC (1): opt-in, one
                               reduction and one kernel per step, the
                               neighbours' new direction formed from gathered z, M^-1 H delta
                               and delta; parity with the standard form at convergence only
                               (2, ABI 7's persistent resident round, was removed in ABI 8:
                               level with these forms)              */
  double rgd_stepsize;      /* RGD: X <- Retr_X(-s * precon(grad f)) (1e-3)              */
  int tile_incidences;      /* incidences per workgroup tile (0: from the handle's local
                               problem, 180..2 chunks; the tile cut orders the per-robot
                               reductions, so handles that must agree bit for bit across
                               placements set the same value)                            */
  int reserved;
} kmx_pgo_params;

/* Per-robot statistics of one RBCD round (what dpgo logs to dpgo_log_*.csv via
 * logIteration, drawio:2136-2142). */
typedef struct kmx_iter_stats {
  int updated;          /* 1 if this robot executed a block update this round  */
  int tcg_iterations;   /* inner iterations of the last RTR iteration          */
  int tcg_stop;         /* KMX_TCG_*                                           */
  int accepted;         /* last RTR step accepted                              */
  double f_init;        /* local cost before the update                        */
  double gradnorm_init; /* Riemannian gradient norm before the update          */
  double f_final;       /* local cost after the update                         */
  double rho;           /* actual / predicted decrease of the last RTR step    */
  double radius;        /* trust radius after the last RTR step                */
  double rel_change;    /* ||X_new - X_old||_F / sqrt(n) (dpgo relativeChange) */
  int64_t edges;        /* edges in the block's local problem (metric unit)    */
  int64_t hessvecs;     /* Hessian-vector products evaluated                   */
} kmx_iter_stats;

#define KMX_TCG_FORM_STANDARD 0
#define KMX_TCG_FORM_ONESYNC 1

#define KMX_TCG_NONE 0
#define KMX_TCG_NEGATIVE_CURVATURE 1
#define KMX_TCG_EXCEEDED_TR 2
#define KMX_TCG_LINEAR 3      /* ||r|| <= ||r0|| kappa        */
#define KMX_TCG_SUPERLINEAR 4 /* ||r|| <= ||r0||^(1+theta)    */
#define KMX_TCG_MAX_ITER 5
#define KMX_TCG_SKIPPED 6     /* gradient below tolerance: no step */

typedef struct kmx_pgo kmx_pgo;

/* Replaces `PGOAgent(id, PGOAgentParameters)` (drawio:1943-1957, 2457).
 * `device` is the HIP ordinal used by this handle. */
int kmx_pgo_create(const kmx_pgo_params* params, int device, kmx_pgo** out);
int kmx_pgo_destroy(kmx_pgo* h);
/* Use the caller's HIP stream (e.g. torch.cuda.current_stream().cuda_stream). */
int kmx_pgo_set_stream(kmx_pgo* h, void* hip_stream);

/* How the host enqueues the tCG steps of a round (dpgo's tCG loop inside
 * PGOAgent::iterate, drawio:2058-2066; the results are identical in every mode):
 *   1  polled: after each step the host waits for the device's progress word
 *      and stops enqueueing once every robot left tCG;
 *   0  blind: all tcg_max_iterations steps are enqueued; the kernels of a
 *      finished robot exit at once; the host never waits inside a round;
 *  -1  adaptive (default): a polled loop that needed nearly tcg_max steps sends
 *      the next loops blind, then one polled loop measures again.
 * The environment variable KMX_POLL=0/1 at handle creation forces 0 / 1. */
int kmx_pgo_set_tcg_poll(kmx_pgo* h, int mode);

/* Native team exchange over RCCL (replaces the ROS topics public_poses +
 * status of dpgo_ros, drawio:2340-2375, for a team with one process per GPU).
 * Rank 0 calls kmx_comm_unique_id and hands the KMX_COMM_ID_BYTES bytes to
 * every rank (any side channel); every rank calls kmx_pgo_comm_init on its
 * handle after kmx_pgo_set_graph, then kmx_pgo_set_exchange with the slot
 * lists of kmx_pgo_exchange_pack / _unpack (host arrays: send_slots grouped by
 * destination rank, recv_slots by source rank, counts[world] each; the own
 * rank's counts equal). From then on every kmx_pgo_iterate /
 * kmx_pgo_iterate_async round starts with the exchange on the handle's stream:
 * gather, one ncclSend / ncclRecv per peer in one group, scatter (rows into the
 * public table, the peers' status words into the team status). Every rank must
 * run the same number of rounds. kmx_pgo_set_graph drops the exchange lists. */
#define KMX_COMM_ID_BYTES 128
int kmx_comm_unique_id(void* out, int64_t nbytes);
/* JSON text: the shared objects libkmx's RCCL and HIP calls resolve to in this
 * process (dladdr of ncclSend / hipMalloc), ncclGetVersion, the RCCL header
 * version kmx was built with, hipRuntimeGetVersion / hipDriverGetVersion. */
int kmx_runtime_info(char* out, int64_t nbytes);
/* The communicator is created non-blocking: a rank whose peers do not all
 * arrive within timeout_s seconds aborts it and returns KMX_EHIP, so one
 * failing rank cannot strand the others in the rendezvous. */
int kmx_pgo_comm_init(kmx_pgo* h, const void* unique_id, int world, int rank, double timeout_s);
/* Drop the communicator and the exchange lists (back to caller-driven
 * exchanges, e.g. after a failed start-up check on another rank). */
int kmx_pgo_comm_destroy(kmx_pgo* h);
int kmx_pgo_set_exchange(kmx_pgo* h, const int32_t* send_slots, const int64_t* send_counts,
                         const int32_t* recv_slots, const int64_t* recv_counts);
/* One exchange now, outside a round (e.g. before kmx_pgo_update_weights);
 * every rank must call it the same number of times. */
int kmx_pgo_exchange(kmx_pgo* h);

/* Replaces the pose-graph intake `PGOAgent::addMeasurement` ->
 * PoseGraph::addOdometry / addPrivateLoopClosure / addSharedLoopClosure
 * (drawio:2142, 2779-2826). Edges are the GLOBAL measurement list of the team:
 * measurement e goes from pose (r1[e],p1[e]) to (r2[e],p2[e]) with rotation
 * R[9e..9e+8] (row-major) and translation t[3e..3e+2], precisions kappa / tau,
 * weight w and fixedWeight flag (odometry). `local[a]` marks robots whose blocks
 * live on this handle; edges with no local endpoint are dropped. Shared loop
 * closures (r1 != r2) are owned by min(r1, r2) for GNC weights (drawio:2198). */
int kmx_pgo_set_graph(kmx_pgo* h, int n_robots, const int32_t* n_poses,
                      const uint8_t* local, int64_t m, const int32_t* r1,
                      const int32_t* p1, const int32_t* r2, const int32_t* p2,
                      const double* R, const double* t, const double* kappa,
                      const double* tau, const double* weight,
                      const uint8_t* fixed_weight);

/* Replaces `initialize(...)` with an injected initial iterate:
 * X is n_poses[robot] * 4r doubles. get_iterate reads the current block back. */
int kmx_pgo_set_iterate(kmx_pgo* h, int robot, const double* X);
int kmx_pgo_get_iterate(kmx_pgo* h, int robot, double* X);

/* Public-pose exchange (publishPublicPoses -> updateNeighborPoses,
 * drawio:2340-2355). The team's public poses (every endpoint of a shared loop
 * closure) form one global table ordered by (robot, pose); its size is
 * kmx_pgo_public_count. pack writes this handle's OWNED rows
 * [first, first+count) of the table (count * 4r doubles) to a caller device
 * buffer; unpack installs a full table (n_public * 4r doubles, device) as the
 * fixed neighbour poses. refresh_local does pack+unpack in-device for the case
 * where every robot is local. set_neighbor_poses is the host-side variant
 * (updateNeighborPoses with a PoseDict): rows for the given (robot,pose). */
int kmx_pgo_public_count(kmx_pgo* h, int64_t* n_public, int64_t* first_owned,
                         int64_t* n_owned);
int kmx_pgo_pack_public(kmx_pgo* h, void* dev_out);
int kmx_pgo_unpack_public(kmx_pgo* h, const void* dev_table);
int kmx_pgo_refresh_local(kmx_pgo* h);
/* Sparse form of the same exchange (one all-to-all instead of an all-gather):
 * gather_public_rows writes the rows of `n` public slots OWNED by this handle
 * (dev_slots: int32 device array of table slots) to dev_out (n * 4r doubles);
 * scatter_public_rows installs n rows received from peers at the given slots.
 * Only the neighbour rows a handle's shared loop closures reference cross the
 * link; refresh_local fills the owned slots. */
int kmx_pgo_gather_public_rows(kmx_pgo* h, const int32_t* dev_slots, int64_t n, void* dev_out);
int kmx_pgo_scatter_public_rows(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const void* dev_rows);
/* The same exchange with the team status piggy-backed (dpgo Status message,
 * drawio:2375, used by shouldUpdateMeasurementWeights' "all agents converged"):
 * the rows are cut into n_seg per-peer segments, segment k = rows
 * [seg[k], seg[k+1]) (dev_seg: n_seg + 1 int32, device), and each segment is
 * followed by ONE double, so segment k starts at double seg[k]*4r + k. pack
 * writes this handle's largest relative change (of its robots' last block
 * updates) after every segment; unpack installs the rows and keeps the n_seg
 * received status values for the next round-begin GNC decision. */
int kmx_pgo_exchange_pack(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const int32_t* dev_seg,
                          int n_seg, void* dev_out);
int kmx_pgo_exchange_unpack(kmx_pgo* h, const int32_t* dev_slots, int64_t n, const int32_t* dev_seg,
                            int n_seg, const void* dev_in);
int kmx_pgo_set_neighbor_poses(kmx_pgo* h, int64_t count, const int32_t* robot,
                               const int32_t* pose, const double* X);
/* The installed public table (n_public * 4r doubles) and, when ext != NULL,
 * the peers' status words of the last exchange (one per per-peer segment):
 * used to check two exchange paths against each other bit for bit. */
int kmx_pgo_get_public(kmx_pgo* h, double* table, double* ext);

/* One RBCD round: `PGOAgent::iterate(doOptimization)` of every robot with
 * active[a] != 0 (drawio:2058-2066, 2513), all using the current neighbour
 * table. stats (may be NULL) receives one record per robot of the team
 * (n_robots records; non-local / inactive robots get updated = 0). */
int kmx_pgo_iterate(kmx_pgo* h, const uint8_t* active, kmx_iter_stats* stats);
/* Enqueue `rounds` concurrent rounds (all local robots active) without any
 * host synchronisation; used by the benchmark. stats are not produced. When
 * refresh_local != 0 the owned public rows are published before the first
 * round (every round republishes the rows it commits): the single-device
 * exchange; otherwise the caller exchanges between rounds. */
int kmx_pgo_iterate_async(kmx_pgo* h, int rounds, int refresh_local);
/* Acceleration (kmx_pgo_params.acceleration = 1, concurrent schedule only):
 * each round first forms the extrapolated point Y = Proj((1 - alpha) X +
 * alpha V) and sets X := Y (the first of refresh_local / exchange_pack /
 * iterate in a round does it, so the exchanged and published rows are Y and
 * the block update starts from Y); after the block updates V = Proj(V +
 * gamma (X - Y)), and every restart_interval rounds V = X, gamma = 0. Between
 * rounds X is the accelerated iterate itself; between the exchange and
 * iterate it holds Y. set_iterate restarts the acceleration (V = X). */
/* Wait for all work enqueued on the handle's stream. */
int kmx_pgo_sync(kmx_pgo* h);
/* As kmx_pgo_sync with a deadline: KMX_ETIMEOUT when the stream has not
 * drained after timeout_s (a round's exchange waiting on a peer that failed);
 * kmx_pgo_comm_destroy then aborts the communicator, which releases it. */
int kmx_pgo_sync_timeout(kmx_pgo* h, double timeout_s);

/* Diagnostic (no reference counterpart): the phase stamps of the one-sync tCG
 * kernel in a KMX_STEP_STAMPS build (`make -C kimera-multi_amd/csrc stamps`):
 * per tile 16 words — 7 wall-clock stamps (100 MHz; pgo.hip body_step), -,
 * poses, incidences, block index, first tile of its robot — of the last launch
 * that formed step 2. KMX_EUNSUP otherwise. */
int kmx_pgo_debug_step_stamps(uint64_t* out, int64_t n);

/* GNC: `updateMeasurementWeights()` (drawio:2215) for every non-fixed edge with
 * a local endpoint, evaluated at the current iterate and neighbour table, then
 * mu <- mu * mu_step, inner iterations <- 0, updates += 1. mu_out (may be
 * NULL) gets the mu used. A shared loop closure is evaluated identically on
 * the handles of both its robots (same two rows), which yields the owner's
 * weight on both sides (publishMeasurementWeights, drawio:2195-2198). */
int kmx_pgo_update_weights(kmx_pgo* h, double* mu_out);
/* GNC schedule run on the device at the start of every round (iterate and
 * iterate_async) when enabled: shouldUpdateMeasurementWeights
 * (drawio:2466-2469) = GNC_TLS cost, fewer than max_updates updates so far,
 * and (more than inner_iters rounds since the last update, or every agent of
 * the team converged: relative change of its last block update <=
 * rel_change_tol, this handle's robots and the statuses received by
 * kmx_pgo_exchange_unpack). Disabled by default (the agent API decides on the
 * host and calls kmx_pgo_update_weights). */
typedef struct kmx_gnc_state {
  int32_t inner_iter;  /* rounds since the last weight update (dpgo mRobustOptInnerIter) */
  int32_t updates;     /* weight updates so far                                         */
  int32_t last_fired;  /* the last round began with a weight update                      */
  int32_t rounds;      /* rounds completed                                               */
  double mu;           /* GNC mu of the next update                                      */
  double reserved[3];
} kmx_gnc_state;
int kmx_pgo_set_gnc_schedule(kmx_pgo* h, int enabled, int inner_iters, int max_updates,
                             double rel_change_tol);
int kmx_pgo_get_gnc_state(kmx_pgo* h, kmx_gnc_state* out);
int kmx_pgo_set_gnc_state(kmx_pgo* h, const kmx_gnc_state* in);
/* Per-robot relative change of the last block update (dpgo Status
 * relativeChange, drawio:2375; +inf before the first update): n_robots
 * doubles, local robots written/read only. */
int kmx_pgo_get_status(kmx_pgo* h, double* rel_change);
int kmx_pgo_set_status(kmx_pgo* h, const double* rel_change);
int kmx_pgo_get_mu(kmx_pgo* h, double* mu);
int kmx_pgo_set_mu(kmx_pgo* h, double mu);
/* `setMeasurementWeight` (drawio:2268) in bulk: weights indexed by global edge
 * id (m doubles). get returns the weights of edges with a local endpoint (others
 * untouched). set installs all; the handle rebuilds its preconditioner. */
int kmx_pgo_get_weights(kmx_pgo* h, double* w);
int kmx_pgo_set_weights(kmx_pgo* h, const double* w);
/* Shared-edge weight exchange for multi-GPU GNC (owner -> peer, drawio:2198):
 * the team's shared loop closures in global edge order; pack writes owned
 * entries and zeros elsewhere (n_shared doubles, device), unpack installs the
 * all-reduced table. */
int kmx_pgo_shared_count(kmx_pgo* h, int64_t* n_shared);
int kmx_pgo_pack_shared_weights(kmx_pgo* h, void* dev_out);
int kmx_pgo_unpack_shared_weights(kmx_pgo* h, const void* dev_table);

/* Rounded trajectory in the anchor frame: `getTrajectoryInGlobalFrame` /
 * publishTrajectory (drawio:2148-2151) with the global anchor of
 * `setGlobalAnchor` (drawio:2396). anchor = 4r doubles [Y0 p0] (lifted pose of
 * robot 0, pose 0). out: n_poses[robot] * 12 doubles = R (row-major 3x3) then t. */
int kmx_pgo_get_trajectory(kmx_pgo* h, int robot, const double* anchor,
                           double* out);

/* Primitive evaluation for parity tests (one robot block, current neighbour
 * table). mode: KMX_EVAL_*. V/out are n_poses[robot]*4r doubles; scalar gets the
 * cost (COST_EGRAD) or <V, out> otherwise. HESS modes evaluate at the current
 * iterate. */
#define KMX_EVAL_COST_EGRAD 0 /* out = Euclidean gradient at X=V, scalar = f(V) */
#define KMX_EVAL_EHESS 1      /* out = Euclidean Hessian-vector product Q V      */
#define KMX_EVAL_RGRAD 2      /* out = Riemannian gradient at X (V ignored)      */
#define KMX_EVAL_RHESS 3      /* out = Riemannian Hessian at X applied to V      */
#define KMX_EVAL_PRECON 4     /* out = preconditioner at X applied to V          */
#define KMX_EVAL_RETRACT 5    /* out = R_X(V)                                    */
int kmx_pgo_eval(kmx_pgo* h, int robot, int mode, const double* V, double* out,
                 double* scalar);

/* Edges in robot `robot`'s local problem (private + shared incident edges). */
int kmx_pgo_local_edges(kmx_pgo* h, int robot, int64_t* m_local);
/* Resident device bytes of the handle and the bytes of one incidence record
 * (68: compact — three components of the rotation's unit quaternion, t,
 * w kappa, w tau with the tail flag in its sign, and the 4-B other endpoint
 * with the fourth component's index; 128: full rotation, when some measurement
 * rotation is not in SO(3) to 1e-12). */
int kmx_pgo_memory(kmx_pgo* h, int64_t* device_bytes, int* record_bytes);
/* Live instrumentation of the dominant kernel (the Hessian-vector product of
 * the tCG loop). When enabled, every Hessian-vector launch enqueued by
 * kmx_pgo_iterate / kmx_pgo_iterate_async is bracketed by a HIP event pair on
 * the handle's stream. read_timing synchronises, sums the event durations and
 * the device-side work counters accumulated since the last read, and resets
 * them. hessvec_alg_bytes follows SURVEY.md §8d: per launch and per robot whose
 * tCG was running, 128 B per local edge + 2 * 8 * r(d+1) B per pose. */
typedef struct kmx_pgo_counters {
  double hessvec_ms_total;     /* summed device time of Hessian-vector launches */
  int64_t hessvec_launches;    /* launches bracketed by events                  */
  double hessvec_alg_bytes;    /* algorithmic bytes those launches processed    */
  int64_t edges_iters;         /* sum over executed block updates of m_alpha    */
  int64_t block_updates;       /* executed block updates (tCG ran)              */
  int64_t hessvecs;            /* robot-level Hessian-vector products           */
  int64_t gnc_updates;         /* GNC weight updates run                        */
} kmx_pgo_counters;
int kmx_pgo_enable_timing(kmx_pgo* h, int enable);
int kmx_pgo_read_counters(kmx_pgo* h, kmx_pgo_counters* out);

/* ------------------------------------------------------------------------- */
/* Kimera-Multi-LCD: descriptor matching + geometric verification             */
/* ------------------------------------------------------------------------- */

#define KMX_NORM_L1 0      /* BruteForce-L1 over bytes: reference build      */
#define KMX_NORM_HAMMING 1 /* BruteForce-Hamming over 256 bits: north_star  */

/* sampler variants of std::uniform_int_distribution<int>(0, INT_MAX) over
 * std::mt19937 (SURVEY.md §0 finding 5) */
#define KMX_RNG_GCC9 0   /* rejection of x >= 2^31, returns x (ROS Noetic)  */
#define KMX_RNG_GCC11 1  /* Lemire: returns x >> 1                          */

/* 5-point minimal solver of the 2D-2D RANSAC (opengv CentralRelativePoseSacProblem). */
#define KMX_ALGO_STEWENIUS 0 /* opengv STEWENIUS: Groebner basis, 10x10 action matrix eigenproblem */
#define KMX_ALGO_NISTER 1    /* opengv NISTER: degree-10 polynomial in z, Sturm roots            */

/* LcdParams (params/D455/LcdParams.yaml:16-17, 51-66). */
typedef struct kmx_lcd_params {
  int norm;                   /* KMX_NORM_* (L1: matcher_type 3 + patch:33-35) */
  double lowe_ratio;          /* 0.7 (compared in double, as LcdParams' double) */
  int min_2d2d_inliers;       /* 10                                            */
  int min_3d3d_inliers;       /* 5                                             */
  double ransac_threshold_2d2d; /* 1e-6 (1 - cos)                              */
  double ransac_threshold_3d3d; /* 0.3 m                                       */
  int ransac_max_iterations;  /* 500                                           */
  double ransac_probability;  /* 0.995                                         */
  int ransac_randomize;       /* 0: fixed seed                                 */
  uint32_t ransac_seed;       /* 12345                                         */
  int rng_variant;            /* KMX_RNG_*                                     */
  int use_1point_3d3d;        /* 1: translation-only 3D-3D given the 2D-2D R   */
  int pose_recovery_type;     /* 0: 3D-3D (reference config), 1: PnP            */
  int min_2d3d_inliers;       /* 20 (LcdParams.yaml:53)                        */
  double ransac_threshold_2d3d; /* PnP inlier threshold in (1 - cos) units: from
                                 a pixel threshold px and focal length f,
                                 1 - cos(atan(px / f)) (LcdParams.yaml:57)     */
  int algorithm_2d2d;         /* KMX_ALGO_* 5-point minimal solver
                                 (ransac_2d2d_algorithm, LcdParams.yaml:73)     */
  int refine_pose;            /* refine_pose (LcdParams.yaml:14): after an accepted
                                 3D-3D recovery (pose_recovery_type 0), T is
                                 re-estimated over all 3D-3D inliers by least
                                 squares (centroids + Kabsch), the restated form
                                 of Kimera-VIO's stereo pose refinement [U]     */
  int rng_stream;             /* LC5, the OpenGV fork's "thread_local" sampler
                                 (README.md:35-36): 0 = every RANSAC problem
                                 seeds its own std::mt19937 with ransac_seed
                                 (opengv's SampleConsensusProblem constructor;
                                 the default); 1 = one engine per verification
                                 thread, seeded once, that every problem
                                 continues in candidate order (2D-2D, then the
                                 Arun / EPnP recovery). Mode 1 is an ordered,
                                 candidate-serial GPU path. */
  int reserved[1];
} kmx_lcd_params;

/* Stages of kmx_lcd_verify_matches. */
#define KMX_LCD_STAGE_2D2D 1    /* geometricVerificationNister (drawio:2589-2592) */
#define KMX_LCD_STAGE_RECOVER 2 /* recoverPose (drawio:2595-2598)                 */

/* computeMatchedIndices (drawio:2583-2586): k=2 brute-force match of every
 * query descriptor against the match frame + Lowe ratio. desc are 32-byte ORB
 * descriptors. Output pairs (i_query, i_match) in query order; *k = count. */
int kmx_lcd_knn2(int norm, double lowe_ratio, const uint8_t* q, int32_t nq,
                 const uint8_t* mdesc, int32_t nm, int32_t* pairs_out,
                 int32_t* k);

/* Batched verification of candidates (verifyLoopSpin -> computeMatchedIndices
 * -> geometricVerificationNister -> recoverPose, drawio:2638-2657). */
typedef struct kmx_lcd_batch_desc {
  int32_t n_frames;       /* frames in the descriptor/feature pool           */
  int32_t max_feats;      /* features per frame (stride)                     */
  const int32_t* n_feats; /* [n_frames]                                       */
  const uint8_t* desc;    /* [n_frames][max_feats][32]                        */
  const double* bearings; /* [n_frames][max_feats][3] unit bearing vectors    */
  const double* points;   /* [n_frames][max_feats][3] stereo points (or NaN)  */
  int32_t n_cand;
  const int32_t* cand_query; /* [n_cand] frame ids */
  const int32_t* cand_match; /* [n_cand] frame ids */
} kmx_lcd_batch_desc;

typedef struct kmx_lcd_result {
  int32_t n_matches;      /* after kNN + Lowe                                 */
  int32_t mono_inliers;   /* 2D-2D RANSAC inliers                             */
  int32_t stereo_inliers; /* 3D-3D inliers                                    */
  int32_t accepted;       /* mono >= min_2d2d && (stereo >= min_3d3d, or
                             pnp >= min_2d3d with pose_recovery_type 1)     */
  int32_t iterations_2d2d;
  int32_t pnp_inliers;    /* 2D-3D inliers (pose_recovery_type 1)              */
  double T_query_match[12]; /* R row-major, t                                 */
} kmx_lcd_result;

typedef struct kmx_lcd kmx_lcd;
int kmx_lcd_create(const kmx_lcd_params* params, int device, kmx_lcd** out);
int kmx_lcd_destroy(kmx_lcd* h);
int kmx_lcd_set_stream(kmx_lcd* h, void* hip_stream);
/* Upload the frame pool (host arrays) to the device; kept until replaced.
 * Replaces every resident frame (a whole-pool reload); frames that arrive one
 * at a time go through kmx_lcd_add_frames. */
int kmx_lcd_set_frames(kmx_lcd* h, const kmx_lcd_batch_desc* pool);
/* LoopClosureDetector::addVLCFrame (drawio:2601; Kimera-Distributed adds each
 * VLC frame as it arrives, drawio:441-505): append n frames (max_feats must
 * equal the pool's, or set it on an empty handle). Resident frames are never
 * re-uploaded: the device pool grows by capacity doubling (one device-to-
 * device copy per doubling), the sampler table is kept (it depends only on
 * the parameters and max_feats). *first_id = id of the first appended frame. */
int kmx_lcd_add_frames(kmx_lcd* h, int32_t n, int32_t max_feats, const int32_t* n_feats,
                       const uint8_t* desc, const double* bearings, const double* points,
                       int32_t* first_id);
/* Frames resident (added or set) and the device capacity in frames. */
int kmx_lcd_pool_info(kmx_lcd* h, int32_t* n_frames, int32_t* capacity, int32_t* max_feats);
/* Verify n_cand candidates against the resident pool. results: n_cand records.
 * inlier masks (optional, may be NULL): [n_cand][max_feats] bytes, bit0 = 2D-2D
 * inlier, bit1 = 3D-3D inlier, indexed by match index (position in the pair
 * list of kmx_lcd_knn2 order). */
int kmx_lcd_verify(kmx_lcd* h, int32_t n_cand, const int32_t* cand_query,
                   const int32_t* cand_match, kmx_lcd_result* results,
                   uint8_t* inlier_masks);
/* Enqueue verification of candidates already resident on the device without
 * host synchronisation (benchmark / streaming path). Up to four calls are in
 * flight (candidate slots used in turn; a fifth waits for the first); calls
 * under 96 candidates per CU run their RANSACs concurrently. Results are not
 * returned: kmx_lcd_sync waits for every call (the synchronous entry points
 * return results). */
int kmx_lcd_verify_async(kmx_lcd* h, int32_t n_cand, const int32_t* cand_query,
                         const int32_t* cand_match);
int kmx_lcd_sync(kmx_lcd* h);
/* computeMatchedIndices (drawio:2583-2586) on resident frames, batched: for
 * candidate i the kNN2 + Lowe pairs of frames cand_query[i] / cand_match[i]
 * in query order, pairs_out[i][k] = (i_query, i_match) for k < k_out[i]
 * (pairs_out: [n_cand][max_feats][2]). */
int kmx_lcd_match(kmx_lcd* h, int32_t n_cand, const int32_t* cand_query, const int32_t* cand_match,
                  int32_t* pairs_out, int32_t* k_out);
/* geometricVerificationNister and / or recoverPose (drawio:2589-2598) on
 * caller-supplied correspondences, batched over candidates, no kNN2: the
 * pairs of candidate i are (i_query[k], i_match[k]) for k in
 * [mptr[i], mptr[i+1]) (feature indices of frames cand_query[i] /
 * cand_match[i]; at most max_feats pairs per candidate). stages: a mask of
 * KMX_LCD_STAGE_*.
 *   - without KMX_LCD_STAGE_2D2D every pair is a 2D-2D inlier (the
 *     correspondences are geometricVerificationNister's inliers) and, for the
 *     1-point 3D-3D recovery, the rotation is T_prior[i] (R row-major, t;
 *     [n][12]; required then, otherwise may be NULL);
 *   - without KMX_LCD_STAGE_RECOVER, accepted = mono_inliers >= min_2d2d and
 *     T_query_match = the 2D-2D pose (unit-norm t).
 * results / inlier_masks as kmx_lcd_verify, masks indexed by pair position. */
int kmx_lcd_verify_matches(kmx_lcd* h, int32_t n_cand, const int32_t* cand_query,
                           const int32_t* cand_match, const int64_t* mptr,
                           const int32_t* i_query, const int32_t* i_match, int stages,
                           const double* T_prior, kmx_lcd_result* results,
                           uint8_t* inlier_masks);
/* Instrumentation: when enabled, every verification brackets its kNN2 launch
 * and its RANSAC launches with HIP events; read_timing synchronises and
 * returns the device times (ms) of the last evented verification. */
int kmx_lcd_enable_timing(kmx_lcd* h, int enable);
int kmx_lcd_read_timing(kmx_lcd* h, double* knn_ms, double* ransac_ms);


/* ------------------------------------------------------------------------- */
/* Kimera-Multi-LCD BoW candidate stage: DBoW2 inverted-file L1 query         */
/* ------------------------------------------------------------------------- */
/* Replaces DBoW2 Database::queryL1 and L1Scoring::score as used by
 * LoopClosureDetector::detectLoop / detectLoopWithRobot (drawio:2574-2580,
 * 2612-2633; LcdParams.yaml:3-12). BowVectors are CSR: vptr[n+1] (int64),
 * words (uint32, strictly increasing per vector) and weights (L1-normalised
 * double). Entry id = position in the database. */
typedef struct kmx_bow kmx_bow;
int kmx_bow_create(int device, kmx_bow** out);
int kmx_bow_destroy(kmx_bow* h);
int kmx_bow_set_stream(kmx_bow* h, void* hip_stream);
/* Build the inverted file of entries 0..n_entries-1 (Database::add in order). */
int kmx_bow_set_database(kmx_bow* h, int32_t n_words, int32_t n_entries,
                         const int64_t* vptr, const uint32_t* words,
                         const double* weights);
/* queryL1 for nq query vectors: results with entry id < max_id[q] (NULL or
 * -1: all), sorted by score descending (ties: lower entry id first), at most
 * max_results (<= 256) each. out_n[nq]; out_ids / out_scores [nq][max_results];
 * score = 1 - 1/2 |v - w|_1. */
int kmx_bow_query(kmx_bow* h, int32_t nq, const int64_t* qptr,
                  const uint32_t* words, const double* weights,
                  const int32_t* max_id, int32_t max_results, int32_t* out_n,
                  int32_t* out_ids, double* out_scores);
/* Enqueue only (benchmark path); kmx_bow_sync waits. */
int kmx_bow_query_async(kmx_bow* h, int32_t nq, const int64_t* qptr,
                        const uint32_t* words, const double* weights,
                        const int32_t* max_id, int32_t max_results);
int kmx_bow_sync(kmx_bow* h);
/* L1Scoring::score of n pairs (a_i, b_i) (the nss factor). */
int kmx_bow_score_pairs(kmx_bow* h, int32_t n, const int64_t* aptr,
                        const uint32_t* aw, const double* av,
                        const int64_t* bptr, const uint32_t* bw,
                        const double* bv, double* out);

#ifdef __cplusplus
}
#endif
#endif /* KMX_ABI_H */
