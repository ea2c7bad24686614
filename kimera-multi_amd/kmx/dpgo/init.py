"""Distributed initialisation: robust alignment of each
robot's locally initialised trajectory to the global frame.

Reference flow (drawio:2271-2307, 2490-2510; images/system_arch.png "Global
Frame Estimation"): every robot first initialises its own block (odometry
chain / local solve) in its own frame; then, once a neighbour that is already
in the global frame publishes the poses at the ends of their shared loop
closures, the robot estimates the rigid transform between the two frames
from every such loop closure and fuses the candidates with GNC-TLS robust
single-pose averaging [U: dpgo's robustSinglePoseAveraging; restated from
the published GNC algorithm]. Robot 0 defines the global frame.

This is host-side control (O(#shared loop closures) per robot, once), like
the reference's.
"""
from __future__ import annotations

import numpy as np

from .params import error_threshold_at_quantile


def project_so3(M: np.ndarray) -> np.ndarray:
    U, _, Vt = np.linalg.svd(M)
    D = np.eye(3)
    D[2, 2] = np.sign(np.linalg.det(U @ Vt))
    return U @ D @ Vt


def single_pose_averaging(R, t, kappa, tau, w):
    """argmin_{R,t} sum_i w_i (kappa_i |R - R_i|_F^2 + tau_i |t - t_i|^2)."""
    Rm = project_so3(np.einsum("i,ijk->jk", w * kappa, R))
    wt = w * tau
    tm = (wt[:, None] * t).sum(0) / max(wt.sum(), 1e-300)
    return Rm, tm


def robust_single_pose_averaging(R, t, kappa, tau, *, barc: float | None = None, mu_step: float = 1.4,
                                 max_iters: int = 1000):
    """GNC-TLS robust averaging of SE(3) candidates (R_i, t_i) with precisions
    (kappa_i, tau_i). Returns (R, t, weights in [0, 1]).
    barc default: chi-square 0.999 quantile of SE(3)'s 6 dof (error_threshold_at_quantile): with
    dpgo's precisions kappa |dR|_F^2 is ~2x a chi-square(3) variable, so tighter quantiles reject
    inliers."""
    R = np.asarray(R, np.float64).reshape(-1, 3, 3)
    t = np.asarray(t, np.float64).reshape(-1, 3)
    n = R.shape[0]
    kappa = np.broadcast_to(np.asarray(kappa, np.float64), (n,)).copy()
    tau = np.broadcast_to(np.asarray(tau, np.float64), (n,)).copy()
    if n == 0:
        raise ValueError("no candidates")
    barc = error_threshold_at_quantile(0.999, 3) if barc is None else barc
    c2 = barc * barc
    w = np.ones(n)
    Rm, tm = single_pose_averaging(R, t, kappa, tau, w)
    if n == 1:
        return Rm, tm, w
    r2 = kappa * ((R - Rm) ** 2).sum((1, 2)) + tau * ((t - tm) ** 2).sum(1)
    mu = c2 / max(2.0 * r2.max() - c2, 1e-12)  # GNC-TLS initial mu (Yang et al. 2020)
    mu = max(mu, 1e-12)
    for _ in range(max_iters):
        lo, hi = mu / (mu + 1.0) * c2, (mu + 1.0) / mu * c2
        w_new = np.where(r2 <= lo, 1.0, np.where(r2 >= hi, 0.0, np.sqrt(c2 * mu * (mu + 1.0) / np.maximum(r2, 1e-300)) - mu))
        if w_new.sum() == 0:  # everything rejected: keep the best single candidate
            w_new = (r2 == r2.min()).astype(float)
        Rm, tm = single_pose_averaging(R, t, kappa, tau, w_new)
        r2 = kappa * ((R - Rm) ** 2).sum((1, 2)) + tau * ((t - tm) ** 2).sum(1)
        converged = np.all((w_new == 0.0) | (w_new == 1.0)) and np.array_equal(w_new, w)
        w = w_new
        if converged:
            break
        mu *= mu_step
    return Rm, tm, w


def alignment_candidates(shared_lcs, own_robot, own_R, own_t, nbr_global):
    """One candidate T_world_own per shared loop closure whose neighbour end is
    known in the world frame.

    shared_lcs: RelativeSEMeasurement-like objects ((r1, p1) -> (r2, p2), R, t,
    kappa, tau) with T_{r1,p1}^{-1} T_{r2,p2} = (R, t).
    own_R / own_t: this robot's trajectory in its own frame ([n, 3, 3], [n, 3]).
    nbr_global: {(robot, pose): (R, t)} neighbour poses in the world frame."""
    Rs, ts, ks, taus = [], [], [], []
    for m in shared_lcs:
        if m.r1 == own_robot and (m.r2, m.p2) in nbr_global:
            # T_W_own(p1) = T_W_nbr(p2) meas^{-1};  T_W_A = T_W_own(p1) T_A_own(p1)^{-1}
            Rn, tn = nbr_global[(m.r2, m.p2)]
            Rw = Rn @ m.R.T
            tw = tn - Rw @ m.t
            Ra, ta = own_R[m.p1], own_t[m.p1]
        elif m.r2 == own_robot and (m.r1, m.p1) in nbr_global:
            # T_W_own(p2) = T_W_nbr(p1) meas
            Rn, tn = nbr_global[(m.r1, m.p1)]
            Rw = Rn @ m.R
            tw = tn + Rn @ m.t
            Ra, ta = own_R[m.p2], own_t[m.p2]
        else:
            continue
        R_WA = Rw @ Ra.T
        Rs.append(R_WA)
        ts.append(tw - R_WA @ ta)
        ks.append(m.kappa)
        taus.append(m.tau)
    return np.array(Rs).reshape(-1, 3, 3), np.array(ts).reshape(-1, 3), np.array(ks), np.array(taus)


def align_to_world(shared_lcs, own_robot, own_R, own_t, nbr_global, **kw):
    """Robust T_world_own = (R, t) and the per-loop-closure inlier weights."""
    Rs, ts, ks, taus = alignment_candidates(shared_lcs, own_robot, own_R, own_t, nbr_global)
    if Rs.shape[0] == 0:
        return None
    return robust_single_pose_averaging(Rs, ts, ks, taus, **kw)


def transform_trajectory(R_WA, t_WA, R, t):
    """Express a trajectory given in frame A in the world frame."""
    return np.einsum("ij,njk->nik", R_WA, R), t @ R_WA.T + t_WA


def chordal_initialization(n: int, edges, anchor: int = 0):
    """Local chordal initialisation of one robot's trajectory (SURVEY.md §8
    row D10; dpgo's local initialisation method Chordal [U: restated from the
    SE-Sync chordal relaxation it uses]).

    edges: iterable of (i, j, R_ij [3x3], t_ij [3], kappa, tau, weight) for the
    robot's own measurements (odometry and private loop closures), with
    R_j = R_i R_ij and t_j = t_i + R_i t_ij. Step 1 minimises
    sum w kappa |R_j - R_i R_ij|_F^2 over unconstrained 3x3 blocks with
    R_anchor = I (sparse normal equations), then projects every block to SO(3);
    step 2 minimises sum w tau |t_j - t_i - R_i t_ij|^2 with t_anchor = 0 for
    the rotations of step 1. Returns (R [n,3,3], t [n,3])."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    E = list(edges)
    if n == 1:
        return np.eye(3)[None], np.zeros((1, 3))
    free = np.array([k for k in range(n) if k != anchor])
    col = -np.ones(n, np.int64)
    col[free] = np.arange(n - 1)
    # rotations: unknowns are the 3x3 blocks of the free poses, row-major, and
    # every edge gives R_j - R_i R_ij = 0, i.e. for each row a of R:
    # R_j[a, :] - R_i[a, :] R_ij = 0 (3 equations per row, same structure per row)
    # row a of every block is an independent problem with the same matrix:
    # s (R_j[a, c] - sum_b R_i[a, b] R_ij[b, c]) = 0 for c = 0..2; the anchor's
    # known row (R_anchor = I) moves to the right-hand side
    rows, cols, vals, rhs = [], [], [], []
    r = 0
    for (i, j, Rij, _t, kap, _tau, w) in E:
        s = np.sqrt(max(w * kap, 0.0))
        Rij = np.asarray(Rij, np.float64)
        for c in range(3):
            if col[j] >= 0:
                rows.append(r); cols.append(3 * col[j] + c); vals.append(s)
            if col[i] >= 0:
                for b in range(3):
                    rows.append(r); cols.append(3 * col[i] + b); vals.append(-s * Rij[b, c])
            rhs.append((c, i, j, s, Rij))
            r += 1
    A = sp.csr_matrix((vals, (rows, cols)), shape=(r, 3 * (n - 1)))
    AtA = (A.T @ A).tocsc()
    solve = spla.factorized(AtA)
    Rs = np.zeros((n, 3, 3))
    Rs[anchor] = np.eye(3)
    for a in range(3):  # one solve per row of the rotation blocks, same matrix
        bvec = np.zeros(r)
        for k, (c, i, j, s, Rij) in enumerate(rhs):
            v = 0.0
            if i == anchor:
                v += s * Rij[a, c]
            if j == anchor:
                v -= s * (1.0 if a == c else 0.0)
            bvec[k] = v
        x = solve(A.T @ bvec)
        Rs[free, a, :] = x.reshape(n - 1, 3)
    for k in free:
        Rs[k] = project_so3(Rs[k])
    # translations
    rows, cols, vals, b = [], [], [], []
    r = 0
    for (i, j, Rij, tij, _kap, tau, w) in E:
        s = np.sqrt(max(w * tau, 0.0))
        d = Rs[i] @ np.asarray(tij, np.float64)
        for c in range(3):
            if col[j] >= 0:
                rows.append(r); cols.append(3 * col[j] + c); vals.append(s)
            if col[i] >= 0:
                rows.append(r); cols.append(3 * col[i] + c); vals.append(-s)
            b.append(s * d[c])
            r += 1
    A = sp.csr_matrix((vals, (rows, cols)), shape=(r, 3 * (n - 1)))
    x = spla.spsolve((A.T @ A).tocsc(), A.T @ np.asarray(b))
    ts = np.zeros((n, 3))
    ts[free] = np.asarray(x).reshape(n - 1, 3)
    return Rs, ts
