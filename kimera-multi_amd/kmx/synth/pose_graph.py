"""Seeded synthetic multi-robot pose graphs.

The Campus bags, GT and vocabularies are external downloads, so
every benchmark and parity case runs on graphs of the same *shape* as the
reference's configs:

* per-robot odometry chains (``fixedWeight`` = 1, the edges dpgo never
  reweights: PoseGraph::addOdometry, drawio:2779-2790);
* loop closures between GT poses within ``lc_radius`` metres — a fraction
  ``f_inter`` of them between different robots (shared loop closures,
  addSharedLoopClosure, drawio:2817);
* ``outlier_frac`` outlier loop closures between random pose pairs with a
  uniform-SO(3) rotation and t ~ U[-10, 10]^3;
* noise sigma_R = 0.01 rad, sigma_t = 0.1 m, so kappa = 1e4 and tau = 1e2
  (params/D455/LcdParams.yaml:29-30 betweenRotation/TranslationPrecision).

Everything is numpy ``PCG64(seed)``; the same call returns bit-identical arrays
on every machine, so GPU runs, the CPU restatement and committed fixtures see
the same inputs.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class PoseGraphData:
    n_robots: int
    n_poses: np.ndarray          # int32 [R]
    r1: np.ndarray               # int32 [m]
    p1: np.ndarray
    r2: np.ndarray
    p2: np.ndarray
    R: np.ndarray                # float64 [m, 3, 3]
    t: np.ndarray                # float64 [m, 3]
    kappa: np.ndarray            # float64 [m]
    tau: np.ndarray
    weight: np.ndarray
    fixed: np.ndarray            # uint8 [m] (1 = odometry)
    outlier: np.ndarray          # bool [m] ground-truth outlier flag
    gt_R: list = field(default_factory=list)   # per robot [n, 3, 3]
    gt_t: list = field(default_factory=list)   # per robot [n, 3]
    init_R: list = field(default_factory=list)  # odometry-chain initial guess
    init_t: list = field(default_factory=list)

    @property
    def m(self) -> int:
        return int(self.r1.shape[0])

    @property
    def n_total(self) -> int:
        return int(self.n_poses.sum())


def _expm_so3(w: np.ndarray) -> np.ndarray:
    """Batched Rodrigues exp map, w [k, 3] -> [k, 3, 3]."""
    th = np.linalg.norm(w, axis=1)
    k = w / np.maximum(th, 1e-300)[:, None]
    K = np.zeros((w.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -k[:, 2], k[:, 1]
    K[:, 1, 0], K[:, 1, 2] = k[:, 2], -k[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -k[:, 1], k[:, 0]
    s, c = np.sin(th)[:, None, None], np.cos(th)[:, None, None]
    out = np.eye(3)[None] + s * K + (1.0 - c) * (K @ K)
    small = th < 1e-12
    if small.any():
        out[small] = np.eye(3)
    return out


def random_rotations(rng: np.random.Generator, k: int) -> np.ndarray:
    """Uniform SO(3) samples via unit quaternions."""
    q = rng.standard_normal((k, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1),
    ], axis=1)


def _compose_scan(Rrel: np.ndarray, trel: np.ndarray, R0: np.ndarray, t0: np.ndarray):
    """Poses T_k = T_0 * prod_{j<k} rel_j as a log-depth batched scan."""
    n = Rrel.shape[0] + 1
    T = np.zeros((n, 4, 4))
    T[:, 3, 3] = 1.0
    T[0, :3, :3] = np.eye(3)
    T[1:, :3, :3] = Rrel
    T[1:, :3, 3] = trel
    s = 1
    while s < n:  # inclusive prefix product, earlier factor on the left
        T[s:] = T[:-s] @ T[s:]
        s *= 2
    T0 = np.eye(4)
    T0[:3, :3], T0[:3, 3] = R0, t0
    T = T0[None] @ T
    return T[:, :3, :3].copy(), T[:, :3, 3].copy()


def _gt_trajectory(rng, n, box, start):
    """Ground-vehicle-like walk: yaw random walk, small pitch/roll, ~1 m steps,
    reflected at the walls of a [-box, box]^2 arena."""
    dyaw = rng.normal(0.0, 0.15, n)
    yaw = np.cumsum(dyaw) + rng.uniform(-np.pi, np.pi)
    pitch = rng.normal(0.0, 0.02, n)
    roll = rng.normal(0.0, 0.02, n)
    cy, sy, cp, sp, cr, sr = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch), np.cos(roll), np.sin(roll)
    R = np.empty((n, 3, 3))
    R[:, 0, 0] = cy * cp; R[:, 0, 1] = cy * sp * sr - sy * cr; R[:, 0, 2] = cy * sp * cr + sy * sr
    R[:, 1, 0] = sy * cp; R[:, 1, 1] = sy * sp * sr + cy * cr; R[:, 1, 2] = sy * sp * cr - cy * sr
    R[:, 2, 0] = -sp;     R[:, 2, 1] = cp * sr;                R[:, 2, 2] = cp * cr
    step = R[:, :, 0] * rng.uniform(0.6, 1.2, n)[:, None]
    p = start[None] + np.cumsum(step, axis=0)
    # reflect into the arena (keeps trajectories overlapping so loop closures exist)
    for ax in range(2):
        x = p[:, ax] + box
        x = np.mod(x, 4 * box)
        p[:, ax] = np.where(x > 2 * box, 4 * box - x, x) - box
    p[:, 2] = 0.3 * np.sin(np.arange(n) / 50.0) + rng.normal(0, 0.01)
    return R, p


def _workers() -> int:
    """Threads for the KD-tree queries (results do not depend on it)."""
    import os
    return max(1, min(16, os.cpu_count() or 1))


def make_pose_graph(n_robots: int, n_poses_total: int, n_edges_total: int, *,
                    outlier_frac: float = 0.2, f_inter: float = 0.10,
                    sigma_R: float = 0.01, sigma_t: float = 0.1,
                    lc_radius: float = 5.0, box: float | None = None,
                    noise_free: bool = False, outlier_scope: str = "team", seed: int = 0) -> PoseGraphData:
    """`outlier_scope` "team": outlier loop closures join random pose pairs of
    the whole team; "robot": both ends on the same robot (the inter-robot loop
    closures of kmx.pipeline come from the verified LCD stream instead)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    R_ = n_robots
    base = n_poses_total // R_
    n_poses = np.full(R_, base, dtype=np.int32)
    n_poses[: n_poses_total - base * R_] += 1
    if box is None:
        box = max(10.0, 0.5 * np.sqrt(n_poses_total))
    gt_R, gt_t = [], []
    for a in range(R_):
        Ra, ta = _gt_trajectory(rng, int(n_poses[a]), box, rng.uniform(-box, box, 3) * np.array([1, 1, 0]))
        gt_R.append(Ra)
        gt_t.append(ta)
    sR = 0.0 if noise_free else sigma_R
    sT = 0.0 if noise_free else sigma_t

    def rel(Ra, ta, Rb, tb):
        Rr = np.einsum("kji,kjl->kil", Ra, Rb)
        tr = np.einsum("kji,kj->ki", Ra, tb - ta)
        return Rr, tr

    def noisy(Rr, tr):
        k = Rr.shape[0]
        if sR > 0:
            Rr = Rr @ _expm_so3(rng.normal(0, sR, (k, 3)))
        if sT > 0:
            tr = tr + rng.normal(0, sT, (k, 3))
        return Rr, tr

    E_r1, E_p1, E_r2, E_p2, E_R, E_t, E_fixed, E_out = [], [], [], [], [], [], [], []
    init_R, init_t = [], []
    # odometry
    for a in range(R_):
        n = int(n_poses[a])
        Rr, tr = rel(gt_R[a][:-1], gt_t[a][:-1], gt_R[a][1:], gt_t[a][1:])
        Rr, tr = noisy(Rr, tr)
        E_r1.append(np.full(n - 1, a)); E_p1.append(np.arange(n - 1))
        E_r2.append(np.full(n - 1, a)); E_p2.append(np.arange(1, n))
        E_R.append(Rr); E_t.append(tr)
        E_fixed.append(np.ones(n - 1, np.uint8)); E_out.append(np.zeros(n - 1, bool))
        Ri, ti = _compose_scan(Rr, tr, gt_R[a][0], gt_t[a][0])
        init_R.append(Ri); init_t.append(ti)
    n_odo = int(n_poses.sum()) - R_
    n_lc = max(0, n_edges_total - n_odo)
    n_out = int(round(outlier_frac * n_lc))
    n_in = n_lc - n_out
    n_inter = int(round(f_inter * n_in)) if R_ > 1 else 0
    n_intra = n_in - n_inter
    # inlier loop closures: pick a random pose, then a partner within lc_radius
    allp = np.concatenate(gt_t)
    rob_of = np.concatenate([np.full(int(n_poses[a]), a) for a in range(R_)])
    idx_of = np.concatenate([np.arange(int(n_poses[a])) for a in range(R_)])
    from scipy.spatial import cKDTree
    tree = cKDTree(allp)

    def sample_pairs(k, inter):
        out_i, out_j = [], []
        need = k
        while need > 0:
            cand = rng.integers(0, allp.shape[0], size=2 * need + 16)
            # k nearest neighbours, then choose one at random among those within radius
            dist, nb = tree.query(allp[cand], k=32, distance_upper_bound=lc_radius, workers=_workers())
            choice = rng.integers(0, 32, size=cand.shape[0])
            j = nb[np.arange(cand.shape[0]), choice]
            ok = j < allp.shape[0]
            jj = np.where(ok, j, 0)
            ok &= jj != cand
            same = rob_of[cand] == rob_of[jj]
            ok &= (~same) if inter else same
            ok &= ~(same & (np.abs(idx_of[cand] - idx_of[jj]) <= 1))  # not an odometry pair
            i_sel, j_sel = cand[ok][:need], jj[ok][:need]
            out_i.append(i_sel); out_j.append(j_sel)
            need -= i_sel.shape[0]
        return np.concatenate(out_i), np.concatenate(out_j)

    flat_R = np.concatenate(gt_R)
    for k, inter in ((n_intra, False), (n_inter, True)):
        if k <= 0:
            continue
        gi, gj = sample_pairs(k, inter)
        Rr, tr = rel(flat_R[gi], allp[gi], flat_R[gj], allp[gj])
        Rr, tr = noisy(Rr, tr)
        E_r1.append(rob_of[gi]); E_p1.append(idx_of[gi]); E_r2.append(rob_of[gj]); E_p2.append(idx_of[gj])
        E_R.append(Rr); E_t.append(tr)
        E_fixed.append(np.zeros(k, np.uint8)); E_out.append(np.zeros(k, bool))
    if n_out > 0:
        gi = rng.integers(0, allp.shape[0], n_out)
        if outlier_scope == "robot":
            off = np.concatenate([[0], np.cumsum(n_poses)[:-1]])
            ri = rob_of[gi]
            gj = off[ri] + (rng.random(n_out) * n_poses[ri]).astype(np.int64)
            bad = gj == gi
            gj[bad] = off[ri[bad]] + (idx_of[gi[bad]] + 2) % n_poses[ri[bad]]
        else:
            gj = rng.integers(0, allp.shape[0], n_out)
            bad = gi == gj
            gj[bad] = (gj[bad] + 1) % allp.shape[0]
        E_r1.append(rob_of[gi]); E_p1.append(idx_of[gi]); E_r2.append(rob_of[gj]); E_p2.append(idx_of[gj])
        E_R.append(random_rotations(rng, n_out)); E_t.append(rng.uniform(-10, 10, (n_out, 3)))
        E_fixed.append(np.zeros(n_out, np.uint8)); E_out.append(np.ones(n_out, bool))
    m = sum(x.shape[0] for x in E_r1)
    kappa = np.full(m, 1.0 / sigma_R ** 2)
    tau = np.full(m, 1.0 / sigma_t ** 2)
    return PoseGraphData(
        n_robots=R_, n_poses=n_poses,
        r1=np.concatenate(E_r1).astype(np.int32), p1=np.concatenate(E_p1).astype(np.int32),
        r2=np.concatenate(E_r2).astype(np.int32), p2=np.concatenate(E_p2).astype(np.int32),
        R=np.ascontiguousarray(np.concatenate(E_R)), t=np.ascontiguousarray(np.concatenate(E_t)),
        kappa=kappa, tau=tau, weight=np.ones(m), fixed=np.concatenate(E_fixed),
        outlier=np.concatenate(E_out), gt_R=gt_R, gt_t=gt_t, init_R=init_R, init_t=init_t)


def lifting_matrix(r: int, d: int = 3, seed: int = 1) -> np.ndarray:
    """Fixed YLift in St(d, r) (r x d, orthonormal columns): dpgo's leader
    publishes a random lifting matrix (publishLiftingMatrix, drawio:2310-2322);
    here it is injected and seeded (SURVEY.md §7 hard part (b))."""
    rng = np.random.Generator(np.random.PCG64(seed))
    A = rng.standard_normal((r, d))
    Q, Rq = np.linalg.qr(A)
    return Q * np.sign(np.diag(Rq))[None, :]


def lift(R: np.ndarray, t: np.ndarray, YLift: np.ndarray) -> np.ndarray:
    """Lifted block X [n, r, 4]: Y_i = YLift R_i, p_i = YLift t_i."""
    n = R.shape[0]
    r = YLift.shape[0]
    X = np.empty((n, r, 4))
    X[:, :, :3] = np.einsum("ad,ndc->nac", YLift, R)
    X[:, :, 3] = t @ YLift.T
    return X


def config(name: str, seed: int = 0) -> PoseGraphData:
    """Named workloads of BASELINE.json configs (synthetic stand-ins)."""
    if name == "campus2":       # configs[0]: 2-robot Campus subset shape
        return make_pose_graph(2, 1000, 1200, seed=seed)
    if name == "campus6":       # configs[1]: 6 robots, 6k poses / 30k edges
        return make_pose_graph(6, 6000, 30000, seed=seed)
    if name == "synth100k":     # configs[3]: 100k poses / 500k edges, 8 robot blocks
        return make_pose_graph(8, 100_000, 500_000, seed=seed)
    if name == "synth8x20k":    # configs[4]: 8 robots x 20k poses, 5 edges/pose
        return make_pose_graph(8, 160_000, 800_000, seed=seed)
    raise KeyError(name)
