"""Distributed initialisation (row f4): frame alignment by GNC-TLS robust
single-pose averaging over shared loop closures (host logic, numpy)."""
import numpy as np

from kmx.dpgo.init import align_to_world, robust_single_pose_averaging, transform_trajectory
from kmx.dpgo.messages import RelativeSEMeasurement
from kmx.synth import make_pose_graph
from kmx.synth.pose_graph import _expm_so3


def test_robust_averaging_rejects_outliers():
    rng = np.random.default_rng(0)
    R0 = _expm_so3(np.array([[0.3, -0.2, 0.5]]))[0]
    t0 = np.array([1.0, -2.0, 0.5])
    n, k = 40, 12
    R = np.einsum("ij,njk->nik", R0, _expm_so3(rng.normal(0, 0.01, (n, 3))))
    t = t0 + rng.normal(0, 0.1, (n, 3))
    R[:k] = _expm_so3(rng.normal(0, 2.0, (k, 3)))
    t[:k] = rng.uniform(-10, 10, (k, 3))
    Rm, tm, w = robust_single_pose_averaging(R, t, 1e4, 1e2)
    assert np.all(w[:k] < 1e-6) and np.all(w[k:] > 0.99)
    assert np.abs(Rm - R0).max() < 1e-2 and np.abs(tm - t0).max() < 0.1  # 28 inliers, sigma 0.01 rad / 0.1 m


def _lcs(g, a):
    out = []
    for e in np.nonzero((g.r1 != g.r2) & ((g.r1 == a) | (g.r2 == a)))[0]:
        out.append(RelativeSEMeasurement(int(g.r1[e]), int(g.r2[e]), int(g.p1[e]), int(g.p2[e]), 3, g.R[e], g.t[e],
                                         float(g.kappa[e]), float(g.tau[e])))
    return out


def test_align_robot_frames_with_outliers():
    # exact measurements (the odometry chains are the ground truth up to each
    # robot's frame), 20 % outlier loop closures
    g = make_pose_graph(3, 900, 3000, outlier_frac=0.2, f_inter=0.3, noise_free=True, seed=5)
    # robot 0 in the world frame (ground truth); robots 1, 2 initialised by
    # their odometry chain in their own frames (first pose at the origin)
    world = {(0, i): (g.gt_R[0][i], g.gt_t[0][i]) for i in range(int(g.n_poses[0]))}
    for a in (1, 2):
        R_loc = np.einsum("ji,njk->nik", g.init_R[a][0], g.init_R[a])
        t_loc = (g.init_t[a] - g.init_t[a][0]) @ g.init_R[a][0]
        out = align_to_world(_lcs(g, a), a, R_loc, t_loc, world)
        assert out is not None
        R_WA, t_WA, w = out
        Rw, tw = transform_trajectory(R_WA, t_WA, R_loc, t_loc)
        # the aligned trajectory starts where the ground truth does
        assert np.abs(Rw - g.gt_R[a]).max() < 1e-9
        assert np.abs(tw - g.gt_t[a]).max() < 1e-8
        assert 0 < w.sum() < len(w)  # some candidates (outlier loop closures) rejected
