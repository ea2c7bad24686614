"""Submap coarsening and the PoseGraph message (row f1)."""
import numpy as np

from kmx.frontend import PoseGraph, SubmapAtlas, measurements_from_pose_graph, pose_graph_from_measurements
from kmx.synth import make_pose_graph


def _atlas(g, a, **kw):
    at = SubmapAtlas(a, **kw)
    for k in range(int(g.n_poses[a])):
        at.add_keyframe(k, 1_000_000 * k, g.gt_R[a][k], g.gt_t[a][k])
    return at


def test_submap_graph_is_consistent_with_keyframes():
    g = make_pose_graph(2, 400, 900, noise_free=True, outlier_frac=0.0, f_inter=0.3, seed=2)
    A = [_atlas(g, a, max_distance=3.0, max_keyframes=10) for a in range(2)]
    for at in A:
        assert 1 < at.n_submaps < len(at.kf_submap)
        # submap odometry = relative submap poses
        for m in at.odometry_edges(1e4, 1e2):
            Ra, ta = at.submap_pose[m.p1]
            Rb, tb = at.submap_pose[m.p2]
            assert np.abs(Ra @ m.R - Rb).max() < 1e-12 and np.abs(Ra @ m.t + ta - tb).max() < 1e-9
        # keyframe poses are recovered from the submap poses
        Rs = np.array([p[0] for p in at.submap_pose])
        ts = np.array([p[1] for p in at.submap_pose])
        R, t = at.keyframe_trajectory(Rs, ts)
        a = at.robot
        assert np.abs(R - g.gt_R[a]).max() < 1e-12 and np.abs(t - g.gt_t[a]).max() < 1e-9
    # keyframe loop closures -> submap edges agree with the submap poses
    for e in np.nonzero(g.fixed == 0)[0][:200]:
        m = SubmapAtlas.submap_loop_closure(A[g.r1[e]], int(g.p1[e]), A[g.r2[e]], int(g.p2[e]), g.R[e], g.t[e],
                                            1e4, 1e2)
        if m is None:  # both keyframes in one submap
            assert g.r1[e] == g.r2[e] and A[g.r1[e]].kf_submap[g.p1[e]] == A[g.r2[e]].kf_submap[g.p2[e]]
            continue
        Ra, ta = A[m.r1].submap_pose[m.p1]
        Rb, tb = A[m.r2].submap_pose[m.p2]
        assert np.abs(Ra @ m.R - Rb).max() < 1e-9 and np.abs(Ra @ m.t + ta - tb).max() < 1e-8


def test_pose_graph_message_round_trip():
    g = make_pose_graph(2, 100, 250, seed=1)
    from tests.test_agent_cpu import _measurements
    ms = _measurements(g, 0)
    msg = pose_graph_from_measurements(ms)
    assert isinstance(msg, PoseGraph) and len(msg.edges) == len(ms)
    back = measurements_from_pose_graph(msg)
    for a, b in zip(ms, back):
        assert (a.r1, a.p1, a.r2, a.p2, a.fixedWeight) == (b.r1, b.p1, b.r2, b.p2, b.fixedWeight)
        assert abs(a.kappa - b.kappa) < 1e-9 * a.kappa and abs(a.tau - b.tau) < 1e-9 * a.tau
        assert np.array_equal(a.R, b.R) and np.array_equal(a.t, b.t)


def test_submap_team_init_and_rounds_on_restatement():
    """f1 -> f4 -> dpgo on the CPU restatement: the submap graph built from
    keyframe odometry and keyframe loop closures (through the PoseGraph
    message), robot 1 aligned to robot 0's frame by robust averaging over the
    shared submap loop closures (exact odometry: the planted frame change is
    recovered to rounding, the outlier closures rejected), then RBCD + GNC
    rounds lower the team cost."""
    from kmx.dpgo.driver import RBCDDriver
    from kmx.dpgo.params import PGOAgentParameters
    from tests.mock_solver import OracleBlockSolver
    from tests.submap_team import planted_alignment, submap_team
    g, atlases, sg, X0, align = submap_team(noise_free=True)
    assert sg.n_robots == 2 and all(1 < at.n_submaps < len(at.kf_submap) for at in atlases)
    assert int((sg.r1 != sg.r2).sum()) > 20
    R_WA, t_WA, w = align[1]
    Rp, tp = planted_alignment(g, 1)
    assert np.abs(R_WA - Rp).max() < 1e-9 and np.abs(t_WA - tp).max() < 1e-8
    assert 0 < w.sum() < len(w)  # outlier loop closures rejected
    P = PGOAgentParameters(r=5)
    drv = RBCDDriver(P, sg, solver=OracleBlockSolver(P))
    drv.initialize(X0)
    st0 = drv.step(with_stats=True)
    for _ in range(15):
        st = drv.step(with_stats=True)
    assert sum(s["f_final"] for s in st) < sum(s["f_init"] for s in st0)
