"""Local chordal initialisation (kmx.dpgo.init):
exact on noise-free measurements, better than the odometry chain on noisy
ones (by the local problem's cost), and selectable on the agent API."""
import numpy as np

from kmx.dpgo.init import chordal_initialization
from kmx.synth import make_pose_graph


def _robot_edges(g, a=0):
    own = (g.r1 == a) & (g.r2 == a)
    return [(int(g.p1[e]), int(g.p2[e]), g.R[e], g.t[e], float(g.kappa[e]), float(g.tau[e]), float(g.weight[e]))
            for e in np.nonzero(own)[0]]


def _cost(Rs, ts, edges):
    c = 0.0
    for (i, j, R, t, k, tau, w) in edges:
        c += w * (k * np.sum((Rs[j] - Rs[i] @ R) ** 2) + tau * np.sum((ts[j] - ts[i] - Rs[i] @ t) ** 2))
    return 0.5 * c


def _relative(Rs, ts):  # gauge: the first pose at the origin
    R0, t0 = Rs[0], ts[0]
    return np.einsum("ij,njk->nik", R0.T, Rs), (ts - t0) @ R0


def test_chordal_exact_on_noise_free_graph():
    g = make_pose_graph(1, 300, 900, outlier_frac=0.0, noise_free=True, seed=2)
    Rs, ts = chordal_initialization(int(g.n_poses[0]), _robot_edges(g))
    Rg, tg = _relative(g.gt_R[0], g.gt_t[0])
    assert np.abs(Rs - Rg).max() < 1e-9
    assert np.abs(ts - tg).max() < 1e-7
    assert np.allclose(np.einsum("nij,nkj->nik", Rs, Rs), np.eye(3), atol=1e-12)


def test_chordal_beats_odometry_on_noisy_graph():
    g = make_pose_graph(1, 400, 1400, outlier_frac=0.0, sigma_R=0.02, sigma_t=0.1, seed=5)
    edges = _robot_edges(g)
    Rs, ts = chordal_initialization(int(g.n_poses[0]), edges)
    Ro, to = _relative(g.init_R[0], g.init_t[0])  # the odometry chain
    assert _cost(Rs, ts, edges) < 0.5 * _cost(Ro, to, edges)
    assert np.all(np.abs(np.linalg.det(Rs) - 1.0) < 1e-12)


def test_agent_chordal_initialization():
    from kmx.dpgo.agent import PGOAgent
    from kmx.dpgo.messages import RelativeSEMeasurement
    from kmx.dpgo.params import PGOAgentParameters
    from tests.mock_solver import OracleBlockSolver
    g = make_pose_graph(1, 200, 700, outlier_frac=0.0, noise_free=True, seed=4)
    P = PGOAgentParameters(r=5, num_robots=1, localInitializationMethod="chordal")
    ag = PGOAgent(0, P, solver=OracleBlockSolver(P))
    for e in range(g.m):
        ag.addMeasurement(RelativeSEMeasurement(0, 0, int(g.p1[e]), int(g.p2[e]), 3, g.R[e], g.t[e],
                                                float(g.kappa[e]), float(g.tau[e]),
                                                fixedWeight=bool(g.fixed[e])))
    ag.initialize()
    T = ag.getTrajectoryInLocalFrame().reshape(3, -1, 4).transpose(1, 0, 2)
    Rg, tg = _relative(g.gt_R[0], g.gt_t[0])
    assert np.abs(T[:, :, :3] - Rg).max() < 1e-8
    assert np.abs(T[:, :, 3] - tg).max() < 1e-6
