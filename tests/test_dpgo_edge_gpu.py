"""Degenerate team graphs on the HIP path against the restatement: a robot
with no poses, a one-pose robot tied to the team by one shared loop closure,
an isolated one-pose robot with no edge (its block update is skipped), a hub
pose with more incidences than two gather chunks (one tile of its own, the
gather loops over many chunks), parallel (duplicate) edges and loop closures
that start at weight 0. Bar as in test_dpgo_gpu.py: equal tCG counts and
acceptance, poses within 1e-6, GNC weights within 1e-9."""
import numpy as np
import pytest

from kmx.dpgo.params import PGOAgentParameters
from kmx.synth import lift, lifting_matrix
from kmx.synth.pose_graph import PoseGraphData, _expm_so3

pytestmark = pytest.mark.gpu


def degenerate_team(seed=0):
    rng = np.random.default_rng(seed)
    n = np.array([200, 1, 0, 1, 900], np.int32)
    gt_R = [_expm_so3(rng.normal(0, 0.3, (int(k), 3))) for k in n]
    gt_t = [np.cumsum(rng.normal(0, 1.0, (int(k), 3)), axis=0) for k in n]
    E = []  # (r1, p1, r2, p2, fixed, weight)
    for a in (0, 4):
        E += [(a, i, a, i + 1, 1, 1.0) for i in range(int(n[a]) - 1)]
    E += [(0, int(i), 0, int(j), 0, 1.0) for i, j in rng.integers(0, 200, (120, 2)) if abs(int(i) - int(j)) > 1]
    E += [(4, 0, 4, int(j), 0, 1.0) for j in range(2, 702)]            # hub: pose 0 of robot 4, 701 incidences
    E += [(4, 10, 4, 20, 0, 1.0), (4, 10, 4, 20, 0, 1.0)]              # parallel edges
    E += [(0, 5, 1, 0, 0, 1.0)]                                        # the one-pose robot's only edge
    E += [(0, int(i), 4, int(j), 0, 0.0) for i, j in zip(rng.integers(0, 200, 30), rng.integers(0, 900, 30))]
    E += [(0, int(i), 4, int(j), 0, 1.0) for i, j in zip(rng.integers(0, 200, 30), rng.integers(0, 900, 30))]
    E = np.array(E, dtype=np.float64)
    r1, p1, r2, p2 = (E[:, k].astype(np.int32) for k in range(4))
    m = len(E)
    R = np.empty((m, 3, 3))
    t = np.empty((m, 3))
    outlier = rng.random(m) < 0.15
    outlier[E[:, 4] == 1] = False
    for e in range(m):
        Ra, ta = gt_R[r1[e]][p1[e]], gt_t[r1[e]][p1[e]]
        Rb, tb = gt_R[r2[e]][p2[e]], gt_t[r2[e]][p2[e]]
        Rr, tr = Ra.T @ Rb, Ra.T @ (tb - ta)
        if outlier[e]:
            Rr, tr = _expm_so3(rng.normal(0, 2.0, (1, 3)))[0], rng.uniform(-10, 10, 3)
        R[e] = Rr @ _expm_so3(rng.normal(0, 0.01, (1, 3)))[0]
        t[e] = tr + rng.normal(0, 0.1, 3)
    # odometry-chain initial guess, perturbed
    init_R, init_t = [], []
    for a, k in enumerate(n):
        Ri = gt_R[a] @ _expm_so3(rng.normal(0, 0.05, (int(k), 3))) if k else np.zeros((0, 3, 3))
        ti = gt_t[a] + rng.normal(0, 0.3, (int(k), 3)) if k else np.zeros((0, 3))
        init_R.append(Ri)
        init_t.append(ti)
    return PoseGraphData(n_robots=len(n), n_poses=n, r1=r1, p1=p1, r2=r2, p2=p2, R=R, t=t,
                         kappa=np.full(m, 1e4), tau=np.full(m, 1e2), weight=E[:, 5].copy(),
                         fixed=E[:, 4].astype(np.uint8), outlier=outlier, gt_R=gt_R, gt_t=gt_t,
                         init_R=init_R, init_t=init_t)


@pytest.mark.parametrize("red", ["0", "2"])
def test_degenerate_team_matches_oracle(gpu, monkeypatch, red):
    from kmx.dpgo.solver import BlockSolver
    from oracle.oracle import OraclePGO
    monkeypatch.setenv("KMX_RED", red)
    g = degenerate_team()
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(P.r, seed=1)
    s = BlockSolver(P, 0)
    try:
        s.set_graph_data(g)
        o = OraclePGO(P.to_c(), g)
        for a in range(g.n_robots):
            if g.n_poses[a]:
                X0 = lift(g.init_R[a], g.init_t[a], Y)
                s.set_iterate(a, X0)
                o.set_iterate(a, X0)
        s.refresh_local()
        o.refresh()
        skipped = 0
        for it in range(20):  # tCG runs 1 -> 10 steps over these rounds
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate()
            for a in range(g.n_robots):
                assert sg[a]["updated"] == so[a]["updated"], (it, a)
                assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
                assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
                if g.n_poses[a]:
                    d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
                    assert d <= 1e-6, (it, a, d)
            skipped += int(sg[3]["tcg_iterations"] == 0)
            if it % 5 == 4:
                s.refresh_local()
                assert s.update_weights() == o.update_weights()
                assert np.abs(s.get_weights() - o.get_weights()).max() <= 1e-9
        assert skipped == 20  # the isolated pose never moves
    finally:
        s.close()
