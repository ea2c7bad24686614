"""configs[4] pipeline host logic (kmx.pipeline) on the CPU restatement: the
loop-closure stream plants ground-truth relative poses, the distributed
initialisation recovers the team from exact loop closures, and a tiny team
run (oracle LCD + oracle RBCD) accepts exactly the planted loop closures and
lowers the trajectory error."""
import numpy as np

from kmx import pipeline as PL
from kmx.synth import make_pose_graph


def _team():
    return make_pose_graph(3, 3000, 12000, f_inter=0.0, outlier_scope="robot", seed=4)


def test_base_graph_has_no_inter_robot_edges():
    g = _team()
    assert not np.any(g.r1 != g.r2)
    assert g.outlier.sum() > 0


def test_stream_plants_ground_truth_poses():
    g = _team()
    st = PL.make_lc_stream(g, 40, 20, n_feats=120, seed=2)
    assert np.all(np.diff(st.r_q) >= 0)              # grouped by query robot
    assert np.all(st.r_q != st.r_m)                  # inter-robot only
    t = np.nonzero(st.truth)[0]
    assert t.shape[0] == 40 and (~st.truth).sum() > 0
    for c in t:
        k = st.cand_query[c] // 2
        assert st.cand_match[c] == 2 * k + 1
        Rq, tq = g.gt_R[st.r_q[c]][st.p_q[c]], g.gt_t[st.r_q[c]][st.p_q[c]]
        Rm, tm = g.gt_R[st.r_m[c]][st.p_m[c]], g.gt_t[st.r_m[c]][st.p_m[c]]
        assert np.allclose(st.pool.R_qm[k], Rq.T @ Rm, atol=1e-12)
        assert np.allclose(st.pool.t_qm[k], Rq.T @ (tm - tq), atol=1e-12)
        assert np.linalg.norm(tm - tq) <= 3.0


def test_global_init_exact_loop_closures():
    g0 = make_pose_graph(3, 3000, 12000, f_inter=0.0, outlier_scope="robot", noise_free=True, seed=4)
    st = PL.make_lc_stream(g0, 30, 0, n_feats=60, seed=2)
    k = st.cand_query // 2
    acc = PL.Accepted(r1=st.r_q, p1=st.p_q, r2=st.r_m, p2=st.p_m, R=st.pool.R_qm[k], t=st.pool.t_qm[k],
                      truth=st.truth, n_verified=30)
    g = PL.team_graph(g0, acc, 1e4, 1e2)
    world, frames = PL.global_init(g, PL.odometry_init(g))
    assert PL.ate_rmse(g, world) < 1e-6
    gt = {a: (g.gt_R[a], g.gt_t[a]) for a in range(3)}
    assert PL.ate_rmse(g, gt) == 0.0


def _oracle_verifier(stream):
    from kmx.lcd import LcdParams
    from oracle import oracle as O

    def verify(cq, cm):
        res, _ = O.lcd_verify(LcdParams().to_c(), stream.pool, cand_query=cq, cand_match=cm, masks=False)
        return [{"accepted": bool(r.accepted), "T_query_match": np.array(r.T_query_match[:])} for r in res]
    return verify


def test_run_pipeline_oracle():
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.lcd import LcdParams
    from tests.mock_solver import OracleBlockSolver
    g0 = _team()
    st = PL.make_lc_stream(g0, 60, 30, n_feats=200, seed=2)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 10
    P.schedule = 1
    out = PL.run_pipeline(g0, st, P, LcdParams(), rounds=40, verifier=_oracle_verifier(st),
                          solver=OracleBlockSolver(P))
    assert out["lcd"]["accepted"] == out["lcd"]["true_positives"] == 60
    assert out["dpgo"]["ate_m"] < out["init"]["ate_m"]
