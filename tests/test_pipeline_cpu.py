"""configs[4] pipeline host logic (kmx.pipeline) on the CPU restatement: the
loop-closure stream plants ground-truth relative poses, the distributed
initialisation recovers the team from exact loop closures, and a tiny team
run (oracle LCD + oracle RBCD) accepts exactly the planted loop closures and
lowers the trajectory error."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

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


def _pipe_inputs():
    from kmx.dpgo.params import PGOAgentParameters
    g0 = make_pose_graph(3, 1500, 6000, f_inter=0.0, outlier_scope="robot", seed=4)
    st = PL.make_lc_stream(g0, 40, 20, n_feats=160, seed=2)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 5
    P.schedule = 1
    return g0, st, P


def _pipe_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.lcd import LcdParams
    from tests.mock_solver import OracleBlockSolver
    g0, st, P = _pipe_inputs()
    out = PL.run_pipeline(g0, st, P, LcdParams(), rank=rank, world=world, rounds=12, verifier=_oracle_verifier(st),
                          solver=OracleBlockSolver(P), exchange_device="cpu", return_trajectory=True)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_run_pipeline_world2_equals_world1():
    """configs[4]'s multi-rank branch: per-rank
    verification of the candidates whose query robot the rank owns,
    all_gather_object of the accepted loop closures, then RBCD over two gloo
    ranks — the same accepted set, initial error and final trajectories (bit
    for bit) as the single-process run."""
    from kmx.lcd import LcdParams
    from tests.mock_solver import OracleBlockSolver
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    g0, st, P = _pipe_inputs()
    ref = PL.run_pipeline(g0, st, P, LcdParams(), rounds=12, verifier=_oracle_verifier(st),
                          solver=OracleBlockSolver(P), return_trajectory=True)
    assert ref["lcd"]["accepted"] == ref["lcd"]["true_positives"] == 40
    for rank, out in got.items():
        for k in ("verified", "accepted", "true_positives"):
            assert out["lcd"][k] == ref["lcd"][k], (rank, k)
        assert out["init"]["ate_m"] == ref["init"]["ate_m"]
        assert out["init"]["shared_loop_closures"] == ref["init"]["shared_loop_closures"]
        assert out["dpgo"]["ate_m"] == ref["dpgo"]["ate_m"]
        for a, (R, t) in ref["trajectory"].items():
            assert np.array_equal(out["trajectory"][a][0], R) and np.array_equal(out["trajectory"][a][1], t), (rank, a)


def test_lcd_results_columnwise_and_structured():
    """kmx_lcd_result records read column by column (detector._results) keep
    every field of the ctypes records, and accepted_from_results takes the
    structured-array form (LoopClosureDetector.verify_arrays) and the dict form
    to the same loop closures."""
    from kmx import abi
    from kmx.lcd.detector import _RES_DT, _results
    n = 37
    res = (abi.LcdResult * n)()
    rng = np.random.default_rng(3)
    for i in range(n):
        r = res[i]
        r.n_matches, r.mono_inliers, r.stereo_inliers = 3 * i, 2 * i, i
        r.pnp_inliers, r.iterations_2d2d, r.accepted = i % 5, 7 * i, int(i % 3 == 0)
        for k in range(12):
            r.T_query_match[k] = rng.standard_normal()
    d = _results(res, n, refines=True)
    for i in range(n):
        r = res[i]
        assert (d[i]["n_matches"], d[i]["mono_inliers"], d[i]["stereo_inliers"], d[i]["pnp_inliers"],
                d[i]["iterations_2d2d"]) == (r.n_matches, r.mono_inliers, r.stereo_inliers, r.pnp_inliers,
                                            r.iterations_2d2d)
        assert d[i]["accepted"] is bool(r.accepted) and d[i]["pose_refined"] is bool(r.accepted)
        assert np.array_equal(d[i]["T_query_match"], np.array(r.T_query_match[:]))
    assert _results(res, 0) == []
    arr = np.frombuffer(res, dtype=_RES_DT, count=n).copy()
    stream = PL.make_lc_stream(_team(), n, 0, n_feats=60, seed=1)
    sel = np.arange(n)
    a1, a2 = PL.accepted_from_results(stream, sel, d), PL.accepted_from_results(stream, sel, arr)
    for k in ("r1", "p1", "r2", "p2", "R", "t", "truth"):
        assert np.array_equal(getattr(a1, k), getattr(a2, k)), k
    assert a1.r1.shape[0] == sum(i % 3 == 0 for i in range(n))
