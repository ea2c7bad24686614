"""GPU parity at every BASELINE.json config size (configs[1]..configs[4]).

The smaller parity tests (test_dpgo_gpu.py, test_lcd_gpu.py, ...) cover the
kernels' corner cases; these run the HIP path on the benchmark workloads
themselves, at full size, against the CPU restatement:

  configs[1] campus6   6 robots, 6k poses / 30k edges: 22 concurrent rounds
                       crossing a GNC weight update; per round every robot's
                       tCG count equal and every pose within 1e-6 (Frobenius)
  configs[3] synth100k 100k poses / 500k edges, 8 robot blocks: 6 full-size
                       rounds and a GNC update, same bar
  configs[2] lcd50k    the real 50k-keyframe x 500-descriptor pool (800 MB of
                       descriptors uploaded whole): 512 candidates spread over
                       the pool, bit-exact results and inlier masks; BoW
                       queries against a 25k-entry database, bit-exact
  configs[4] 8x20k     the pipeline on 8 robots x 20k poses: identical accepted
                       loop-closure set, team graph and initial error; rounds
                       within 1e-6 m of the restatement
"""
import numpy as np
import pytest

from kmx.dpgo.params import PGOAgentParameters
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share; the oracle's per-robot threads


def _rounds_vs_oracle(g, P, rounds, gnc_at):
    from oracle.oracle import OraclePGO
    Y = lifting_matrix(P.r, seed=1)
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        X0 = lift(g.init_R[a], g.init_t[a], Y)
        s.set_iterate(a, X0)
        o.set_iterate(a, X0)
    worst = 0.0
    try:
        for it in range(rounds):
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate(threads=THREADS)
            for a in range(g.n_robots):
                assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
                assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
                d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
                worst = max(worst, d)
                assert d <= 1e-6, (it, a, d)
            if it in gnc_at:
                s.refresh_local()
                assert s.update_weights() == o.update_weights()
                wg, wo = s.get_weights(), o.get_weights()
                assert np.abs(wg - wo).max() <= 1e-9
    finally:
        s.close()
    return worst


@pytest.mark.timeout(600)
def test_configs1_campus6_rounds(gpu):
    g = config("campus6", seed=0)
    assert g.n_robots == 6 and g.n_total == 6000 and g.m == 30000
    P = PGOAgentParameters(r=5)
    _rounds_vs_oracle(g, P, 22, gnc_at={19})


@pytest.mark.timeout(900)
def test_configs3_synth100k_rounds(gpu):
    g = config("synth100k", seed=0)
    assert g.n_robots == 8 and g.n_total == 100_000 and g.m == 500_000
    P = PGOAgentParameters(r=5)
    _rounds_vs_oracle(g, P, 6, gnc_at={3})


@pytest.fixture(scope="module")
def lcd_pool():
    from kmx.synth.lcd import make_lcd_pool
    return make_lcd_pool(50_000, 500, seed=0)


@pytest.mark.timeout(900)
def test_configs2_lcd_pool_bit_exact(gpu, lcd_pool):
    from kmx.lcd import LcdParams, LoopClosureDetector
    from oracle import oracle as O
    pool = lcd_pool
    rng = np.random.default_rng(12)
    # 512 candidates across the whole pool, including its last frames (full-size indexing)
    nc = pool.cand_query.shape[0]
    idx = np.concatenate([np.sort(rng.choice(nc - 12, 500, replace=False)), np.arange(nc - 12, nc)])
    cq, cm = pool.cand_query[idx].copy(), pool.cand_match[idx].copy()
    p = LcdParams()
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(cq, cm, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool, cand_query=cq, cand_match=cm)
    assert len(got) == len(ref) == idx.shape[0] >= 512
    for i in range(len(got)):
        g, r = got[i], ref[i]
        assert (g["n_matches"], g["mono_inliers"], g["stereo_inliers"], g["accepted"], g["iterations_2d2d"]) == \
            (r.n_matches, r.mono_inliers, r.stereo_inliers, bool(r.accepted), r.iterations_2d2d), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i
    assert np.array_equal(gm, rm)
    acc = np.array([g["accepted"] for g in got])
    planted = cq % 2 == 0
    assert acc[planted].mean() > 0.9 and not acc[~planted].any()


@pytest.mark.timeout(600)
def test_configs2_bow_queries_bit_exact(gpu):
    """The bench's BoW leg shape: robot 1 queries robot 0's 25k-entry database
    (100k words); 1024 of its 25k queries against the restatement."""
    from kmx.lcd.bow import BowDatabase
    from kmx.synth.bow import make_bow_stream
    from oracle import oracle as O
    st = make_bow_stream(2, 25_000, n_words=100_000, seed=0)
    db = st.subset(np.nonzero(st.robot == 0)[0])
    assert db.n == 25_000
    qi = np.nonzero(st.robot == 1)[0]
    qs = st.subset(qi[np.random.default_rng(3).choice(qi.shape[0], 1024, replace=False)])
    G = BowDatabase(st.n_words)
    G.set_entries(db.vptr, db.words, db.weights)
    n, ids, sc = G.query(qs.vptr, qs.words, qs.weights, 50)
    D = O.OracleBowDb(st.n_words, db.vptr, db.words, db.weights)
    n0, ids0, sc0 = D.query(qs.vptr, qs.words, qs.weights, 50)
    assert np.array_equal(n, n0)
    for q in range(qs.n):
        assert np.array_equal(ids[q, :n[q]], ids0[q, :n[q]]), q
        assert np.array_equal(sc[q, :n[q]], sc0[q, :n[q]]), q


@pytest.mark.timeout(900)
def test_configs4_pipeline_8x20k(gpu):
    from kmx import pipeline as PL
    from kmx.lcd import LcdParams
    from kmx.synth import make_pose_graph
    from tests.mock_solver import OracleBlockSolver
    from tests.test_pipeline_cpu import _oracle_verifier
    g0 = make_pose_graph(8, 160_000, 800_000, f_inter=0.0, outlier_scope="robot", sigma_R=0.002,
                         sigma_t=0.02, seed=0)
    st = PL.make_lc_stream(g0, 8 * 60, 8 * 30, seed=1)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 3
    P.schedule = 1
    gpu_out = PL.run_pipeline(g0, st, P, LcdParams(), rounds=6, device=0)
    cpu_out = PL.run_pipeline(g0, st, P, LcdParams(), rounds=6, verifier=_oracle_verifier(st),
                              solver=OracleBlockSolver(P))
    for k in ("verified", "accepted", "true_positives"):
        assert gpu_out["lcd"][k] == cpu_out["lcd"][k], k
    assert gpu_out["lcd"]["accepted"] == gpu_out["lcd"]["true_positives"] == 8 * 60
    assert gpu_out["init"]["ate_m"] == cpu_out["init"]["ate_m"]
    assert gpu_out["init"]["edges"] == cpu_out["init"]["edges"]
    assert abs(gpu_out["dpgo"]["ate_m"] - cpu_out["dpgo"]["ate_m"]) < 1e-6
