"""Edge cases of the HIP path against the CPU restatement.

dpgo: robot blocks of very different sizes (a 4-pose robot next to a 700-pose
one), a hub pose with hundreds of loop closures (a tile of one pose; the
degree-balanced gather splits it over every lane group), every gather variant
and both tilings. LCD: ragged feature counts (0 ... max), a candidate whose
query and match frame are the same, max_feats = 1024, and an empty batch."""
import numpy as np
import pytest

from kmx.synth import lift, lifting_matrix, make_pose_graph
from kmx.synth.pose_graph import PoseGraphData, _expm_so3, random_rotations

pytestmark = pytest.mark.gpu


def _hub_graph(seed=9):
    g = make_pose_graph(3, 1200, 4000, seed=seed)
    # shrink robot 0 to 4 poses: drop its edges beyond pose 3
    keep = ~(((g.r1 == 0) & (g.p1 > 3)) | ((g.r2 == 0) & (g.p2 > 3)))
    n_poses = g.n_poses.copy()
    n_poses[0] = 4
    rng = np.random.default_rng(seed)
    # hub: pose 17 of robot 1 gets 400 extra loop closures to random poses of robots 1 and 2
    k = 400
    r2 = rng.integers(1, 3, k).astype(np.int32)
    p2 = np.array([rng.integers(0, n_poses[r]) for r in r2], np.int32)
    ok = ~((r2 == 1) & (p2 == 17))
    r2, p2 = r2[ok], p2[ok]
    k = r2.shape[0]
    sel = lambda a: a[keep]  # noqa: E731
    return PoseGraphData(
        n_robots=3, n_poses=n_poses,
        r1=np.concatenate([sel(g.r1), np.full(k, 1, np.int32)]), p1=np.concatenate([sel(g.p1), np.full(k, 17, np.int32)]),
        r2=np.concatenate([sel(g.r2), r2]), p2=np.concatenate([sel(g.p2), p2]),
        R=np.ascontiguousarray(np.concatenate([sel(g.R), random_rotations(rng, k)])),
        t=np.ascontiguousarray(np.concatenate([sel(g.t), rng.uniform(-3, 3, (k, 3))])),
        kappa=np.concatenate([sel(g.kappa), np.full(k, 1e4)]), tau=np.concatenate([sel(g.tau), np.full(k, 1e2)]),
        weight=np.concatenate([sel(g.weight), np.ones(k)]), fixed=np.concatenate([sel(g.fixed), np.zeros(k, np.uint8)]),
        outlier=np.concatenate([sel(g.outlier), np.ones(k, bool)]),
        gt_R=[g.gt_R[0][:4], g.gt_R[1], g.gt_R[2]], gt_t=[g.gt_t[0][:4], g.gt_t[1], g.gt_t[2]],
        init_R=[g.init_R[0][:4], g.init_R[1], g.init_R[2]], init_t=[g.init_t[0][:4], g.init_t[1], g.init_t[2]])


@pytest.mark.parametrize("records", ["compact", "full"])
def test_hub_pose_and_tiny_robot(gpu, records):
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.dpgo.solver import BlockSolver
    from oracle.oracle import OraclePGO
    g = _hub_graph()
    if records == "full":  # one non-rotation measurement: 128-B records
        g.R[3] = g.R[3] + 1e-6 * np.random.default_rng(1).standard_normal((3, 3))
    assert np.bincount(np.concatenate([g.p1[g.r1 == 1], g.p2[g.r2 == 1]]))[17] > 300
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5, seed=1)
    rng = np.random.default_rng(2)
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    o = OraclePGO(P.to_c(), g)
    for a in range(3):
        k = int(g.n_poses[a])
        X = lift(g.init_R[a] @ _expm_so3(rng.normal(0, 0.05, (k, 3))), g.init_t[a] + rng.normal(0, 0.2, (k, 3)), Y)
        s.set_iterate(a, X)
        o.set_iterate(a, X)
    for it in range(8):
        s.refresh_local()
        o.refresh()
        sg, so = s.iterate(), o.iterate()
        for a in range(3):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a)
            d = np.abs(s.get_iterate(a) - o.get_iterate(a)).max()
            assert d <= 1e-6, (it, a, d)
        if it == 3:
            s.refresh_local()
            o.refresh()
            assert s.update_weights() == o.update_weights()
            assert np.abs(s.get_weights() - o.get_weights()).max() <= 1e-9
    s.close()


def test_lcd_ragged_and_limits(gpu):
    from kmx.lcd import LcdParams, LoopClosureDetector
    from kmx.synth.lcd import make_lcd_pool
    from oracle import oracle as O
    pool = make_lcd_pool(20, 1024, seed=6)
    pool.n_feats = np.array([1024, 1024, 0, 300, 4, 300, 5, 300, 9, 9, 10, 300, 300, 0, 700, 700, 1, 1, 64, 1024],
                            np.int32)
    cq = np.array([0, 2, 3, 4, 6, 8, 10, 12, 14, 16, 18, 19, 5, 7, 0], np.int32)
    cm = np.array([1, 3, 2, 5, 7, 9, 11, 13, 15, 17, 19, 18, 5, 3, 19], np.int32)  # incl. q == m
    p = LcdParams()
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(cq, cm, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool, cand_query=cq, cand_match=cm)
    for i in range(cq.shape[0]):
        r = ref[i]
        g = got[i]
        assert (g["n_matches"], g["mono_inliers"], g["stereo_inliers"], g["accepted"], g["iterations_2d2d"]) == \
            (r.n_matches, r.mono_inliers, r.stereo_inliers, bool(r.accepted), r.iterations_2d2d), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:]), equal_nan=True), i
    assert np.array_equal(gm, rm)
    assert got[0]["accepted"]                      # planted pair at max_feats = 1024
    assert not got[1]["accepted"] and got[1]["n_matches"] == 0   # empty query frame
    empty, _ = det.verify(np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert empty == []
