"""The HIP path against the frozen fixtures tests/golden/{dpgo,lcd}_small.npz
(outputs of the CPU restatement at the commit that made them): the GPU is
checked against stored data, not only against the oracle of the day.

Bars: LCD bit-exact (masks, counts, iterations, poses); dpgo tCG counts and
accept flags equal, per-pose Frobenius <= 1e-6 after every round (north_star),
weights <= 1e-9, mu identical."""
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLD))
import make_golden as MG  # noqa: E402


def test_dpgo_gpu_matches_fixture(gpu):
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.dpgo.solver import BlockSolver
    d = np.load(GOLD / "dpgo_small.npz")
    g = MG.graph_from(d)
    P = PGOAgentParameters(r=int(d["r"]))
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    for a, Xa in enumerate(MG.split_rows(g, d["X0"])):
        s.set_iterate(a, Xa)
    u = 0
    for it in range(MG.DPGO_ROUNDS):
        s.refresh_local()
        st = s.iterate()
        for a in range(g.n_robots):
            assert [st[a]["tcg_iterations"], st[a]["accepted"], st[a]["updated"]] == d["round_ints"][it, a, :3].tolist()
            f0 = d["round_f"][it, a, 0]
            assert abs(st[a]["f_init"] - f0) <= 1e-9 * max(1.0, abs(f0))
        if it % MG.DPGO_GNC_EVERY == MG.DPGO_GNC_EVERY - 1:
            s.refresh_local()
            assert s.update_weights() == d["mu"][u]
            assert np.abs(s.get_weights() - d["weights"][u]).max() <= 1e-9
            u += 1
    X = np.concatenate([s.get_iterate(a) for a in range(g.n_robots)])
    dist = np.linalg.norm((X - d["X_final"]).reshape(X.shape[0], -1), axis=1).max()
    assert dist <= 1e-6, dist


@pytest.mark.parametrize("k", range(len(MG.LCD_CASES)))
def test_lcd_gpu_matches_fixture(gpu, k):
    from kmx.lcd import LoopClosureDetector
    d = np.load(GOLD / "lcd_small.npz")
    pool = MG.pool_from(d)
    det = LoopClosureDetector(MG.lcd_params(MG.LCD_CASES[k]))
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ints = np.array([[r["n_matches"], r["mono_inliers"], r["stereo_inliers"], r["pnp_inliers"], int(r["accepted"]),
                      r["iterations_2d2d"]] for r in got], np.int32)
    assert np.array_equal(ints, d[f"ints_{k}"])
    assert np.array_equal(gm, d[f"masks_{k}"])
    assert np.array_equal(np.array([r["T_query_match"] for r in got]), d[f"T_{k}"])


@pytest.mark.parametrize("k", range(len(MG.LCD_REFINE_CASES)))
def test_lcd_refine_gpu_matches_fixture(gpu, k):
    """refine_pose 1 (the reference LcdParams.yaml:14): the HIP refit equals
    the frozen restatement output bit for bit."""
    from kmx.lcd import LoopClosureDetector
    d = np.load(GOLD / "lcd_small.npz")
    r = np.load(GOLD / "lcd_refine.npz")
    pool = MG.pool_from(d)
    det = LoopClosureDetector(MG.lcd_params(MG.LCD_REFINE_CASES[k], refine=1))
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ints = np.array([[x["n_matches"], x["mono_inliers"], x["stereo_inliers"], x["pnp_inliers"], int(x["accepted"]),
                      x["iterations_2d2d"]] for x in got], np.int32)
    assert np.array_equal(ints, r[f"ints_{k}"])
    assert np.array_equal(gm, r[f"masks_{k}"])
    assert np.array_equal(np.array([x["T_query_match"] for x in got]), r[f"T_{k}"])


@pytest.mark.parametrize("k", range(len(MG.LCD_CASES)))
def test_lcd_stream_gpu_matches_fixture(gpu, k):
    """rng_stream 1 (the ordered, candidate-serial sampler) against the frozen
    restatement output of the persistent-engine reading, bit for bit."""
    from kmx.lcd import LoopClosureDetector
    d = np.load(GOLD / "lcd_small.npz")
    r = np.load(GOLD / "lcd_stream.npz")
    pool = MG.pool_from(d)
    det = LoopClosureDetector(MG.lcd_params(MG.LCD_CASES[k], stream=1))
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ints = np.array([[x["n_matches"], x["mono_inliers"], x["stereo_inliers"], x["pnp_inliers"], int(x["accepted"]),
                      x["iterations_2d2d"]] for x in got], np.int32)
    assert np.array_equal(ints, r[f"ints_{k}"])
    assert np.array_equal(gm, r[f"masks_{k}"])
    assert np.array_equal(np.array([x["T_query_match"] for x in got]), r[f"T_{k}"])
