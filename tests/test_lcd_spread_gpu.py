"""The spread form of the 2D-2D RANSAC (lcd.hip k_rs_hyps, whose last wave per candidate replays the control, /
k_rs_finish): a synchronous call of a few candidates — the
reference verifies one candidate per call — computes ranges of each
candidate's hypotheses on many waves at once and replays the serial loop's
control over them.

Bar: bit-exact against the restatement (oracle/lcd_oracle.c, one hypothesis at
a time) and against the work-queue kernel on the same candidates: identical
match counts, 2D-2D / 3D-3D / PnP inlier counts and masks, iteration counts and
poses — including candidates that run to the iteration cap (look-alikes that
fail geometry), caps that end a range part way, and short loops that stop
inside the first range."""
import numpy as np
import pytest

from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool

pytestmark = pytest.mark.gpu

FIELDS = ("n_matches", "mono_inliers", "stereo_inliers", "pnp_inliers", "iterations_2d2d")


def _det(p, pool, spread, monkeypatch):
    monkeypatch.setenv("KMX_LCD_SPREAD", str(spread))
    d = LoopClosureDetector(p)
    d.set_pool(pool)
    return d


def _params(algo, recovery, **kw):
    return LcdParams(ransac_2d2d_algorithm=algo, pose_recovery_type=int(recovery == 1),
                     ransac_use_1point_3d3d=int(recovery != 2), refine_pose=int(recovery != 1), **kw)


def _same_as_oracle(got, gm, ref, rm):
    for i, (g, r) in enumerate(zip(got, ref)):
        assert tuple(g[k] for k in FIELDS) == tuple(getattr(r, k) for k in FIELDS), (i, g, r.iterations_2d2d)
        assert g["accepted"] == bool(r.accepted), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i
    assert np.array_equal(gm, rm)


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
@pytest.mark.parametrize("recovery", [0, 1, 2], ids=["1point", "pnp", "arun"])
def test_spread_matches_oracle_and_work_queue(gpu, monkeypatch, algo, recovery):
    """Planted loop closures (short loops), random pairs (few matches) and
    look-alike pairs (true_frac 0.15: long loops) through the spread form
    (every candidate of the call) and the work-queue kernel."""
    from oracle import oracle as O
    pool = make_lcd_pool(24, 300, true_frac=0.15, false_frac=0.35, seed=21)
    p = _params(algo, recovery)
    ds = _det(p, pool, 64, monkeypatch)
    dq = _det(p, pool, 0, monkeypatch)
    try:
        got, gm = ds.verify(pool.cand_query, pool.cand_match, with_masks=True)
        ref, rm = O.lcd_verify(p.to_c(), pool)
        _same_as_oracle(got, gm, ref, rm)
        wq, wm = dq.verify(pool.cand_query, pool.cand_match, with_masks=True)
        for i, (a, b) in enumerate(zip(got, wq)):
            assert tuple(a[k] for k in FIELDS) == tuple(b[k] for k in FIELDS), i
            assert a["accepted"] == b["accepted"], i
            assert np.array_equal(a["T_query_match"], b["T_query_match"]), i
        assert np.array_equal(gm, wm)
        its = [g["iterations_2d2d"] for g in got]
        assert max(its) > 66, its  # some loops run past the first range
    finally:
        ds.close()
        dq.close()


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
@pytest.mark.parametrize("max_iter", [1, 7, 70, 500])
def test_spread_hard_candidates_to_the_cap(gpu, monkeypatch, algo, max_iter):
    """Look-alike pairs (150 descriptor look-alikes, no true correspondence):
    every loop runs to its cap, across range boundaries (66, 510) and inside
    the first range; one candidate per call as the reference's verification
    thread does, and all of them in one call."""
    from oracle import oracle as O
    pool = make_lcd_pool(12, 500, true_frac=0.0, false_frac=0.3, seed=3)
    cq, cm = pool.cand_query[0::2], pool.cand_match[0::2]
    p = _params(algo, 0, ransac_max_iterations=max_iter)
    d = _det(p, pool, 8, monkeypatch)
    try:
        ref, rm = O.lcd_verify(p.to_c(), pool, cand_query=cq, cand_match=cm)
        got, gm = d.verify(cq, cm, with_masks=True)
        _same_as_oracle(got, gm, ref, rm)
        assert all(not g["accepted"] for g in got)
        assert all(g["n_matches"] >= 100 for g in got)
        for i in range(len(cq)):  # one call each
            g1, m1 = d.verify(cq[i:i + 1], cm[i:i + 1], with_masks=True)
            assert tuple(g1[0][k] for k in FIELDS) == tuple(got[i][k] for k in FIELDS), i
            assert np.array_equal(m1[0], gm[i])
    finally:
        d.close()


def test_spread_call_chain_equals_batched(gpu, monkeypatch):
    """computeMatchedIndices -> geometricVerificationNister -> recoverPose one
    candidate at a time (kmx_lcd_match, then kmx_lcd_verify_matches with one
    candidate: the spread form) against the batched work-queue verify."""
    pool = make_lcd_pool(16, 300, true_frac=0.3, false_frac=0.3, seed=8)
    p = _params(0, 0)
    d1 = _det(p, pool, 8, monkeypatch)
    dq = _det(p, pool, 0, monkeypatch)
    try:
        ref, _ = dq.verify(pool.cand_query, pool.cand_match)
        for i, (a, b) in enumerate(zip(pool.cand_query, pool.cand_match)):
            iq, im = d1.computeMatchedIndices(int(a), int(b))
            assert len(iq) == ref[i]["n_matches"]
            ok, iq2, im2, T = d1.geometricVerificationNister(int(a), int(b), iq, im)
            assert len(iq2) == ref[i]["mono_inliers"], i
            if not ok:
                assert not ref[i]["accepted"], i
                continue
            ok2, T2, inl = d1.recoverPose(int(a), int(b), iq2, im2, T)
            assert ok2 == ref[i]["accepted"], i
            assert int(inl.sum()) == ref[i]["stereo_inliers"], i
            if ok2:
                assert np.array_equal(T2[:3, :3].reshape(9), ref[i]["T_query_match"][:9]), i
                assert np.array_equal(T2[:3, 3], ref[i]["T_query_match"][9:]), i
    finally:
        d1.close()
        dq.close()


@pytest.mark.parametrize("refine", [0, 1], ids=["keep", "refine"])
def test_spread_max_feats_1024_and_refine_off(gpu, monkeypatch, refine):
    """One candidate per call at max_feats = 1024 (the 1-point recovery's
    staging then needs 75 KB of LDS: the launch raises the dynamic limit) and
    ragged frames, with refine_pose on and off (the recovery sums T_j itself,
    or re-forms it from the staged points): bit-exact against the
    restatement."""
    from oracle import oracle as O
    pool = make_lcd_pool(20, 1024, seed=6)
    pool.n_feats = np.array([1024, 1024, 0, 300, 4, 300, 5, 300, 9, 9, 10, 300, 300, 0, 700, 700, 1, 1, 64, 1024],
                            np.int32)
    cq = np.array([0, 2, 3, 4, 6, 8, 10, 12, 14, 16, 18, 19, 5, 7, 0], np.int32)
    cm = np.array([1, 3, 2, 5, 7, 9, 11, 13, 15, 17, 19, 18, 5, 3, 19], np.int32)
    p = LcdParams(refine_pose=refine)
    d = _det(p, pool, 8, monkeypatch)
    try:
        ref, rm = O.lcd_verify(p.to_c(), pool, cand_query=cq, cand_match=cm)
        for i in range(cq.shape[0]):
            g, gm = d.verify(cq[i:i + 1], cm[i:i + 1], with_masks=True)
            r = ref[i]
            assert tuple(g[0][k] for k in FIELDS) == tuple(getattr(r, k) for k in FIELDS), i
            assert g[0]["accepted"] == bool(r.accepted), i
            assert np.array_equal(g[0]["T_query_match"], np.array(r.T_query_match[:]), equal_nan=True), i
            assert np.array_equal(gm[0], rm[i]), i
        assert ref[0].accepted  # the planted pair at max_feats = 1024 went through the recovery
    finally:
        d.close()
