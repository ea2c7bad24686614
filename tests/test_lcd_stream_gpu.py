"""The LCD boundary the way Kimera-Distributed drives it:
frames added one at a time (addVLCFrame, drawio:2601) and the two
verification calls on caller-supplied correspondences
(geometricVerificationNister / recoverPose, drawio:2589-2598), through the C
ABI, bit-exact against the CPU restatement (oracle/lcd_oracle.c
orc_lcd_verify_pairs_batch). Also the LC5 ordered sampler (rng_stream 1, the
OpenGV fork's thread_local engine, README.md:35-36) against the restatement's
persistent-engine reading."""
import numpy as np
import pytest

from kmx import abi
from kmx.lcd import LcdParams, LoopClosureDetector, VLCFrame
from kmx.synth.lcd import make_lcd_pool

pytestmark = pytest.mark.gpu

FIELDS = ("n_matches", "mono_inliers", "stereo_inliers", "pnp_inliers", "iterations_2d2d")


def _same(g, r, i):
    assert tuple(g[k] for k in FIELDS) == tuple(getattr(r, k) for k in FIELDS), i
    assert g["accepted"] == bool(r.accepted), i
    assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i


def _params(recovery, algo=0, **kw):
    """recovery 0: 1-point 3D-3D (reference config), 1: EPnP, 2: Arun."""
    return LcdParams(pose_recovery_type=int(recovery == 1), ransac_2d2d_algorithm=algo,
                     ransac_use_1point_3d3d=int(recovery != 2), refine_pose=int(recovery != 1), **kw)


def test_frames_added_one_at_a_time_match_whole_pool(gpu):
    """1,000 frames added one by one (capacity doubling, no re-upload) give
    the same verification results, bit for bit, as the whole-pool upload."""
    pool = make_lcd_pool(1000, 120, seed=21)
    p = LcdParams()
    whole = LoopClosureDetector(p)
    whole.set_pool(pool)
    ref, rm = whole.verify(pool.cand_query, pool.cand_match, with_masks=True)
    stream = LoopClosureDetector(p)
    caps = set()
    for f in range(pool.n_frames):
        fid = stream.add_frames(pool.n_feats[f:f + 1], pool.desc[f:f + 1], pool.bearings[f:f + 1],
                                pool.points[f:f + 1])
        assert fid == f
        caps.add(stream.pool_info()["capacity"])
    info = stream.pool_info()
    assert info["n_frames"] == 1000 and info["max_feats"] == 120
    assert sorted(caps) == [64, 128, 256, 512, 1024]  # doubling, not one allocation per frame
    got, gm = stream.verify(pool.cand_query, pool.cand_match, with_masks=True)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert all(np.array_equal(g[k], r[k]) for k in g), i
    assert np.array_equal(gm, rm)
    # frames added after verification stay usable, and the earlier ones unchanged
    extra = make_lcd_pool(4, 120, seed=22)
    fid = stream.add_frames(extra.n_feats, extra.desc, extra.bearings, extra.points)
    assert fid == 1000
    g2, _ = stream.verify(extra.cand_query + 1000, extra.cand_match + 1000)
    e = LoopClosureDetector(p)
    e.set_pool(extra)
    r2, _ = e.verify(extra.cand_query, extra.cand_match)
    for a, b in zip(g2, r2):
        assert a["accepted"] == b["accepted"] and np.array_equal(a["T_query_match"], b["T_query_match"])
    # a frame of another feature stride is refused
    with pytest.raises(abi.KmxError):
        stream.add_frames(extra.n_feats[:1], np.zeros((1, 200, 32), np.uint8), np.zeros((1, 200, 3)),
                          np.zeros((1, 200, 3)))


def test_frames_added_while_calls_are_in_flight(gpu):
    """The streaming pattern: a frame arrives, the candidates among the frames
    so far are verified asynchronously, the next frame arrives. Appends that
    double the pool (device-to-device copy, old pool freed) run while up to
    four small calls' RANSACs read it from their own streams; the synchronous
    results at the end, and of a call made between appends, equal the
    whole-pool path's bit for bit."""
    pool = make_lcd_pool(200, 120, seed=31)
    p = LcdParams()
    whole = LoopClosureDetector(p)
    whole.set_pool(pool)
    ref, rm = whole.verify(pool.cand_query, pool.cand_match, with_masks=True)
    stream = LoopClosureDetector(p)
    cq, cm = pool.cand_query, pool.cand_match
    mid = None
    for f in range(pool.n_frames):
        stream.add_frames(pool.n_feats[f:f + 1], pool.desc[f:f + 1], pool.bearings[f:f + 1], pool.points[f:f + 1])
        ready = np.flatnonzero(np.maximum(cq, cm) <= f)
        if len(ready):
            stream.verify_async(cq[ready], cm[ready])
        if f == 120:
            mid = (ready, stream.verify(cq[ready], cm[ready], with_masks=True))
    stream.sync()
    ready, (g1, m1) = mid
    assert np.array_equal(m1, rm[ready][:, :m1.shape[1]])
    for i, g in zip(ready, g1):
        assert all(np.array_equal(g[k], ref[i][k]) for k in g), i
    got, gm = stream.verify(cq, cm, with_masks=True)
    assert np.array_equal(gm, rm)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert all(np.array_equal(g[k], r[k]) for k in g), i


def test_add_vlc_frame_vertices(gpu):
    """addVLCFrame keys frames by (robot_id, pose_id) and pads them to the
    pool stride (LcdParams nfeatures); computeMatchedIndices on vertices is
    the pool kNN2 and agrees with the stand-alone matcher."""
    pool = make_lcd_pool(6, 150, seed=4)
    det = LoopClosureDetector(LcdParams(nfeatures=200))
    for f in range(pool.n_frames):
        n = int(pool.n_feats[f])
        det.addVLCFrame(VLCFrame(robot_id=f % 2, pose_id=100 + f, descriptors=pool.desc[f, :n],
                                 versors=pool.bearings[f, :n], keypoints=pool.points[f, :n]))
    assert det.pool_info()["max_feats"] == 200
    iq, im = det.computeMatchedIndices((0, 100), (1, 101))
    sq, sm = LoopClosureDetector.compute_matched_indices(pool.desc[0], pool.desc[1])
    assert np.array_equal(iq, sq) and np.array_equal(im, sm) and len(iq) > 20


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
@pytest.mark.parametrize("recovery", [0, 1, 2], ids=["1point", "pnp", "arun"])
def test_verify_matches_stages_match_oracle(gpu, recovery, algo):
    from oracle import oracle as O
    pool = make_lcd_pool(24, 300, seed=3)
    p = _params(recovery, algo)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    cq, cm = pool.cand_query, pool.cand_match
    pairs, k = det.match(cq, cm)
    corr = [(pairs[i, :k[i], 0], pairs[i, :k[i], 1]) for i in range(len(cq))]
    # both stages on the kNN2 pairs = the fused verify
    full, fm = det.verify(cq, cm, with_masks=True)
    got, gm = det.verify_matches(cq, cm, corr, stages=3, with_masks=True)
    ref, rm = O.lcd_verify_pairs(p.to_c(), pool, cq, cm, corr, stages=3)
    for i in range(len(cq)):
        _same(got[i], ref[i], i)
        assert got[i]["accepted"] == full[i]["accepted"]
        assert np.array_equal(got[i]["T_query_match"], full[i]["T_query_match"])
    assert np.array_equal(gm, rm) and np.array_equal(gm, fm)
    # geometricVerificationNister alone
    g1, m1 = det.verify_matches(cq, cm, corr, stages=abi.KMX_LCD_STAGE_2D2D, with_masks=True)
    r1, rm1 = O.lcd_verify_pairs(p.to_c(), pool, cq, cm, corr, stages=1)
    for i in range(len(cq)):
        _same(g1[i], r1[i], i)
    assert np.array_equal(m1, rm1)
    # recoverPose alone on the 2D-2D inliers, rotation from the 2D-2D pose
    inl = [(a[(m1[i, :len(a)] & 1) > 0], b[(m1[i, :len(a)] & 1) > 0]) for i, (a, b) in enumerate(corr)]
    prior = np.array([g["T_query_match"] for g in g1])
    g2, m2 = det.verify_matches(cq, cm, inl, stages=abi.KMX_LCD_STAGE_RECOVER, T_prior=prior, with_masks=True)
    r2, rm2 = O.lcd_verify_pairs(p.to_c(), pool, cq, cm, inl, stages=2, T_prior=prior)
    for i in range(len(cq)):
        _same(g2[i], r2[i], i)
    assert np.array_equal(m2, rm2)
    # the chain recovers what the fused path recovers wherever the 2D-2D gate passed
    for i in range(len(cq)):
        if g1[i]["accepted"]:
            assert g2[i]["accepted"] == full[i]["accepted"], i
            assert g2[i]["stereo_inliers"] == full[i]["stereo_inliers"], i
            assert g2[i]["pnp_inliers"] == full[i]["pnp_inliers"], i
            assert np.array_equal(g2[i]["T_query_match"], full[i]["T_query_match"]), i


def test_structured_results_equal_dicts(gpu):
    """verify_arrays and verify_matches_csr(as_arrays=True) return the same
    kmx_lcd_result records as the dict forms, field for field."""
    pool = make_lcd_pool(16, 200, seed=5)
    det = LoopClosureDetector(LcdParams())
    det.set_pool(pool)
    cq, cm = pool.cand_query, pool.cand_match
    full, _ = det.verify(cq, cm)
    arr = det.verify_arrays(cq, cm)
    pairs, k = det.match(cq, cm)
    mptr = np.r_[0, np.cumsum(k)].astype(np.int64)
    sel = np.arange(pairs.shape[1])[None, :] < k[:, None]
    iq, im = pairs[:, :, 0][sel], pairs[:, :, 1][sel]
    dres, _ = det.verify_matches_csr(cq, cm, mptr, iq, im)
    ares, _ = det.verify_matches_csr(cq, cm, mptr, iq, im, as_arrays=True)
    assert arr.shape == (len(cq),) and ares.shape == (len(cq),) and sum(r["accepted"] for r in full) > 0
    for d, a in ((full, arr), (dres, ares)):
        for i, r in enumerate(d):
            for f in ("n_matches", "mono_inliers", "stereo_inliers", "pnp_inliers", "iterations_2d2d"):
                assert r[f] == int(a[f][i]), (f, i)
            assert r["accepted"] == bool(a["accepted"][i])
            assert np.array_equal(r["T_query_match"], a["T_query_match"][i])
    assert det.verify_arrays(cq[:0], cm[:0]).shape == (0,)


def test_reference_shaped_single_calls(gpu):
    """computeMatchedIndices -> geometricVerificationNister -> recoverPose on
    vertices, as verifyLoopSpin calls them (drawio:2638-2657)."""
    pool = make_lcd_pool(8, 300, seed=7)
    det = LoopClosureDetector(LcdParams())
    det.set_pool(pool)
    full, _ = det.verify(pool.cand_query, pool.cand_match)
    for i, (q, m) in enumerate(zip(pool.cand_query, pool.cand_match)):
        iq, im = det.computeMatchedIndices(int(q), int(m))
        ok, iq2, im2, T_mono = det.geometricVerificationNister(int(q), int(m), iq, im)
        assert ok == (full[i]["mono_inliers"] >= 10)
        assert len(iq2) == full[i]["mono_inliers"] or not ok
        if not ok:
            continue
        ok3, T, inl3 = det.recoverPose(int(q), int(m), iq2, im2, T_mono)
        assert ok3 == full[i]["accepted"] and int(inl3.sum()) == full[i]["stereo_inliers"]
        assert np.array_equal(T[:3, :3].reshape(9), full[i]["T_query_match"][:9])
        assert np.array_equal(T[:3, 3], full[i]["T_query_match"][9:])


def test_verify_matches_edge_cases(gpu):
    from oracle import oracle as O
    pool = make_lcd_pool(8, 64, seed=11)
    p = LcdParams()
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    e = np.zeros(0, np.int32)
    corr = [(e, e), (np.arange(3), np.arange(3)), (np.arange(64), np.arange(64)),
            (np.zeros(10, np.int32), np.arange(10))]  # empty, below 5, the maximum, repeated query index
    cq, cm = pool.cand_query[:4], pool.cand_match[:4]
    for st in (1, 2, 3):
        prior = np.tile(np.r_[np.eye(3).ravel(), 0, 0, 0], (4, 1))
        got, gm = det.verify_matches(cq, cm, corr, stages=st, T_prior=prior, with_masks=True)
        ref, rm = O.lcd_verify_pairs(p.to_c(), pool, cq, cm, corr, stages=st, T_prior=prior)
        for i in range(4):
            _same(got[i], ref[i], (st, i))
        assert np.array_equal(gm, rm)
    with pytest.raises(abi.KmxError):  # index outside the frame
        det.verify_matches(cq[:1], cm[:1], [(np.array([64]), np.array([0]))])
    with pytest.raises(abi.KmxError):  # more pairs than max_feats
        det.verify_matches(cq[:1], cm[:1], [(np.zeros(65, np.int32), np.zeros(65, np.int32))])
    with pytest.raises(abi.KmxError):  # 1-point recovery alone needs the 2D-2D rotation
        det.verify_matches(cq[:1], cm[:1], corr[2:3], stages=2)


@pytest.mark.parametrize("recovery,algo,variant", [(0, 0, "gcc9"), (2, 0, "gcc11"), (1, 1, "gcc9"), (2, 1, "gcc9")],
                         ids=["1point-stew", "arun-stew", "pnp-nister", "arun-nister"])
def test_ordered_sampler_matches_oracle_stream(gpu, recovery, algo, variant):
    """rng_stream 1: the verification thread's engine continues from problem
    to problem in candidate order; bit-exact against the restatement's
    persistent engine, and different from the per-problem reseed after the
    first drawing problem (so the flag really selects the other reading)."""
    from oracle import oracle as O
    pool = make_lcd_pool(16, 200, seed=13)
    p = _params(recovery, algo, rng_variant=variant, rng_stream=1)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool)
    for i in range(len(got)):
        _same(got[i], ref[i], i)
    assert np.array_equal(gm, rm)
    p0 = _params(recovery, algo, rng_variant=variant, rng_stream=0)
    ref0, _ = O.lcd_verify(p0.to_c(), pool)
    assert (got[0]["mono_inliers"], got[0]["iterations_2d2d"]) == (ref0[0].mono_inliers, ref0[0].iterations_2d2d)
    assert any(got[i]["iterations_2d2d"] != ref0[i].iterations_2d2d or
               not np.array_equal(got[i]["T_query_match"], np.array(ref0[i].T_query_match[:]))
               for i in range(2, len(got), 2))
    # the engine persists across calls: two calls = one call over both halves
    det2 = LoopClosureDetector(p)
    det2.set_pool(pool)
    h = len(pool.cand_query) // 2
    a, _ = det2.verify(pool.cand_query[:h], pool.cand_match[:h])
    b, _ = det2.verify(pool.cand_query[h:], pool.cand_match[h:])
    for i, g in enumerate(a + b):
        _same(g, ref[i], i)
