"""GPU parity of the LCD verification path against the CPU restatement.

Bar: bit-exact — identical match lists, identical 2D-2D / 3D-3D inlier sets
(masks), identical iteration counts and identical poses (the RANSAC file is
built with -ffp-contract=off and ports the oracle line by line)."""
import numpy as np
import pytest

from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("norm", ["l1", "hamming"])
def test_knn2_matches_oracle(gpu, norm):
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    for nq, nm in [(0, 10), (10, 0), (1, 1), (7, 2), (300, 500), (500, 300), (64, 1024)]:
        q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
        m = rng.integers(0, 256, (nm, 32), dtype=np.uint8)
        if nq and nm:  # plant near-duplicates and exact ties
            k = min(nq, nm) // 2
            q[:k] = m[:k] ^ (rng.random((k, 32)) < 0.02).astype(np.uint8)
            if nm > 3:
                m[nm - 1] = m[0]
        gi, gj = LoopClosureDetector.compute_matched_indices(q, m, 0.7, norm)
        nrm = 1 if norm == "hamming" else 0
        ref = O.knn2(nrm, 0.7, q, m)
        assert np.array_equal(gi, ref[:, 0]) and np.array_equal(gj, ref[:, 1]), (nq, nm)


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
@pytest.mark.parametrize("variant,norm,recovery", [("gcc9", "l1", 0), ("gcc11", "hamming", 0), ("gcc9", "l1", 1),
                                                   ("gcc11", "l1", 2)])
def test_verify_bit_exact(gpu, variant, norm, recovery, algo):
    """recovery 0: 1-point 3D-3D (reference config); 1: EPnP RANSAC (LC4);
    2: Arun 3-point 3D-3D RANSAC (ransac_use_1point_3d3d 0).
    algo: ransac_2d2d_algorithm (0 Stewenius, the reference config; 1 Nister)."""
    from oracle import oracle as O
    pool = make_lcd_pool(24, 300, seed=3)
    p = LcdParams(rng_variant=variant, norm=norm, pose_recovery_type=int(recovery == 1),
                  ransac_2d2d_algorithm=algo, ransac_use_1point_3d3d=int(recovery != 2),
                  refine_pose=int(recovery != 1))  # the 3D-3D recoveries with the reference's refinement
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool)
    for i in range(len(got)):
        r = ref[i]
        g = got[i]
        assert (g["n_matches"], g["mono_inliers"], g["stereo_inliers"], g["pnp_inliers"], g["accepted"],
                g["iterations_2d2d"]) == (r.n_matches, r.mono_inliers, r.stereo_inliers, r.pnp_inliers,
                                          bool(r.accepted), r.iterations_2d2d), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i
    assert np.array_equal(gm, rm)
    # planted loop closures are found, random pairs rejected
    acc = np.array([g["accepted"] for g in got])
    assert acc[0::2].all() and not acc[1::2].any()


@pytest.mark.parametrize("max_iter,true_frac,false_frac", [(1, 0.5, 0.2), (7, 0.25, 0.5), (40, 0.25, 0.4),
                                                           (500, 0.3, 0.4)])
def test_stewenius_batches_stop_like_the_serial_loop(gpu, max_iter, true_frac, false_frac):
    """k_ransac_coop computes Stewenius hypotheses six at a time and scores
    them in order under the serial loop's tests (iterations < k, skipped <
    max_skip, iterations > max_iter): iteration caps that end a batch part
    way, and low inlier ratios (long runs, adaptive k shrinking mid-batch),
    give the one-at-a-time restatement's iteration counts, inlier sets and
    poses bit for bit."""
    from oracle import oracle as O
    pool = make_lcd_pool(24, 300, true_frac=true_frac, false_frac=false_frac, seed=9)
    p = LcdParams(ransac_2d2d_algorithm=0, ransac_max_iterations=max_iter)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool)
    its = []
    for i in range(len(got)):
        r, g = ref[i], got[i]
        assert (g["n_matches"], g["mono_inliers"], g["stereo_inliers"], g["accepted"], g["iterations_2d2d"]) == \
            (r.n_matches, r.mono_inliers, r.stereo_inliers, bool(r.accepted), r.iterations_2d2d), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i
        its.append(r.iterations_2d2d)
    assert np.array_equal(gm, rm)
    its = np.array(its[0::2])
    assert its.max() <= max_iter + 1
    if max_iter == 500:  # the adaptive bound ends the runs (345 .. 486 iterations), inside batches of six
        assert its.max() < max_iter and (its % 6 != 0).any()


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
@pytest.mark.parametrize("max_iter", [50, 500])
@pytest.mark.parametrize("frames", ["match", "both"])
def test_degenerate_samples_skip_like_the_serial_loop(gpu, algo, max_iter, frames):
    """Every bearing of one candidate's match frame (and, with "both", of its
    query frame) points the same way. "both": no sample gives a solvable
    5-point system, every hypothesis counts as skipped and the loop ends at
    max_skip = 10 x max_iter with no model (Stewenius: six skipped hypotheses
    per batch, each checked against the serial stopping rule); "match": the
    solvers return degenerate models the loop scores and rejects. The other
    candidates are unaffected. Bit for bit against the restatement."""
    from oracle import oracle as O
    pool = make_lcd_pool(4, 120, seed=5)
    pool.bearings[int(pool.cand_match[0]), :, :] = np.array([0.0, 0.0, 1.0])
    if frames == "both":
        pool.bearings[int(pool.cand_query[0]), :, :] = np.array([0.0, 1.0, 0.0])
    p = LcdParams(ransac_2d2d_algorithm=algo, ransac_max_iterations=max_iter)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    ref, rm = O.lcd_verify(p.to_c(), pool)
    for i in range(len(got)):
        r, g = ref[i], got[i]
        assert (g["n_matches"], g["mono_inliers"], g["stereo_inliers"], g["accepted"], g["iterations_2d2d"]) == \
            (r.n_matches, r.mono_inliers, r.stereo_inliers, bool(r.accepted), r.iterations_2d2d), i
        assert np.array_equal(g["T_query_match"], np.array(r.T_query_match[:])), i
    assert np.array_equal(gm, rm)
    assert got[0]["n_matches"] >= 5 and not got[0]["accepted"]
    if frames == "both":
        assert got[0]["iterations_2d2d"] == 0
    assert got[2]["accepted"]


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
def test_longest_first_queue_is_bit_exact(gpu, monkeypatch, algo):
    """KMX_LCD_ORDER=1: the RANSAC work queue takes candidates by match count,
    largest first (k_order); each candidate's result is independent of when
    it is taken, so results and masks equal the index-order queue's."""
    pool = make_lcd_pool(40, 300, seed=17)
    p = LcdParams(ransac_2d2d_algorithm=algo)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    monkeypatch.delenv("KMX_LCD_ORDER", raising=False)
    a, am = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    monkeypatch.setenv("KMX_LCD_ORDER", "1")
    b, bm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    assert np.array_equal(am, bm)
    for x, y in zip(a, b):
        assert all(np.array_equal(x[k], y[k]) for k in x)


def test_back_to_back_calls_overlap_safely(gpu):
    """Successive calls use the detector's candidate slots in turn and a
    call's kNN2 runs on a side stream while the previous call's RANSAC
    drains: back-to-back async calls, a call that grows the buffers while
    another is in flight, and the synchronous results after them equal a
    fresh detector's."""
    pool = make_lcd_pool(64, 200, seed=23)
    p = LcdParams()
    ref = LoopClosureDetector(p)
    ref.set_pool(pool)
    want, wm = ref.verify(pool.cand_query, pool.cand_match, with_masks=True)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    rng = np.random.default_rng(0)
    for _ in range(3):
        sel = rng.permutation(pool.cand_query.shape[0])[:20]
        det.verify_async(pool.cand_query[sel], pool.cand_match[sel])
    det.verify_async(np.tile(pool.cand_query, 40), np.tile(pool.cand_match, 40))  # > 1024: regrows in flight
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    det.sync()
    assert np.array_equal(gm, wm)
    for g, w in zip(got, want):
        assert all(np.array_equal(g[k], w[k]) for k in g)


@pytest.mark.parametrize("env", ["1", "0"], ids=["rsx", "one_stream"])
def test_concurrent_slots_mixed_sizes(gpu, monkeypatch, env):
    """Slots 1-3's RANSACs run on their own streams for calls under 96
    candidates per CU (lcd.hip rs_stream), so which stream a slot last used
    changes from call to call: async calls on either side of that size, then match and
    verify_matches (which write the slot from its stream) and a synchronous
    verify; every result equals a fresh detector's. KMX_LCD_RSX=0 keeps every
    slot on the handle's stream."""
    monkeypatch.setenv("KMX_LCD_RSX", env)
    pool = make_lcd_pool(64, 200, seed=29)
    p = LcdParams()
    ref = LoopClosureDetector(p)
    ref.set_pool(pool)
    want, wm = ref.verify(pool.cand_query, pool.cand_match, with_masks=True)
    wp, wk = ref.match(pool.cand_query, pool.cand_match)
    corr = [(wp[i, :wk[i], 0], wp[i, :wk[i], 1]) for i in range(len(wk))]
    wv, wvm = ref.verify_matches(pool.cand_query, pool.cand_match, corr, with_masks=True)
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    big = -(-(96 * 256 + 1) // pool.cand_query.shape[0])  # above the cut on a 256-CU part
    for reps in (1, big, 2, big, 1):
        det.verify_async(np.tile(pool.cand_query, reps), np.tile(pool.cand_match, reps))
        gp, gk = det.match(pool.cand_query, pool.cand_match)
        assert np.array_equal(gk, wk) and np.array_equal(gp, wp)
    det.verify_async(np.tile(pool.cand_query, big), np.tile(pool.cand_match, big))
    gv, gvm = det.verify_matches(pool.cand_query, pool.cand_match, corr, with_masks=True)
    assert np.array_equal(gvm, wvm)
    for g, w in zip(gv, wv):
        assert all(np.array_equal(g[k], w[k]) for k in g)
    det.verify_async(pool.cand_query, pool.cand_match)
    got, gm = det.verify(pool.cand_query, pool.cand_match, with_masks=True)
    det.sync()
    assert np.array_equal(gm, wm)
    for g, w in zip(got, want):
        assert all(np.array_equal(g[k], w[k]) for k in g)


@pytest.mark.parametrize("norm", ["l1", "hamming"])
def test_split_knn2_matches_oracle(gpu, monkeypatch, norm):
    """kmx_lcd_match on resident frames: the small-call kNN2 (k_knn2s, a
    candidate's queries over ceil(N / 64) workgroups, each query's match set
    over 4 waves, merged as ordered keys; KMX_LCD_KSPLIT) gives k_knn2's rows
    and counts bit for bit, and both give the restatement's, across feature
    counts that end a 64-query block or a match quarter part way, frames with
    0 / 1 features, planted near-duplicates and exact ties, at N = 1024 (16
    blocks) — and a call of 65 candidates takes k_knn2."""
    from oracle import oracle as O
    rng = np.random.default_rng(11)
    N = 1024
    counts = [0, 1, 2, 3, 63, 64, 65, 127, 300, 500, 1023, 1024]
    F = len(counts)
    desc = rng.integers(0, 256, (F, N, 32), dtype=np.uint8)
    for f in range(1, F):  # near-duplicates of frame f - 1 and an exact tie
        k = min(counts[f], counts[f - 1]) // 2
        desc[f, :k] = desc[f - 1, :k] ^ (rng.random((k, 32)) < 0.02).astype(np.uint8)
        if counts[f] > 3:
            desc[f, counts[f] - 1] = desc[f, 0]
    bear = np.zeros((F, N, 3))
    bear[..., 2] = 1.0
    pts = np.ones((F, N, 3))
    p = LcdParams(norm=norm)
    cand = [(a, b) for a in range(F) for b in range(F) if a != b]
    res = {}
    for split in ("1", "0"):
        monkeypatch.setenv("KMX_LCD_KSPLIT", split)
        d = LoopClosureDetector(p)
        d.add_frames(np.array(counts, np.int32), desc, bear, pts)
        out = []
        for i in range(0, len(cand), 40):  # calls of 40 candidates (split), then one of 65 (k_knn2)
            cq = np.array([c[0] for c in cand[i:i + 40]], np.int32)
            cm = np.array([c[1] for c in cand[i:i + 40]], np.int32)
            out.append(d.match(cq, cm))
        cq = np.array([c[0] for c in cand[:65]], np.int32)
        cm = np.array([c[1] for c in cand[:65]], np.int32)
        out.append(d.match(cq, cm))
        d.close()
        res[split] = out
    for (pa, ka), (pb, kb) in zip(res["1"], res["0"]):
        assert np.array_equal(ka, kb)
        for i in range(len(ka)):
            assert np.array_equal(pa[i, :ka[i]], pb[i, :kb[i]]), i
    nrm = 1 if norm == "hamming" else 0
    for i, (a, b) in enumerate(cand):
        pa, ka = res["1"][i // 40]
        ref = O.knn2(nrm, 0.7, desc[a, :counts[a]], desc[b, :counts[b]])
        got = pa[i % 40, :ka[i % 40]]
        assert np.array_equal(got[:, 0], ref[:, 0]) and np.array_equal(got[:, 1], ref[:, 1]), (a, b)


@pytest.mark.parametrize("N", [300, 512, 513])
def test_knn2q_hamming_matches_oracle(gpu, monkeypatch, N):
    """The Hamming matcher's batched kNN2 (k_knn2q: four queries per thread,
    N <= 512; above it, and with KMX_LCD_KNNQ=0, k_knn2): calls of more than
    64 candidates, feature counts that end a thread's four queries part way,
    frames with 0 / 1 features, near-duplicates and exact ties — the
    restatement's rows and counts, and k_knn2's."""
    from oracle import oracle as O
    rng = np.random.default_rng(17)
    counts = [0, 1, 2, 3, 5, 127, 128, 129, min(N, 300), N - 1, N]
    F = len(counts)
    desc = rng.integers(0, 256, (F, N, 32), dtype=np.uint8)
    for f in range(1, F):
        k = min(counts[f], counts[f - 1]) // 2
        desc[f, :k] = desc[f - 1, :k] ^ (rng.random((k, 32)) < 0.02).astype(np.uint8)
        if counts[f] > 3:
            desc[f, counts[f] - 1] = desc[f, 0]
    bear = np.zeros((F, N, 3))
    bear[..., 2] = 1.0
    pts = np.ones((F, N, 3))
    cand = [(a, b) for a in range(F) for b in range(F) if a != b]  # 110 > 64: the batched kernels
    cq = np.array([c[0] for c in cand], np.int32)
    cm = np.array([c[1] for c in cand], np.int32)
    res = {}
    for q in ("1", "0"):
        monkeypatch.setenv("KMX_LCD_KNNQ", q)
        d = LoopClosureDetector(LcdParams(norm="hamming"))
        d.add_frames(np.array(counts, np.int32), desc, bear, pts)
        res[q] = d.match(cq, cm)
        d.close()
    (pa, ka), (pb, kb) = res["1"], res["0"]
    assert np.array_equal(ka, kb)
    for i, (a, b) in enumerate(cand):
        assert np.array_equal(pa[i, :ka[i]], pb[i, :kb[i]]), (a, b)
        ref = O.knn2(1, 0.7, desc[a, :counts[a]], desc[b, :counts[b]])
        assert np.array_equal(pa[i, :ka[i], 0], ref[:, 0]) and np.array_equal(pa[i, :ka[i], 1], ref[:, 1]), (a, b)
