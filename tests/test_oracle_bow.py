"""CPU checks of the BoW restatement (oracle/bow_oracle.c).

DBoW2 is not vendored (parity unpinned); the restatement of queryL1 /
L1Scoring::score is pinned against an independent scipy formulation: for
L1-normalised positive weights, 1 - 1/2 |v - w|_1 = sum_i min(v_i, w_i)
(histogram intersection), evaluated with sparse column slicing."""
import numpy as np
import pytest
import scipy.sparse as sp

from kmx.synth.bow import make_bow_stream
from oracle import oracle as O


def _csr(st):
    return sp.csr_matrix((st.weights, st.words.astype(np.int64), st.vptr), shape=(st.n, st.n_words))


def _intersection_scores(Md, qw, qv):
    sub = Md[:, qw.astype(np.int64)].tocoo()
    vals = np.minimum(sub.data, qv[sub.col])
    sc = np.bincount(sub.row, vals, minlength=Md.shape[0])
    touched = np.bincount(sub.row, minlength=Md.shape[0]) > 0
    return sc, touched


@pytest.fixture(scope="module")
def stream():
    return make_bow_stream(2, 400, n_words=20_000, seed=3)


def test_l1_score_is_histogram_intersection(stream):
    rng = np.random.default_rng(0)
    for _ in range(50):
        i, j = rng.integers(0, stream.n, 2)
        wi, vi = stream.vector(i)
        wj, vj = stream.vector(j)
        ref = np.minimum(*np.broadcast_arrays(*[
            np.zeros(stream.n_words) + np.bincount(w.astype(np.int64), v, stream.n_words) for w, v in
            ((wi, vi), (wj, vj))])).sum()
        assert abs(O.bow_score(wi, vi, wj, vj) - ref) < 1e-12


def test_query_matches_intersection_ranking(stream):
    db = stream.subset(np.nonzero(stream.robot == 1)[0])
    qs = stream.subset(np.nonzero(stream.robot == 0)[0][:120])
    Md = _csr(db)
    D = O.OracleBowDb(stream.n_words, db.vptr, db.words, db.weights)
    K = 50
    n, ids, sc = D.query(qs.vptr, qs.words, qs.weights, K)
    for q in range(qs.n):
        qw, qv = qs.vector(q)
        ref, touched = _intersection_scores(Md, qw, qv)
        k = n[q]
        assert k == min(K, touched.sum())
        got = ids[q, :k]
        assert np.all(touched[got])
        assert np.abs(sc[q, :k] - ref[got]).max() < 1e-12
        # sorted by score descending, ties by id ascending (on its own values)
        for a, b in zip(range(k - 1), range(1, k)):
            assert sc[q, a] > sc[q, b] or (sc[q, a] == sc[q, b] and got[a] < got[b])
        # nothing left out scores clearly above the cut
        rest = np.setdiff1d(np.nonzero(touched)[0], got)
        if rest.size and k == K:
            assert ref[rest].max() <= sc[q, k - 1] + 1e-12


def test_query_max_id_and_empty(stream):
    db = stream.subset(np.arange(300))
    D = O.OracleBowDb(stream.n_words, db.vptr, db.words, db.weights)
    qs = stream.subset(np.arange(150, 160))
    max_id = np.array([0, 1, 5, 50, 100, 151, 152, 200, -1, 10], np.int32)
    n, ids, sc = D.query(qs.vptr, qs.words, qs.weights, 20, max_id)
    assert n[0] == 0
    for q in range(qs.n):
        if max_id[q] >= 0:
            assert np.all(ids[q, :n[q]] < max_id[q])
    # a frame finds itself first when allowed (score 1)
    assert ids[8, 0] == 158 and abs(sc[8, 0] - 1.0) < 1e-12
    # an empty query touches nothing
    n0, _, _ = D.query(np.array([0, 0]), np.zeros(0, np.uint32), np.zeros(0), 5)
    assert n0[0] == 0


def test_detect_with_robot_finds_revisited_places(stream):
    db = stream.subset(np.nonzero(stream.robot == 0)[0])
    qi = np.nonzero((stream.robot == 1) & (stream.pose > 0))[0]
    qs, prev = stream.subset(qi), stream.subset(qi - 1)
    D = O.OracleBowDb(stream.n_words, db.vptr, db.words, db.weights)
    match, score, nss = D.detect_batch(qs.vptr, qs.words, qs.weights, prev.vptr, prev.words, prev.weights)
    revisit = qs.place < (db.place.max() + 1)
    same = qs.place == prev.place  # previous keyframe at the same place: meaningful nss
    hit = match >= 0
    assert np.all(hit[nss < 0.05] == False)  # noqa: E712  (nss gate)
    assert hit[revisit & same].mean() > 0.9
    assert np.mean(db.place[match[hit & revisit]] == qs.place[hit & revisit]) > 0.95
    assert hit[~revisit].mean() < 0.2


def test_host_islands_and_temporal_match_restatement():
    """The product's host-side control (kmx.lcd.bow islands / temporal gate)
    against the C restatement, on random result lists."""
    import ctypes as C
    from kmx.lcd import LcdParams
    from kmx.lcd.bow import TemporalConstraint, compute_islands
    L = O.lib()
    p = LcdParams()
    rng = np.random.default_rng(5)
    isl = (O._Island * 64)()
    state = np.zeros(4, np.int32)
    tc = TemporalConstraint(p)
    for trial in range(300):
        k = int(rng.integers(1, 40))
        ids = np.ascontiguousarray(rng.choice(400, k, replace=False).astype(np.int32))
        sc = np.ascontiguousarray(np.sort(rng.random(k))[::-1].copy())
        ni = L.orc_bow_islands(k, O._i(ids), O._f(sc), p.max_intraisland_gap, p.min_matches_per_island,
                               C.byref(isl))
        got = compute_islands(ids, sc, p)
        assert len(got) == ni
        for g, j in zip(got, range(ni)):
            assert (g.start_id, g.end_id, g.best_id) == (isl[j].start, isl[j].end, isl[j].best_id)
            assert g.island_score == isl[j].score and g.best_score == isl[j].best_score
        best = got[max(range(ni), key=lambda j: got[j].island_score)]
        fid = 100 + trial + int(rng.integers(0, 3))
        a = bool(L.orc_bow_temporal(O._i(state), fid, best.start_id, best.end_id, p.max_nrFrames_between_queries,
                                    p.max_nrFrames_between_islands, p.min_temporal_matches))
        assert tc.check(fid, best) == a
