"""BoW candidate stage on MI355X vs the CPU restatement: bit-exact (==) ids,
scores, nss factors and detection decisions."""
import numpy as np
import pytest

from kmx.lcd import LcdParams
from kmx.lcd.bow import BowDatabase, BowDetector
from kmx.synth.bow import make_bow_stream
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stream():
    return make_bow_stream(2, 1500, n_words=50_000, seed=7)


@pytest.mark.parametrize("env", [{}, {"KMX_BOW_CHUNK": "512"}, {"KMX_BOW_CHUNK": "97"}, {"KMX_BOW_LDS": "0"}])
def test_query_bit_exact(gpu, stream, env, monkeypatch):
    """Default: LDS accumulator in one chunk (1500 entries); small chunks cover
    the per-chunk selection and the merge (and max_id cutting a chunk);
    KMX_BOW_LDS=0 is the HBM-accumulator kernel."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    db = stream.subset(np.nonzero(stream.robot == 1)[0])
    qs = stream.subset(np.nonzero(stream.robot == 0)[0])
    G = BowDatabase(stream.n_words)
    G.set_entries(db.vptr, db.words, db.weights)
    D = O.OracleBowDb(stream.n_words, db.vptr, db.words, db.weights)
    for K, max_id in ((50, None), (7, np.random.default_rng(1).integers(-1, db.n, qs.n).astype(np.int32)),
                      (256, None)):
        n, ids, sc = G.query(qs.vptr, qs.words, qs.weights, K, max_id)
        n0, ids0, sc0 = D.query(qs.vptr, qs.words, qs.weights, K, max_id)
        assert np.array_equal(n, n0)
        for q in range(qs.n):
            assert np.array_equal(ids[q, :n[q]], ids0[q, :n[q]]), (K, q)
            assert np.array_equal(sc[q, :n[q]], sc0[q, :n[q]]), (K, q)


@pytest.mark.parametrize("env", [{}, {"KMX_BOW_CHUNK": "7"}, {"KMX_BOW_LDS": "0"}])
def test_edge_cases(gpu, stream, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    G = BowDatabase(stream.n_words)
    G.set_entries(np.zeros(1, np.int64), np.zeros(0, np.uint32), np.zeros(0))  # empty database
    n, _, _ = G.query(stream.vptr[:3], stream.words, stream.weights, 10)
    assert np.all(n == 0)
    db = stream.subset(np.arange(40))
    G.set_entries(db.vptr, db.words, db.weights)
    # empty query vector, out-of-vocabulary word, max_id 0
    qptr = np.array([0, 0, 1, 1 + (db.vptr[6] - db.vptr[5])], np.int64)
    w5, v5 = db.vector(5)
    words = np.concatenate([[stream.n_words + 5], w5]).astype(np.uint32)
    weights = np.concatenate([[0.5], v5])
    n, ids, sc = G.query(qptr, words, weights, 5, np.array([-1, -1, -1], np.int32))
    assert n[0] == 0 and n[1] == 0 and ids[2, 0] == 5 and abs(sc[2, 0] - 1.0) < 1e-12
    n, _, _ = G.query(qptr, words, weights, 5, np.array([0, 0, 0], np.int32))
    assert np.all(n == 0)


def test_pair_scores_and_detect_with_robot(gpu, stream):
    db = stream.subset(np.nonzero(stream.robot == 0)[0])
    qi = np.nonzero((stream.robot == 1) & (stream.pose > 0))[0]
    qs, prev = stream.subset(qi), stream.subset(qi - 1)
    det = BowDetector(LcdParams(), n_words=stream.n_words)
    det.set_robot_database(0, db.vptr, db.words, db.weights)
    m, s, nss = det.detectLoopWithRobot(0, (qs.vptr, qs.words, qs.weights), (prev.vptr, prev.words, prev.weights))
    D = O.OracleBowDb(stream.n_words, db.vptr, db.words, db.weights)
    m0, s0, nss0 = D.detect_batch(qs.vptr, qs.words, qs.weights, prev.vptr, prev.words, prev.weights)
    assert np.array_equal(nss, nss0)
    assert np.array_equal(m, m0) and np.array_equal(s, s0)
    assert (m >= 0).sum() > qs.n // 4


def test_detect_loop_stream(gpu, stream):
    r0 = np.nonzero(stream.robot == 0)[0]
    own = stream.subset(r0)
    # robot 0 revisits its own places: append a second pass over its first places
    again = stream.subset(r0[:400])
    allf = stream.subset(np.concatenate([r0, r0[:400]]))
    p = LcdParams()
    det = BowDetector(p, n_words=stream.n_words)
    det.set_robot_database(0, allf.vptr, allf.words, allf.weights)
    first = own.n
    got = det.detectLoop(0, (again.vptr, again.words, again.weights), first_frame=first)
    D = O.OracleBowDb(stream.n_words, allf.vptr, allf.words, allf.weights)
    ref = O.detect_loop_stream(D, again.vptr, again.words, again.weights, first, p)
    assert got == ref
    assert sum(1 for g in got if g[1] == "LOOP_DETECTED") > 100
