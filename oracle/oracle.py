"""ctypes wrapper of the CPU restatement (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package. It mirrors the
product handle (kmx.dpgo.solver.BlockSolver) so parity tests read the same on
both sides. Parity status: see the header of dpgo_oracle.c ("parity unpinned"
against upstream dpgo; pinned by analytic known answers).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
import os  # noqa: E402

# ORC_LIB selects another build of the same sources (bench.py's -march=native one)
LIB = Path(os.environ.get("ORC_LIB", HERE / "build" / "liborc.so"))

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _setup(_lib)
    return _lib


def _setup(L):
    import sys
    sys.path.insert(0, str(HERE.parent / "kimera-multi_amd"))
    from kmx.abi import IterStats, PgoParams, LcdParams, LcdResult  # struct layouts only
    P, i32, i64, f64, u8 = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_uint8
    pi32, pf64, pu8 = C.POINTER(i32), C.POINTER(f64), C.POINTER(u8)
    sigs = {
        "orc_pgo_create": ([C.POINTER(PgoParams)], P),
        "orc_pgo_destroy": ([P], None),
        "orc_pgo_set_graph": ([P, C.c_int, pi32, i64, pi32, pi32, pi32, pi32, pf64, pf64, pf64, pf64, pf64, pu8], C.c_int),
        "orc_pgo_set_iterate": ([P, C.c_int, pf64], C.c_int),
        "orc_pgo_get_iterate": ([P, C.c_int, pf64], C.c_int),
        "orc_pgo_refresh": ([P], C.c_int),
        "orc_pgo_get_weights": ([P, pf64], C.c_int),
        "orc_pgo_set_weights": ([P, pf64], C.c_int),
        "orc_pgo_get_mu": ([P], f64),
        "orc_pgo_set_mu": ([P, f64], None),
        "orc_pgo_local_edges": ([P, C.c_int], i64),
        "orc_pgo_round": ([P, pu8, C.POINTER(IterStats)], C.c_int),
        "orc_pgo_round_mt": ([P, pu8, C.POINTER(IterStats), C.c_int], C.c_int),
        "orc_pgo_round_mt2": ([P, pu8, C.POINTER(IterStats), C.c_int, C.c_int], C.c_int),
        "orc_pgo_round_nbr": ([P, pu8, C.POINTER(IterStats)], C.c_int),
        "orc_pgo_update_weights_owned": ([P, pu8, pf64], C.c_int),
        "orc_pgo_update_weights_local": ([P, pu8, pf64], C.c_int),
        "orc_pgo_set_nbr_rows": ([P, i64, pi32, pi32, pf64], C.c_int),
        "orc_pgo_get_x_rows": ([P, i64, pi32, pi32, pf64], C.c_int),
        "orc_pgo_update_weights": ([P, pf64], C.c_int),
        "orc_pgo_get_trajectory": ([P, C.c_int, pf64, pf64], C.c_int),
        "orc_pgo_eval": ([P, C.c_int, C.c_int, pf64, pf64, pf64], C.c_int),
        "orc_pgo_accel_pre": ([P, pu8], C.c_int),
        "orc_pgo_accel_post": ([P, pu8], C.c_int),
        "orc_pgo_accel_gamma": ([P], f64),
    }
    for name, (a, r) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = a
        fn.restype = r
    _lcd_setup(L)
    _bow_setup(L)


def _bow_setup(L):
    P, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    pi32, pi64, pf64, pu32 = C.POINTER(i32), C.POINTER(i64), C.POINTER(f64), C.POINTER(C.c_uint32)
    sigs = {
        "orc_bow_score": ([pu32, pf64, C.c_int, pu32, pf64, C.c_int], f64),
        "orc_bowdb_create": ([C.c_int, C.c_int, pi64, pu32, pf64], P),
        "orc_bowdb_destroy": ([P], None),
        "orc_bowdb_query": ([P, pu32, pf64, C.c_int, C.c_int, C.c_int, pi32, pf64], C.c_int),
        "orc_bow_islands": ([C.c_int, pi32, pf64, C.c_int, C.c_int, C.c_void_p], C.c_int),
        "orc_bow_temporal": ([pi32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int], C.c_int),
        "orc_bow_detect_batch": ([P, C.c_int, pi64, pu32, pf64, pi64, pu32, pf64, C.c_int, f64, f64, pi32, pf64,
                                  pf64], None),
    }
    for name, (a, r) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = a
        fn.restype = r


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _u(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


class OraclePGO:
    """All robots of the team in one CPU process (Jacobi rounds like the GPU)."""

    def __init__(self, params, graph):
        from kmx.abi import PgoParams, IterStats  # noqa: F401
        self.L = lib()
        self.params = params
        self.r = params.r
        self.h = self.L.orc_pgo_create(C.byref(params))
        g = graph
        self.n_robots = g.n_robots
        self.n_poses = np.ascontiguousarray(g.n_poses, dtype=np.int32)
        self._keep = [np.ascontiguousarray(x) for x in (g.r1, g.p1, g.r2, g.p2)]
        self._R = np.ascontiguousarray(g.R.reshape(-1), dtype=np.float64)
        self._t = np.ascontiguousarray(g.t.reshape(-1), dtype=np.float64)
        self._k = np.ascontiguousarray(g.kappa, dtype=np.float64)
        self._tau = np.ascontiguousarray(g.tau, dtype=np.float64)
        self._w = np.ascontiguousarray(g.weight, dtype=np.float64)
        self._fx = np.ascontiguousarray(g.fixed, dtype=np.uint8)
        r1, p1, r2, p2 = self._keep
        rc = self.L.orc_pgo_set_graph(self.h, g.n_robots, _i(self.n_poses), g.m, _i(r1), _i(p1), _i(r2), _i(p2),
                                      _f(self._R), _f(self._t), _f(self._k), _f(self._tau), _f(self._w), _u(self._fx))
        assert rc == 0, rc
        self.m = g.m

    def __del__(self):
        try:
            self.L.orc_pgo_destroy(self.h)
        except Exception:
            pass

    def set_iterate(self, robot, X):
        X = np.ascontiguousarray(X, dtype=np.float64)
        assert X.size == self.n_poses[robot] * 4 * self.r
        self.L.orc_pgo_set_iterate(self.h, robot, _f(X))

    def get_iterate(self, robot):
        X = np.empty((self.n_poses[robot], self.r, 4))
        self.L.orc_pgo_get_iterate(self.h, robot, _f(X))
        return X

    def refresh(self):
        self.L.orc_pgo_refresh(self.h)

    def iterate(self, active=None, threads=1, inner=1):
        """threads: robot blocks over OpenMP threads (results identical to the
        serial round); inner > 1: each block update over `inner` more threads,
        the all-cores timing variant (results equal to rounding only)."""
        from kmx.abi import IterStats
        act = np.ones(self.n_robots, np.uint8) if active is None else np.ascontiguousarray(active, dtype=np.uint8)
        stats = (IterStats * self.n_robots)()
        if inner > 1:
            self.L.orc_pgo_round_mt2(self.h, _u(act), stats, max(threads, 1), inner)
        elif threads > 1:
            self.L.orc_pgo_round_mt(self.h, _u(act), stats, threads)
        else:
            self.L.orc_pgo_round(self.h, _u(act), stats)
        return [s.as_dict() for s in stats]

    def iterate_nbr(self, active=None):
        """Round against the installed neighbour table (no refresh)."""
        from kmx.abi import IterStats
        act = np.ones(self.n_robots, np.uint8) if active is None else np.ascontiguousarray(active, dtype=np.uint8)
        stats = (IterStats * self.n_robots)()
        self.L.orc_pgo_round_nbr(self.h, _u(act), stats)
        return [s.as_dict() for s in stats]

    def accel_pre(self, mask=None):
        """Form the accelerated extrapolation Y for the next round (X := Y)."""
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self.L.orc_pgo_accel_pre(self.h, None if m is None else _u(m))

    def accel_post(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self.L.orc_pgo_accel_post(self.h, None if m is None else _u(m))

    @property
    def accel_gamma(self):
        return self.L.orc_pgo_accel_gamma(self.h)

    def set_nbr_rows(self, robots, poses, X):
        r = np.ascontiguousarray(robots, dtype=np.int32); p = np.ascontiguousarray(poses, dtype=np.int32)
        X = np.ascontiguousarray(X, dtype=np.float64)
        self.L.orc_pgo_set_nbr_rows(self.h, r.shape[0], _i(r), _i(p), _f(X))

    def get_x_rows(self, robots, poses):
        r = np.ascontiguousarray(robots, dtype=np.int32); p = np.ascontiguousarray(poses, dtype=np.int32)
        X = np.empty((r.shape[0], self.r, 4))
        self.L.orc_pgo_get_x_rows(self.h, r.shape[0], _i(r), _i(p), _f(X))
        return X

    def update_weights(self):
        mu = C.c_double(0)
        self.L.orc_pgo_update_weights(self.h, C.byref(mu))
        return mu.value

    def update_weights_owned(self, local):
        loc = np.ascontiguousarray(local, dtype=np.uint8)
        mu = C.c_double(0)
        self.L.orc_pgo_update_weights_owned(self.h, _u(loc), C.byref(mu))
        return mu.value

    def update_weights_local(self, local):
        loc = np.ascontiguousarray(local, dtype=np.uint8)
        mu = C.c_double(0)
        self.L.orc_pgo_update_weights_local(self.h, _u(loc), C.byref(mu))
        return mu.value

    def get_weights(self):
        w = np.empty(self.m)
        self.L.orc_pgo_get_weights(self.h, _f(w))
        return w

    def set_weights(self, w):
        w = np.ascontiguousarray(w, dtype=np.float64)
        self.L.orc_pgo_set_weights(self.h, _f(w))

    @property
    def mu(self):
        return self.L.orc_pgo_get_mu(self.h)

    @mu.setter
    def mu(self, v):
        self.L.orc_pgo_set_mu(self.h, float(v))

    def local_edges(self, robot):
        return int(self.L.orc_pgo_local_edges(self.h, robot))

    def trajectory(self, robot, anchor):
        anchor = np.ascontiguousarray(anchor, dtype=np.float64)
        out = np.empty((self.n_poses[robot], 12))
        self.L.orc_pgo_get_trajectory(self.h, robot, _f(anchor), _f(out))
        return out

    def eval(self, robot, mode, V=None):
        n = int(self.n_poses[robot])
        Vin = np.zeros((n, self.r, 4)) if V is None else np.ascontiguousarray(V, dtype=np.float64)
        out = np.empty((n, self.r, 4))
        s = C.c_double(0)
        self.L.orc_pgo_eval(self.h, robot, mode, _f(Vin), _f(out), C.byref(s))
        return out, s.value


# ------------------------------------------------------------------ LCD ---
class LcdBatchDesc(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32), ("max_feats", C.c_int32), ("n_feats", C.POINTER(C.c_int32)),
        ("desc", C.POINTER(C.c_uint8)), ("bearings", C.POINTER(C.c_double)), ("points", C.POINTER(C.c_double)),
        ("n_cand", C.c_int32), ("cand_query", C.POINTER(C.c_int32)), ("cand_match", C.POINTER(C.c_int32)),
    ]


def batch_desc(pool):
    """ctypes view of an LcdPool (keeps references alive on the struct)."""
    d = LcdBatchDesc()
    d._keep = [np.ascontiguousarray(pool.n_feats, dtype=np.int32), np.ascontiguousarray(pool.desc, dtype=np.uint8),
               np.ascontiguousarray(pool.bearings, dtype=np.float64), np.ascontiguousarray(pool.points, dtype=np.float64),
               np.ascontiguousarray(pool.cand_query, dtype=np.int32), np.ascontiguousarray(pool.cand_match, dtype=np.int32)]
    nf, de, be, pt, cq, cm = d._keep
    d.n_frames, d.max_feats = pool.n_frames, pool.max_feats
    d.n_feats, d.desc, d.bearings, d.points = _i(nf), _u(de), _f(be), _f(pt)
    d.n_cand, d.cand_query, d.cand_match = cq.shape[0], _i(cq), _i(cm)
    return d


def _lcd_setup(L):
    from kmx.abi import LcdParams, LcdResult
    i32, u8, f64 = C.c_int32, C.c_uint8, C.c_double
    L.orc_mt19937_stream.argtypes = [C.c_uint32, C.c_int, i32, C.POINTER(i32)]
    L.orc_ransac_samples.argtypes = [C.c_uint32, C.c_int, i32, i32, C.POINTER(i32)]
    L.orc_lcd_knn2.argtypes = [C.c_int, f64, C.POINTER(u8), i32, C.POINTER(u8), i32, C.POINTER(i32), C.POINTER(i32)]
    L.orc_fivept_nister.argtypes = [C.POINTER(f64), C.POINTER(f64), C.POINTER(f64)]
    L.orc_fivept_stewenius.argtypes = [C.POINTER(f64), C.POINTER(f64), C.POINTER(f64)]
    L.orc_lcd_verify_batch.argtypes = [C.POINTER(LcdParams), C.POINTER(LcdBatchDesc), i32, C.POINTER(i32),
                                       C.POINTER(i32), C.POINTER(LcdResult), C.POINTER(u8)]
    L.orc_lcd_verify_pairs_batch.argtypes = [C.POINTER(LcdParams), C.POINTER(LcdBatchDesc), i32, C.POINTER(i32),
                                             C.POINTER(i32), C.POINTER(C.c_int64), C.POINTER(i32), C.POINTER(i32),
                                             C.c_int, C.POINTER(f64), C.POINTER(LcdResult), C.POINTER(u8)]
    for n in ("orc_mt19937_stream", "orc_ransac_samples", "orc_lcd_knn2", "orc_fivept_nister", "orc_fivept_stewenius",
              "orc_lcd_verify_batch", "orc_lcd_verify_pairs_batch"):
        getattr(L, n).restype = C.c_int


def mt19937_stream(seed, variant, n):
    L = lib(); _lcd_setup(L)
    out = np.empty(n, np.int32)
    L.orc_mt19937_stream(seed, variant, n, _i(out))
    return out


def ransac_samples(seed, variant, K, passes):
    L = lib(); _lcd_setup(L)
    out = np.empty((passes, 5), np.int32)
    rc = L.orc_ransac_samples(seed, variant, K, passes, _i(out))
    assert rc == 0
    return out


def knn2(norm, lowe, q, m):
    L = lib(); _lcd_setup(L)
    q = np.ascontiguousarray(q, dtype=np.uint8); m = np.ascontiguousarray(m, dtype=np.uint8)
    pairs = np.empty((max(q.shape[0], 1), 2), np.int32)
    k = C.c_int32()
    L.orc_lcd_knn2(norm, lowe, _u(q), q.shape[0], _u(m), m.shape[0], _i(pairs), C.byref(k))
    return pairs[: k.value].copy()


def fivept(f1, f2, algo=1):
    """5-point essentials: algo 1 Nister (real roots), 0 Stewenius (every
    eigen-solution, complex ones by their real part)."""
    L = lib(); _lcd_setup(L)
    f1 = np.ascontiguousarray(f1, dtype=np.float64); f2 = np.ascontiguousarray(f2, dtype=np.float64)
    Es = np.empty((10, 9))
    fn = L.orc_fivept_nister if algo == 1 else L.orc_fivept_stewenius
    n = fn(_f(f1), _f(f2), _f(Es))
    return Es[:n].reshape(-1, 3, 3)


def epnp(pw, f):
    """EPnP restatement (oracle/lcd_oracle.c orc_epnp): camera pose (R_wc, t_wc)
    in the world frame of the points, or None."""
    L = lib()
    L.orc_epnp.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                           C.POINTER(C.c_double)]
    L.orc_epnp.restype = C.c_int
    pw = np.ascontiguousarray(pw, np.float64)
    f = np.ascontiguousarray(f, np.float64)
    R = np.empty((3, 3))
    t = np.empty(3)
    ok = L.orc_epnp(pw.shape[0], _f(pw), _f(f), _f(R), _f(t))
    return (R, t) if ok else None


def lcd_verify(params, pool, cand_query=None, cand_match=None, masks=True):
    from kmx.abi import LcdResult
    L = lib(); _lcd_setup(L)
    cq = np.ascontiguousarray(pool.cand_query if cand_query is None else cand_query, dtype=np.int32)
    cm = np.ascontiguousarray(pool.cand_match if cand_match is None else cand_match, dtype=np.int32)
    d = batch_desc(pool)
    res = (LcdResult * cq.shape[0])()
    mk = np.zeros((cq.shape[0], pool.max_feats), np.uint8) if masks else None
    L.orc_lcd_verify_batch(C.byref(params), C.byref(d), cq.shape[0], _i(cq), _i(cm), res,
                           _u(mk) if masks else None)
    return res, mk


def lcd_verify_pairs(params, pool, cand_query, cand_match, correspondences, stages=3, T_prior=None, masks=True):
    """geometricVerificationNister / recoverPose restated on caller-supplied
    correspondences (oracle/lcd_oracle.c orc_lcd_verify_pairs_batch)."""
    from kmx.abi import LcdResult
    L = lib(); _lcd_setup(L)
    cq = np.ascontiguousarray(cand_query, dtype=np.int32)
    cm = np.ascontiguousarray(cand_match, dtype=np.int32)
    n = cq.shape[0]
    lens = [len(a) for a, _ in correspondences]
    mptr = np.zeros(n + 1, np.int64)
    mptr[1:] = np.cumsum(lens)
    iq = np.ascontiguousarray(np.concatenate([np.asarray(a, np.int32) for a, _ in correspondences] + [np.zeros(1, np.int32)]))
    im = np.ascontiguousarray(np.concatenate([np.asarray(b, np.int32) for _, b in correspondences] + [np.zeros(1, np.int32)]))
    pr = None if T_prior is None else np.ascontiguousarray(T_prior, np.float64).reshape(n, 12)
    d = batch_desc(pool)
    res = (LcdResult * max(n, 1))()
    mk = np.zeros((max(n, 1), pool.max_feats), np.uint8) if masks else None
    L.orc_lcd_verify_pairs_batch(C.byref(params), C.byref(d), n, _i(cq), _i(cm),
                                 mptr.ctypes.data_as(C.POINTER(C.c_int64)), _i(iq), _i(im), int(stages),
                                 _f(pr) if pr is not None else None, res, _u(mk) if masks else None)
    return res, (mk[:n] if masks else None)


# ------------------------------------------------------------------ BoW ----
def _u32(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def _i64(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def bow_score(w1, v1, w2, v2):
    """DBoW2 L1Scoring::score (restated in oracle/bow_oracle.c)."""
    L = lib()
    w1, w2 = np.ascontiguousarray(w1, np.uint32), np.ascontiguousarray(w2, np.uint32)
    v1, v2 = np.ascontiguousarray(v1, np.float64), np.ascontiguousarray(v2, np.float64)
    return L.orc_bow_score(_u32(w1), _f(v1), w1.shape[0], _u32(w2), _f(v2), w2.shape[0])


class OracleBowDb:
    """DBoW2 Database (L1) restatement: inverted file + queryL1."""

    def __init__(self, n_words, vptr, words, weights):
        self.L = lib()
        self.vptr = np.ascontiguousarray(vptr, np.int64)
        self.words = np.ascontiguousarray(words, np.uint32)
        self.weights = np.ascontiguousarray(weights, np.float64)
        self.n = self.vptr.shape[0] - 1
        self.h = self.L.orc_bowdb_create(int(n_words), self.n, _i64(self.vptr), _u32(self.words), _f(self.weights))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_bowdb_destroy(self.h)
            self.h = None

    def query(self, qptr, words, weights, max_results=50, max_id=None):
        qptr = np.ascontiguousarray(qptr, np.int64)
        words = np.ascontiguousarray(words, np.uint32)
        weights = np.ascontiguousarray(weights, np.float64)
        nq = qptr.shape[0] - 1
        n = np.zeros(nq, np.int32)
        ids = np.full((nq, max_results), -1, np.int32)
        sc = np.zeros((nq, max_results))
        for q in range(nq):
            mid = -1 if max_id is None else int(max_id[q])
            a, b = qptr[q], qptr[q + 1]
            n[q] = self.L.orc_bowdb_query(self.h, _u32(words[a:]), _f(weights[a:]), int(b - a), max_results, mid,
                                          _i(ids[q]), _f(sc[q]))
        return n, ids, sc

    def detect_batch(self, qptr, qw, qv, pptr, pw, pv, max_results=50, alpha=0.4, min_nss=0.05):
        """detectLoopWithRobot over a batch (previous-keyframe vectors in p*)."""
        qptr, pptr = np.ascontiguousarray(qptr, np.int64), np.ascontiguousarray(pptr, np.int64)
        qw, pw = np.ascontiguousarray(qw, np.uint32), np.ascontiguousarray(pw, np.uint32)
        qv, pv = np.ascontiguousarray(qv, np.float64), np.ascontiguousarray(pv, np.float64)
        nq = qptr.shape[0] - 1
        match = np.zeros(nq, np.int32)
        score = np.zeros(nq)
        nss = np.zeros(nq)
        self.L.orc_bow_detect_batch(self.h, nq, _i64(qptr), _u32(qw), _f(qv), _i64(pptr), _u32(pw), _f(pv),
                                    max_results, alpha, min_nss, _i(match), _f(score), _f(nss))
        return match, score, nss


class _Island(C.Structure):
    _fields_ = [("start", C.c_int), ("end", C.c_int), ("best_id", C.c_int), ("score", C.c_double),
                ("best_score", C.c_double)]


def detect_loop_stream(db: "OracleBowDb", vptr, words, weights, first_frame, p):
    """Single-robot detectLoop over consecutive keyframes (restated control:
    max_id = frame - recent_frames_window, nss vs the previous keyframe,
    alpha cut, islands, temporal constraint). p: kmx.lcd.LcdParams."""
    L = lib()
    vptr = np.ascontiguousarray(vptr, np.int64)
    words = np.ascontiguousarray(words, np.uint32)
    weights = np.ascontiguousarray(weights, np.float64)
    nq = vptr.shape[0] - 1
    fids = np.arange(first_frame, first_frame + nq)
    max_id = np.maximum(fids - p.recent_frames_window, 0)
    n, ids, sc = db.query(vptr, words, weights, p.max_db_results, max_id)
    state = np.zeros(4, np.int32)
    isl = (_Island * max(p.max_db_results, 1))()
    out = []
    for q in range(nq):
        fid = int(fids[q])
        if n[q] == 0:
            out.append((fid, "NO_MATCHES", -1, 0.0))
            continue
        nss = 1.0
        if p.use_nss:
            if q == 0:
                out.append((fid, "LOW_NSS_FACTOR", -1, 0.0))
                continue
            a, b = slice(vptr[q], vptr[q + 1]), slice(vptr[q - 1], vptr[q])
            nss = bow_score(words[a], weights[a], words[b], weights[b])
            if nss < p.min_nss_factor:
                out.append((fid, "LOW_NSS_FACTOR", -1, 0.0))
                continue
        k = 0
        while k < n[q] and sc[q, k] >= p.alpha * nss:
            k += 1
        if k == 0:
            out.append((fid, "LOW_SCORE", -1, 0.0))
            continue
        qi = np.ascontiguousarray(ids[q, :k])
        qs = np.ascontiguousarray(sc[q, :k])
        ni = L.orc_bow_islands(k, _i(qi), _f(qs), p.max_intraisland_gap, p.min_matches_per_island, C.byref(isl))
        if ni == 0:
            out.append((fid, "NO_GROUPS", -1, 0.0))
            continue
        best = max(range(ni), key=lambda j: isl[j].score)  # first maximum, like std::max_element
        b = isl[best]
        if not L.orc_bow_temporal(_i(state), fid, b.start, b.end, p.max_nrFrames_between_queries,
                                  p.max_nrFrames_between_islands, p.min_temporal_matches):
            out.append((fid, "FAILED_TEMPORAL_CONSTRAINT", b.best_id, b.best_score))
            continue
        out.append((fid, "LOOP_DETECTED", b.best_id, b.best_score))
    return out
