"""BoW candidate stage of Kimera-Multi-LCD on MI355X.

Mirrors the reference's detection calls (drawio:2574-2580, 2612-2633,
drawio:1565) on top of kmx_bow_* (C ABI, bow.hip):

  BowDatabase.query          DBoW2 Database::queryL1 (batched; GPU)
  BowDatabase.score_pairs    L1Scoring::score (the nss factor; GPU)
  BowDetector.detectLoopWithRobot   nss vs the previous keyframe of the query
                             robot, min_nss_factor gate, max_db_results query,
                             alpha * nss cut, best result (batched)
  BowDetector.detectLoop     single-robot stream: query with
                             max_id = frame - recent_frames_window, nss / alpha
                             cut, computeIslands, checkTemporalConstraint
                             (sequential control on the host, queries batched)

Constants are LcdParams (params/D455/LcdParams.yaml:3-12). DBoW2 and
kimera_multi_lcd are not vendored: the restatement is "parity unpinned" and
checked bit-exact against oracle/bow_oracle.c (tests/test_bow_gpu.py).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .. import abi
from ..abi import check, fptr, i64ptr, iptr, u32ptr
from .detector import LcdParams


def _csr(vptr, words, weights):
    return (np.ascontiguousarray(vptr, np.int64), np.ascontiguousarray(words, np.uint32),
            np.ascontiguousarray(weights, np.float64))


class BowDatabase:
    """An L1 DBoW2 database of BowVectors (entry id = insertion index) on one GPU."""

    def __init__(self, n_words: int, device: int = 0):
        L = abi.lib()
        if abi.device_count() <= device:
            raise abi.KmxError(f"no HIP device {device} visible (kmx has no CPU fallback)")
        h = C.c_void_p()
        check(L.kmx_bow_create(device, C.byref(h)), "kmx_bow_create")
        self.L, self.h, self.n_words, self.n = L, h, int(n_words), 0

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.kmx_bow_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_entries(self, vptr, words, weights):
        """Database::add of every vector, in order (replaces the database)."""
        vptr, words, weights = _csr(vptr, words, weights)
        self.n = vptr.shape[0] - 1
        check(self.L.kmx_bow_set_database(self.h, self.n_words, self.n, i64ptr(vptr), u32ptr(words),
                                          fptr(weights)), "kmx_bow_set_database")

    def query(self, qptr, words, weights, max_results: int = 50, max_id=None):
        """queryL1 of each query vector -> (n [nq], ids [nq, K], scores [nq, K])."""
        qptr, words, weights = _csr(qptr, words, weights)
        nq = qptr.shape[0] - 1
        mid = None if max_id is None else np.ascontiguousarray(max_id, np.int32)
        n = np.zeros(nq, np.int32)
        ids = np.full((nq, max_results), -1, np.int32)
        sc = np.zeros((nq, max_results))
        check(self.L.kmx_bow_query(self.h, nq, i64ptr(qptr), u32ptr(words), fptr(weights),
                                   iptr(mid) if mid is not None else None, max_results, iptr(n), iptr(ids),
                                   fptr(sc)), "kmx_bow_query")
        return n, ids, sc

    def query_async(self, qptr, words, weights, max_results: int = 50, max_id=None):
        qptr, words, weights = _csr(qptr, words, weights)
        self._keep = (qptr, words, weights)
        mid = None if max_id is None else np.ascontiguousarray(max_id, np.int32)
        check(self.L.kmx_bow_query_async(self.h, qptr.shape[0] - 1, i64ptr(qptr), u32ptr(words), fptr(weights),
                                         iptr(mid) if mid is not None else None, max_results),
              "kmx_bow_query_async")

    def sync(self):
        check(self.L.kmx_bow_sync(self.h), "kmx_bow_sync")

    def score_pairs(self, a, b):
        """L1 scores of pairs: a, b = (vptr, words, weights) with the same count."""
        aptr, aw, av = _csr(*a)
        bptr, bw, bv = _csr(*b)
        n = aptr.shape[0] - 1
        out = np.zeros(n)
        check(self.L.kmx_bow_score_pairs(self.h, n, i64ptr(aptr), u32ptr(aw), fptr(av), i64ptr(bptr),
                                         u32ptr(bw), fptr(bv), fptr(out)), "kmx_bow_score_pairs")
        return out


@dataclass
class MatchIsland:
    start_id: int
    end_id: int
    island_score: float
    best_id: int
    best_score: float


def compute_islands(ids, scores, p: LcdParams) -> list[MatchIsland]:
    """LcdThirdPartyWrapper::computeIslands (DLoopDetector islands) [U]."""
    n = len(ids)
    if n == 0:
        return []
    if n == 1:
        return [MatchIsland(int(ids[0]), int(ids[0]), float(scores[0]), int(ids[0]), float(scores[0]))]
    order = np.argsort(np.asarray(ids), kind="stable")
    ids = [int(ids[i]) for i in order]
    sc = [float(scores[i]) for i in order]
    out = []
    first = last = ids[0]
    i_first = i_last = 0
    best_s, best_e = sc[0], ids[0]
    for idx in range(1, n + 1):
        if idx < n and ids[idx] - last < p.max_intraisland_gap:
            last, i_last = ids[idx], idx
            if sc[idx] > best_s:
                best_s, best_e = sc[idx], ids[idx]
            continue
        if last - first + 1 >= p.min_matches_per_island:
            s = 0.0
            for k in range(i_first, i_last + 1):
                s += sc[k]
            out.append(MatchIsland(first, last, s, best_e, best_s))
        if idx < n:
            first = last = ids[idx]
            i_first = i_last = idx
            best_s, best_e = sc[idx], ids[idx]
    return out


class TemporalConstraint:
    """LcdThirdPartyWrapper::checkTemporalConstraint state [U]."""

    def __init__(self, p: LcdParams):
        self.p = p
        self.entries = 0
        self.latest_query = 0
        self.latest = None

    def check(self, query_id: int, island: MatchIsland) -> bool:
        p = self.p
        if self.entries == 0 or query_id - self.latest_query > p.max_nrFrames_between_queries:
            self.entries = 1
        else:
            a1, a2 = self.latest.start_id, self.latest.end_id
            b1, b2 = island.start_id, island.end_id
            if (b1 <= a1 <= b2) or (a1 <= b1 <= a2) or (b1 <= a2 <= b2) or (a1 <= b2 <= a2):
                self.entries += 1
            else:
                gap = max(a1 - b2, b1 - a2)
                self.entries = self.entries + 1 if gap <= p.max_nrFrames_between_islands else 1
        self.latest, self.latest_query = island, query_id
        return self.entries > p.min_temporal_matches


class BowDetector:
    """Loop-candidate detection on BowVectors (one database per robot)."""

    def __init__(self, params: LcdParams | None = None, n_words: int = 1_000_000, device: int = 0):
        self.p = params or LcdParams()
        self.n_words = n_words
        self.device = device
        self.db: dict[int, BowDatabase] = {}

    def set_robot_database(self, robot: int, vptr, words, weights):
        db = self.db.get(robot) or BowDatabase(self.n_words, self.device)
        db.set_entries(vptr, words, weights)
        self.db[robot] = db

    def detectLoopWithRobot(self, robot: int, query, prev):
        """Batched detectLoopWithRobot: query / prev = (vptr, words, weights) of the
        query keyframes and of their robots' previous keyframes (empty vector =
        no previous keyframe). Returns (match entry id or -1, score, nss)."""
        p = self.p
        db = self.db[robot]
        nq = len(query[0]) - 1
        nss = db.score_pairs(query, prev) if p.use_nss else np.ones(nq)
        has_prev = np.diff(np.asarray(prev[0])) > 0
        ok = has_prev & (nss >= p.min_nss_factor) if p.use_nss else np.ones(nq, bool)
        n, ids, sc = db.query(*query, max_results=p.max_db_results)
        match = np.full(nq, -1, np.int32)
        score = np.zeros(nq)
        thr = p.alpha * nss
        good = ok & (n > 0) & (sc[:, 0] >= thr)
        match[good] = ids[good, 0]
        score[good] = sc[good, 0]
        return match, score, np.where(has_prev, nss, 0.0)

    def detectLoop(self, robot: int, frames, first_frame: int = 0):
        """Single-robot detectLoop over keyframes first_frame.. of `robot`'s
        database (frames = (vptr, words, weights) of the same keyframes, in
        order). The queries run as one GPU batch with max_id = frame -
        recent_frames_window (entries added after their own query are invisible,
        as in the sequential loop); nss, islands and the temporal constraint are
        the sequential host logic. Returns a list of (frame, status, match, score)."""
        p = self.p
        db = self.db[robot]
        vptr, words, weights = _csr(*frames)
        nq = vptr.shape[0] - 1
        fids = np.arange(first_frame, first_frame + nq)
        max_id = np.maximum(fids - p.recent_frames_window, 0).astype(np.int32)
        n, ids, sc = db.query(vptr, words, weights, p.max_db_results, max_id)
        # nss of keyframe q against keyframe q - 1 (the latest BoW vector)
        if nq > 1:
            a = (vptr[1:] - vptr[1], words[vptr[1]:vptr[-1]], weights[vptr[1]:vptr[-1]])
            b = (vptr[:-1] - vptr[0], words[vptr[0]:vptr[-2]], weights[vptr[0]:vptr[-2]])
            nss_tail = db.score_pairs(a, b)
        else:
            nss_tail = np.zeros(0)
        tc = TemporalConstraint(p)
        out = []
        for q in range(nq):
            fid = int(fids[q])
            if n[q] == 0:
                out.append((fid, "NO_MATCHES", -1, 0.0))
                continue
            nss = 1.0
            if p.use_nss:
                nss = nss_tail[q - 1] if q > 0 else 0.0
                if q == 0 or nss < p.min_nss_factor:
                    out.append((fid, "LOW_NSS_FACTOR", -1, 0.0))
                    continue
            keep = sc[q, :n[q]] >= p.alpha * nss
            if not keep.any():
                out.append((fid, "LOW_SCORE", -1, 0.0))
                continue
            k = int(np.argmin(keep)) if not keep.all() else int(n[q])  # results are sorted: a prefix
            islands = compute_islands(ids[q, :k], sc[q, :k], p)
            if not islands:
                out.append((fid, "NO_GROUPS", -1, 0.0))
                continue
            best = max(islands, key=lambda isl: isl.island_score)
            if not tc.check(fid, best):
                out.append((fid, "FAILED_TEMPORAL_CONSTRAINT", best.best_id, best.best_score))
                continue
            out.append((fid, "LOOP_DETECTED", best.best_id, best.best_score))
        return out
