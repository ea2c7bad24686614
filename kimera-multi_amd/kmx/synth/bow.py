"""Seeded synthetic BoW keyframe streams (configs[2] "BoW query").

The reference's vocabulary (mit_voc.yml, kimera_vio_jackal.launch:40) and the
Campus keyframes are offline downloads, so BowVectors are generated with the
same structure: a robot walks through "places"; a place owns a set of
landmark words drawn with a skewed (Zipf-like) word popularity over
`n_words`; a keyframe observes a random subset of its place's words plus a few
random words, with positive tf-idf-like weights, L1-normalised (DBoW2 L1
scoring normalises with L1). Keyframe i of a robot is at place i // dwell, so
consecutive keyframes overlap (a meaningful nss factor), and robot b > 0
revisits a fraction `revisit` of robot 0's places (inter-robot loop closures).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class BowStream:
    n_words: int
    vptr: np.ndarray      # int64 [F + 1]
    words: np.ndarray     # uint32 [nnz], strictly increasing per vector
    weights: np.ndarray   # float64 [nnz], L1-normalised per vector
    robot: np.ndarray     # int32 [F]
    pose: np.ndarray      # int32 [F] keyframe index within its robot
    place: np.ndarray     # int32 [F] ground-truth place

    @property
    def n(self) -> int:
        return int(self.robot.shape[0])

    def subset(self, idx) -> "BowStream":
        idx = np.asarray(idx)
        lens = self.vptr[idx + 1] - self.vptr[idx]
        vptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        sel = np.concatenate([np.arange(self.vptr[i], self.vptr[i + 1]) for i in idx]) if idx.size else \
            np.zeros(0, np.int64)
        return BowStream(self.n_words, vptr, self.words[sel], self.weights[sel], self.robot[idx], self.pose[idx],
                         self.place[idx])

    def vector(self, i):
        s = slice(self.vptr[i], self.vptr[i + 1])
        return self.words[s], self.weights[s]


def make_bow_stream(n_robots: int = 2, frames_per_robot: int = 1000, *, n_words: int = 100_000,
                    place_words: int = 400, words_per_frame: int = 300, noise_words: int = 30, dwell: int = 4,
                    revisit: float = 0.5, skew: float = 1.5, seed: int = 0) -> BowStream:
    rng = np.random.Generator(np.random.PCG64(seed))
    places_per_robot = (frames_per_robot + dwell - 1) // dwell
    base = places_per_robot  # robot 0 owns places [0, base)
    place_of = []
    next_place = base
    for r in range(n_robots):
        if r == 0:
            seq = np.arange(places_per_robot)
        else:
            seq = np.empty(places_per_robot, np.int64)
            rev = rng.random(places_per_robot) < revisit
            seq[rev] = rng.integers(0, base, int(rev.sum()))
            seq[~rev] = next_place + np.arange(int((~rev).sum()))
            next_place += int((~rev).sum())
        place_of.append(np.repeat(seq, dwell)[:frames_per_robot])
    n_places = next_place if n_robots > 1 else base

    def skewed(k):  # popular words have small ids
        return np.minimum((n_words * rng.random(k) ** skew).astype(np.int64), n_words - 1)

    pw = skewed(n_places * place_words).reshape(n_places, place_words)
    pwt = rng.gamma(2.0, 1.0, (n_places, place_words))
    vptr, words, weights, robot, pose, place = [0], [], [], [], [], []
    for r in range(n_robots):
        for i, pl in enumerate(place_of[r]):
            pick = rng.choice(place_words, words_per_frame, replace=False)
            w = np.concatenate([pw[pl, pick], skewed(noise_words)])
            v = np.concatenate([pwt[pl, pick] * rng.uniform(0.7, 1.3, words_per_frame),
                                rng.gamma(2.0, 1.0, noise_words)])
            w, first = np.unique(w, return_index=True)  # sorted, duplicates dropped
            v = v[first]
            v = v / v.sum()
            words.append(w.astype(np.uint32))
            weights.append(v)
            vptr.append(vptr[-1] + w.shape[0])
            robot.append(r)
            pose.append(i)
            place.append(pl)
    return BowStream(n_words, np.asarray(vptr, np.int64), np.concatenate(words), np.concatenate(weights),
                     np.asarray(robot, np.int32), np.asarray(pose, np.int32), np.asarray(place, np.int32))
