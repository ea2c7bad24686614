"""Seeded synthetic loop-closure candidates.

The D455 keyframes, ORB descriptors and vocabulary are not available offline,
so configs[2] runs on frames of the same shape: `n_feats` 32-byte ORB-like
descriptors per keyframe, a unit bearing vector and a stereo 3D point per
feature (camera frame, z forward).

Frames come in pairs (2k, 2k+1) that observe a common scene under a planted
relative pose (|theta| <= 30 deg, |t| <= 2 m, points 1-20 m ahead):
  * `true_frac` of the features are true correspondences: the match frame's
    descriptor with `flip_frac` of its 256 bits flipped, geometry consistent;
  * `false_frac` are descriptor look-alikes with inconsistent geometry (they
    pass Lowe's test and must be rejected by RANSAC);
  * the rest are independent random features.
Candidate i pairs query frame i with its partner (even i) or with a random
unrelated frame (odd i), so half of the candidates are true loop closures.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .pose_graph import _expm_so3


@dataclass
class LcdPool:
    n_frames: int
    max_feats: int
    n_feats: np.ndarray    # int32 [F]
    desc: np.ndarray       # uint8 [F, N, 32]
    bearings: np.ndarray   # float64 [F, N, 3]
    points: np.ndarray     # float64 [F, N, 3]
    cand_query: np.ndarray  # int32 [C]
    cand_match: np.ndarray
    R_qm: np.ndarray       # planted pose of pair k: p_q = R p_m + t
    t_qm: np.ndarray
    true_idx: np.ndarray   # [pairs, n_true, 2] (query feature, match feature)


def _bearing(p, rng, sigma):
    f = p / np.linalg.norm(p, axis=-1, keepdims=True)
    if sigma > 0:
        f = f + rng.normal(0, sigma, f.shape)
        f = f / np.linalg.norm(f, axis=-1, keepdims=True)
    return f


def make_lcd_pool(n_frames: int, n_feats: int = 500, *, true_frac: float = 0.5, false_frac: float = 0.2,
                  flip_frac: float = 0.05, bearing_sigma: float = 1e-4, point_sigma: float = 0.05,
                  noise_free: bool = False, seed: int = 0, R_qm: np.ndarray | None = None,
                  t_qm: np.ndarray | None = None) -> LcdPool:
    """`R_qm` / `t_qm` ([n_frames / 2, 3, 3] / [.., 3]) plant given relative
    poses instead of random ones (the loop-closure stream of kmx.pipeline);
    the random draws are made either way, so every other array is unchanged."""
    if n_frames % 2:
        raise ValueError("n_frames must be even (frames come in pairs)")
    rng = np.random.Generator(np.random.PCG64(seed))
    P, N = n_frames // 2, n_feats
    nt, nf = int(round(true_frac * N)), int(round(false_frac * N))
    # planted relative poses
    axis = rng.normal(size=(P, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(-np.pi / 6, np.pi / 6, P)
    R = _expm_so3(axis * ang[:, None])
    tdir = rng.normal(size=(P, 3))
    tdir /= np.linalg.norm(tdir, axis=1, keepdims=True)
    t = tdir * rng.uniform(0.2, 2.0, P)[:, None]
    if R_qm is not None:
        R = np.ascontiguousarray(np.asarray(R_qm, np.float64).reshape(P, 3, 3))
        t = np.ascontiguousarray(np.asarray(t_qm, np.float64).reshape(P, 3))
    # scene points in the match frame, in front of both cameras
    def scene(k):
        z = rng.uniform(1.0, 20.0, (P, k))
        xy = rng.uniform(-0.6, 0.6, (P, k, 2)) * z[..., None]
        pm = np.concatenate([xy, z[..., None]], axis=-1)
        pq = np.einsum("pij,pkj->pki", R, pm) + t[:, None, :]
        bad = pq[..., 2] < 0.5
        pq[bad] = pm[bad]  # rare: keep a valid bearing (becomes a geometric outlier)
        return pm, pq
    pm_true, pq_true = scene(nt)
    sb = 0.0 if noise_free else bearing_sigma
    sp = 0.0 if noise_free else point_sigma
    desc = rng.integers(0, 256, size=(n_frames, N, 32), dtype=np.uint8)
    pts = np.empty((n_frames, N, 3))
    # random scene for all features, then overwrite the planted ones
    z = rng.uniform(1.0, 20.0, (n_frames, N))
    pts[..., :2] = rng.uniform(-0.6, 0.6, (n_frames, N, 2)) * z[..., None]
    pts[..., 2] = z
    qf = np.arange(0, n_frames, 2)
    mf = qf + 1
    perm_q = np.argsort(rng.random((P, N)), axis=1)  # feature slot permutations
    perm_m = np.argsort(rng.random((P, N)), axis=1)
    iq_true, im_true = perm_q[:, :nt], perm_m[:, :nt]
    iq_false, im_false = perm_q[:, nt:nt + nf], perm_m[:, nt:nt + nf]
    rows = np.arange(P)[:, None]
    # true correspondences: same scene point, similar descriptor
    pts[mf[:, None], im_true] = pm_true
    pts[qf[:, None], iq_true] = pq_true

    def flip_masks(k):  # uint8 [P, k, 32] with each bit set w.p. flip_frac (chunked: bounded memory)
        out = np.empty((P, k, 32), np.uint8)
        for c0 in range(0, P, 1024):
            c1 = min(P, c0 + 1024)
            out[c0:c1] = np.packbits(rng.integers(0, 1 << 16, (c1 - c0, k, 256), dtype=np.uint16)
                                     < int(flip_frac * (1 << 16)), axis=-1)
        return out
    desc[qf[:, None], iq_true] = desc[mf[:, None], im_true] ^ flip_masks(nt)
    # false look-alikes: similar descriptor, unrelated geometry
    desc[qf[:, None], iq_false] = desc[mf[:, None], im_false] ^ flip_masks(nf)
    bearings = _bearing(pts, rng, sb)
    if sp > 0:
        pts = pts + rng.normal(0, sp, pts.shape)
    cq = np.arange(n_frames, dtype=np.int32)
    cm = np.where(cq % 2 == 0, cq + 1, 0).astype(np.int32)
    odd = cq % 2 == 1
    other = rng.integers(0, n_frames, odd.sum())
    clash = (other == cq[odd]) | (other == cq[odd] - 1)
    other[clash] = (other[clash] + 2) % n_frames
    cm[odd] = other
    true_idx = np.stack([iq_true, im_true], axis=-1).astype(np.int32)
    del rows
    return LcdPool(n_frames=n_frames, max_feats=N, n_feats=np.full(n_frames, N, np.int32),
                   desc=np.ascontiguousarray(desc), bearings=np.ascontiguousarray(bearings),
                   points=np.ascontiguousarray(pts), cand_query=cq, cand_match=cm, R_qm=R, t_qm=t,
                   true_idx=true_idx)
