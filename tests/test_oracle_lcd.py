"""CPU checks of the LCD restatement (oracle/lcd_oracle.c).

Pinned by (1) the real libstdc++ of this container (golden fixture made by
tests/golden/gen_mt19937_gcc11.py) for the GCC-11 sampler variant, (2) the
GCC-9 libstdc++ rejection path restated in Python, (3) numpy brute force for
kNN + Lowe, (4) known answers: noise-free 5-point instances recover the true
essential matrix; planted loop closures are verified with the planted pose and
exactly the planted inlier set."""
import json
from pathlib import Path

import numpy as np
import pytest

from kmx.lcd.detector import LcdParams
from kmx.synth.lcd import make_lcd_pool
from kmx.synth.pose_graph import _expm_so3
from oracle import oracle as O

GOLD = json.loads((Path(__file__).parent / "golden" / "mt19937_gcc11.json").read_text())


def test_mt19937_known_answer_and_raw_stream():
    assert GOLD["kat_10000"] == 4123659995  # C++ standard [rand.predef]
    for seed, raw in GOLD["raw"].items():
        got = O.mt19937_stream(int(seed), -1, len(raw)).astype(np.int64) & 0xFFFFFFFF
        assert np.array_equal(got, np.array(raw, dtype=np.int64))


def test_uniform_int_variants():
    for seed, uid in GOLD["uid"].items():
        assert GOLD["gcc_major"] == 11
        assert np.array_equal(O.mt19937_stream(int(seed), 1, len(uid)), np.array(uid))  # GCC 11: real libstdc++
        raw = np.array(GOLD["raw"][seed], dtype=np.int64)
        gcc9 = raw[raw < (1 << 31)]  # uniform_int_dist.h fallback: scaling 1, reject >= 2^31
        got = O.mt19937_stream(int(seed), 0, gcc9.shape[0])
        assert np.array_equal(got, gcc9)


def test_ransac_sample_shuffle():
    K, passes = 37, 50
    for variant in (0, 1):
        seq = O.mt19937_stream(12345, variant, passes * 5)
        sh = list(range(K))
        for p in range(passes):
            for i in range(5):
                j = i + seq[p * 5 + i] % (K - i)
                sh[i], sh[j] = sh[j], sh[i]
            assert O.ransac_samples(12345, variant, K, passes)[p].tolist() == sh[:5]


def _brute_knn(q, m, lowe, hamming):
    if hamming:
        d = np.unpackbits(q[:, None, :] ^ m[None, :, :], axis=-1).sum(-1)
    else:
        d = np.abs(q[:, None, :].astype(int) - m[None, :, :].astype(int)).sum(-1)
    out = []
    if m.shape[0] < 2:
        return np.zeros((0, 2), int)
    for i in range(q.shape[0]):
        order = np.lexsort((np.arange(m.shape[0]), d[i]))  # (distance, index)
        d0, d1 = d[i, order[0]], d[i, order[1]]
        if float(np.float32(d0)) < lowe * float(np.float32(d1)):
            out.append((i, order[0]))
    return np.array(out, int).reshape(-1, 2)


@pytest.mark.parametrize("hamming", [False, True])
def test_knn2_vs_bruteforce(hamming):
    rng = np.random.default_rng(0)
    for nq, nm in [(0, 5), (5, 1), (40, 60), (120, 80)]:
        q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
        m = rng.integers(0, 256, (nm, 32), dtype=np.uint8)
        if nq and nm > 3:
            k = min(nq, nm) // 2
            q[:k] = m[:k] ^ (rng.random((k, 32)) < 0.02).astype(np.uint8)
            m[-1] = m[0]  # exact tie in the second neighbour
        got = O.knn2(1 if hamming else 0, 0.7, q, m)
        assert np.array_equal(got, _brute_knn(q, m, 0.7, hamming))


def test_lowe_boundary_is_strict_in_double():
    # d0 / d1 = 7 / 10: 7 < 0.7 * 10 in double (0.7 * 10 = 7.000000000000001)
    m = np.zeros((2, 32), np.uint8)
    m[1, :10] = 1
    q = np.zeros((1, 32), np.uint8)
    q[0, :3] = 1  # L1 to m0 = 3 ... build exact 7 vs 10 below
    q = np.zeros((1, 32), np.uint8); q[0, 0] = 7
    m = np.zeros((2, 32), np.uint8); m[1, 0] = 17  # d(q, m0) = 7, d(q, m1) = 10
    assert O.knn2(0, 0.7, q, m).tolist() == ([[0, 0]] if 7 < 0.7 * 10 else [])


def test_fivept_recovers_true_essential():
    rng = np.random.default_rng(3)
    for trial in range(20):
        R = _expm_so3(rng.normal(0, 0.4, (1, 3)))[0]
        t = rng.normal(size=3)
        pm = np.c_[rng.uniform(-3, 3, (5, 2)), rng.uniform(2, 15, 5)]
        pq = pm @ R.T + t
        f1 = pq / np.linalg.norm(pq, axis=1, keepdims=True)
        f2 = pm / np.linalg.norm(pm, axis=1, keepdims=True)
        Es = O.fivept(f1, f2)
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        Et = tx @ R
        Et /= np.linalg.norm(Et)
        assert len(Es) >= 1
        assert min(min(np.abs(E - Et).max(), np.abs(E + Et).max()) for E in Es) < 1e-8, trial
        for E in Es:
            assert np.abs(np.einsum("ni,ij,nj->n", f1, E, f2)).max() < 1e-12


@pytest.mark.parametrize("seed", [3, 11])
def test_fivept_stewenius_contains_every_real_solution(seed):
    """Stewenius (action-matrix eigen-decomposition) vs Nister (Sturm roots of
    the degree-10 polynomial) on the same samples: the planted E is among the
    Stewenius solutions, every Nister root is one of them (independent
    root-finding methods agree), the count is #real + #complex pairs, and
    every E (real parts included) satisfies the five epipolar constraints."""
    rng = np.random.default_rng(seed)
    for trial in range(60):
        R = _expm_so3(rng.normal(0, 0.4, (1, 3)))[0]
        t = rng.normal(size=3)
        pm = np.c_[rng.uniform(-3, 3, (5, 2)), rng.uniform(2, 15, 5)]
        pq = pm @ R.T + t
        f1 = pq / np.linalg.norm(pq, axis=1, keepdims=True)
        f2 = pm / np.linalg.norm(pm, axis=1, keepdims=True)
        Es, En = O.fivept(f1, f2, 0), O.fivept(f1, f2, 1)
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        Et = tx @ R
        Et /= np.linalg.norm(Et)
        d = lambda A, B: min(np.abs(A - B).max(), np.abs(A + B).max())
        assert min(d(E, Et) for E in Es) < 1e-10, trial
        assert all(min(d(E, F) for F in Es) < 1e-5 for E in En), trial
        assert len(En) + (10 - len(En)) // 2 == len(Es), trial
        assert np.abs(np.einsum("ni,kij,nj->kn", f1, Es, f2)).max() < 1e-12


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
def test_verify_noise_free_pool(algo):
    pool = make_lcd_pool(12, 200, noise_free=True, seed=4)
    p = LcdParams(ransac_2d2d_algorithm=algo).to_c()
    res, masks = O.lcd_verify(p, pool)
    for c in range(len(res)):
        r = res[c]
        if c % 2 == 0:
            k = c // 2
            assert r.accepted
            T = np.array(r.T_query_match[:])
            assert np.abs(T[:9].reshape(3, 3) - pool.R_qm[k]).max() < 1e-7  # Sturm-bisection root precision
            assert np.abs(T[9:] - pool.t_qm[k]).max() < 1e-6
            # the 2D-2D inliers are exactly the planted true correspondences
            pairs = O.knn2(0, 0.7, pool.desc[c], pool.desc[c + 1])
            ti = pool.true_idx[k]
            cons = np.abs(pool.points[c, ti[:, 0]] - pool.points[c + 1, ti[:, 1]] @ pool.R_qm[k].T
                          - pool.t_qm[k]).max(1) < 1e-9  # drop the rare planted points behind the query camera
            true = {tuple(x) for x in ti[cons].tolist()}
            inl = {tuple(pairs[j]) for j in range(len(pairs)) if masks[c, j] & 1}
            assert inl == true & {tuple(x) for x in pairs.tolist()}
        else:
            assert not r.accepted


@pytest.mark.parametrize("noise_free", [True, False])
def test_verify_arun_3d3d(noise_free):
    """Arun 3-point 3D-3D RANSAC (ransac_use_1point_3d3d: 0): planted pairs
    accepted with the planted pose (exact without noise, within the point
    noise otherwise), random pairs rejected."""
    pool = make_lcd_pool(12, 200, noise_free=noise_free, seed=4)
    res, masks = O.lcd_verify(LcdParams(ransac_use_1point_3d3d=0).to_c(), pool)
    for c in range(len(res)):
        r = res[c]
        if c % 2 == 0:
            T = np.array(r.T_query_match[:])
            assert r.accepted and r.stereo_inliers >= 0.95 * r.mono_inliers
            assert np.abs(T[:9].reshape(3, 3) - pool.R_qm[c // 2]).max() < (1e-12 if noise_free else 0.02)
            assert np.abs(T[9:] - pool.t_qm[c // 2]).max() < (1e-12 if noise_free else 0.2)
            assert int(((masks[c] & 2) > 0).sum()) == r.stereo_inliers
        else:
            assert not r.accepted


def test_epnp_recovers_camera_pose():
    """EPnP restatement (LC4): noise-free correspondences give the exact camera
    pose (R_wc, t_wc) for 6..40 points."""
    rng = np.random.default_rng(0)
    for trial in range(100):
        R = _expm_so3(rng.normal(0, 0.5, (1, 3)))[0]
        t = rng.normal(0, 1, 3)
        n = int(rng.integers(6, 40))
        pc = np.c_[rng.uniform(-3, 3, (n, 2)), rng.uniform(2, 15, n)]  # camera frame
        pw = (pc - t) @ R  # pc = R pw + t
        Rwc, twc = O.epnp(pw, pc / np.linalg.norm(pc, axis=1, keepdims=True))
        assert np.abs(Rwc - R.T).max() < 1e-9 and np.abs(twc + R.T @ t).max() < 1e-8, trial


def test_verify_pnp_noise_free_pool():
    pool = make_lcd_pool(12, 200, noise_free=True, seed=4)
    p = LcdParams(pose_recovery_type=1, refine_pose=0).to_c()
    res, masks = O.lcd_verify(p, pool)
    for c in range(len(res)):
        r = res[c]
        if c % 2 == 0:
            assert r.accepted and r.pnp_inliers >= 90 and r.stereo_inliers == 0
            T = np.array(r.T_query_match[:])
            assert np.abs(T[:9].reshape(3, 3) - pool.R_qm[c // 2]).max() < 1e-9
            assert np.abs(T[9:] - pool.t_qm[c // 2]).max() < 1e-8
            assert np.count_nonzero(masks[c] & 2) == r.pnp_inliers
        else:
            assert not r.accepted


@pytest.mark.parametrize("algo", [0, 1], ids=["stewenius", "nister"])
def test_fivept_solutions_are_essential_matrices(algo):
    """Known-answer properties that hold whatever root finder or eigen-solver
    computes them (so they pin the restatement independently of the kernels):
    every real solution E of a random (noisy, not planted) 5-point problem
    satisfies the five epipolar constraints, det(E) = 0 and the trace
    constraint 2 E E^T E - tr(E E^T) E = 0 (Nister 2004, eq. 9), up to rounding.
    Nister's count of real solutions is even-parity consistent (<= 10)."""
    rng = np.random.default_rng(21 + algo)
    seen = 0
    for trial in range(80):
        f1 = rng.normal(size=(5, 3))
        f2 = f1 + rng.normal(0, 0.3, (5, 3))
        f1 /= np.linalg.norm(f1, axis=1, keepdims=True)
        f2 /= np.linalg.norm(f2, axis=1, keepdims=True)
        Es = O.fivept(f1, f2, algo)
        assert len(Es) <= 10
        for E in Es:
            if algo == 0 and abs(np.linalg.det(E)) > 1e-6:
                continue  # Stewenius also returns the real parts of complex pairs
            seen += 1
            E = E / np.linalg.norm(E)
            assert np.abs(np.einsum("ni,ij,nj->n", f1, E, f2)).max() < 1e-9, trial
            assert abs(np.linalg.det(E)) < 1e-9, trial
            EEt = E @ E.T
            assert np.abs(2 * EEt @ E - np.trace(EEt) * E).max() < 1e-8, trial
    assert seen > 80
