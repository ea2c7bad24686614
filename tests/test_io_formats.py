"""Output / input formats: round trips and the column
layout the reference's evaluation scripts read."""
import numpy as np

from kmx.io import (LoopClosureRecord, quat_to_rot, read_g2o, read_loop_closures_csv, read_tum, rot_to_quat,
                    write_g2o, write_keyframes_csv, write_loop_closures_csv, write_tum)
from kmx.synth import make_pose_graph
from kmx.synth.pose_graph import _expm_so3


def test_quaternion_round_trip():
    R = _expm_so3(np.random.default_rng(0).normal(0, 2.0, (200, 3)))
    q = rot_to_quat(R)
    assert np.all(q[:, 3] >= 0) and np.allclose(np.linalg.norm(q, axis=1), 1)
    assert np.abs(quat_to_rot(q) - R).max() < 1e-12
    from scipy.spatial.transform import Rotation  # same (x, y, z, w) convention as lc_result.py
    assert np.abs(Rotation.from_quat(q).as_matrix() - R).max() < 1e-12


def test_tum_round_trip_and_columns(tmp_path):
    import pandas as pd
    R = _expm_so3(np.random.default_rng(1).normal(0, 1, (20, 3)))
    T = np.concatenate([R.reshape(-1, 9), np.random.default_rng(2).normal(size=(20, 3))], axis=1)
    stamps = 1.6e9 + np.arange(20) * 0.5
    f = tmp_path / "kimera_distributed_poses_tum_0.tum"
    write_tum(f, stamps, T)
    s, T2 = read_tum(f)
    assert np.allclose(s, stamps) and np.abs(T2 - T).max() < 1e-8
    df = pd.read_csv(f, sep=" ", header=None)  # lc_result.py:49-55
    df.columns = ["timestamp", "tx", "ty", "tz", "qx", "qy", "qz", "qw"]
    assert np.allclose(df[["tx", "ty", "tz"]].values, T[:, 9:])


def test_loop_closure_and_keyframe_csv(tmp_path):
    import csv
    R = _expm_so3(np.array([[0.1, -0.2, 0.3]]))[0]
    recs = [LoopClosureRecord(0, 12, 1, 40, R, np.array([1.0, 2.0, -0.5]), 0.31, 55, 23, 1665000000123456789)]
    f = tmp_path / "loop_closures.csv"
    write_loop_closures_csv(f, recs)
    row = next(csv.DictReader(open(f)))
    assert set(row) == {"robot1", "pose1", "robot2", "pose2", "qx", "qy", "qz", "qw", "tx", "ty", "tz",
                        "norm_bow_score", "mono_inliers", "stereo_inliers", "stamp_ns"}
    back = read_loop_closures_csv(f)[0]
    assert (back.robot1, back.pose1, back.robot2, back.pose2, back.mono_inliers, back.stamp_ns) == \
        (0, 12, 1, 40, 55, 1665000000123456789)
    assert np.abs(back.R - R).max() < 1e-10
    k = tmp_path / "kimera_distributed_keyframes.csv"
    write_keyframes_csv(k, [0, 1, 2], [10, 20, 30])
    rows = list(csv.DictReader(open(k)))
    assert rows[2] == {"keyframe_id": "2", "keyframe_stamp_ns": "30"}


def test_g2o_round_trip(tmp_path):
    g = make_pose_graph(2, 60, 150, seed=4)
    f = tmp_path / "graph.g2o"
    write_g2o(f, g)
    h = read_g2o(f)
    assert h.m == g.m and np.array_equal(h.n_poses, g.n_poses)
    for k in ("r1", "p1", "r2", "p2"):
        assert np.array_equal(getattr(h, k), getattr(g, k))
    assert np.abs(h.R - g.R).max() < 1e-10 and np.abs(h.t - g.t).max() < 1e-10
    assert np.allclose(h.kappa, g.kappa) and np.allclose(h.tau, g.tau)
    assert len(h.init_R) == 2 and np.abs(h.init_R[1] - g.init_R[1]).max() < 1e-10
