"""TUM / CSV / g2o formats of the Kimera-Multi outputs.

* TUM trajectory (`kimera_distributed_poses_tum_*.tum`, evo_real_time.py:67,
  101-107; read by lc_result.py:49-55 with columns
  timestamp tx ty tz qx qy qz qw, space separated, no header).
* loop_closures.csv (lc_result.py:118-138): robot1,pose1,robot2,pose2,
  qx,qy,qz,qw,tx,ty,tz,norm_bow_score,mono_inliers,stereo_inliers,stamp_ns;
  the relative pose T_1_2 maps pose2's frame into pose1's.
* kimera_distributed_keyframes.csv (lc_result.py:606-615): keyframe_id,
  keyframe_stamp_ns.
* output_lcd_status.csv / output_lcd_result.csv (the LCD logger files
  lc_result.py:140-183 reads): one status row per verified candidate
  (lcd_status, query_id, match_id, mono_inliers, stereo_inliers) and one
  result row (isLoop, queryKfId, matchKfId, timestamp_query, timestamp_match,
  x, y, z, qx, qy, qz, qw); LOOP_DETECTED rows and isLoop == 1 rows pair up
  in order.
* dpgo_log_<robot>.csv (dpgo_ros createIterationLog / logIteration,
  drawio:2018, 2136-2142): one row per RBCD round of the robot; the dpgo_ros
  sources are not vendored, the columns restate its iteration log [U]:
  robot_id, cluster_id, num_active_robots, iteration, num_poses,
  bytes_received, iter_success, rel_change.
* g2o (VERTEX_SE3:QUAT / EDGE_SE3:QUAT with the 6x6 upper-triangular
  information, translation block first) as the pose-graph input format: a
  real graph can replace the synthetic configs (SURVEY.md §8d configs[0]).
Quaternions are (x, y, z, w) (scipy / Eigen coefficient order).
"""
from __future__ import annotations

import csv
from dataclasses import dataclass

import numpy as np


def quat_to_rot(q: np.ndarray) -> np.ndarray:
    """(x, y, z, w) [n, 4] -> rotation matrices [n, 3, 3] (normalises q)."""
    q = np.asarray(q, np.float64).reshape(-1, 4)
    q = q / np.linalg.norm(q, axis=1, keepdims=True)
    x, y, z, w = q.T
    R = np.empty((q.shape[0], 3, 3))
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - z * w)
    R[:, 0, 2] = 2 * (x * z + y * w)
    R[:, 1, 0] = 2 * (x * y + z * w)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - x * w)
    R[:, 2, 0] = 2 * (x * z - y * w)
    R[:, 2, 1] = 2 * (y * z + x * w)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def rot_to_quat(R: np.ndarray) -> np.ndarray:
    """Rotation matrices [n, 3, 3] -> (x, y, z, w) [n, 4] with w >= 0 (Shepperd)."""
    R = np.asarray(R, np.float64).reshape(-1, 3, 3)
    n = R.shape[0]
    q = np.empty((n, 4))
    tr = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]
    for i in range(n):
        m = R[i]
        if tr[i] > 0:
            s = 2.0 * np.sqrt(tr[i] + 1.0)
            q[i] = [(m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s, 0.25 * s]
        elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
            s = 2.0 * np.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2])
            q[i] = [0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s, (m[2, 1] - m[1, 2]) / s]
        elif m[1, 1] > m[2, 2]:
            s = 2.0 * np.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2])
            q[i] = [(m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s, (m[0, 2] - m[2, 0]) / s]
        else:
            s = 2.0 * np.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1])
            q[i] = [(m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s, (m[1, 0] - m[0, 1]) / s]
    q *= np.where(q[:, 3:4] < 0, -1.0, 1.0)
    return q


# -------------------------------------------------------------------- TUM --
def write_tum(path, stamps, T):
    """T: [n, 12] (R row-major, t) as returned by PGOAgent / kmx_pgo_get_trajectory,
    or [n, 3, 4]."""
    T = np.asarray(T, np.float64)
    if T.ndim == 3:
        T = np.concatenate([T[:, :, :3].reshape(-1, 9), T[:, :, 3]], axis=1)
    q = rot_to_quat(T[:, :9].reshape(-1, 3, 3))
    with open(path, "w") as f:
        for s, t, qq in zip(np.asarray(stamps, np.float64), T[:, 9:], q):
            f.write("%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n" % (s, t[0], t[1], t[2], qq[0], qq[1], qq[2], qq[3]))


def read_tum(path):
    """-> (stamps [n], T [n, 12])."""
    a = np.loadtxt(path, ndmin=2)
    R = quat_to_rot(a[:, 4:8])
    return a[:, 0], np.concatenate([R.reshape(-1, 9), a[:, 1:4]], axis=1)


# ----------------------------------------------------------- LC / keyframes --
LC_FIELDS = ["robot1", "pose1", "robot2", "pose2", "qx", "qy", "qz", "qw", "tx", "ty", "tz", "norm_bow_score",
             "mono_inliers", "stereo_inliers", "stamp_ns"]


@dataclass
class LoopClosureRecord:
    robot1: int
    pose1: int
    robot2: int
    pose2: int
    R: np.ndarray          # T_1_2 rotation (3x3)
    t: np.ndarray          # T_1_2 translation
    norm_bow_score: float = 0.0
    mono_inliers: int = 0
    stereo_inliers: int = 0
    stamp_ns: int = 0


def write_loop_closures_csv(path, records):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(LC_FIELDS)
        for r in records:
            q = rot_to_quat(r.R)[0]
            w.writerow([r.robot1, r.pose1, r.robot2, r.pose2, *("%.12g" % v for v in q),
                        *("%.12g" % v for v in np.asarray(r.t, np.float64)), "%.12g" % r.norm_bow_score,
                        r.mono_inliers, r.stereo_inliers, r.stamp_ns])


def read_loop_closures_csv(path):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            q = np.array([float(row[k]) for k in ("qx", "qy", "qz", "qw")])
            out.append(LoopClosureRecord(int(row["robot1"]), int(row["pose1"]), int(row["robot2"]),
                                         int(row["pose2"]), quat_to_rot(q)[0],
                                         np.array([float(row[k]) for k in ("tx", "ty", "tz")]),
                                         float(row["norm_bow_score"]), int(row["mono_inliers"]),
                                         int(row["stereo_inliers"]), int(row["stamp_ns"])))
    return out


def write_keyframes_csv(path, keyframe_ids, stamps_ns):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["keyframe_id", "keyframe_stamp_ns"])
        for k, s in zip(keyframe_ids, stamps_ns):
            w.writerow([int(k), int(s)])


# ------------------------------------------------------------- LCD logs --
LCD_STATUS_FIELDS = ["timestamp_kf", "lcd_status", "query_id", "match_id", "mono_inliers", "stereo_inliers"]
LCD_RESULT_FIELDS = ["timestamp_kf", "isLoop", "queryKfId", "matchKfId", "timestamp_query", "timestamp_match", "x",
                     "y", "z", "qx", "qy", "qz", "qw"]


def lcd_status_name(result: dict, min_2d2d: int = 10) -> str:
    """LCDStatus of one verification (geometricVerificationNister ->
    recoverPose, drawio:2589-2598)."""
    if result["accepted"]:
        return "LOOP_DETECTED"
    if result["mono_inliers"] < min_2d2d:
        return "FAILED_GEOM_VERIFICATION"
    return "FAILED_POSE_RECOVERY"


def write_lcd_logs(status_path, result_path, query_ids, match_ids, results, stamps_ns=None, min_2d2d: int = 10):
    """output_lcd_status.csv + output_lcd_result.csv from LoopClosureDetector
    .verify results (T_query_match: p_q = R p_m + t)."""
    n = len(results)
    st = np.zeros(n, np.int64) if stamps_ns is None else np.asarray(stamps_ns, np.int64)
    with open(status_path, "w", newline="") as fs, open(result_path, "w", newline="") as fr:
        ws, wr = csv.writer(fs), csv.writer(fr)
        ws.writerow(LCD_STATUS_FIELDS)
        wr.writerow(LCD_RESULT_FIELDS)
        for k, r in enumerate(results):
            q_id, m_id = int(query_ids[k]), int(match_ids[k])
            ws.writerow([int(st[q_id]) if st.size > q_id else 0, lcd_status_name(r, min_2d2d), q_id, m_id,
                         int(r["mono_inliers"]), int(r["stereo_inliers"])])
            T = np.asarray(r["T_query_match"], np.float64)
            qq = rot_to_quat(T[:9].reshape(3, 3))[0] if r["accepted"] else np.array([0.0, 0.0, 0.0, 1.0])
            wr.writerow([int(st[q_id]) if st.size > q_id else 0, 1 if r["accepted"] else 0, q_id, m_id,
                         int(st[q_id]) if st.size > q_id else 0, int(st[m_id]) if st.size > m_id else 0,
                         *("%.12g" % v for v in T[9:]), *("%.12g" % v for v in qq)])


# ------------------------------------------------------------- dpgo log --
DPGO_LOG_FIELDS = ["robot_id", "cluster_id", "num_active_robots", "iteration", "num_poses", "bytes_received",
                   "iter_success", "rel_change"]


class DpgoIterationLog:
    """dpgo_log_<robot>.csv writer (one per robot; logIteration appends a row
    per round in which the robot's stats are known)."""

    def __init__(self, directory, robot_id: int, cluster_id: int = 0):
        import os
        self.path = os.path.join(str(directory), f"dpgo_log_{int(robot_id)}.csv")
        self.robot_id, self.cluster_id = int(robot_id), int(cluster_id)
        with open(self.path, "w", newline="") as f:
            csv.writer(f).writerow(DPGO_LOG_FIELDS)

    def log_iteration(self, iteration: int, num_active_robots: int, num_poses: int, bytes_received: int,
                      stats: dict):
        with open(self.path, "a", newline="") as f:
            csv.writer(f).writerow([self.robot_id, self.cluster_id, int(num_active_robots), int(iteration),
                                    int(num_poses), int(bytes_received), int(bool(stats.get("accepted", 0))),
                                    "%.12g" % float(stats.get("rel_change", 0.0))])


def read_dpgo_log(path):
    with open(path) as f:
        return [{k: (float(v) if k == "rel_change" else int(v)) for k, v in row.items()} for row in csv.DictReader(f)]


# -------------------------------------------------------------------- g2o --
def _info_from_precisions(kappa, tau):
    """Isotropic dpgo precisions -> 6x6 information (translation first, g2o)."""
    I = np.zeros((6, 6))
    I[:3, :3] = np.eye(3) * tau
    I[3:, 3:] = np.eye(3) * (kappa / 2.0)  # rotation block: 2 kappa |dR|_F^2 ~ kappa/2 |dtheta|^2 [U]
    return I


def write_g2o(path, graph, key_of=lambda r, p: (r << 56) | p):
    """Write a PoseGraphData as EDGE_SE3:QUAT lines (+ VERTEX_SE3:QUAT of the
    initial guess when present). Keys encode (robot, pose) as gtsam::Symbol-like
    integers by default."""
    q = rot_to_quat(graph.R)
    with open(path, "w") as f:
        if graph.init_R:
            for a in range(graph.n_robots):
                qa = rot_to_quat(graph.init_R[a])
                for i in range(int(graph.n_poses[a])):
                    t = graph.init_t[a][i]
                    f.write("VERTEX_SE3:QUAT %d %.12g %.12g %.12g %.12g %.12g %.12g %.12g\n"
                            % (key_of(a, i), *t, *qa[i]))
        iu = np.triu_indices(6)
        for e in range(graph.m):
            I = _info_from_precisions(graph.kappa[e], graph.tau[e])
            f.write("EDGE_SE3:QUAT %d %d %.12g %.12g %.12g %.12g %.12g %.12g %.12g %s\n"
                    % (key_of(int(graph.r1[e]), int(graph.p1[e])), key_of(int(graph.r2[e]), int(graph.p2[e])),
                       *graph.t[e], *q[e], " ".join("%.12g" % v for v in I[iu])))


def read_g2o(path, split=lambda key: (key >> 56, key & ((1 << 56) - 1))):
    """Read EDGE_SE3:QUAT / VERTEX_SE3:QUAT into a PoseGraphData (kappa / tau
    from the mean of the rotation / translation information diagonals; odometry
    = consecutive poses of one robot, fixedWeight)."""
    from ..synth.pose_graph import PoseGraphData
    edges, verts = [], {}
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "VERTEX_SE3:QUAT":
                verts[int(tok[1])] = np.array([float(x) for x in tok[2:9]])
            elif tok[0] == "EDGE_SE3:QUAT":
                edges.append((int(tok[1]), int(tok[2]), np.array([float(x) for x in tok[3:10]]),
                              np.array([float(x) for x in tok[10:31]])))
    m = len(edges)
    r1 = np.empty(m, np.int32); p1 = np.empty(m, np.int32); r2 = np.empty(m, np.int32); p2 = np.empty(m, np.int32)
    t = np.empty((m, 3)); qs = np.empty((m, 4)); kappa = np.empty(m); tau = np.empty(m)
    iu = np.triu_indices(6)
    for e, (a, b, meas, info) in enumerate(edges):
        r1[e], p1[e] = split(a)
        r2[e], p2[e] = split(b)
        t[e], qs[e] = meas[:3], meas[3:]
        I = np.zeros((6, 6))
        I[iu] = info
        tau[e] = np.mean(np.diag(I)[:3])
        kappa[e] = 2.0 * np.mean(np.diag(I)[3:])
    n_robots = int(max(r1.max(), r2.max())) + 1 if m else 0
    n_poses = np.zeros(n_robots, np.int32)
    for rr, pp in ((r1, p1), (r2, p2)):
        np.maximum.at(n_poses, rr, pp + 1)
    fixed = ((r1 == r2) & (p2 == p1 + 1)).astype(np.uint8)
    g = PoseGraphData(n_robots=n_robots, n_poses=n_poses, r1=r1, p1=p1, r2=r2, p2=p2, R=quat_to_rot(qs), t=t,
                      kappa=kappa, tau=tau, weight=np.ones(m), fixed=fixed, outlier=np.zeros(m, bool))
    if verts:
        for a in range(n_robots):
            Ra, ta = [], []
            for i in range(int(n_poses[a])):
                v = verts.get(int((a << 56) | i))
                if v is None:
                    break
                ta.append(v[:3]); Ra.append(quat_to_rot(v[3:])[0])
            if len(Ra) == n_poses[a]:
                g.init_R.append(np.array(Ra)); g.init_t.append(np.array(ta))
        if len(g.init_R) != n_robots:
            g.init_R, g.init_t = [], []
    return g
