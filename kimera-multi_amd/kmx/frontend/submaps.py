"""Kimera-Distributed submap coarsening and the PoseGraph wire format
(drawio:557-574, 623-632; pose_graph_tools,
kimera_multi.repos:110-113).

Kimera-Distributed does not hand dpgo its keyframe graph: keyframes are
grouped into submaps ("create a submap representing the new keyframe and the
frames after it", drawio:623) and `getSubmapPoseGraph` (drawio:560-574)
serves the sparse graph "new loop closures of submap_loop_closures_ + edges
between submaps" through `request_pose_graph` (drawio:629-632):

* a submap's pose is the odometry pose of its first keyframe; every keyframe
  keeps its pose relative to its submap (T_S_k);
* odometry edges join consecutive submaps of a robot (relative odometry);
* a keyframe loop closure (a, k_a) -> (b, k_b) with T_ka_kb becomes the submap
  edge T_Sa_Sb = T_Sa_ka T_ka_kb T_Sb_kb^-1;
* after optimisation a keyframe's pose is T_W_S T_S_k (the TUM output).

A new submap starts when the current one spans more than `max_distance`
metres or `max_keyframes` keyframes [U: Kimera-Distributed's thresholds are
named submap_dist_threshold / submap_time_threshold in its launch files,
which are not part of this reference tree].

PoseGraph / PoseGraphNode / PoseGraphEdge mirror pose_graph_tools_msgs
(edge types ODOM = 0, LOOPCLOSE = 1, ...; 6x6 covariance, rotation block
last as in GTSAM's Pose3 tangent order [U]).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ..dpgo.messages import RelativeSEMeasurement


def _inv(R, t):
    return R.T, -R.T @ t


def _mul(Ra, ta, Rb, tb):
    return Ra @ Rb, Ra @ tb + ta


class SubmapAtlas:
    """Keyframes of one robot grouped into submaps."""

    def __init__(self, robot_id: int, *, max_distance: float = 5.0, max_keyframes: int = 20):
        self.robot = robot_id
        self.max_distance = max_distance
        self.max_keyframes = max_keyframes
        self.kf_submap: list[int] = []          # keyframe id -> submap id
        self.kf_rel: list[tuple] = []           # keyframe id -> T_S_k
        self.kf_stamp: list[int] = []
        self.submap_pose: list[tuple] = []      # submap id -> T_odom_S (first keyframe's odometry pose)
        self.submap_kfs: list[list[int]] = []
        self._loop_closures: list[RelativeSEMeasurement] = []

    @property
    def n_submaps(self) -> int:
        return len(self.submap_pose)

    def add_keyframe(self, kf_id: int, stamp_ns: int, R_odom, t_odom) -> int:
        """Keyframes arrive in order (kf_id = 0, 1, ...). Returns the submap id."""
        if kf_id != len(self.kf_submap):
            raise ValueError("keyframes must be added in order")
        R_odom, t_odom = np.asarray(R_odom, np.float64), np.asarray(t_odom, np.float64)
        new = not self.submap_pose
        if not new:
            Rs, ts = self.submap_pose[-1]
            new = (np.linalg.norm(t_odom - ts) > self.max_distance or
                   len(self.submap_kfs[-1]) >= self.max_keyframes)
        if new:
            self.submap_pose.append((R_odom, t_odom))
            self.submap_kfs.append([])
        s = self.n_submaps - 1
        Rs, ts = self.submap_pose[s]
        self.kf_rel.append(_mul(*_inv(Rs, ts), R_odom, t_odom))
        self.kf_submap.append(s)
        self.kf_stamp.append(int(stamp_ns))
        self.submap_kfs[s].append(kf_id)
        return s

    def odometry_edges(self, kappa: float, tau: float) -> list[RelativeSEMeasurement]:
        out = []
        for s in range(self.n_submaps - 1):
            R, t = _mul(*_inv(*self.submap_pose[s]), *self.submap_pose[s + 1])
            out.append(RelativeSEMeasurement(self.robot, self.robot, s, s + 1, 3, R, t, kappa, tau, True, 1.0))
        return out

    def keyframe_in_submap(self, kf_id: int):
        return self.kf_submap[kf_id], self.kf_rel[kf_id]

    @staticmethod
    def submap_loop_closure(atlas_a: "SubmapAtlas", kf_a: int, atlas_b: "SubmapAtlas", kf_b: int, R_ab, t_ab,
                            kappa: float, tau: float) -> RelativeSEMeasurement | None:
        """Keyframe loop closure T_ka_kb -> submap edge T_Sa_Sb; None when both
        keyframes lie in the same submap of one robot (a self-loop carries no
        constraint between submap poses, and kmx_pgo_set_graph rejects it) [U:
        Kimera-Distributed's own handling is not vendored]."""
        sa, (Ra, ta) = atlas_a.keyframe_in_submap(kf_a)
        sb, (Rb, tb) = atlas_b.keyframe_in_submap(kf_b)
        if atlas_a.robot == atlas_b.robot and sa == sb:
            return None
        R, t = _mul(*_mul(Ra, ta, np.asarray(R_ab, np.float64), np.asarray(t_ab, np.float64)), *_inv(Rb, tb))
        return RelativeSEMeasurement(atlas_a.robot, atlas_b.robot, sa, sb, 3, R, t, kappa, tau, False, 1.0)

    def keyframe_trajectory(self, R_sub, t_sub):
        """Keyframe poses from optimised submap poses ([n_submaps, 3, 3], [n_submaps, 3])."""
        n = len(self.kf_submap)
        R = np.empty((n, 3, 3))
        t = np.empty((n, 3))
        for k in range(n):
            s = self.kf_submap[k]
            R[k], t[k] = _mul(R_sub[s], t_sub[s], *self.kf_rel[k])
        return R, t


# --------------------------------------------------------- PoseGraph msg ---
ODOM, LOOPCLOSE, LANDMARK, REJECTED_LOOPCLOSE, MESH, POSE_MESH, MESH_POSE = range(7)


@dataclass
class PoseGraphNode:
    robot_id: int
    key: int
    R: np.ndarray
    t: np.ndarray
    stamp_ns: int = 0


@dataclass
class PoseGraphEdge:
    robot_from: int
    key_from: int
    robot_to: int
    key_to: int
    type: int
    R: np.ndarray
    t: np.ndarray
    covariance: np.ndarray = field(default_factory=lambda: np.eye(6))  # [t (3), rot (3)] [U]


@dataclass
class PoseGraph:
    nodes: list = field(default_factory=list)
    edges: list = field(default_factory=list)


def _cov_from_precisions(kappa: float, tau: float) -> np.ndarray:
    """dpgo's isotropic precisions -> 6x6 covariance (translation, rotation).
    kappa |dR|_F^2 ~ 2 kappa |dtheta|^2 => rotation variance 1 / (2 kappa)."""
    C = np.zeros((6, 6))
    C[:3, :3] = np.eye(3) / tau
    C[3:, 3:] = np.eye(3) / (2.0 * kappa)
    return C


def _precisions_from_cov(C: np.ndarray):
    C = np.asarray(C, np.float64).reshape(6, 6)
    tau = 3.0 / np.trace(C[:3, :3])
    kappa = 3.0 / (2.0 * np.trace(C[3:, 3:]))
    return kappa, tau


def pose_graph_from_measurements(measurements, nodes=()) -> PoseGraph:
    g = PoseGraph(nodes=list(nodes))
    for m in measurements:
        typ = ODOM if (m.fixedWeight and m.r1 == m.r2 and m.p2 == m.p1 + 1) else LOOPCLOSE
        g.edges.append(PoseGraphEdge(m.r1, m.p1, m.r2, m.p2, typ, np.asarray(m.R), np.asarray(m.t),
                                     _cov_from_precisions(m.kappa, m.tau)))
    return g


def measurements_from_pose_graph(g: PoseGraph) -> list[RelativeSEMeasurement]:
    """PoseGraph edges -> dpgo measurements (odometry edges keep a fixed weight;
    REJECTED_LOOPCLOSE and mesh edges are dropped)."""
    out = []
    for e in g.edges:
        if e.type not in (ODOM, LOOPCLOSE):
            continue
        kappa, tau = _precisions_from_cov(e.covariance)
        out.append(RelativeSEMeasurement(e.robot_from, e.robot_to, e.key_from, e.key_to, 3, np.asarray(e.R),
                                         np.asarray(e.t), kappa, tau, e.type == ODOM, 1.0))
    return out


def graph_data(measurements, n_poses=None):
    """dpgo measurements (e.g. measurements_from_pose_graph of a
    request_pose_graph reply) -> the team graph kmx_pgo_set_graph takes
    (PoseGraphData; pose counts from the largest pose index per robot unless
    given)."""
    from ..synth.pose_graph import PoseGraphData
    ms = list(measurements)
    if not ms:
        raise ValueError("no measurements")
    nr = max(max(m.r1, m.r2) for m in ms) + 1 if n_poses is None else len(n_poses)
    npose = np.zeros(nr, np.int32)
    if n_poses is not None:
        npose[:] = np.asarray(n_poses, np.int32)
    for m in ms:
        npose[m.r1] = max(npose[m.r1], m.p1 + 1)
        npose[m.r2] = max(npose[m.r2], m.p2 + 1)
    f = lambda key, dt: np.array([getattr(m, key) for m in ms], dtype=dt)
    return PoseGraphData(
        n_robots=nr, n_poses=npose, r1=f("r1", np.int32), p1=f("p1", np.int32), r2=f("r2", np.int32),
        p2=f("p2", np.int32), R=np.array([np.asarray(m.R, np.float64) for m in ms]).reshape(-1, 3, 3),
        t=np.array([np.asarray(m.t, np.float64) for m in ms]).reshape(-1, 3), kappa=f("kappa", np.float64),
        tau=f("tau", np.float64), weight=f("weight", np.float64), fixed=f("fixedWeight", np.uint8),
        outlier=np.zeros(len(ms), bool))

