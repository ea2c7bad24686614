"""dpgo_ros message types and the PGOAgent status record, as plain dataclasses.

The ROS wire API of dpgo_ros (drawio:1986, 2151, 2313-2393):
topics ~/command, ~/public_poses, ~/lifting_matrix, ~/measurement_weights,
~/status, ~/anchor. Inside one node of this framework these become
collectives (kmx.dpgo.driver); across processes a ROS bridge fills these
records field for field. Command type values follow the order in which the
survey lists them [U: the .msg constants themselves are not in the reference
tree]."""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np


class CommandType(IntEnum):
    REQUEST_POSE_GRAPH = 0  # drawio:2124
    INITIALIZE = 1          # drawio:2307
    UPDATE = 2              # drawio:2369
    UPDATE_WEIGHT = 3       # drawio:2212
    TERMINATE = 4           # drawio:2180
    HARD_TERMINATE = 5      # drawio:2433
    RECOVER = 6             # drawio:2448
    NOOP = 7                # drawio:2402
    SET_ACTIVE_ROBOTS = 8   # drawio:2405


class PGOAgentState(IntEnum):
    WAIT_FOR_DATA = 0
    WAIT_FOR_INITIALIZATION = 1
    INITIALIZED = 2


@dataclass(frozen=True, order=True)
class PoseID:
    robot_id: int
    frame_id: int


@dataclass
class RelativeSEMeasurement:
    """dpgo RelativeSEMeasurement (drawio:2779-2826): pose (r1,p1) -> (r2,p2)
    with p_2 = p_1 + R_1 t, R_2 = R_1 R; precisions kappa (rotation) and tau
    (translation); `weight` is the GNC weight, `fixedWeight` exempts the edge
    (odometry) from reweighting."""
    r1: int
    r2: int
    p1: int
    p2: int
    d: int
    R: np.ndarray
    t: np.ndarray
    kappa: float
    tau: float
    fixedWeight: bool = False
    weight: float = 1.0


@dataclass
class PGOAgentStatus:
    agentID: int
    state: PGOAgentState = PGOAgentState.WAIT_FOR_DATA
    instanceNumber: int = 0
    iterationNumber: int = 0
    readyToTerminate: bool = False
    relativeChange: float = 0.0


@dataclass
class Command:
    publishing_robot: int
    command: CommandType
    executing_robot: int = -1
    executing_iteration: int = 0
    active_robots: list = field(default_factory=list)


@dataclass
class PublicPoses:
    """~/public_poses: lifted public poses of one robot (r x (d+1) each)."""
    robot_id: int
    instance_number: int
    iteration_number: int
    pose_ids: list          # [PoseID]
    poses: list             # [np.ndarray r x (d+1)]
    is_auxiliary: bool = False

    def as_dict(self) -> dict:
        return dict(zip(self.pose_ids, self.poses))


@dataclass
class LiftingMatrix:
    rows: int
    cols: int
    data: np.ndarray        # r x d, column-orthonormal


@dataclass
class MeasurementWeights:
    """~/measurement_weights: owner -> peer weights of shared loop closures."""
    robot_id: int
    instance_number: int
    src: list               # [PoseID]
    dst: list               # [PoseID]
    weights: list           # [float]
    fixed: list             # [bool]
