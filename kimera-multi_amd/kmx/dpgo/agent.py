"""PGOAgent — the dpgo agent API over the MI355X block solver.

One agent = one robot (dpgo_ros runs one per process, drawio:1954-1966). The
agent keeps the reference's call surface and semantics:

  PGOAgent(ID, params)                      dpgo::PGOAgent ctor
  addMeasurement / setMeasurements          PoseGraph::addMeasurement (drawio:2142, 2337, 2779-2826)
  setLiftingMatrix                          drawio:2310-2322
  initialize(TInit=None)                    INITIALIZE (drawio:2271-2307); odometry chain when no TInit (D10)
  iterate(doOptimization)                   drawio:2513 (one RBCD block update)
  getSharedPoseDict / updateNeighborPoses   drawio:2340-2355
  shouldUpdateMeasurementWeights /
  updateMeasurementWeights                  drawio:2466-2469, 2215 (owner re-weights its loop closures)
  getSharedMeasurementWeights /
  setMeasurementWeight                      drawio:2195-2268 (owner -> peer)
  setGlobalAnchor / getTrajectoryIn*Frame   drawio:2396, 2148-2151
  getStatus / setNeighborStatus /
  shouldTerminate / reset                   drawio:2030, 2375-2387, 2436

Errors: the C++ agent returns `false` or aborts via CHECK; here a call made in
the wrong state raises ValueError, getters that dpgo reports via `bool`
return None. There is no CPU fallback: the default solver is the HIP
BlockSolver and fails loudly without a GPU (tests inject the oracle-backed
stand-in in tests/mock_solver.py).

Edge order inside the solver: odometry, then private loop closures, then
shared loop closures, each in insertion order (dpgo's odometry_, private_lcs_,
shared_lcs_ vectors).
"""
from __future__ import annotations

import numpy as np

from ..synth.pose_graph import PoseGraphData, lift, lifting_matrix
from .messages import (MeasurementWeights, PGOAgentState, PGOAgentStatus, PoseID, PublicPoses,
                       RelativeSEMeasurement)
from .params import PGOAgentParameters
from .schedule import GncSchedule


class PGOAgent:
    def __init__(self, ID: int, params: PGOAgentParameters, *, device: int = 0, solver=None):
        self.mID = int(ID)
        self.params = params
        self.d, self.r = params.d, params.r
        self._device = device
        self._solver_factory = (lambda: solver) if solver is not None else None
        self.instance = 0
        self._reset_state()

    # ------------------------------------------------------------- state ---
    def _reset_state(self):
        self.odometry: list[RelativeSEMeasurement] = []
        self.private_lcs: list[RelativeSEMeasurement] = []
        self.shared_lcs: list[RelativeSEMeasurement] = []
        self.state = PGOAgentState.WAIT_FOR_DATA
        self.iteration = 0
        self._gnc = GncSchedule.from_params(self.params)
        self.YLift = None
        self.globalAnchor = None
        self.solver = None
        self.n = 0
        self._edge_index = {}
        self._have_nbr = set()
        self.neighbor_status: dict[int, PGOAgentStatus] = {}
        self._rel_change = float("inf")

    def getID(self) -> int:
        return self.mID

    def num_poses(self) -> int:
        return self.n

    def dimension(self) -> int:
        return self.d

    def relaxation_rank(self) -> int:
        return self.r

    def instance_number(self) -> int:
        return self.instance

    def iteration_number(self) -> int:
        return self.iteration

    def getState(self) -> PGOAgentState:
        return self.state

    # ------------------------------------------------------ measurements ---
    def addMeasurement(self, m: RelativeSEMeasurement):
        """PoseGraph::addMeasurement: odometry if same robot and p2 == p1 + 1,
        private loop closure if same robot, shared loop closure otherwise."""
        if self.state == PGOAgentState.INITIALIZED:
            raise ValueError("addMeasurement after initialize (call reset first)")
        if m.r1 != self.mID and m.r2 != self.mID:
            raise ValueError(f"measurement ({m.r1},{m.p1})->({m.r2},{m.p2}) does not involve robot {self.mID}")
        if m.r1 == m.r2:
            if m.p2 == m.p1 + 1:
                self.odometry.append(m)
            else:
                self.private_lcs.append(m)
        else:
            self.shared_lcs.append(m)
        self.state = PGOAgentState.WAIT_FOR_INITIALIZATION

    def setMeasurements(self, odometry, private_lcs, shared_lcs):
        self.odometry, self.private_lcs, self.shared_lcs = list(odometry), list(private_lcs), list(shared_lcs)
        self.state = PGOAgentState.WAIT_FOR_INITIALIZATION

    def _all(self):
        return self.odometry + self.private_lcs + self.shared_lcs

    # ---------------------------------------------------- initialisation ---
    def setLiftingMatrix(self, M):
        M = np.asarray(M, dtype=np.float64)
        if M.shape != (self.r, self.d):
            raise ValueError(f"lifting matrix must be {self.r}x{self.d}")
        self.YLift = M

    def getLiftingMatrix(self):
        return self.YLift

    def _graph(self) -> PoseGraphData:
        ms = self._all()
        if not ms:
            raise ValueError("no measurements")
        nr = max(max(m.r1, m.r2) for m in ms) + 1
        npose = np.zeros(nr, np.int32)
        for m in ms:
            npose[m.r1] = max(npose[m.r1], m.p1 + 1)
            npose[m.r2] = max(npose[m.r2], m.p2 + 1)
        f = lambda key, dt: np.array([getattr(m, key) for m in ms], dtype=dt)
        return PoseGraphData(
            n_robots=nr, n_poses=npose, r1=f("r1", np.int32), p1=f("p1", np.int32), r2=f("r2", np.int32),
            p2=f("p2", np.int32), R=np.array([np.asarray(m.R, np.float64) for m in ms]).reshape(-1, 3, 3),
            t=np.array([np.asarray(m.t, np.float64) for m in ms]).reshape(-1, 3), kappa=f("kappa", np.float64),
            tau=f("tau", np.float64), weight=f("weight", np.float64),
            fixed=f("fixedWeight", np.uint8), outlier=np.zeros(len(ms), bool))

    def _odometry_chain(self):
        Rs = np.zeros((self.n, 3, 3))
        ts = np.zeros((self.n, 3))
        Rs[0] = np.eye(3)
        step = {}
        for m in sorted(self.odometry, key=lambda m: not m.fixedWeight):  # true odometry first
            step.setdefault(m.p1, m)
        for i in range(self.n - 1):
            m = step.get(i)
            if m is None:
                raise ValueError(f"odometry chain broken at pose {i}; pass TInit")
            Rs[i + 1] = Rs[i] @ m.R
            ts[i + 1] = ts[i] + Rs[i] @ m.t
        return Rs, ts

    def initialize(self, TInit=None, neighbor_global_poses=None):
        """INITIALIZE: build the local problem and the initial lifted iterate.
        TInit: dpgo PoseArray (d x (d+1)n) or [n, 3, 4]; default: the odometry
        chain or, with localInitializationMethod "chordal", the chordal
        relaxation over the robot's own measurements (kmx.dpgo.init).
        neighbor_global_poses: {(robot, pose): (R, t)} of neighbours already in
        the global frame -> the local trajectory is aligned to it by robust
        single-pose averaging over the shared loop closures (kmx.dpgo.init;
        drawio:2271-2307). Robot 0 defines the global frame."""
        if self.state == PGOAgentState.WAIT_FOR_DATA:
            raise ValueError("no measurements")
        if self.YLift is None:
            if self.mID != 0:
                raise ValueError("lifting matrix not set (the leader publishes it, drawio:2310-2322)")
            self.YLift = lifting_matrix(self.r, self.d)
        g = self._graph()
        self.graph = g
        self.n = int(g.n_poses[self.mID])
        local = np.zeros(g.n_robots, np.uint8)
        local[self.mID] = 1
        if self._solver_factory is not None:
            self.solver = self._solver_factory()
        else:
            from .solver import BlockSolver
            self.solver = BlockSolver(self.params, self._device)
        self.solver.set_graph_data(g, local)
        # (src, dst) -> edge indices; a key can repeat (two measurements between
        # the same poses): lookups by key address the first, weight messages
        # are applied in order
        self._edge_index, self._edge_dups = {}, {}
        for k, m in enumerate(self._all()):
            key = (m.r1, m.p1, m.r2, m.p2)
            self._edge_index.setdefault(key, k)
            self._edge_dups.setdefault(key, []).append(k)
        self._base_w = g.weight.copy()
        # shared loop closures: public poses (own end) and neighbour poses (other end)
        self._own_public = sorted({PoseID(m.r1, m.p1) if m.r1 == self.mID else PoseID(m.r2, m.p2)
                                   for m in self.shared_lcs})
        self._nbr_public = sorted({PoseID(m.r2, m.p2) if m.r1 == self.mID else PoseID(m.r1, m.p1)
                                   for m in self.shared_lcs})
        self._have_nbr = set()
        self._weights = g.weight.copy()
        if TInit is None:
            if self.params.localInitializationMethod == "chordal":
                from .init import chordal_initialization
                own = self.odometry + self.private_lcs
                Rs, ts = chordal_initialization(self.n, [(m.p1, m.p2, m.R, m.t, m.kappa, m.tau, m.weight) for m in own])
            elif self.params.localInitializationMethod == "odometry":
                Rs, ts = self._odometry_chain()
            else:
                raise ValueError(f"unknown localInitializationMethod {self.params.localInitializationMethod!r}")
        else:
            T = np.asarray(TInit, dtype=np.float64)
            if T.shape == (self.d, (self.d + 1) * self.n):
                T = T.reshape(self.d, self.n, self.d + 1).transpose(1, 0, 2)
            Rs, ts = T[:, :, :3], T[:, :, 3]
        self.alignment = None
        if neighbor_global_poses and self.mID != 0:
            from .init import align_to_world, transform_trajectory
            out = align_to_world(self.shared_lcs, self.mID, Rs, ts, neighbor_global_poses)
            if out is not None:
                R_WA, t_WA, w = out
                Rs, ts = transform_trajectory(R_WA, t_WA, Rs, ts)
                self.alignment = (R_WA, t_WA, w)
        self.solver.set_iterate(self.mID, lift(Rs, ts, self.YLift))
        self._apply_missing_neighbours()
        self.iteration = 0
        self.state = PGOAgentState.INITIALIZED

    def _apply_missing_neighbours(self):
        """Shared loop closures whose neighbour pose has not arrived yet carry
        weight 0 in the local problem (they become active with the first
        updateNeighborPoses that contains the neighbour pose)."""
        w = self._weights.copy()
        for m in self.shared_lcs:
            other = PoseID(m.r2, m.p2) if m.r1 == self.mID else PoseID(m.r1, m.p1)
            if other not in self._have_nbr:
                w[self._edge_dups[(m.r1, m.p1, m.r2, m.p2)]] = 0.0
        self.solver.set_weights(w)

    # ------------------------------------------------------------ rounds ---
    @property
    def weight_updates(self) -> int:
        return self._gnc.updates

    def iterate(self, doOptimization: bool = True) -> bool:
        if self.state != PGOAgentState.INITIALIZED:
            return False
        self.iteration += 1
        self._gnc.round_done()  # every iterate counts as a GNC inner iteration
        if doOptimization:
            act = np.zeros(self.graph.n_robots, np.uint8)
            act[self.mID] = 1
            st = self.solver.iterate(act)[self.mID]
            self.last_stats = st
            if st["updated"]:
                self._rel_change = st["rel_change"]
        return True

    def setX(self, X):
        self.solver.set_iterate(self.mID, np.asarray(X, np.float64).reshape(self.n, self.r, self.d + 1))

    def getX(self):
        return self.solver.get_iterate(self.mID) if self.state == PGOAgentState.INITIALIZED else None

    def getNeighbors(self) -> list[int]:
        return sorted({p.robot_id for p in self._nbr_public}) if self.state == PGOAgentState.INITIALIZED else []

    def getSharedPoseDict(self):
        """Own poses that are endpoints of shared loop closures (publishPublicPoses)."""
        if self.state != PGOAgentState.INITIALIZED:
            return None
        X = self.solver.get_iterate(self.mID)
        return {p: X[p.frame_id].copy() for p in self._own_public}

    def publicPosesMessage(self) -> PublicPoses | None:
        D = self.getSharedPoseDict()
        if D is None:
            return None
        return PublicPoses(self.mID, self.instance, self.iteration, list(D), list(D.values()))

    def updateNeighborPoses(self, neighborID: int, poseDict: dict):
        if self.state != PGOAgentState.INITIALIZED or neighborID == self.mID:
            return
        want = [p for p in self._nbr_public if p.robot_id == neighborID and p in poseDict]
        if not want:
            return
        self.solver.set_neighbor_poses([p.robot_id for p in want], [p.frame_id for p in want],
                                       np.stack([np.asarray(poseDict[p], np.float64) for p in want]))
        new = set(want) - self._have_nbr
        if new:
            self._have_nbr |= new
            self._apply_missing_neighbours()

    # --------------------------------------------------------------- GNC ---
    def shouldUpdateMeasurementWeights(self) -> bool:
        """drawio:2466-2469: never for L2 or after robustOptNumWeightUpdates
        updates; true once more than robustOptInnerIters iterations ran since
        the last update, or when every agent of the team (num_robots; own
        status and the statuses received by setNeighborStatus) has converged
        (relative change <= relChangeTol)."""
        team = []
        for rid in range(max(self.params.num_robots, self.mID + 1)):
            if rid == self.mID:
                team.append(self._rel_change)
            else:
                st = self.neighbor_status.get(rid)
                team.append(st.relativeChange if st is not None and st.iterationNumber > 0 else float("inf"))
        return self._gnc.should_update(team)

    def updateMeasurementWeights(self):
        """GNC-TLS update of the loop closures this robot owns (non-fixed,
        owner = lower robot id for shared ones), then mu <- mu * mu_step."""
        if self.state != PGOAgentState.INITIALIZED:
            raise ValueError("updateMeasurementWeights before initialize")
        self.solver.update_weights()
        w = self.solver.get_weights(self._weights)
        for m in self.shared_lcs:  # no neighbour pose yet: keep the previous weight
            other = PoseID(m.r2, m.p2) if m.r1 == self.mID else PoseID(m.r1, m.p1)
            if other not in self._have_nbr:
                k = self._edge_dups[(m.r1, m.p1, m.r2, m.p2)]
                w[k] = self._weights[k]
        self._weights = w
        self._apply_missing_neighbours()
        self._gnc.updated()

    def setMeasurementWeight(self, src: PoseID, dst: PoseID, weight: float, fixed_weight: bool = False):
        k = self._edge_index.get((src.robot_id, src.frame_id, dst.robot_id, dst.frame_id))
        if k is None:
            return False
        self._weights[k] = weight
        if self.state == PGOAgentState.INITIALIZED:
            self._apply_missing_neighbours()
        return True

    def getMeasurementWeight(self, src: PoseID, dst: PoseID):
        k = self._edge_index.get((src.robot_id, src.frame_id, dst.robot_id, dst.frame_id))
        return None if k is None else float(self._weights[k])

    def getSharedMeasurementWeights(self) -> MeasurementWeights:
        """Weights of the shared loop closures this robot owns (publishMeasurementWeights)."""
        src, dst, w, fx = [], [], [], []
        base = len(self.odometry) + len(self.private_lcs)
        for k, m in enumerate(self.shared_lcs):
            if min(m.r1, m.r2) != self.mID:
                continue
            src.append(PoseID(m.r1, m.p1))
            dst.append(PoseID(m.r2, m.p2))
            w.append(float(self._weights[base + k]))
            fx.append(bool(m.fixedWeight))
        return MeasurementWeights(self.mID, self.instance, src, dst, w, fx)

    def measurementWeightsCallback(self, msg: MeasurementWeights):
        seen = {}
        for s, t, w, f in zip(msg.src, msg.dst, msg.weights, msg.fixed):
            if min(s.robot_id, t.robot_id) != msg.robot_id:  # only the owner's word counts
                continue
            key = (s.robot_id, s.frame_id, t.robot_id, t.frame_id)
            ks = self._edge_dups.get(key)
            if not ks:
                continue
            i = seen.get(key, 0)  # repeated keys: the j-th weight goes to the j-th copy
            seen[key] = i + 1
            self._weights[ks[min(i, len(ks) - 1)]] = w
        if self.state == PGOAgentState.INITIALIZED:
            self._apply_missing_neighbours()

    # ----------------------------------------------------------- outputs ---
    def setGlobalAnchor(self, M):
        M = np.asarray(M, np.float64)
        if M.shape != (self.r, self.d + 1):
            raise ValueError(f"anchor must be {self.r}x{self.d + 1} (lifted pose)")
        self.globalAnchor = M

    def _traj(self, anchor):
        T = self.solver.trajectory(self.mID, anchor)  # [n, 12]: R row-major, t
        out = np.empty((self.d, (self.d + 1) * self.n))
        out.reshape(self.d, self.n, self.d + 1)[:] = np.concatenate(
            [T[:, :9].reshape(-1, 3, 3), T[:, 9:, None]], axis=2).transpose(1, 0, 2)
        return out

    def getTrajectoryInLocalFrame(self):
        """d x (d+1)n, expressed relative to this robot's first pose."""
        if self.state != PGOAgentState.INITIALIZED:
            return None
        return self._traj(self.solver.get_iterate(self.mID)[0])

    def getTrajectoryInGlobalFrame(self):
        """d x (d+1)n relative to the global anchor (leader's first pose)."""
        if self.state != PGOAgentState.INITIALIZED or self.globalAnchor is None:
            return None
        return self._traj(self.globalAnchor)

    # ---------------------------------------------------------- status ---
    def getStatus(self) -> PGOAgentStatus:
        ready = (self.state == PGOAgentState.INITIALIZED and self.iteration > 0
                 and self._rel_change < self.params.relChangeTol)
        return PGOAgentStatus(self.mID, self.state, self.instance, self.iteration, bool(ready),
                              float(self._rel_change) if np.isfinite(self._rel_change) else 0.0)

    def setNeighborStatus(self, status: PGOAgentStatus):
        self.neighbor_status[status.agentID] = status

    def shouldTerminate(self) -> bool:
        """drawio:2030: past maxNumIters, or this agent and every neighbour ready."""
        if self.iteration >= self.params.maxNumIters:
            return True
        if not self.getStatus().readyToTerminate:
            return False
        for nb in self.getNeighbors():
            st = self.neighbor_status.get(nb)
            if st is None or not st.readyToTerminate:
                return False
        return True

    def reset(self):
        """drawio:2436: drop measurements and iterate; next instance."""
        if self.solver is not None and hasattr(self.solver, "close"):
            self.solver.close()
        self.instance += 1
        self._reset_state()
