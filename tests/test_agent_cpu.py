"""PGOAgent (dpgo API mirror) driven the dpgo_ros way — one agent per robot,
PublicPoses / MeasurementWeights messages between them — on the oracle-backed
solver stand-in, against the single-process team restatement."""
import numpy as np
import pytest

from kmx.dpgo.agent import PGOAgent
from kmx.dpgo.messages import PGOAgentState, PoseID, RelativeSEMeasurement
from kmx.dpgo.params import PGOAgentParameters
from kmx.synth import lift, lifting_matrix, make_pose_graph
from tests.mock_solver import OracleBlockSolver


def _measurements(g, a):
    out = []
    for e in np.nonzero((g.r1 == a) | (g.r2 == a))[0]:
        out.append(RelativeSEMeasurement(int(g.r1[e]), int(g.r2[e]), int(g.p1[e]), int(g.p2[e]), 3, g.R[e].copy(),
                                         g.t[e].copy(), float(g.kappa[e]), float(g.tau[e]), bool(g.fixed[e]),
                                         float(g.weight[e])))
    return out


def _team(g, P, TInit=True):
    Y = lifting_matrix(P.r)
    agents = []
    for a in range(g.n_robots):
        ag = PGOAgent(a, P, solver=OracleBlockSolver(P))
        for m in _measurements(g, a):
            ag.addMeasurement(m)
        ag.setLiftingMatrix(Y)
        T = np.concatenate([g.init_R[a], g.init_t[a][:, :, None]], axis=2) if TInit else None
        ag.initialize(T)
        agents.append(ag)
    return agents, Y


def _exchange(agents):
    msgs = [ag.publicPosesMessage() for ag in agents]
    for ag in agents:
        for m in msgs:
            ag.updateNeighborPoses(m.robot_id, m.as_dict())


def test_agents_match_team_restatement():
    from oracle.oracle import OraclePGO
    g = make_pose_graph(3, 300, 900, seed=7)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 4
    agents, Y = _team(g, P)
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        o.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    rounds = 12
    for k in range(1, rounds + 1):
        _exchange(agents)
        for ag in agents:
            ag.iterate(True)
        o.iterate()
        if all(ag.shouldUpdateMeasurementWeights() for ag in agents):
            _exchange(agents)
            for ag in agents:
                ag.updateMeasurementWeights()
            wmsgs = [ag.getSharedMeasurementWeights() for ag in agents]
            for ag in agents:
                for m in wmsgs:
                    if m.robot_id != ag.getID():
                        ag.measurementWeightsCallback(m)
            o.refresh()
            o.update_weights()
        # drawio:2466-2469: an update once MORE than InnerIters iterations ran (no
        # team statuses exchanged here, so the convergence branch never fires)
        assert agents[0].weight_updates == k // (P.robustOptInnerIters + 1), k
    for a, ag in enumerate(agents):
        # different edge order inside each agent -> summation order differs at ~1 ulp
        assert np.abs(ag.getX() - o.get_iterate(a)).max() < 1e-9
    w = o.get_weights()
    from collections import Counter
    dup = Counter(zip(g.r1.tolist(), g.p1.tolist(), g.r2.tolist(), g.p2.tolist()))
    for ag in agents:
        for m in ag.shared_lcs + ag.private_lcs:
            if dup[(m.r1, m.p1, m.r2, m.p2)] > 1:
                continue  # repeated (src, dst) key: the lookup by key is ambiguous
            e = np.nonzero((g.r1 == m.r1) & (g.p1 == m.p1) & (g.r2 == m.r2) & (g.p2 == m.p2))[0][0]
            assert abs(ag.getMeasurementWeight(PoseID(m.r1, m.p1), PoseID(m.r2, m.p2)) - w[e]) < 1e-9


def test_agent_states_outputs_and_reset():
    g = make_pose_graph(2, 120, 300, seed=3)
    P = PGOAgentParameters(r=5)
    P.maxNumIters = 5
    ag = PGOAgent(1, P, solver=OracleBlockSolver(P))
    assert ag.getState() == PGOAgentState.WAIT_FOR_DATA
    assert not ag.iterate()
    for m in _measurements(g, 1):
        ag.addMeasurement(m)
    assert ag.getState() == PGOAgentState.WAIT_FOR_INITIALIZATION
    with pytest.raises(ValueError):
        ag.initialize()  # non-leader without a lifting matrix
    assert len(ag.odometry) == g.n_poses[1] - 1
    Y = lifting_matrix(5)
    ag.setLiftingMatrix(Y)
    ag.initialize()  # odometry chain
    assert ag.num_poses() == g.n_poses[1]
    # the odometry chain starts at the identity and composes the odometry measurements
    T = ag.getTrajectoryInLocalFrame()
    assert T.shape == (3, 4 * ag.num_poses())
    R0, t0 = g.init_R[1][0], g.init_t[1][0]
    ref = np.einsum("ji,njk->nik", R0, g.init_R[1])
    assert np.abs(T.reshape(3, -1, 4).transpose(1, 0, 2)[:, :, :3] - ref).max() < 1e-9
    assert ag.getNeighbors() == [0]
    D = ag.getSharedPoseDict()
    assert all(p.robot_id == 1 and v.shape == (5, 4) for p, v in D.items())
    assert ag.getTrajectoryInGlobalFrame() is None
    ag.setGlobalAnchor(lift(np.eye(3)[None], np.zeros((1, 3)), Y)[0])
    for _ in range(5):
        ag.iterate()
    assert ag.shouldTerminate()  # maxNumIters
    st = ag.getStatus()
    assert st.agentID == 1 and st.iterationNumber == 5
    ag.reset()
    assert ag.getState() == PGOAgentState.WAIT_FOR_DATA and ag.instance_number() == 1


def test_agent_initialize_in_global_frame():
    """Robot 1 aligns its odometry-chain initialisation to robot 0's global
    frame through the shared loop closures (row f4)."""
    g = make_pose_graph(2, 400, 1200, outlier_frac=0.2, f_inter=0.3, noise_free=True, seed=9)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5)
    a0 = PGOAgent(0, P, solver=OracleBlockSolver(P))
    a1 = PGOAgent(1, P, solver=OracleBlockSolver(P))
    for ag in (a0, a1):
        for m in _measurements(g, ag.getID()):
            ag.addMeasurement(m)
        ag.setLiftingMatrix(Y)
    T0 = np.concatenate([g.gt_R[0], g.gt_t[0][:, :, None]], axis=2)
    a0.initialize(T0)
    world = {(0, i): (g.gt_R[0][i], g.gt_t[0][i]) for i in range(int(g.n_poses[0]))}
    a1.initialize(neighbor_global_poses=world)
    X = a1.getX()
    Rw = np.einsum("ab,nac->nbc", Y, X[:, :, :3])
    assert np.abs(Rw - g.gt_R[1]).max() < 1e-8
    assert a1.alignment is not None and 0 < a1.alignment[2].sum() < len(a1.alignment[2])
