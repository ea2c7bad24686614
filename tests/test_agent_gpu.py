"""PGOAgent on the HIP BlockSolver (one agent = one robot, messages between
agents) against the CPU team restatement: poses within 1e-6, GNC weights within 1e-6."""
import numpy as np
import pytest

from kmx.dpgo.agent import PGOAgent
from kmx.dpgo.params import PGOAgentParameters
from kmx.synth import lift, lifting_matrix, make_pose_graph
from tests.test_agent_cpu import _exchange, _measurements

pytestmark = pytest.mark.gpu


def test_gpu_agents_match_team_restatement(gpu):
    from oracle.oracle import OraclePGO
    g = make_pose_graph(3, 1500, 4500, seed=11)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 5
    Y = lifting_matrix(5)
    agents = []
    for a in range(g.n_robots):
        ag = PGOAgent(a, P, device=0)
        for m in _measurements(g, a):
            ag.addMeasurement(m)
        ag.setLiftingMatrix(Y)
        ag.initialize(np.concatenate([g.init_R[a], g.init_t[a][:, :, None]], axis=2))
        agents.append(ag)
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        o.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    for k in range(1, 16):
        _exchange(agents)
        for ag in agents:
            ag.iterate(True)
        o.iterate()
        if agents[0].shouldUpdateMeasurementWeights():
            _exchange(agents)
            for ag in agents:
                ag.updateMeasurementWeights()
            msgs = [ag.getSharedMeasurementWeights() for ag in agents]
            for ag in agents:
                for m in msgs:
                    if m.robot_id != ag.getID():
                        ag.measurementWeightsCallback(m)
            o.refresh()
            o.update_weights()
    for a, ag in enumerate(agents):
        assert np.abs(ag.getX() - o.get_iterate(a)).max() < 1e-6
    anchor = agents[0].getX()[0]
    for ag in agents:
        ag.setGlobalAnchor(anchor)
        T = ag.getTrajectoryInGlobalFrame()
        ref = o.trajectory(ag.getID(), anchor)
        got = T.reshape(3, -1, 4).transpose(1, 0, 2)
        assert np.abs(got[:, :, :3].reshape(-1, 9) - ref[:, :9]).max() < 1e-6
        assert np.abs(got[:, :, 3] - ref[:, 9:]).max() < 1e-6
