"""The dpgo_ros command channel on the driver:
checkTimeout's decision (drawio:2417-2451), TERMINATE / HARD_TERMINATE /
RECOVER / SET_ACTIVE_ROBOTS / UPDATE / INITIALIZE applied to the solver state,
and the leader's decision broadcast to a gloo world of 2. CPU restatement as
the solver (tests/mock_solver.py). The ROS parameter defaults are [U]
(dpgo_ros is not vendored); the rule itself is the drawio's."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from kmx.dpgo.command import TimeoutMonitor, TimeoutParameters
from kmx.dpgo.messages import Command, CommandType, PGOAgentState
from kmx.synth import lift, lifting_matrix, make_pose_graph

S = PGOAgentState


def _setup(schedule=1):
    from kmx.dpgo.driver import RBCDDriver
    from kmx.dpgo.params import PGOAgentParameters
    from tests.mock_solver import OracleBlockSolver
    g = make_pose_graph(3, 300, 800, seed=6)
    P = PGOAgentParameters(r=5, schedule=schedule)
    P.robustOptInnerIters, P.robustOptNumWeightUpdates = 2, 4
    Y = lifting_matrix(5, seed=1)
    X0 = {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}
    drv = RBCDDriver(P, g, solver=OracleBlockSolver(P))
    drv.monitor = TimeoutMonitor(TimeoutParameters(timeoutThreshold=10.0), now=0.0)
    drv.initialize(X0)
    return drv, X0


def _iterates(drv):
    return [drv.iterate_of(a) for a in range(drv.graph.n_robots)]


def test_timeout_rule():
    m = TimeoutMonitor(TimeoutParameters(timeoutThreshold=10.0, enableRecovery=True), now=0.0)
    m.note_update(5.0)
    assert m.check(10.0, S.INITIALIZED, 7, 3) is None                  # quiet for exactly the threshold
    assert m.check(11.0, S.INITIALIZED, 7, 3) == CommandType.RECOVER
    assert m.check(11.0, S.INITIALIZED, 7, 0) == CommandType.HARD_TERMINATE        # 1) no active robot
    assert m.check(11.0, S.WAIT_FOR_INITIALIZATION, 7, 3) == CommandType.HARD_TERMINATE  # 3) not initialised
    assert m.check(11.0, S.INITIALIZED, 0, 3) == CommandType.HARD_TERMINATE        # 3) no iteration yet
    assert m.check(35.1, S.INITIALIZED, 7, 3) == CommandType.HARD_TERMINATE        # 4) no update for 3x thr
    assert m.check(35.0, S.INITIALIZED, 7, 3) == CommandType.RECOVER
    m.params.enableRecovery = False
    assert m.check(11.0, S.INITIALIZED, 7, 3) == CommandType.HARD_TERMINATE        # 2) recovery disabled
    m.note_command(20.0)
    assert m.check(29.0, S.INITIALIZED, 7, 3) is None


def test_terminate_then_recover():
    drv, _ = _setup()
    drv.run(max_rounds=4, check_every=2)
    X = _iterates(drv)
    drv.handle_command(Command(0, CommandType.TERMINATE), now=1.0)
    assert drv.terminated
    with pytest.raises(ValueError):
        drv.step()
    assert drv.run(max_rounds=5) == 0
    assert all(np.array_equal(a, b) for a, b in zip(X, _iterates(drv)))     # the final iterate stays readable
    drv.handle_command(Command(0, CommandType.RECOVER, executing_iteration=2, active_robots=[0, 2]), now=2.0)
    assert not drv.terminated and drv.round_index == 2 and drv.active_robots == {0, 2}
    drv.step()
    assert drv.round_index == 3
    Y = _iterates(drv)
    assert np.array_equal(Y[1], X[1]) and not np.array_equal(Y[0], X[0])


def test_hard_terminate_resets_to_a_fresh_run():
    """HARD_TERMINATE then INITIALIZE: the next rounds equal a fresh driver's
    bit for bit (weights, mu, GNC counters and status restored)."""
    drv, _ = _setup()
    drv.run(max_rounds=8, check_every=4)
    assert drv.weight_updates >= 2
    drv.handle_command(Command(0, CommandType.HARD_TERMINATE), now=1.0)
    assert drv.state == S.WAIT_FOR_INITIALIZATION and drv.instance == 1 and drv.round_index == 0
    assert drv.weight_updates == 0 and np.all(np.isinf(drv.solver.status()))
    with pytest.raises(ValueError):
        drv.step()
    drv.handle_command(Command(0, CommandType.INITIALIZE), now=2.0)
    assert drv.state == S.INITIALIZED
    drv.run(max_rounds=8, check_every=4)
    fresh, _ = _setup()
    fresh.run(max_rounds=8, check_every=4)
    assert drv.weight_updates == fresh.weight_updates
    assert np.array_equal(drv.solver.get_weights(), fresh.solver.get_weights())
    assert all(np.array_equal(a, b) for a, b in zip(_iterates(drv), _iterates(fresh)))


def test_active_robots_and_update():
    drv, _ = _setup()
    drv.handle_command(Command(0, CommandType.SET_ACTIVE_ROBOTS, active_robots=[0, 2]), now=1.0)
    X = _iterates(drv)
    drv.run(max_rounds=3)
    Y = _iterates(drv)
    assert np.array_equal(Y[1], X[1]) and not np.array_equal(Y[0], X[0]) and not np.array_equal(Y[2], X[2])
    with pytest.raises(ValueError):
        drv.handle_command(Command(0, CommandType.UPDATE, executing_robot=1))
    with pytest.raises(ValueError):
        drv.handle_command(Command(0, CommandType.SET_ACTIVE_ROBOTS, active_robots=[5]))
    drv.handle_command(Command(0, CommandType.SET_ACTIVE_ROBOTS, active_robots=[0, 1, 2]), now=2.0)
    st = drv.handle_command(Command(0, CommandType.UPDATE, executing_robot=1), now=3.0)
    Z = _iterates(drv)
    assert [bool(s["updated"]) for s in st] == [False, True, False]
    assert np.array_equal(Z[0], Y[0]) and np.array_equal(Z[2], Y[2]) and not np.array_equal(Z[1], Y[1])
    assert drv.active_robots == {0, 1, 2} and drv.monitor.last_update == 3.0
    n = drv.weight_updates
    drv.handle_command(Command(0, CommandType.UPDATE_WEIGHT), now=4.0)
    assert drv.weight_updates == n + 1


def test_check_timeout_on_the_driver():
    drv, _ = _setup()
    assert drv.check_timeout(now=5.0) is None
    assert drv.check_timeout(now=11.0).command == CommandType.HARD_TERMINATE  # no round ran yet
    assert drv.state == S.WAIT_FOR_INITIALIZATION
    drv.handle_command(Command(0, CommandType.INITIALIZE), now=12.0)
    for k in range(3):
        drv.handle_command(Command(0, CommandType.UPDATE), now=13.0 + k)
    c = drv.check_timeout(now=26.0)
    assert c.command == CommandType.RECOVER and c.executing_iteration == 3
    assert drv.state == S.INITIALIZED and drv.round_index == 3 and drv.monitor.last_command == 26.0
    assert drv.check_timeout(now=70.0).command == CommandType.HARD_TERMINATE  # no update for > 3x threshold


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    from kmx.dpgo.params import PGOAgentParameters
    from tests.mock_solver import OracleBlockSolver
    g = make_pose_graph(4, 400, 1000, seed=2)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5, seed=1)
    drv = RBCDDriver(P, g, rank=rank, world=world, solver=OracleBlockSolver(P), exchange_device="cpu")
    drv.monitor = TimeoutMonitor(TimeoutParameters(timeoutThreshold=10.0), now=0.0)
    drv.initialize({a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)})
    drv.step()
    drv.monitor.note_update(1.0)
    # only the leader's clock has run out; rank 1's would say "no timeout"
    c = drv.check_timeout(now=12.0 if rank == 0 else 3.0)
    q.put((rank, None if c is None else int(c.command), drv.round_index, drv.state == PGOAgentState.INITIALIZED))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_leader_timeout_decision():
    from tests.test_distributed_cpu import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in procs:
            rank, c, it, init = q.get(timeout=100)
            got[rank] = (c, it, init)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert got[0] == got[1] == (int(CommandType.RECOVER), 1, True)


def test_team_tile_incidences_rule():
    """The cut the multi-rank driver hands every rank (csrc/pgo.hip set_graph's
    automatic rule for 1/world of the team's incidences): about 736 tiles,
    between 180 incidences and two 240-incidence chunks (r = 5)."""
    from kmx.dpgo.driver import team_tile_incidences
    from kmx.synth import make_pose_graph
    g = make_pose_graph(8, 100_000, 500_000, seed=0)  # 1M incidences
    assert team_tile_incidences(g, 1, 5) == 480       # capped at two chunks
    assert team_tile_incidences(g, 2, 5) == 480
    assert team_tile_incidences(g, 4, 5) == 340       # ceil(250000 / 736)
    assert team_tile_incidences(g, 8, 5) == 180       # not below 180
    assert team_tile_incidences(g, 1, 3) == 2 * 4 * 21 * 3  # r = 3: tiles of 84 poses
