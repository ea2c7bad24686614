"""dpgo_ros scheduling rules on the host:
the executing-robot choice of the synchronous mode (round-robin and uniform,
drawio:2478-2481) pinned against this container's real libstdc++, and team
termination (shouldTerminate, drawio:2027-2030) through the driver, single
process and over gloo with the all_reduce(MAX) of the ranks' statuses."""
import json
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

from kmx.dpgo.schedule import MT19937, RNG_GCC11, ROUND_ROBIN, UNIFORM, ExecutingRobot, uniform_int

GOLD = Path(__file__).resolve().parent / "golden" / "mt19937_gcc11.json"


def test_uniform_small_ranges_match_libstdcxx():
    d = json.loads(GOLD.read_text())
    assert d["gcc_major"] >= 11 and d["small"]
    for key, draws in d["small"].items():
        seed, n = (int(x) for x in key.split(":"))
        gen = MT19937(seed)
        assert [uniform_int(gen, 0, n - 1, RNG_GCC11) for _ in draws] == draws, key


def test_executing_robot_rules():
    d = json.loads(GOLD.read_text())
    rr = ExecutingRobot(ROUND_ROBIN)
    assert [rr.next(range(4)) for _ in range(9)] == [0, 1, 2, 3, 0, 1, 2, 3, 0]
    rr2 = ExecutingRobot(ROUND_ROBIN)
    assert [rr2.next([1, 3, 6]) for _ in range(5)] == [1, 3, 6, 1, 3]
    un = ExecutingRobot(UNIFORM, seed=7, variant=RNG_GCC11)
    act = [2, 4, 5, 9, 11, 12]
    assert [un.next(act) for _ in range(200)] == [act[i] for i in d["small"]["7:6"]]
    with pytest.raises(ValueError):
        ExecutingRobot(5)


def _problem():
    from kmx.dpgo.params import PGOAgentParameters, RobustCostType
    from kmx.synth import lift, lifting_matrix, make_pose_graph
    g = make_pose_graph(4, 400, 1000, seed=2)
    P = PGOAgentParameters(r=5)
    P.robustCostParams.costType = RobustCostType.L2
    Y = lifting_matrix(5, seed=1)
    return g, P, {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}


def _team_max(rounds):
    """Largest relative change of the team after each round (single process)."""
    from oracle.oracle import OraclePGO
    g, P, X0 = _problem()
    o = OraclePGO(P.to_c(), g)
    for a, X in X0.items():
        o.set_iterate(a, X)
    return np.array([max(s["rel_change"] for s in o.iterate()) for _ in range(rounds)])


def test_driver_terminates_single_process():
    from kmx.dpgo.driver import RBCDDriver
    from tests.mock_solver import OracleBlockSolver
    tm = _team_max(30)
    g, P, X0 = _problem()
    P.relChangeTol = float(tm[19]) * (1 + 1e-9)  # reached at the round-20 check at the latest
    expect = next(k for k in range(5, 31, 5) if tm[k - 1] < P.relChangeTol)
    drv = RBCDDriver(P, g, solver=OracleBlockSolver(P))
    drv.initialize(X0)
    assert drv.run(max_rounds=30, check_every=5) == expect
    P2 = _problem()[1]
    P2.maxNumIters = 7
    drv2 = RBCDDriver(P2, g, solver=OracleBlockSolver(P2))
    drv2.initialize(X0)
    assert drv2.run(check_every=5) == 7  # maxNumIters


def _worker(rank, world, port, tol, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    from tests.mock_solver import OracleBlockSolver
    g, P, X0 = _problem()
    P.relChangeTol = tol
    drv = RBCDDriver(P, g, rank=rank, world=world, solver=OracleBlockSolver(P), exchange_device="cpu")
    drv.initialize(X0)
    n = drv.run(max_rounds=30, check_every=5)
    q.put((rank, n, drv.team_max_rel_change()))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_team_termination_over_gloo():
    """Both ranks stop at the same check, the one where the team's largest
    relative change (all_reduce MAX of the ranks' statuses) first falls below
    relChangeTol, as in the single-process run."""
    tm = _team_max(30)
    tol = float(tm[14]) * (1 + 1e-9)
    expect = next(k for k in range(5, 31, 5) if tm[k - 1] < tol)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, tol, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in procs:
            rank, n, m = q.get(timeout=240)
            out[rank] = (n, m)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert out[0][0] == out[1][0] == expect
    assert out[0][1] == out[1][1] == tm[expect - 1]


def test_gnc_run_does_not_stop_before_gnc_is_done():
    """Robust cost: the team's relative change can fall below relChangeTol
    while GNC weight updates are still pending (that convergence is what fires
    the next update, drawio:2466-2469). run() keeps going until
    robustOptNumWeightUpdates updates ran, unless robustOptMinConvergenceRatio
    of the loop-closure weights already sit at 0 / 1."""
    from kmx.dpgo.driver import RBCDDriver
    from kmx.dpgo.params import RobustCostType
    from tests.mock_solver import OracleBlockSolver
    g, P, X0 = _problem()
    P.robustCostParams.costType = RobustCostType.GNC_TLS
    P.relChangeTol = 1e9              # every block update counts as converged
    P.robustOptInnerIters = 3
    P.robustOptNumWeightUpdates = 3
    P.robustOptMinConvergenceRatio = 1.01  # unreachable: only the update count ends GNC
    drv = RBCDDriver(P, g, solver=OracleBlockSolver(P))
    drv.initialize(X0)
    # round 1 (no status yet: no update), rounds 2-4 each fire ("all converged")
    assert drv.run(max_rounds=50, check_every=1) == 4
    assert drv.weight_updates == 3
    P.robustOptMinConvergenceRatio = 0.0  # GNC counts as done at once: the L2 rule
    drv2 = RBCDDriver(P, g, solver=OracleBlockSolver(P))
    drv2.initialize(X0)
    assert drv2.run(max_rounds=50, check_every=1) == 1
    assert 0.0 <= drv2.converged_weight_ratio() <= 1.0
