"""Two ranks on one MI355X (gloo exchange staged through host copies) running
the real HIP solver: the distributed RBCD iterates and GNC weights must equal
the single-process GPU run bit for bit (per-robot reductions are ordered the
same whatever the rank placement; the GNC schedule is decided on each rank's
device from the statuses carried by the exchange)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kmx.synth import lift, lifting_matrix, make_pose_graph

pytestmark = pytest.mark.gpu


def _graph():
    return make_pose_graph(4, 2000, 5000, seed=3)


def _params(rel_tol=1e-3, form="standard"):
    from kmx.dpgo.params import PGOAgentParameters
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 4
    P.relChangeTol = rel_tol
    P.schedule = 1
    P.localOptimizationParams.tCG_form = form
    return P


def _x0(g):
    Y = lifting_matrix(5, seed=1)
    return {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}


def _run(drv, rounds):
    for _ in range(rounds):
        drv.step(with_stats=True)
    drv.solver.sync()
    return {a: drv.iterate_of(a) for a in drv.robots}, drv.solver.get_weights()


def _worker(rank, world, port, rounds, q, rel_tol, form="standard"):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    g, P = _graph(), _params(rel_tol, form)
    drv = RBCDDriver(P, g, rank=rank, world=world, device=0, exchange_device="cpu")
    drv.initialize(_x0(g))
    X, w = _run(drv, rounds)
    q.put((rank, X, w, list(drv.robots)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("rel_tol,form", [(1e-3, "standard"), (30.0, "standard"), (1e-3, "onesync")])
def test_two_ranks_one_gpu_match_single_process(gpu, rel_tol, form):
    """(onesync: the opt-in one-sync tCG keeps the same placement independence:
    its 8-wide robot sums are ordered like the standard form's.)"""
    from kmx.dpgo.driver import RBCDDriver
    rounds = 11
    g, P = _graph(), _params(rel_tol, form)
    drv = RBCDDriver(P, g, device=0)
    drv.initialize(_x0(g))
    X1, w1 = _run(drv, rounds)
    assert drv.weight_updates >= 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, rounds, q, rel_tol, form), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in procs:  # drain the queue before asserting, so workers can exit
            results.append(q.get(timeout=420))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    got = {}
    for rank, X, w, robots in results:
        got.update(X)
        sel = np.isin(g.r1, robots) | np.isin(g.r2, robots)  # edges this rank's blocks see
        assert np.array_equal(w[sel], w1[sel]), rank
    for a in range(g.n_robots):
        assert np.array_equal(got[a], X1[a]), a


@pytest.mark.timeout(300)
def test_commands_on_device(gpu):
    """HARD_TERMINATE resets the device state (weights, mu, GNC counters,
    status) so that INITIALIZE + the same rounds reproduce a fresh handle bit
    for bit; SET_ACTIVE_ROBOTS freezes the inactive blocks on the device."""
    from kmx.dpgo.driver import RBCDDriver
    from kmx.dpgo.messages import Command, CommandType
    g, P = _graph(), _params()
    drv = RBCDDriver(P, g, device=0)
    drv.initialize(_x0(g))
    drv.run(max_rounds=12, check_every=6)
    assert drv.weight_updates >= 2
    drv.handle_command(Command(0, CommandType.HARD_TERMINATE))
    assert drv.weight_updates == 0 and np.all(np.isinf(drv.solver.status()))
    drv.handle_command(Command(0, CommandType.INITIALIZE))
    X1, w1 = _run(drv, 12)
    fresh = RBCDDriver(P, g, device=0)
    fresh.initialize(_x0(g))
    X2, w2 = _run(fresh, 12)
    assert drv.weight_updates == fresh.weight_updates >= 2
    assert np.array_equal(w1, w2)
    for a in range(g.n_robots):
        assert np.array_equal(X1[a], X2[a]), a
    drv.handle_command(Command(0, CommandType.SET_ACTIVE_ROBOTS, active_robots=[1, 3]))
    drv.run(max_rounds=4)
    drv.solver.sync()
    for a in range(g.n_robots):
        same = np.array_equal(drv.iterate_of(a), X1[a])
        assert same == (a in (0, 2)), a


@pytest.mark.timeout(300)
def test_tile_cut_rule_matches_handle(gpu):
    """The driver's team_tile_incidences (what every rank of a multi-rank team
    is given) reproduces the cut kmx_pgo_set_graph picks on its own for the
    whole team: passing it explicitly leaves a single-handle run bit for bit
    unchanged (25k poses, 250k incidences: a cut above the 180 floor)."""
    import dataclasses
    from kmx.dpgo.driver import RBCDDriver, team_tile_incidences
    g = make_pose_graph(2, 25_000, 125_000, seed=7)
    P = _params()
    cap = team_tile_incidences(g, 1, P.r)
    assert 180 < cap < 480
    out = []
    for Pk in (P, dataclasses.replace(P, tileIncidences=cap)):
        drv = RBCDDriver(Pk, g, device=0)
        drv.initialize(_x0(g))
        out.append(_run(drv, 6))
        drv.solver.close()
    for a in range(g.n_robots):
        assert np.array_equal(out[0][0][a], out[1][0][a]), a


@pytest.mark.parametrize("self_p2p", ["0", "1"])
def test_native_exchange_world1_matches_plain_rounds(gpu, monkeypatch, self_p2p):
    """The RCCL exchange inside the round (kmx_pgo_comm_init / set_exchange) on a
    world-1 communicator: the own segment (this handle's status word) is copied,
    or with KMX_XCHG_SELF_P2P=1 sent to itself by ncclSend / ncclRecv. Rounds,
    an explicit exchange and a GNC update give the same iterates bit for bit as
    the handle without a communicator (the multi-peer path is the same group with
    more peers; the 8-GPU run is the driver's)."""
    import numpy as np
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.dpgo.solver import BlockSolver
    from kmx.synth import lift, lifting_matrix, make_pose_graph
    monkeypatch.setenv("KMX_XCHG_SELF_P2P", self_p2p)
    g = make_pose_graph(2, 400, 1200, seed=2)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5, seed=1)
    out = []
    for native in (False, True):
        s = BlockSolver(P, 0)
        s.set_graph_data(g)
        s.set_gnc_schedule(True, 3, 50, P.relChangeTol)
        if native:
            s.comm_init(BlockSolver.comm_unique_id(), 1, 0)
            s.set_exchange(np.zeros(0, np.int32), [0], np.zeros(0, np.int32), [0])
        for a in range(g.n_robots):
            s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
        s.iterate_async(5, refresh_local=True)
        if native:
            s.exchange()
        s.update_weights()
        s.iterate_async(4, refresh_local=False)
        s.sync()
        out.append([s.get_iterate(a) for a in range(g.n_robots)] + [s.get_weights()])
        s.close()
    for a, b in zip(*out):
        assert np.array_equal(a, b)


def test_native_exchange_checks(gpu):
    import numpy as np
    from kmx import abi
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.dpgo.solver import BlockSolver
    from kmx.synth import make_pose_graph
    g = make_pose_graph(2, 50, 120, seed=1)
    s = BlockSolver(PGOAgentParameters(r=5), 0)
    s.set_graph_data(g)
    with pytest.raises(abi.KmxError):  # before comm_init
        s.set_exchange(np.zeros(0, np.int32), [0], np.zeros(0, np.int32), [0])
    with pytest.raises(abi.KmxError):
        s.exchange()
    s.comm_init(BlockSolver.comm_unique_id(), 1, 0)
    with pytest.raises(abi.KmxError):  # own segment counts differ
        s.set_exchange(np.zeros(1, np.int32), [1], np.zeros(0, np.int32), [0])
    with pytest.raises(abi.KmxError):  # slot out of range
        s.set_exchange(np.array([10**6], np.int32), [1], np.array([0], np.int32), [1])
    s.close()
