"""world_size-2 gloo run of the multi-process RBCD driver (public-pose
all-gather + owner -> peer GNC weight all-reduce) on the CPU restatement:
the distributed iterates must equal the single-process team run bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kmx.synth import lift, lifting_matrix, make_pose_graph


def _graph():
    return make_pose_graph(4, 400, 1000, seed=2)


def _params():
    from kmx.dpgo.params import PGOAgentParameters
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 3
    return P


def _x0(g):
    Y = lifting_matrix(5, seed=1)
    return {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}


def _worker(rank, world, port, rounds, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    from tests.mock_solver import OracleBlockSolver
    g, P = _graph(), _params()
    drv = RBCDDriver(P, g, rank=rank, world=world, solver=OracleBlockSolver(P), exchange_device="cpu")
    drv.initialize(_x0(g))
    for _ in range(rounds):
        drv.step(with_stats=True)
    q.put((rank, {a: drv.iterate_of(a) for a in drv.robots}, drv.weight_updates))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process():
    from oracle.oracle import OraclePGO
    rounds = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, rounds, q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    wu = []
    try:
        for _ in procs:
            rank, X, w = q.get(timeout=240)
            got.update(X)
            wu.append(w)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    # single-process reference: same rounds, same GNC schedule
    g, P = _graph(), _params()
    o = OraclePGO(P.to_c(), g)
    for a, X in _x0(g).items():
        o.set_iterate(a, X)
    for k in range(1, rounds + 1):
        o.iterate()
        if k % P.robustOptInnerIters == 0:
            o.refresh()
            o.update_weights()
    assert wu == [rounds // P.robustOptInnerIters] * 2
    for a in range(g.n_robots):
        assert np.array_equal(got[a], o.get_iterate(a)), a
