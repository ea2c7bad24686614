"""world_size-2/3 gloo runs of the multi-process RBCD driver (one public-pose
all-to-all per round carrying the status words; GNC decided per round from
the schedule and the team status; shared loop closures re-weighted on both
ranks) on the CPU restatement: the distributed iterates must equal the
single-process team run bit for bit. Plus the host-side consistency of the
sparse exchange plan."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kmx.synth import lift, lifting_matrix, make_pose_graph


def _graph(big=False):
    if big:  # configs[3] shape: 8 robot blocks, 100k poses, 500k edges (20 % outliers)
        return make_pose_graph(8, 100_000, 500_000, seed=0)
    return make_pose_graph(4, 400, 1000, seed=2)


def _params(rel_tol=1e-3, accel=False):
    from kmx.dpgo.params import PGOAgentParameters
    P = PGOAgentParameters(r=5, acceleration=accel, restartInterval=4)
    P.robustOptInnerIters = 3
    P.robustOptNumWeightUpdates = 3
    P.relChangeTol = rel_tol
    return P


def _x0(g):
    Y = lifting_matrix(5, seed=1)
    return {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}


def _worker(rank, world, port, rounds, q, rel_tol, accel=False, big=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    from tests.mock_solver import OracleBlockSolver
    g, P = _graph(big), _params(rel_tol, accel)
    drv = RBCDDriver(P, g, rank=rank, world=world, solver=OracleBlockSolver(P), exchange_device="cpu")
    drv.initialize(_x0(g))
    for _ in range(rounds):
        drv.step(with_stats=True)
    q.put((rank, {a: drv.iterate_of(a) for a in drv.robots}, drv.weight_updates, drv.exchange_rows))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def reference_rounds(g, P, rounds):
    """Single-process team run with the host mirror of the GNC schedule."""
    from kmx.dpgo.schedule import GncSchedule
    from oracle.oracle import OraclePGO
    o = OraclePGO(P.to_c(), g)
    for a, X in _x0(g).items():
        o.set_iterate(a, X)
    sched = GncSchedule.from_params(P)
    relc = np.full(g.n_robots, np.inf)
    for _ in range(rounds):
        o.accel_pre()  # accelerated rounds: Y first (the GNC decision and the exchange see Y)
        if sched.should_update(relc):
            o.refresh()
            o.update_weights()
            sched.updated()
        relc = np.array([x["rel_change"] for x in o.iterate()])
        sched.round_done()
    return o, sched


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,rel_tol,accel", [(2, 1e-3, False), (3, 1e-3, False), (2, 30.0, False),
                                                (2, 1e-3, True)])
def test_gloo_ranks_match_single_process(world, rel_tol, accel):
    from oracle.oracle import OraclePGO
    rounds = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rounds, q, rel_tol, accel), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    wu = []
    try:
        for _ in procs:
            rank, X, w, _ = q.get(timeout=240)
            got.update(X)
            wu.append(w)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    # single-process reference: same rounds, same GNC schedule
    g, P = _graph(), _params(rel_tol, accel)
    o, sched = reference_rounds(g, P, rounds)
    assert sched.updates >= 2
    assert wu == [sched.updates] * world
    for a in range(g.n_robots):
        assert np.array_equal(got[a], o.get_iterate(a)), a


@pytest.mark.timeout(600)
def test_gloo_ws2_configs3_shape():
    """world_size 2 on the configs[3]-shaped graph (8 blocks, 100k poses, 500k
    edges, 4 blocks per rank, ~34k public rows each way per round) across a
    GNC weight update: bitwise equal to the single-process team run."""
    rounds, world = 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rounds, q, 1e-3, False, True), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    got, wu, rows = {}, [], []
    try:
        for _ in procs:
            rank, X, w, xr = q.get(timeout=500)
            got.update(X)
            wu.append(w)
            rows.append(xr)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    g, P = _graph(True), _params(1e-3)
    o, sched = reference_rounds(g, P, rounds)
    assert sched.updates >= 1 and wu == [sched.updates] * world
    assert all(20_000 < a < 60_000 and 20_000 < b < 60_000 for a, b in rows)
    for a in range(g.n_robots):
        assert np.array_equal(got[a], o.get_iterate(a)), a


@pytest.mark.parametrize("world", [2, 3, 4])
def test_exchange_plan_consistent(world):
    """Every rank receives exactly the foreign public poses its shared loop
    closures reference, in the order its peers send them."""
    from kmx.dpgo.driver import exchange_plan, robot_ranges
    g = make_pose_graph(6, 1200, 4000, seed=5)
    plans = [exchange_plan(g, world, k) for k in range(world)]
    sh = g.r1 != g.r2
    keys = np.unique(np.concatenate([(g.r1[sh].astype(np.int64) << 32) | g.p1[sh],
                                     (g.r2[sh].astype(np.int64) << 32) | g.p2[sh]]))
    rank_of = np.empty(g.n_robots, np.int64)
    for k, (lo, hi) in enumerate(robot_ranges(g.n_robots, world)):
        rank_of[lo:hi] = k
    for q in range(world):
        send_q, sc_q, recv_q, rc_q = plans[q]
        assert int(sc_q.sum()) == send_q.shape[0] and int(rc_q.sum()) == recv_q.shape[0]
        # what q must receive: the foreign endpoints of its shared loop closures
        need = set()
        for e in np.nonzero(sh)[0]:
            a, b = rank_of[g.r1[e]], rank_of[g.r2[e]]
            if a == b:
                continue
            if a == q:
                need.add(int(np.searchsorted(keys, (int(g.r2[e]) << 32) | int(g.p2[e]))))
            if b == q:
                need.add(int(np.searchsorted(keys, (int(g.r1[e]) << 32) | int(g.p1[e]))))
        assert sorted(need) == recv_q.tolist()
        off_r = np.concatenate([[0], np.cumsum(rc_q)])
        for k in range(world):
            send_k, sc_k, _, _ = plans[k]
            off_s = np.concatenate([[0], np.cumsum(sc_k)])
            seg_sent = send_k[off_s[q]:off_s[q + 1]]
            seg_recv = recv_q[off_r[k]:off_r[k + 1]]
            assert np.array_equal(seg_sent, seg_recv), (k, q)
            assert np.all(rank_of[keys[seg_sent] >> 32] == k)


def _native_worker(rank, world, port, rounds, q, fail_rank=-1, corrupt_rank=-1, raise_rank=-1, store=None,
                   destroy_raises=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if store:
        os.environ.update(KMX_MOCK_STORE=store, KMX_XCHG_TIMEOUT="5")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kmx.dpgo.driver import RBCDDriver
    from tests.mock_solver import NativeOracleBlockSolver
    g, P = _graph(False), _params(1e-3, False)
    s = NativeOracleBlockSolver(P)
    if rank == fail_rank:  # this rank's communicator cannot be created
        def fail(*a, **k):
            raise RuntimeError("no RCCL")
        s.comm_init = fail
    s.corrupt = rank == corrupt_rank  # this rank's transport delivers a wrong bit
    s.raise_in_exchange = rank == raise_rank  # this rank's first exchange raises after its peers posted
    s.raise_in_destroy = destroy_raises and rank == raise_rank  # and then its abort raises too
    drv = RBCDDriver(P, g, rank=rank, world=world, solver=s, exchange_device="cuda")
    drv.initialize(_x0(g))
    drv.step(with_stats=True)          # one exchange (the round's own)
    drv.run_async(rounds - 2)          # one solver call for all its rounds
    drv.step(with_stats=True)
    q.put((rank, {a: drv.iterate_of(a) for a in drv.robots}, drv.weight_updates, drv.native,
           getattr(s, "comm_inits", 0), getattr(s, "exchanges", 0), getattr(s, "async_calls", 0),
           drv.exchange_mode, getattr(s, "comm_destroys", 0)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_native_exchange_branch_matches_single_process():
    """RBCDDriver's native branch (the exchange inside the solver's rounds, the
    RCCL path of a GPU team; here the mock solver runs it over gloo): the unique
    id reaches every rank, each round exchanges exactly once (no extra exchange
    from step(), run_async is one solver call), and the iterates equal the
    single-process team run bit for bit."""
    world, rounds = 2, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_native_worker, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    g, P = _graph(False), _params(1e-3, False)
    o, sched = reference_rounds(g, P, rounds)
    for rank, X, wu, native, inits, exchanges, async_calls, mode, destroys in res:
        assert native and inits == 1 and destroys == 0
        assert exchanges == rounds + 1 and async_calls == 1  # + the first round's start-up check
        assert "checked bitwise" in mode
        assert wu == sched.updates
        for a, Xa in X.items():
            assert np.array_equal(Xa, o.get_iterate(a)), (rank, a)


@pytest.mark.timeout(300)
def test_native_exchange_falls_back_together():
    """One rank cannot create its communicator: every rank agrees (MIN
    all-reduce) to use the torch.distributed exchange, and the team still
    matches the single-process run bit for bit."""
    world, rounds = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_native_worker, args=(r, world, port, rounds, q, 1)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    g, P = _graph(False), _params(1e-3, False)
    o, _ = reference_rounds(g, P, rounds)
    for rank, X, wu, native, inits, exchanges, async_calls, mode, destroys in res:
        assert not native and exchanges == 0
        assert "fallback" in mode and destroys == (1 if rank == 0 else 0)
        for a, Xa in X.items():
            assert np.array_equal(Xa, o.get_iterate(a)), (rank, a)


@pytest.mark.timeout(300)
def test_native_exchange_checked_at_first_round():
    """One rank's in-round transport delivers a wrong bit: the first round's
    check (native exchange vs the torch.distributed all_to_all, public table
    and status words compared bitwise) fails there, every rank drops the
    native exchange together, and the team still matches the single-process
    run bit for bit."""
    world, rounds = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_native_worker, args=(r, world, port, rounds, q, -1, 1)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    g, P = _graph(False), _params(1e-3, False)
    o, _ = reference_rounds(g, P, rounds)
    for rank, X, wu, native, inits, exchanges, async_calls, mode, destroys in res:
        assert not native and inits == 1 and destroys == 1 and exchanges == 1
        assert "differed" in mode
        for a, Xa in X.items():
            assert np.array_equal(Xa, o.get_iterate(a)), (rank, a)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("destroy_raises", [False, True], ids=["abort_ok", "abort_raises"])
def test_native_exchange_raise_after_peers_posted(tmp_path, destroy_raises):
    """one rank's first native exchange raises after its
    peer has posted its half (a posted, asynchronous transport as ncclSend /
    ncclRecv on the stream). The peer's wait is bounded (sync_timeout,
    KMX_XCHG_TIMEOUT), both ranks reach the agreement, drop the native
    exchange together, exchange_mode reports the exception (not a bitwise
    mismatch), and the team still matches the single-process run bit for
    bit."""
    world, rounds = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    store = str(tmp_path / "xchg_store")
    ps = [ctx.Process(target=_native_worker, args=(r, world, port, rounds, q, -1, -1, 1, store, destroy_raises))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    g, P = _graph(False), _params(1e-3, False)
    o, _ = reference_rounds(g, P, rounds)
    for rank, X, wu, native, inits, exchanges, async_calls, mode, destroys in res:
        assert not native and inits == 1 and destroys == 1
        assert "failed" in mode and "rank 1" in mode and "injected" in mode and "differed" not in mode
        # an abort that raises is reported, and the peers still agree
        assert ("comm_destroy on rank 1" in mode) == destroy_raises
        assert exchanges == (1 if rank == 0 else 0)  # rank 0 posted; rank 1 raised first
        for a, Xa in X.items():
            assert np.array_equal(Xa, o.get_iterate(a)), (rank, a)
