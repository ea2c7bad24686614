"""The opt-in one-sync tCG (kmx_pgo_params.tcg_form = KMX_TCG_FORM_ONESYNC,
VERDICT r3 next-round item 2): one k_step launch per tCG step, every scalar
of the next step from one reduction (pgo.hip body_step), restated by
oracle/dpgo_oracle.c tcg_onesync.

Bars:
  * against the restatement's same form, per round: equal tCG iteration
    counts and acceptance, every lifted pose within 1e-6 (the standard form's
    bar), on the round structures the standard form is tested on (tCG capped
    at 1 / 3 steps, two RTR iterations, 25-step tCG with direction folds,
    ranks 3 and 8, full records, a 12.5k-pose block whose 8-wide robot sums
    take the looped path);
  * polled, blind and adaptive enqueueing agree bit for bit;
  * SURVEY.md §8e "at convergence": configs[1] run to relChangeTol across its
    GNC updates, every round compared with the restatement's same form,
    rounded trajectories within 1e-6, and rounds to converge within 10 % of
    the standard (ROPTLIB) form's.
"""
import numpy as np
import pytest

from kmx.dpgo.params import PGOAgentParameters
from kmx.dpgo.schedule import GncSchedule
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix
from tests.test_dpgo_gpu import _full_records, _pair, _setup

pytestmark = pytest.mark.gpu


def _onesync(P):
    P.localOptimizationParams.tCG_form = "onesync"
    return P


def _rounds(s, o, g, P, n, robust=True):
    for it in range(n):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            assert sg[a]["tcg_stop"] == so[a]["tcg_stop"], (it, a, sg[a], so[a])
            assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
        if robust and it % 4 == 3:
            s.refresh_local()
            assert s.update_weights() == o.update_weights()
            assert np.abs(s.get_weights() - o.get_weights()).max() <= 1e-9


@pytest.mark.parametrize("case", ["default", "tcg1", "tcg3", "rtr2", "r3", "r8", "full", "l2"])
def test_onesync_rounds_match_oracle(gpu, case):
    r = 3 if case == "r3" else 8 if case == "r8" else 5
    g, P, X0 = _setup(r=r, robust=case != "l2", seed=3)
    if case == "full":
        _full_records(g)
    lo = _onesync(P).localOptimizationParams
    if case == "tcg1":
        lo.RTR_tCG_iterations = 1
    elif case == "tcg3":
        lo.RTR_tCG_iterations = 3
    elif case == "rtr2":
        lo.RTR_iterations = 2
    s, o = _pair(g, P, X0)
    try:
        _rounds(s, o, g, P, 10, robust=case != "l2")
        # the asynchronous form (every round from one host call)
        s.iterate_async(3, refresh_local=True)
        s.sync()
        for _ in range(3):
            o.refresh()
            o.iterate()
        for a in range(g.n_robots):
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (a, d)
    finally:
        s.close()


def test_onesync_long_tcg_folds_directions(gpu):
    """25-step tCG on the residual test: k_step folds the two kept directions
    into eta at every second step, the newest with its own launch's
    coefficient, and k_retract adds the rest."""
    g, P, X0 = _setup(robust=False, seed=4, perturb=0.01, outlier=0.0)
    lo = _onesync(P).localOptimizationParams
    lo.RTR_tCG_iterations = 25
    lo.tCG_kappa = 1e-8
    lo.RTR_initial_radius, lo.RTR_max_radius = 1e4, 1e6
    s, o = _pair(g, P, X0)
    longest = 0
    try:
        for it in range(8):
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate()
            for a in range(g.n_robots):
                assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
                longest = max(longest, sg[a]["tcg_iterations"])
                d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
                assert d <= 1e-6, (it, a, d)
        assert longest > 10, longest
    finally:
        s.close()


@pytest.mark.parametrize("tile_incidences", [0, 60])
def test_onesync_large_robot_block(gpu, tile_incidences):
    """One 12.5k-pose block: ~700 tiles with the automatic cut (one pass of
    RobotSum8, four tiles per thread), ~2,100 with 60 incidences per tile (more
    than the 1,024 one pass holds: the looped path)."""
    g, P, X0 = _setup(n_robots=1, n=12_500, m=62_500, seed=5)
    _onesync(P)
    P.tileIncidences = tile_incidences
    s, o = _pair(g, P, X0)
    try:
        for it in range(4):
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate()
            assert sg[0]["tcg_iterations"] == so[0]["tcg_iterations"], (it, sg[0], so[0])
            d = np.linalg.norm((s.get_iterate(0) - o.get_iterate(0)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, d)
    finally:
        s.close()


@pytest.mark.parametrize("tile_incidences", [24, 40])
def test_onesync_partials_double_buffered(gpu, tile_incidences):
    """a k_step launch reads step k's 8-wide partials of
    every tile of its robot while each tile writes step k + 1's; with the
    partials in one buffer, a tile dispatched after a same-robot tile finished
    read the new partial. Cut so fine that a robot's tiles span several
    generations of resident workgroups (~3,000-5,000 tiles for one 12.5k-pose
    block, against 768 resident at 3 per CU), every round must still match the
    restatement's one-sync form: the same tCG count and stop reason, and every
    lifted pose within 1e-9 (the per-round drift of a correct run is ~1e-12; a
    torn robot sum changes alpha / beta in some tiles only)."""
    g, P, X0 = _setup(n_robots=1, n=12_500, m=62_500, seed=7)
    _onesync(P)
    P.tileIncidences = tile_incidences
    s, o = _pair(g, P, X0)
    try:
        for it in range(5):
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate()
            assert sg[0]["tcg_iterations"] == so[0]["tcg_iterations"], (it, sg[0], so[0])
            assert sg[0]["tcg_stop"] == so[0]["tcg_stop"], (it, sg[0], so[0])
            assert sg[0]["accepted"] == so[0]["accepted"], it
            d = np.linalg.norm((s.get_iterate(0) - o.get_iterate(0)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-9, (it, d)
    finally:
        s.close()


@pytest.mark.parametrize("robust", [False, True])
def test_onesync_accelerated_rounds_match_oracle(gpu, robust):
    """Nesterov-accelerated RBCD with the one-sync tCG: the extrapolated point
    the round starts from and the momentum update around it are the standard
    form's; the rounds match the restatement's same form across two restarts."""
    g, P, X0 = _setup(robust=robust)
    _onesync(P)
    P.acceleration, P.restartInterval = True, 5
    s, o = _pair(g, P, X0)
    try:
        for it in range(12):
            s.refresh_local()
            sg = s.iterate()
            so = o.iterate()
            for a in range(g.n_robots):
                assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
                d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
                assert d <= 1e-6, (it, a, d)
            if robust and it % 4 == 3:
                s.refresh_local()
                o.accel_pre()
                o.refresh()
                assert s.update_weights() == o.update_weights()
    finally:
        s.close()


def test_onesync_poll_modes_agree_bitwise(gpu):
    g, P, X0 = _setup(robust=True, seed=6)
    _onesync(P)
    out = []
    for mode in (1, 0, -1):
        s = BlockSolver(P, 0)
        s.set_tcg_poll(mode)
        s.set_graph_data(g)
        s.set_gnc_schedule(True, 3, 50, P.relChangeTol)
        for a in range(g.n_robots):
            s.set_iterate(a, X0[a])
        s.read_counters()
        s.iterate_async(14, refresh_local=True)
        s.sync()
        c = s.read_counters()
        out.append([s.get_iterate(a) for a in range(g.n_robots)] + [s.get_weights(), s.status(),
                   np.array([c["hessvecs"], c["edges_iters"], c["block_updates"], c["gnc_updates"]])])
        s.close()
    for other in out[1:]:
        for a, b in zip(out[0], other):
            assert np.array_equal(a, b)


def _converge(g, P, Y, oracle=True, cap=1500):
    """configs[1] rounds until the GNC schedule ran its updates and every
    robot's relative change is below relChangeTol; with the restatement of the
    same form compared at every round. Returns (rounds, solver, oracle)."""
    from oracle.oracle import OraclePGO
    from tests.test_parity_long_gpu import _rounds_both
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
    o = OraclePGO(P.to_c(), g) if oracle else None
    for a in range(g.n_robots):
        X0 = lift(g.init_R[a], g.init_t[a], Y)
        s.set_iterate(a, X0)
        if o:
            o.set_iterate(a, X0)
    sched = GncSchedule.from_params(P)
    relc = np.full(g.n_robots, np.inf)
    done = 0
    while done < cap:
        if o:
            relc, _ = _rounds_both(s, o, sched, relc, g, P, 1, done)
        else:
            s.refresh_local()
            s.iterate()
            relc = np.array(s.status(), dtype=np.float64)
            sched.updates = s.gnc_state()["updates"]
        done += 1
        if sched.updates >= P.robustOptNumWeightUpdates and relc.max() < P.relChangeTol:
            break
    return done, s, o


@pytest.mark.timeout(900)
def test_onesync_configs1_converged(gpu):
    g = config("campus6", seed=0)
    Y = lifting_matrix(5, seed=1)

    def params(form):
        P = PGOAgentParameters(r=5)
        P.robustOptInnerIters = 20
        P.robustOptNumWeightUpdates = 8
        P.relChangeTol = 1e-3
        P.localOptimizationParams.tCG_form = form
        return P

    n_std, s_std, _ = _converge(g, params("standard"), Y, oracle=False)
    s_std.close()
    P = params("onesync")
    n_os, s, o = _converge(g, P, Y)
    try:
        assert n_std < 1500 and n_os < 1500, (n_std, n_os)
        assert abs(n_os - n_std) <= 0.1 * n_std, (n_os, n_std)
        print(f"configs[1] rounds to converge: standard {n_std}, one-sync {n_os}")
        from tests.test_parity_long_gpu import _trajectories_agree
        _trajectories_agree(s, o, g, Y, P.r)
    finally:
        s.close()
