"""GPU parity: the HIP path (through the C ABI) vs the CPU restatement.

Tolerances (north_star: "optimized poses within 1e-6 Frobenius of reference"):
  * primitives (cost / egrad / Hess-vec / projections / retraction): the
    kernels accumulate every output element in the oracle's order with
    -ffp-contract=off, so they must agree to 1e-12 relative (bit-exact in
    practice; reductions differ only in summation order);
  * full RBCD rounds: per-pose Frobenius difference <= 1e-6 after every round.
"""
import numpy as np
import pytest

from kmx import abi
from kmx.dpgo.params import PGOAgentParameters, RobustCostType
from kmx.dpgo.solver import BlockSolver
from kmx.synth import lift, lifting_matrix, make_pose_graph
from kmx.synth.pose_graph import _expm_so3

pytestmark = pytest.mark.gpu


def _setup(n_robots=3, n=300, m=900, r=5, robust=True, seed=0, perturb=0.05, outlier=0.2):
    g = make_pose_graph(n_robots, n, m, outlier_frac=outlier, seed=seed)
    P = PGOAgentParameters(r=r)
    if not robust:
        P.robustCostParams.costType = RobustCostType.L2
    Y = lifting_matrix(r, seed=1)
    rng = np.random.default_rng(seed + 7)
    X0 = {}
    for a in range(g.n_robots):
        k = int(g.n_poses[a])
        Rp = g.init_R[a] @ _expm_so3(rng.normal(0, perturb, (k, 3)))
        X0[a] = lift(Rp, g.init_t[a] + rng.normal(0, 5 * perturb, (k, 3)), Y)
    return g, P, X0


def _pair(g, P, X0):
    from oracle.oracle import OraclePGO
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        s.set_iterate(a, X0[a])
        o.set_iterate(a, X0[a])
    s.refresh_local()
    o.refresh()
    return s, o


def _full_records(g):
    """Make one measurement rotation a non-rotation (1e-6 off SO(3)), so the
    handle stores the full 128-B records instead of the compact ones."""
    g.R[5] = g.R[5] + 1e-6 * np.random.default_rng(1).standard_normal((3, 3))
    return g


@pytest.mark.parametrize("r,records", [(3, "compact"), (5, "compact"), (8, "compact"), (5, "full")])
def test_primitives_match_oracle(gpu, r, records):
    g, P, X0 = _setup(r=r)
    if records == "full":
        _full_records(g)
    # non-trivial GNC weights so w*kappa paths are exercised
    g.weight = np.random.default_rng(3).uniform(0.0, 1.0, g.m)
    s, o = _pair(g, P, X0)
    rng = np.random.default_rng(11)
    for a in range(g.n_robots):
        V = rng.standard_normal(X0[a].shape)
        for mode in (abi.KMX_EVAL_COST_EGRAD, abi.KMX_EVAL_EHESS, abi.KMX_EVAL_RGRAD, abi.KMX_EVAL_RHESS,
                     abi.KMX_EVAL_PRECON, abi.KMX_EVAL_RETRACT):
            Vin = X0[a] if mode == abi.KMX_EVAL_COST_EGRAD else V
            if mode == abi.KMX_EVAL_RETRACT:
                Vin = 0.1 * V
            gout, gs = s.eval(a, mode, Vin)
            oout, os_ = o.eval(a, mode, Vin)
            scale = max(1.0, np.abs(oout).max())
            assert np.abs(gout - oout).max() <= 1e-12 * scale, (mode, np.abs(gout - oout).max())
            assert abs(gs - os_) <= 1e-10 * max(1.0, abs(os_)), (mode, gs, os_)


def _rot(axis, angle):
    return _expm_so3((np.asarray(axis, float) / np.linalg.norm(axis) * angle)[None])[0]


def test_compact_record_quaternion_cases(gpu):
    """The 68-B record stores three quaternion components and rebuilds the
    largest: measurement rotations whose largest component is each of w, x, y,
    z, of either sign before the flip, and ties (180 degrees about a diagonal:
    |x| = |y|), against the restatement's primitives to 1e-12."""
    g, P, X0 = _setup(robust=False)
    cases = [np.eye(3), _rot([1, 0, 0], np.pi), _rot([0, 1, 0], np.pi), _rot([0, 0, 1], np.pi),
             _rot([1, 1, 0], np.pi), _rot([1, 1, 1], np.pi), _rot([0, 1, 1], 2.0), _rot([1, 0, 0], 3.0),
             _rot([0, -1, 0], 3.1), _rot([0, 0, -1], 2.9), _rot([-1, 2, 0.5], -2.5), _rot([1, 1, 1], 2 * np.pi / 3)]
    for i, R in enumerate(cases * 4):
        g.R[7 * i + 3] = R
    s, o = _pair(g, P, X0)
    assert s.memory()[1] == 68
    rng = np.random.default_rng(2)
    for a in range(g.n_robots):
        V = rng.standard_normal(X0[a].shape)
        for mode in (abi.KMX_EVAL_COST_EGRAD, abi.KMX_EVAL_EHESS):
            Vin = X0[a] if mode == abi.KMX_EVAL_COST_EGRAD else V
            gout, gs = s.eval(a, mode, Vin)
            oout, os_ = o.eval(a, mode, Vin)
            assert np.abs(gout - oout).max() <= 1e-12 * max(1.0, np.abs(oout).max()), mode
    s.close()


@pytest.mark.parametrize("records", ["compact", "full"])
def test_zero_weights_keep_incidence_direction(gpu, records):
    """The compact record keeps the tail flag in w tau's sign bit (a zero weight
    is -0.0 on the tail's record): edges set to weight exactly 0 and back to 1
    through kmx_pgo_set_weights (k_apply_weights rewrites both records), with the
    Hessian, gradient and whole rounds against the restatement after each change."""
    g, P, X0 = _setup(robust=False)
    if records == "full":
        _full_records(g)
    s, o = _pair(g, P, X0)
    rng = np.random.default_rng(5)
    w = np.ones(g.m)
    w[rng.random(g.m) < 0.4] = 0.0  # tails and heads of private and shared edges alike
    for wv in (w, np.ones(g.m), w):
        s.set_weights(wv)
        o.set_weights(wv)
        s.refresh_local()
        o.refresh()
        for a in range(g.n_robots):
            V = rng.standard_normal(X0[a].shape)
            for mode in (abi.KMX_EVAL_COST_EGRAD, abi.KMX_EVAL_EHESS):
                Vin = s.get_iterate(a) if mode == abi.KMX_EVAL_COST_EGRAD else V
                gout, _ = s.eval(a, mode, Vin)
                oout, _ = o.eval(a, mode, Vin)
                assert np.abs(gout - oout).max() <= 1e-12 * max(1.0, np.abs(oout).max()), (records, mode)
        sg, so = s.iterate(), o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (a, sg[a], so[a])
            d = np.abs(s.get_iterate(a) - o.get_iterate(a)).max()
            assert d <= 1e-6, (a, d)
        assert np.array_equal(s.get_weights(), o.get_weights())
    s.close()


@pytest.mark.parametrize("robust,records", [(False, "compact"), (True, "compact"), (True, "full")])
def test_rounds_match_oracle(gpu, robust, records):
    """compact: 68-B records (SO(3) input, rotation rebuilt from its quaternion); full: the
    128-B records of a graph with a non-rotation measurement."""
    g, P, X0 = _setup(robust=robust)
    if records == "full":
        _full_records(g)
    s, o = _pair(g, P, X0)
    assert s.memory()[1] == (68 if records == "compact" else 128)
    for it in range(12):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            assert sg[a]["accepted"] == so[a]["accepted"]
            assert abs(sg[a]["f_init"] - so[a]["f_init"]) <= 1e-9 * max(1.0, abs(so[a]["f_init"]))
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
        if robust and it % 4 == 3:
            s.refresh_local()
            mu_g = s.update_weights()
            mu_o = o.update_weights()
            assert mu_g == mu_o
            wg, wo = s.get_weights(), o.get_weights()
            assert np.abs(wg - wo).max() <= 1e-9, np.abs(wg - wo).max()


@pytest.mark.parametrize("r", [3, 4, 8])
def test_rounds_match_oracle_rank(gpu, r):
    """The incidence-parallel kernels (and their LDS layouts: chunk of TP*r
    incidences, 64 // r poses per wave) at other relaxation ranks, GNC on."""
    g, P, X0 = _setup(r=r)
    s, o = _pair(g, P, X0)
    for it in range(8):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
        if it % 4 == 3:
            s.refresh_local()
            assert s.update_weights() == o.update_weights()


def test_sequential_schedule(gpu):
    g, P, X0 = _setup()
    s, o = _pair(g, P, X0)
    for it in range(6):
        act = np.zeros(g.n_robots, np.uint8)
        act[it % g.n_robots] = 1
        s.refresh_local()
        sg = s.iterate(act)
        so = o.iterate(act)
        for a in range(g.n_robots):
            assert sg[a]["updated"] == act[a] == so[a]["updated"]
            d = np.abs(s.get_iterate(a) - o.get_iterate(a)).max()
            assert d <= 1e-8, (it, a, d)


def test_trajectory_matches_oracle(gpu):
    g, P, X0 = _setup()
    s, o = _pair(g, P, X0)
    for _ in range(3):
        s.refresh_local()
        s.iterate()
        o.iterate()
    anchor = s.get_iterate(0)[0]
    for a in range(g.n_robots):
        tg, to = s.trajectory(a, anchor), o.trajectory(a, anchor)
        assert np.abs(tg - to).max() <= 1e-9
        Rg = tg[:, :9].reshape(-1, 3, 3)
        assert np.abs(np.einsum("nji,njk->nik", Rg, Rg) - np.eye(3)).max() < 1e-9
        assert np.all(np.linalg.det(Rg) > 0)


def test_async_rounds_equal_sync_rounds(gpu):
    """The benchmark path (no host sync, device-side control) computes the same
    iterates as the stats path."""
    g, P, X0 = _setup()
    s1 = BlockSolver(P, 0)
    s1.set_graph_data(g)
    s2 = BlockSolver(P, 0)
    s2.set_graph_data(g)
    for a in range(g.n_robots):
        s1.set_iterate(a, X0[a])
        s2.set_iterate(a, X0[a])
    for _ in range(5):
        s1.refresh_local()
        s1.iterate()
    s2.iterate_async(5, refresh_local=True)
    s2.sync()
    for a in range(g.n_robots):
        assert np.array_equal(s1.get_iterate(a), s2.get_iterate(a))
    c = s2.read_counters()
    assert c["block_updates"] == 5 * g.n_robots


def test_noise_free_converges_to_ground_truth(gpu):
    g = make_pose_graph(2, 200, 300, outlier_frac=0.0, noise_free=True, seed=0)
    P = PGOAgentParameters(r=5)
    P.robustCostParams.costType = RobustCostType.L2
    P.localOptimizationParams.RTR_tCG_iterations = 50
    Y = lifting_matrix(5)
    rng = np.random.default_rng(0)
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    for a in range(2):
        k = int(g.n_poses[a])
        Rp = g.init_R[a] @ _expm_so3(rng.normal(0, 0.1, (k, 3)))
        s.set_iterate(a, lift(Rp, g.init_t[a] + rng.normal(0, 0.5, (k, 3)), Y))
    s.iterate_async(200, refresh_local=True)
    s.sync()
    anchor = s.get_iterate(0)[0]
    R0, t0 = g.gt_R[0][0], g.gt_t[0][0]
    for a in range(2):
        T = s.trajectory(a, anchor)
        Rg = np.einsum("ji,njk->nik", R0, g.gt_R[a])
        tg = (g.gt_t[a] - t0) @ R0
        assert np.abs(T[:, 9:] - tg).max() < 1e-4
        assert np.abs(T[:, :9].reshape(-1, 3, 3) - Rg).max() < 1e-4


def test_non_rotation_measurement_uses_full_records(gpu):
    """A measurement whose rotation is not in SO(3) to 1e-12 must not go
    through the compact records (which rebuild row 2 = row0 x row1)."""
    g, P, X0 = _setup()
    _full_records(g)
    s, o = _pair(g, P, X0)
    assert s.memory()[1] == 128
    rng = np.random.default_rng(2)
    for a in range(g.n_robots):
        V = rng.standard_normal(X0[a].shape)
        for mode in (abi.KMX_EVAL_COST_EGRAD, abi.KMX_EVAL_EHESS):
            Vin = X0[a] if mode == abi.KMX_EVAL_COST_EGRAD else V
            gout, _ = s.eval(a, mode, Vin)
            oout, _ = o.eval(a, mode, Vin)
            assert np.abs(gout - oout).max() <= 1e-12 * max(1.0, np.abs(oout).max()), mode


@pytest.mark.parametrize("rel_tol", [1e-3, 30.0])
def test_device_gnc_schedule_matches_host_rule(gpu, rel_tol):
    """shouldUpdateMeasurementWeights evaluated on the device at every round
    begin (kmx_pgo_set_gnc_schedule + iterate_async) against the host mirror
    (kmx.dpgo.schedule.GncSchedule) driving the restatement: the same rounds
    fire, the same weights and iterates follow. rel_tol 1e-3 fires on the
    inner-iteration count only; 30 also by team convergence."""
    from kmx.dpgo.schedule import GncSchedule
    g, P, X0 = _setup(robust=True)
    P.robustOptInnerIters = 3
    P.robustOptNumWeightUpdates = 4
    P.relChangeTol = rel_tol
    s, o = _pair(g, P, X0)
    s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, rel_tol)
    sched = GncSchedule.from_params(P)
    relc = np.full(g.n_robots, np.inf)
    fired = []
    for it in range(14):
        if sched.should_update(relc):
            o.refresh()
            o.update_weights()
            sched.updated()
            fired.append(it)
        st = o.iterate()
        relc = np.array([x["rel_change"] for x in st])
        sched.round_done()
        s.iterate_async(1, refresh_local=True)
        gs = s.gnc_state()
        assert gs["updates"] == sched.updates and gs["inner_iter"] == sched.inner, (it, gs)
        assert bool(gs["last_fired"]) == (it in fired), it
        for a in range(g.n_robots):
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
        assert np.abs(s.get_weights() - o.get_weights()).max() <= 1e-9
        assert np.abs(s.status() - relc).max() <= 1e-9
    assert sched.updates == P.robustOptNumWeightUpdates or rel_tol < 1
    assert len(fired) >= 3


@pytest.mark.parametrize("robust", [False, True])
def test_accelerated_rounds_match_oracle(gpu, robust):
    """Nesterov-accelerated RBCD (k_accel: Y before the round, V after it,
    restart every restartInterval rounds) vs the oracle's orc_pgo_accel_*:
    tCG counts equal and poses within 1e-6 every round, across two restarts
    and (robust) two explicit GNC updates."""
    g, P, X0 = _setup(robust=robust)
    P.acceleration, P.restartInterval = True, 5
    s, o = _pair(g, P, X0)
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
    assert s.memory()[0] > 0


def test_accelerated_async_equals_sync(gpu):
    g, P, X0 = _setup()
    P.acceleration, P.restartInterval = True, 4
    s1, s2 = BlockSolver(P, 0), BlockSolver(P, 0)
    for s in (s1, s2):
        s.set_graph_data(g)
        for a in range(g.n_robots):
            s.set_iterate(a, X0[a])
    for _ in range(9):
        s1.refresh_local()
        s1.iterate()
    s2.iterate_async(9, refresh_local=True)
    s2.sync()
    for a in range(g.n_robots):
        assert np.array_equal(s1.get_iterate(a), s2.get_iterate(a))


@pytest.mark.parametrize("robust", [False, True])
def test_rgd_rounds_match_oracle(gpu, robust):
    """ROptMethod RGD on the device (k_grad -> k_retract with eta = -s z, no tCG
    launches, always accepted) vs the oracle's gradientDescent restatement."""
    from kmx.dpgo.params import ROptMethod
    g, P, X0 = _setup(robust=robust)
    P.localOptimizationParams.method = ROptMethod.RGD
    P.localOptimizationParams.RGD_stepsize = 1e-4
    s, o = _pair(g, P, X0)
    for it in range(8):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert (sg[a]["tcg_iterations"], sg[a]["accepted"]) == (so[a]["tcg_iterations"], so[a]["accepted"])
            assert abs(sg[a]["f_final"] - so[a]["f_final"]) <= 1e-9 * max(1.0, abs(so[a]["f_final"]))
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
        if robust and it % 4 == 3:
            s.refresh_local()
            assert s.update_weights() == o.update_weights()


@pytest.mark.parametrize("red", ["0", "2"])
@pytest.mark.parametrize("case", ["rtr2", "tcg1", "tcg3"])
def test_round_structure_matches_oracle(gpu, monkeypatch, red, case):
    """Both reduction forms (KMX_RED=0: a k_reduce launch per reduction; 2: the
    consumer form with every reduction folded into the next kernel) on round
    structures the default parameters never produce: two RTR iterations per
    block update (the trial cost is reduced by a launch and the second
    iteration's gradient folded into its first k_hess), and tCG capped at one /
    three steps (the last update reduced in k_retract). Synchronous rounds
    (kmx_pgo_iterate) and the asynchronous form (kmx_pgo_iterate_async) both
    match the CPU restatement."""
    monkeypatch.setenv("KMX_RED", red)
    g, P, X0 = _setup(robust=True, seed=3)
    lo = P.localOptimizationParams
    if case == "rtr2":
        lo.RTR_iterations = 2
    else:
        lo.RTR_tCG_iterations = 1 if case == "tcg1" else 3
    s, o = _pair(g, P, X0)
    for it in range(6):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
    s.iterate_async(3, refresh_local=True)
    s.sync()
    for _ in range(3):
        o.refresh()
        o.iterate()
    for a in range(g.n_robots):
        d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
        assert d <= 1e-6, (a, d)


@pytest.mark.parametrize("red", ["0", "2"])
def test_long_tcg_folds_directions(gpu, monkeypatch, red):
    """Long tCG (25-step cap, residual test at kappa 1e-8): k_hess folds the kept
    directions (DHMAX, pgo.hip) into eta before their buffers are reused, at
    every DHMAX-th step, and k_retract adds the rest, in step order; the rounds
    match the restatement, whose eta is one running sum."""
    monkeypatch.setenv("KMX_RED", red)
    # no outliers, start near the optimum: positive curvature, so tCG stops on
    # its residual test (kappa 1e-8) rather than at the trust-region boundary
    g, P, X0 = _setup(robust=False, seed=4, perturb=0.01, outlier=0.0)
    lo = P.localOptimizationParams
    lo.RTR_tCG_iterations = 25
    lo.tCG_kappa = 1e-8  # long inner solves: the residual test needs many steps
    lo.RTR_initial_radius, lo.RTR_max_radius = 1e4, 1e6
    s, o = _pair(g, P, X0)
    longest = 0
    for it in range(8):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
            longest = max(longest, sg[a]["tcg_iterations"])
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= 1e-6, (it, a, d)
    assert longest > 10, longest  # the fold ran


@pytest.mark.parametrize("tile_incidences", [0, 60])
def test_large_robot_block_matches_oracle(gpu, tile_incidences):
    """One 12.5k-pose robot block (the per-GPU share of configs[3] at N = 8): the
    finer tile cut gives it ~700 tiles, more than the 2 x 256 partials the
    consumer k_hess's one-shot robot sums hold, so its folded reductions take
    the looped robot_sum path (k_update's four-tile-per-thread sum holds them);
    with 60 incidences per tile (~2,100 tiles) every consumer sum loops. Rounds
    (GNC on) still match the restatement."""
    g, P, X0 = _setup(n_robots=1, n=12_500, m=62_500, seed=5)
    P.tileIncidences = tile_incidences
    s, o = _pair(g, P, X0)
    for it in range(4):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        assert sg[0]["tcg_iterations"] == so[0]["tcg_iterations"], (it, sg[0], so[0])
        assert sg[0]["accepted"] == so[0]["accepted"]
        d = np.linalg.norm((s.get_iterate(0) - o.get_iterate(0)).reshape(-1, 4 * P.r), axis=1).max()
        assert d <= 1e-6, (it, d)


def test_reduction_forms_agree_bitwise(gpu, monkeypatch):
    """The consumer kernels reduce every robot's partials in k_reduce's order and
    take the same decisions, so both forms give the same iterates bit for bit
    (what keeps a team's result independent of how its ranks' sizes fall on
    either side of the form's size threshold). Gated k_hess launches
    (KMX_HESS_GATE: the phase test before the first records are fetched in
    every launch after a tCG's first; 0 turns it off) only reorder loads, so
    both give the same bits in both forms."""
    g, P, X0 = _setup(robust=True, seed=4)
    out = []
    for red, gate in (("0", "1"), ("2", "1"), ("0", "0"), ("2", "0")):
        monkeypatch.setenv("KMX_RED", red)
        monkeypatch.setenv("KMX_HESS_GATE", gate)
        s = BlockSolver(P, 0)
        s.set_graph_data(g)
        s.set_gnc_schedule(True, 3, 50, P.relChangeTol)
        for a in range(g.n_robots):
            s.set_iterate(a, X0[a])
        s.iterate_async(9, refresh_local=True)
        s.sync()
        out.append([s.get_iterate(a) for a in range(g.n_robots)] + [s.get_weights()])
        s.close()
    for other in out[1:]:
        for a, b in zip(out[0], other):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("red", ["0", "2", "ungated"])
def test_tcg_poll_modes_agree_bitwise(gpu, monkeypatch, red):
    """Polled, blind and adaptive tCG enqueueing (kmx_pgo_set_tcg_poll 1 / 0 /
    -1) launch the same work that matters: a blind step of a robot that already
    left tCG exits at once. Iterates, GNC weights and work counters agree bit
    for bit over rounds that cross GNC updates, in both reduction forms, and
    the team status a multi-rank exchange carries is the same ("ungated":
    KMX_HESS_GATE=0, every k_hess launch fetches its first records before the
    phase test)."""
    monkeypatch.setenv("KMX_RED", "0" if red == "ungated" else red)
    monkeypatch.setenv("KMX_HESS_GATE", "0" if red == "ungated" else "1")
    g, P, X0 = _setup(robust=True, seed=6)
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


def test_tcg_poll_mode_checked(gpu):
    P = PGOAgentParameters(r=5)
    s = BlockSolver(P, 0)
    with pytest.raises(abi.KmxError):
        s.set_tcg_poll(2)
    s.close()
