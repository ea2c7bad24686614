"""The resident round (kmx_pgo_params.tcg_form = KMX_TCG_FORM_RESIDENT, VERDICT
r4 next-round item 1): the one-sync tCG's arithmetic with the whole block
update in ONE persistent launch per round (pgo.hip body_round), each tile's
rows resident in registers / LDS, one grid barrier per tCG step.

Bars:
  * against the launched one-sync form on the same tile cut: every round's
    statistics and every lifted pose bit for bit (same expressions, the robot
    sums in the same order), GNC weight updates included;
  * against the restatement's one-sync form (oracle/dpgo_oracle.c
    tcg_onesync): per round equal tCG counts, stop reasons and acceptance,
    every lifted pose within 1e-6, on the round structures the launched form
    is tested on, and on a 12.5k-pose block (configs[3]'s shard at 8 GPUs);
  * the asynchronous enqueueing (iterate_async, the driver's path) equals the
    per-round calls bit for bit;
  * what the resident form cannot run (rtr_iterations 2, RGD) falls back to
    the launched one-sync form and says why.
"""
import numpy as np
import pytest

from kmx.dpgo.solver import BlockSolver
from tests.test_dpgo_gpu import _full_records, _pair, _setup

pytestmark = pytest.mark.gpu


def _tile_inc(r):
    """The resident form's automatic cut: full tiles of 4 waves x (64 // r)
    poses, two gather chunks (pgo.hip set_graph)."""
    return 2 * 4 * (64 // r) * r


def _form(P, form, same_cut=True):
    P.localOptimizationParams.tCG_form = form
    if same_cut:
        P.tileIncidences = _tile_inc(P.r)
    return P


def _make(g, P, X0, gnc=False):
    s = BlockSolver(P, 0)
    s.set_graph_data(g)
    if gnc:
        s.set_gnc_schedule(True, 3, 50, P.relChangeTol)
    for a in range(g.n_robots):
        s.set_iterate(a, X0[a])
    s.refresh_local()
    return s


STAT_KEYS = ("updated", "tcg_iterations", "tcg_stop", "accepted", "f_init", "gradnorm_init", "f_final", "rho",
             "radius", "rel_change", "hessvecs")


@pytest.mark.parametrize("case", ["default", "tcg3", "r3", "r8", "full", "l2"])
def test_resident_equals_launched_onesync_bitwise(gpu, case):
    r = 3 if case == "r3" else 8 if case == "r8" else 5
    g, P, X0 = _setup(r=r, robust=case != "l2", seed=11)
    if case == "full":
        _full_records(g)
    if case == "tcg3":
        P.localOptimizationParams.RTR_tCG_iterations = 3
    import copy
    Pr, Pl = _form(copy.deepcopy(P), "resident"), _form(copy.deepcopy(P), "onesync")
    sr, sl = _make(g, Pr, X0), _make(g, Pl, X0)
    try:
        info = sr.resident_info()
        assert info["resident"], info
        assert info["ntiles"] <= info["capacity"], info
        assert not sl.resident_info()["resident"]
        for it in range(10):
            sr.refresh_local()
            sl.refresh_local()
            a_r, a_l = sr.iterate(), sl.iterate()
            for a in range(g.n_robots):
                for k in STAT_KEYS:
                    assert a_r[a][k] == a_l[a][k], (it, a, k, a_r[a][k], a_l[a][k])
                assert np.array_equal(sr.get_iterate(a), sl.get_iterate(a)), (it, a)
            if case != "l2" and it % 4 == 3:
                sr.refresh_local()
                sl.refresh_local()
                assert sr.update_weights() == sl.update_weights()
                assert np.array_equal(sr.get_weights(), sl.get_weights())
        cr, cl = sr.read_counters(), sl.read_counters()
        for k in ("hessvecs", "edges_iters", "block_updates"):
            assert cr[k] == cl[k], (k, cr[k], cl[k])
    finally:
        sr.close()
        sl.close()


def _rounds_vs_oracle(s, o, g, P, n, robust=True, tol=1e-6):
    for it in range(n):
        s.refresh_local()
        sg = s.iterate()
        so = o.iterate()
        for a in range(g.n_robots):
            assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a, sg[a], so[a])
            assert sg[a]["tcg_stop"] == so[a]["tcg_stop"], (it, a, sg[a], so[a])
            assert sg[a]["accepted"] == so[a]["accepted"], (it, a)
            d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
            assert d <= tol, (it, a, d)
        if robust and it % 4 == 3:
            s.refresh_local()
            assert s.update_weights() == o.update_weights()
            assert np.abs(s.get_weights() - o.get_weights()).max() <= 1e-9


@pytest.mark.parametrize("case", ["default", "tcg1", "long_tcg", "two_robots_one_idle"])
def test_resident_rounds_match_oracle(gpu, case):
    if case == "long_tcg":
        g, P, X0 = _setup(robust=False, seed=4, perturb=0.01, outlier=0.0)
        lo = P.localOptimizationParams
        lo.RTR_tCG_iterations = 25
        lo.tCG_kappa = 1e-8
        lo.RTR_initial_radius, lo.RTR_max_radius = 1e4, 1e6
    else:
        g, P, X0 = _setup(seed=12)
    if case == "tcg1":
        P.localOptimizationParams.RTR_tCG_iterations = 1
    _form(P, "resident", same_cut=False)
    s, o = _pair(g, P, X0)
    try:
        assert s.resident_info()["resident"], s.resident_info()
        if case == "two_robots_one_idle":
            # one robot inactive (the sequential schedule's shape): it still takes every grid barrier
            active = np.zeros(g.n_robots, np.uint8)
            active[1] = 1
            for it in range(6):
                s.refresh_local()
                sg = s.iterate(active)
                so = o.iterate(active)
                for a in range(g.n_robots):
                    assert sg[a]["updated"] == so[a]["updated"] == int(active[a])
                    assert sg[a]["tcg_iterations"] == so[a]["tcg_iterations"], (it, a)
                    d = np.linalg.norm((s.get_iterate(a) - o.get_iterate(a)).reshape(-1, 4 * P.r), axis=1).max()
                    assert d <= 1e-6, (it, a, d)
            return
        _rounds_vs_oracle(s, o, g, P, 10 if case != "long_tcg" else 8, robust=case != "long_tcg")
    finally:
        s.close()


def test_resident_shard_of_configs3(gpu):
    """One 12.5k-pose / 62.5k-edge block, the per-GPU shard of configs[3] at 8
    GPUs: every tile resident, rounds match the restatement."""
    g, P, X0 = _setup(n_robots=1, n=12_500, m=62_500, seed=5)
    _form(P, "resident", same_cut=False)
    s, o = _pair(g, P, X0)
    try:
        info = s.resident_info()
        assert info["resident"] and info["ntiles"] <= info["capacity"], info
        _rounds_vs_oracle(s, o, g, P, 4, robust=False)
    finally:
        s.close()


def test_resident_async_equals_iterate(gpu):
    """iterate_async (every round from one host call; the GNC schedule decided
    on the device) against the same rounds one iterate() call at a time."""
    g, P, X0 = _setup(seed=13)
    _form(P, "resident", same_cut=False)
    sa, si = _make(g, P, X0, gnc=True), _make(g, P, X0, gnc=True)
    try:
        sa.iterate_async(14, refresh_local=True)
        sa.sync()
        for _ in range(14):
            si.refresh_local()
            si.iterate()
        for a in range(g.n_robots):
            assert np.array_equal(sa.get_iterate(a), si.get_iterate(a)), a
        assert np.array_equal(sa.get_weights(), si.get_weights())
        assert sa.gnc_state() == si.gnc_state()
        assert sa.gnc_state()["updates"] >= 2
    finally:
        sa.close()
        si.close()


@pytest.mark.parametrize("what", ["rtr2", "rgd"])
def test_resident_fallback_says_why(gpu, what):
    g, P, X0 = _setup(seed=14)
    from kmx.dpgo.params import ROptMethod
    if what == "rtr2":
        P.localOptimizationParams.RTR_iterations = 2
    else:
        P.localOptimizationParams.method = ROptMethod.RGD
    _form(P, "resident", same_cut=False)
    s, o = _pair(g, P, X0)
    try:
        info = s.resident_info()
        assert not info["resident"] and info["reason"], info
        _rounds_vs_oracle(s, o, g, P, 4)
    finally:
        s.close()
