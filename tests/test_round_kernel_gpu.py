"""The persistent round (k_round: one launch per RBCD round, the phases
between grid barriers) against the launched form it replaces (one kernel per
phase, host-enqueued tCG steps): same tiles, same bodies, same summation
order. Integers (tCG counts and stops, acceptance, Hess-vecs, edges, GNC
updates) must be equal; floating point agrees to rounding (pgo.hip is built
with FMA contraction, whose fusion choices depend on the code around an
expression, so the inlined round may round a sum differently in the last
bit): 1e-12 relative on statistics, 1e-9 on poses. The launched form carries
the oracle parity (test_dpgo_gpu.py, test_configs_gpu.py,
test_parity_long_gpu.py); this carries it over.

Shapes: a small 4-robot team (every phase, a GNC update, robots stopping tCG
at different steps), and the configs[3] rank handle of an 8-GPU team (robot 0's
12.5k-pose block with the team's tile cut), synchronous and batched rounds.
"""
import numpy as np
import pytest

from kmx.dpgo.params import PGOAgentParameters
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix, make_pose_graph

pytestmark = pytest.mark.gpu


def _pair(g, P, local=None, tile=0):
    import dataclasses
    P = dataclasses.replace(P, tileIncidences=tile)
    Y = lifting_matrix(P.r, seed=1)
    out = []
    for form in (0, 1):
        s = BlockSolver(P, 0)
        s.set_round_form(form)
        s.set_graph_data(g, local)
        s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
        loc = range(g.n_robots) if local is None else np.nonzero(local)[0]
        for a in loc:
            s.set_iterate(int(a), lift(g.init_R[a], g.init_t[a], Y))
        s.refresh_local()
        out.append(s)
    assert not out[0].round_form()["persistent"]
    f = out[1].round_form()
    assert f["persistent"], f
    return out, list(loc)


INTS = ("updated", "tcg_iterations", "tcg_stop", "accepted", "edges", "hessvecs")
FLTS = ("f_init", "gradnorm_init", "f_final", "rho", "radius", "rel_change")


def _stats_agree(a, b, it):
    for x, y in zip(a, b):
        for k in INTS:
            assert x[k] == y[k], (it, k, x, y)
        for k in FLTS:
            assert abs(x[k] - y[k]) <= 1e-12 * max(1.0, abs(x[k])), (it, k, x[k], y[k])


def _same(sl, sp, robots):
    for a in robots:
        d = np.abs(sl.get_iterate(a) - sp.get_iterate(a)).max()
        assert d <= 1e-9, (a, d)
    assert np.abs(sl.get_weights() - sp.get_weights()).max() <= 1e-9
    gl, gp = sl.gnc_state(), sp.gnc_state()
    assert {k: v for k, v in gl.items() if k != "mu"} == {k: v for k, v in gp.items() if k != "mu"}
    assert gl["mu"] == gp["mu"]
    sa, sb = sl.status(), sp.status()
    assert np.allclose(sa, sb, rtol=1e-9, atol=1e-12)


@pytest.mark.timeout(300)
def test_round_kernel_matches_launched_small_team(gpu):
    g = make_pose_graph(4, 4000, 12000, seed=3)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 4
    (sl, sp), robots = _pair(g, P, tile=180)
    try:
        for it in range(14):
            _stats_agree(sl.iterate(), sp.iterate(), it)
        _same(sl, sp, robots)
        assert sp.gnc_state()["updates"] >= 2
        cl, cp = sl.read_counters(), sp.read_counters()
        for k in ("edges_iters", "block_updates", "hessvecs", "gnc_updates"):
            assert cl[k] == cp[k], k
        sl.iterate_async(25, refresh_local=True)
        sp.iterate_async(25, refresh_local=True)
        sl.sync()
        sp.sync()
        _same(sl, sp, robots)
    finally:
        sl.close()
        sp.close()


@pytest.mark.timeout(300)
def test_round_kernel_matches_launched_rank_handle(gpu):
    """Robot 0's block of configs[3] as rank 0 of an 8-GPU team holds it (the
    team's tile cut, foreign public rows frozen): 60 batched rounds, the
    many-Hess-vec regime included."""
    from kmx.dpgo.driver import team_tile_incidences
    g = config("synth100k", seed=0)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 20
    local = np.zeros(g.n_robots, np.uint8)
    local[0] = 1
    (sl, sp), robots = _pair(g, P, local, team_tile_incidences(g, 8, P.r))
    try:
        for it in range(3):
            _stats_agree(sl.iterate(), sp.iterate(), it)
        sl.iterate_async(60, refresh_local=False)
        sp.iterate_async(60, refresh_local=False)
        sl.sync()
        sp.sync()
        _same(sl, sp, robots)
        cl, cp = sl.read_counters(), sp.read_counters()
        assert cl["hessvecs"] == cp["hessvecs"] and cl["hessvecs"] > 60 * 3
    finally:
        sl.close()
        sp.close()
