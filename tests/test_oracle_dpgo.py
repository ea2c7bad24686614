"""CPU checks of the dpgo restatement (oracle/dpgo_oracle.c).

The reference ships no dpgo fixtures (parity unpinned), so
the oracle is pinned by (1) an independent vectorised numpy restatement of the
cost / gradient / Hessian of SURVEY.md §9.1, (2) finite differences,
(3) manifold identities, (4) known answers: a noise-free graph converges to
ground truth; GNC-TLS rejects planted outliers."""
import numpy as np
import pytest

from kmx.abi import (KMX_EVAL_COST_EGRAD, KMX_EVAL_EHESS, KMX_EVAL_PRECON, KMX_EVAL_RETRACT, KMX_EVAL_RGRAD,
                     KMX_EVAL_RHESS)
from kmx.dpgo.params import PGOAgentParameters, RobustCostType
from kmx.synth import lift, lifting_matrix, make_pose_graph
from kmx.synth.pose_graph import _expm_so3
from oracle.oracle import OraclePGO


def _problem(seed=0, r=5, robots=3, n=240, m=700, weights=True):
    g = make_pose_graph(robots, n, m, seed=seed)
    if weights:
        g.weight = np.random.default_rng(seed).uniform(0.1, 1.0, g.m)
    P = PGOAgentParameters(r=r)
    Y = lifting_matrix(r, seed=1)
    rng = np.random.default_rng(seed + 1)
    X = {}
    for a in range(g.n_robots):
        k = int(g.n_poses[a])
        X[a] = lift(g.init_R[a] @ _expm_so3(rng.normal(0, 0.05, (k, 3))), g.init_t[a] + rng.normal(0, 0.2, (k, 3)), Y)
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        o.set_iterate(a, X[a])
    o.refresh()
    return g, P, o, X


def numpy_block(g, X, a, V=None, hess=False):
    """Independent restatement: f = 1/2 sum_e w(k|Y_j - Y_i R|^2 + t|p_j - p_i - Y_i t|^2)."""
    off = np.concatenate([[0], np.cumsum(g.n_poses)])
    allX = np.concatenate([X[b] for b in range(g.n_robots)])
    Vb = X[a] if V is None else V
    sel = (g.r1 == a) | (g.r2 == a)
    e = np.nonzero(sel)[0]
    gi, gj = off[g.r1[e]] + g.p1[e], off[g.r2[e]] + g.p2[e]
    Xi, Xj = allX[gi].copy(), allX[gj].copy()
    ti, tj = g.r1[e] == a, g.r2[e] == a
    Xi[ti] = Vb[g.p1[e][ti]]
    Xj[tj] = Vb[g.p2[e][tj]]
    if hess:
        Xi[~ti] = 0.0
        Xj[~tj] = 0.0
    wk = (g.weight * g.kappa)[e][:, None, None]
    wt = (g.weight * g.tau)[e][:, None]
    ER = Xj[:, :, :3] - Xi[:, :, :3] @ g.R[e]
    Et = Xj[:, :, 3] - Xi[:, :, 3] - np.einsum("nac,nc->na", Xi[:, :, :3], g.t[e])
    cost = 0.5 * (np.sum(wk * ER ** 2) + np.sum(wt * Et ** 2))
    G = np.zeros_like(Vb)
    np.add.at(G, (g.p2[e][tj], slice(None), slice(0, 3)), (wk * ER)[tj])
    np.add.at(G, (g.p2[e][tj], slice(None), 3), (wt * Et)[tj])
    gi_Y = -(wk * np.einsum("nac,nkc->nak", ER, g.R[e])) - (wt * Et)[:, :, None] * g.t[e][:, None, :]
    np.add.at(G, (g.p1[e][ti], slice(None), slice(0, 3)), gi_Y[ti])
    np.add.at(G, (g.p1[e][ti], slice(None), 3), -(wt * Et)[ti])
    return cost, G


def test_cost_grad_hess_vs_numpy():
    g, P, o, X = _problem()
    rng = np.random.default_rng(4)
    for a in range(g.n_robots):
        eg, f = o.eval(a, KMX_EVAL_COST_EGRAD, X[a])
        fn, Gn = numpy_block(g, X, a)
        assert abs(f - fn) <= 1e-10 * abs(fn)
        assert np.abs(eg - Gn).max() <= 1e-9 * max(1.0, np.abs(Gn).max())
        V = rng.standard_normal(X[a].shape)
        H, _ = o.eval(a, KMX_EVAL_EHESS, V)
        _, Hn = numpy_block(g, X, a, V=V, hess=True)
        assert np.abs(H - Hn).max() <= 1e-9 * max(1.0, np.abs(Hn).max())


def test_finite_differences():
    g, P, o, X = _problem(seed=3)
    rng = np.random.default_rng(7)
    a = 1
    V = rng.standard_normal(X[a].shape)
    eg, f = o.eval(a, KMX_EVAL_COST_EGRAD, X[a])
    eps = 1e-6
    _, fp = o.eval(a, KMX_EVAL_COST_EGRAD, X[a] + eps * V)
    _, fm = o.eval(a, KMX_EVAL_COST_EGRAD, X[a] - eps * V)
    assert abs((fp - fm) / (2 * eps) - np.sum(eg * V)) <= 1e-6 * abs(np.sum(eg * V))
    gp, _ = o.eval(a, KMX_EVAL_COST_EGRAD, X[a] + eps * V)
    gm, _ = o.eval(a, KMX_EVAL_COST_EGRAD, X[a] - eps * V)
    H, _ = o.eval(a, KMX_EVAL_EHESS, V)
    assert np.abs((gp - gm) / (2 * eps) - H).max() <= 1e-5 * np.abs(H).max()


def test_manifold_identities():
    g, P, o, X = _problem(seed=5)
    rng = np.random.default_rng(9)
    a = 0
    Y = X[a][:, :, :3]
    rg, _ = o.eval(a, KMX_EVAL_RGRAD)
    M = np.einsum("nac,nak->nck", Y, rg[:, :, :3])
    assert np.abs(M + M.transpose(0, 2, 1)).max() < 1e-8 * max(1.0, np.abs(rg).max())  # tangent

    def tangent(Z):
        S = np.einsum("nac,nak->nck", Y, Z[:, :, :3])
        S = 0.5 * (S + S.transpose(0, 2, 1))
        T = Z.copy()
        T[:, :, :3] -= np.einsum("nac,nck->nak", Y, S)
        return T
    U, V = tangent(rng.standard_normal(X[a].shape)), tangent(rng.standard_normal(X[a].shape))
    HU, _ = o.eval(a, KMX_EVAL_RHESS, U)
    HV, _ = o.eval(a, KMX_EVAL_RHESS, V)
    assert abs(np.sum(U * HV) - np.sum(V * HU)) <= 1e-9 * abs(np.sum(U * HV))  # symmetric
    PV, s = o.eval(a, KMX_EVAL_PRECON, V)
    assert s > 0
    Xt, _ = o.eval(a, KMX_EVAL_RETRACT, 0.1 * V)
    YtY = np.einsum("nac,nak->nck", Xt[:, :, :3], Xt[:, :, :3])
    assert np.abs(YtY - np.eye(3)).max() < 1e-12


def test_noise_free_converges_to_ground_truth():
    g = make_pose_graph(2, 160, 240, outlier_frac=0.0, noise_free=True, seed=0)
    P = PGOAgentParameters(r=5)
    P.robustCostParams.costType = RobustCostType.L2
    P.localOptimizationParams.RTR_tCG_iterations = 50
    Y = lifting_matrix(5)
    rng = np.random.default_rng(0)
    o = OraclePGO(P.to_c(), g)
    for a in range(2):
        k = int(g.n_poses[a])
        o.set_iterate(a, lift(g.init_R[a] @ _expm_so3(rng.normal(0, 0.1, (k, 3))),
                              g.init_t[a] + rng.normal(0, 0.5, (k, 3)), Y))
    for _ in range(250):
        o.iterate()
    anchor = o.get_iterate(0)[0]
    R0, t0 = g.gt_R[0][0], g.gt_t[0][0]
    for a in range(2):
        T = o.trajectory(a, anchor)
        assert np.abs(T[:, 9:] - (g.gt_t[a] - t0) @ R0).max() < 1e-4
        assert np.abs(T[:, :9].reshape(-1, 3, 3) - np.einsum("ji,njk->nik", R0, g.gt_R[a])).max() < 1e-4


def test_gnc_rejects_outliers():
    g = make_pose_graph(2, 200, 500, outlier_frac=0.2, seed=1)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5)
    o = OraclePGO(P.to_c(), g)
    for a in range(2):
        o.set_iterate(a, lift(g.gt_R[a], g.gt_t[a], Y))  # start at ground truth
    for k in range(1, 401):
        o.iterate()
        if k % 10 == 0:
            o.refresh()
            o.update_weights()
    w = o.get_weights()
    lc = g.fixed == 0
    assert np.mean(w[lc & g.outlier] < 1e-3) > 0.95
    assert np.mean(w[lc & ~g.outlier] > 0.999) > 0.95


@pytest.mark.parametrize("rSq,mu,barc,expect", [
    (0.0, 1e-5, 5.0, 1.0),            # below the lower bound
    (1e9, 1e-5, 5.0, None),           # between the bounds: formula
    (1e12, 1e-5, 5.0, 0.0),           # above the upper bound
    (24.9, 1e6, 5.0, 1.0), (25.1, 1e6, 5.0, 0.0),  # mu -> inf: TLS step at barc^2
])
def test_gnc_tls_weight_known_answers(rSq, mu, barc, expect):
    """RobustCost::weight for GNC_TLS (drawio:2215), via a 1-edge graph."""
    import math
    lo, hi = mu / (mu + 1) * barc ** 2, (mu + 1) / mu * barc ** 2
    ref = 1.0 if rSq <= lo else 0.0 if rSq >= hi else math.sqrt(barc ** 2 * mu * (mu + 1) / rSq) - mu
    if expect is not None:
        assert ref == expect
    from kmx.synth.pose_graph import PoseGraphData
    # one loop closure with residual^2 = rSq (tau-only translation residual)
    d = math.sqrt(rSq / 100.0)
    g = PoseGraphData(n_robots=1, n_poses=np.array([2], np.int32), r1=np.array([0], np.int32),
                      p1=np.array([0], np.int32), r2=np.array([0], np.int32), p2=np.array([1], np.int32),
                      R=np.eye(3)[None].copy(), t=np.array([[d, 0.0, 0.0]]), kappa=np.array([1e4]),
                      tau=np.array([100.0]), weight=np.array([1.0]), fixed=np.array([0], np.uint8),
                      outlier=np.array([False]))
    P = PGOAgentParameters(r=3)
    P.robustCostParams.GNCBarc, P.robustCostParams.GNCInitMu = barc, mu
    o = OraclePGO(P.to_c(), g)
    o.set_iterate(0, np.stack([np.c_[np.eye(3), np.zeros(3)]] * 2))
    o.update_weights()
    assert abs(o.get_weights()[0] - ref) <= 1e-12 * max(1.0, ref)


def _accel_run(accel, rounds, restart=30, seed=1):
    g = make_pose_graph(4, 800, 2400, outlier_frac=0.0, seed=seed)
    P = PGOAgentParameters(r=5, acceleration=accel, restartInterval=restart)
    P.robustCostParams.costType = RobustCostType.L2
    o = OraclePGO(P.to_c(), g)
    Y = lifting_matrix(5, seed=1)
    for a in range(g.n_robots):
        o.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    costs, gammas = [], []
    for _ in range(rounds):
        costs.append(sum(s["f_final"] for s in o.iterate()))
        gammas.append(o.accel_gamma)
    return o, g, np.array(costs), np.array(gammas)


def test_acceleration_schedule_and_speedup():
    """Nesterov-accelerated RBCD (dpgo acceleration): gamma follows
    gamma' = (1 + sqrt(1 + 4 N^2 gamma^2)) / (2N) from 0, restarts to 0 every
    restartInterval rounds, the momentum V stays on the manifold, and on the
    same graph the accelerated rounds reach a lower cost than plain RBCD."""
    N, restart = 4, 10
    o, g, ca, ga = _accel_run(True, 40, restart)
    gam, exp = 0.0, []
    for k in range(40):
        gn = (1 + np.sqrt(1 + 4 * N * N * gam * gam)) / (2 * N)
        gam = 0.0 if (k + 1) % restart == 0 else gn
        exp.append(gam)
    assert np.allclose(ga, exp, rtol=0, atol=1e-15)
    for a in range(g.n_robots):  # iterates stay on the lifted manifold
        X = o.get_iterate(a)[:, :, :3]
        assert np.abs(np.einsum("nai,naj->nij", X, X) - np.eye(3)).max() < 1e-10
    _, _, c0, _ = _accel_run(False, 40)
    _, _, c1, _ = _accel_run(True, 40, restart=30)
    assert c1[-1] < c0[-1] and c1[20] < c0[20]


def test_rgd_method_descends():
    """ROptMethod RGD (dpgo QuadraticOptimizer::gradientDescent): one
    preconditioned Riemannian gradient step of size s per block update, always
    accepted; the cost decreases monotonically from the odometry start for a
    small step, no tCG runs, and the iterate stays on the manifold."""
    from kmx.dpgo.params import ROptMethod
    g = make_pose_graph(3, 300, 900, outlier_frac=0.0, seed=2)
    P = PGOAgentParameters(r=5)
    P.robustCostParams.costType = RobustCostType.L2
    P.localOptimizationParams.method = ROptMethod.RGD
    P.localOptimizationParams.RGD_stepsize = 1e-4
    o = OraclePGO(P.to_c(), g)
    Y = lifting_matrix(5, seed=1)
    for a in range(g.n_robots):
        o.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    costs = []
    for _ in range(15):
        st = o.iterate()
        assert all(s["tcg_iterations"] == 0 and s["accepted"] == 1 for s in st)
        assert all(s["f_final"] < s["f_init"] for s in st)
        costs.append(sum(s["f_final"] for s in st))
    assert all(b < a for a, b in zip(costs, costs[1:]))
    for a in range(g.n_robots):
        X = o.get_iterate(a)[:, :, :3]
        assert np.abs(np.einsum("nai,naj->nij", X, X) - np.eye(3)).max() < 1e-10


def test_all_cores_variant_agrees_with_serial_round():
    """orc_pgo_round_mt2 (bench.py's all-cores CPU baseline: blocks over outer
    threads, each block update over inner threads, edge terms gathered per pose)
    follows the serial restatement to rounding: equal tCG counts and acceptance,
    poses within 1e-9 over 10 rounds."""
    from oracle.oracle import OraclePGO
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.synth import lift, lifting_matrix, make_pose_graph
    g = make_pose_graph(4, 4000, 16000, outlier_frac=0.2, seed=2)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5, seed=1)
    a_, b_ = OraclePGO(P.to_c(), g), OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        X0 = lift(g.init_R[a], g.init_t[a], Y)
        a_.set_iterate(a, X0)
        b_.set_iterate(a, X0)
    for it in range(10):
        sa = a_.iterate()
        sb = b_.iterate(threads=2, inner=2)
        for r in range(g.n_robots):
            assert sa[r]["tcg_iterations"] == sb[r]["tcg_iterations"] and sa[r]["accepted"] == sb[r]["accepted"]
            d = np.abs(a_.get_iterate(r) - b_.get_iterate(r)).max()
            assert d <= 1e-9, (it, r, d)


def test_onesync_tcg_form_tracks_standard_form():
    """The one-sync tCG restatement (tcg_onesync, KMX_TCG_FORM_ONESYNC): the
    same Steihaug-Toint decisions from one reduction per step. In exact
    arithmetic it is the standard iteration; in floating point the two stay
    within rounding over a run to relChangeTol: equal Hess-vec counts per
    round here, the same round count to converge, costs within 1e-9."""
    runs = {}
    for form in ("standard", "onesync"):
        g, P, o, X = _problem(seed=2, robots=3, n=300, m=900)
        P.localOptimizationParams.tCG_form = form
        o = OraclePGO(P.to_c(), g)
        for a in range(g.n_robots):
            o.set_iterate(a, X[a])
        o.refresh()
        hist = []
        for it in range(200):
            st = o.iterate()
            hist.append((max(s["rel_change"] for s in st), [s["hessvecs"] for s in st],
                         sum(s["f_final"] for s in st)))
            if it % 10 == 9:
                o.refresh()
                o.update_weights()
        runs[form] = hist
    conv = {f: next(i for i, x in enumerate(h) if x[0] < 1e-3) for f, h in runs.items()}
    assert conv["onesync"] == conv["standard"], conv
    for a, b in zip(runs["standard"], runs["onesync"]):
        assert a[1] == b[1]
        assert abs(a[2] - b[2]) <= 1e-9 * abs(a[2])


def test_tcg_form_is_checked():
    P = PGOAgentParameters(r=5)
    P.localOptimizationParams.tCG_form = "pipelined"
    with pytest.raises(ValueError):
        P.to_c()
