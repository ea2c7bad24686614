"""Generate the frozen parity fixtures tests/golden/{dpgo,lcd}_small.npz.

Inputs (graph / frame pool / initial iterate) and the CPU restatement's
outputs are stored together, so a later change of oracle/ (or of the
synthetic generators) cannot move the bar: tests/test_golden_cpu.py fails
when the oracle no longer reproduces these files, and tests/test_golden_gpu.py
checks the HIP path against the stored outputs directly.

Run from the repo root:  python tests/golden/make_golden.py
(the fixtures were made with the oracle at the commit that added them;
regenerate only for a deliberate, reviewed change of restated behaviour).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "kimera-multi_amd"), str(ROOT)]
OUT = Path(__file__).resolve().parent

DPGO_ROUNDS = 12
DPGO_GNC_EVERY = 4       # update_weights after rounds 3, 7, 11 (as test_rounds_match_oracle)
LCD_CASES = [            # (ransac_2d2d_algorithm, rng_variant, norm, recovery: 0 1-point 3D-3D, 1 PnP, 2 Arun)
    (0, "gcc9", "l1", 0), (1, "gcc9", "l1", 0), (0, "gcc11", "hamming", 0), (1, "gcc11", "hamming", 0),
    (0, "gcc9", "l1", 1), (0, "gcc9", "l1", 2),
]


def dpgo_inputs():
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.synth import lift, lifting_matrix, make_pose_graph
    from kmx.synth.pose_graph import _expm_so3
    g = make_pose_graph(3, 300, 900, outlier_frac=0.2, seed=0)
    P = PGOAgentParameters(r=5)
    Y = lifting_matrix(5, seed=1)
    rng = np.random.default_rng(7)
    X0 = []
    for a in range(g.n_robots):
        k = int(g.n_poses[a])
        Rp = g.init_R[a] @ _expm_so3(rng.normal(0, 0.05, (k, 3)))
        X0.append(lift(Rp, g.init_t[a] + rng.normal(0, 0.25, (k, 3)), Y))
    return g, P, np.concatenate(X0)


def graph_from(d):
    from kmx.synth.pose_graph import PoseGraphData
    return PoseGraphData(n_robots=int(d["n_poses"].shape[0]), n_poses=d["n_poses"], r1=d["r1"], p1=d["p1"],
                         r2=d["r2"], p2=d["p2"], R=d["R"], t=d["t"], kappa=d["kappa"], tau=d["tau"],
                         weight=d["weight"].copy(), fixed=d["fixed"], outlier=np.zeros(d["r1"].shape[0], bool))


def split_rows(g, X):
    off = np.concatenate([[0], np.cumsum(g.n_poses)])
    return [X[off[a]:off[a + 1]] for a in range(g.n_robots)]


def run_dpgo_oracle(g, r, X0):
    """The restatement's concurrent rounds with an explicit GNC update every
    DPGO_GNC_EVERY rounds: per round and robot (tcg_iterations, accepted, updated, hessvecs;
    f_init, gradnorm_init, f_final, rel_change), the weights and mu after each update, the
    final iterate."""
    from kmx.dpgo.params import PGOAgentParameters
    from oracle.oracle import OraclePGO
    P = PGOAgentParameters(r=r)
    o = OraclePGO(P.to_c(), g)
    for a, Xa in enumerate(split_rows(g, X0)):
        o.set_iterate(a, Xa)
    ints, flts, mus, ws = [], [], [], []
    for it in range(DPGO_ROUNDS):
        o.refresh()
        st = o.iterate()
        ints.append([[s["tcg_iterations"], s["accepted"], s["updated"], s["hessvecs"]] for s in st])
        flts.append([[s["f_init"], s["gradnorm_init"], s["f_final"], s["rel_change"]] for s in st])
        if it % DPGO_GNC_EVERY == DPGO_GNC_EVERY - 1:
            o.refresh()
            mus.append(o.update_weights())
            ws.append(o.get_weights())
    X = np.concatenate([o.get_iterate(a) for a in range(g.n_robots)])
    return {"round_ints": np.array(ints, np.int32), "round_f": np.array(flts, np.float64),
            "mu": np.array(mus), "weights": np.array(ws), "X_final": X}


def lcd_inputs():
    from kmx.synth.lcd import make_lcd_pool
    return make_lcd_pool(16, 200, seed=3)


def pool_from(d):
    from kmx.synth.lcd import LcdPool
    F, N = d["desc"].shape[:2]
    z = np.zeros((0, 3))
    return LcdPool(n_frames=F, max_feats=N, n_feats=d["n_feats"], desc=d["desc"], bearings=d["bearings"],
                   points=d["points"], cand_query=d["cand_query"], cand_match=d["cand_match"], R_qm=z, t_qm=z,
                   true_idx=np.zeros((0, 0, 2), np.int32))


LCD_REFINE_CASES = [     # refine_pose 1 (LcdParams.yaml:14) on the 3D-3D recoveries: lcd_refine.npz
    (0, "gcc9", "l1", 0), (1, "gcc11", "hamming", 0), (0, "gcc9", "l1", 2),
]


def lcd_params(case, refine=0, stream=0):
    from kmx.lcd import LcdParams
    algo, variant, norm, rec = case
    # focal_length 380: the value the frozen PnP fixtures were generated with
    # (before the default became the D455 fu, 377.229); it only sets the 2D-3D
    # inlier threshold, so the fixtures stay valid vectors for that parameter
    return LcdParams(ransac_2d2d_algorithm=algo, rng_variant=variant, norm=norm, pose_recovery_type=int(rec == 1),
                     ransac_use_1point_3d3d=int(rec != 2), refine_pose=refine, rng_stream=stream, focal_length=380.0)


def run_lcd_oracle(pool, case, refine=0, stream=0):
    from oracle import oracle as O
    res, masks = O.lcd_verify(lcd_params(case, refine, stream).to_c(), pool)
    ints = np.array([[r.n_matches, r.mono_inliers, r.stereo_inliers, r.pnp_inliers, r.accepted, r.iterations_2d2d]
                     for r in res], np.int32)
    T = np.array([list(r.T_query_match[:]) for r in res], np.float64)
    return ints, T, masks


def make_refine():
    """lcd_refine.npz: the refine_pose cases on the same pool (added with the
    refinement; the earlier fixtures are not regenerated)."""
    pool = lcd_inputs()
    arrs = {}
    for k, case in enumerate(LCD_REFINE_CASES):
        ints, T, masks = run_lcd_oracle(pool, case, refine=1)
        arrs[f"ints_{k}"], arrs[f"T_{k}"], arrs[f"masks_{k}"] = ints, T, masks
    np.savez_compressed(OUT / "lcd_refine.npz",
                        cases=np.array([[a, v == "gcc11", n == "hamming", r] for a, v, n, r in LCD_REFINE_CASES],
                                       np.int32), **arrs)
    print("lcd_refine.npz", (OUT / "lcd_refine.npz").stat().st_size, "bytes")


def make_stream():
    """lcd_stream.npz: every LCD case under the other LC5 reading (rng_stream
    1, the fork's thread_local engine continued across problems; README.md:35-36)
    on the same pool (added in round 4; the earlier fixtures are not
    regenerated)."""
    pool = lcd_inputs()
    arrs = {}
    for k, case in enumerate(LCD_CASES):
        ints, T, masks = run_lcd_oracle(pool, case, stream=1)
        arrs[f"ints_{k}"], arrs[f"T_{k}"], arrs[f"masks_{k}"] = ints, T, masks
    np.savez_compressed(OUT / "lcd_stream.npz",
                        cases=np.array([[a, v == "gcc11", n == "hamming", r] for a, v, n, r in LCD_CASES], np.int32),
                        **arrs)
    print("lcd_stream.npz", (OUT / "lcd_stream.npz").stat().st_size, "bytes")


def main():
    g, P, X0 = dpgo_inputs()
    out = run_dpgo_oracle(g, P.r, X0)
    np.savez_compressed(OUT / "dpgo_small.npz", r=np.int32(P.r), n_poses=g.n_poses, r1=g.r1, p1=g.p1, r2=g.r2,
                        p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau, weight=g.weight, fixed=g.fixed, X0=X0,
                        **out)
    pool = lcd_inputs()
    arrs = {}
    for k, case in enumerate(LCD_CASES):
        ints, T, masks = run_lcd_oracle(pool, case)
        arrs[f"ints_{k}"], arrs[f"T_{k}"], arrs[f"masks_{k}"] = ints, T, masks
    np.savez_compressed(OUT / "lcd_small.npz", n_feats=pool.n_feats, desc=pool.desc, bearings=pool.bearings,
                        points=pool.points, cand_query=pool.cand_query, cand_match=pool.cand_match,
                        cases=np.array([[a, v == "gcc11", n == "hamming", r] for a, v, n, r in LCD_CASES], np.int32),
                        **arrs)
    for f in ("dpgo_small.npz", "lcd_small.npz"):
        print(f, (OUT / f).stat().st_size, "bytes")


if __name__ == "__main__":
    if sys.argv[1:] == ["--refine"]:
        make_refine()
    elif sys.argv[1:] == ["--stream"]:
        make_stream()
    else:
        main()
