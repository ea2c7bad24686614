"""The callers either side of the path, with the HIP path in the middle
(VERDICT r2 "next round" item 7):

  f1 + f4 + dpgo + f3  a keyframe-level 2-robot team taken through submap
      coarsening and the PoseGraph message (f1), robot 1 aligned to robot 0's
      frame by robust single-pose averaging (f4), RBCD + GNC rounds on the HIP
      solver with dpgo_log_<robot>.csv written by RBCDDriver(log_dir=...),
      keyframe trajectories rebuilt from the optimised submap poses and written
      as kimera_distributed_poses_tum_<robot>.tum; everything compared with the
      same flow on the CPU restatement: per-round tCG counts equal, poses and
      TUM rows within 1e-6, dpgo_log rows equal (rel_change within 1e-9 abs);
  f3 (LCD)  the LCD logs and loop_closures.csv written from the HIP
      verification and read back through the lc_result.py:115-196 reader
      contract: identical to the files written from the restatement.
"""
import numpy as np
import pytest

from kmx.dpgo.params import PGOAgentParameters

pytestmark = pytest.mark.gpu


def _run(sg, X0, P, log_dir, solver=None, rounds=25):
    from kmx.dpgo.driver import RBCDDriver
    drv = RBCDDriver(P, sg, device=0, solver=solver, log_dir=str(log_dir))
    drv.initialize(X0)
    return drv, [drv.step(with_stats=True) for _ in range(rounds)]


@pytest.mark.timeout(600)
def test_submap_team_through_hip_to_tum_and_dpgo_log(gpu, tmp_path):
    from kmx.io import read_dpgo_log, write_tum
    from tests.mock_solver import OracleBlockSolver
    from tests.submap_team import submap_team
    from tests.test_eval_readers_cpu import _ReaderContract
    g, atlases, sg, X0, align = submap_team()
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 6
    (tmp_path / "gpu").mkdir()
    (tmp_path / "cpu").mkdir()
    dg, sgs = _run(sg, X0, P, tmp_path / "gpu")
    do, sos = _run(sg, X0, P, tmp_path / "cpu", solver=OracleBlockSolver(P))
    try:
        for it, (a, b) in enumerate(zip(sgs, sos)):
            for r in range(sg.n_robots):
                assert a[r]["tcg_iterations"] == b[r]["tcg_iterations"], (it, r)
                assert a[r]["accepted"] == b[r]["accepted"], (it, r)
        assert dg.weight_updates == do.weight_updates >= 2
        anchor = dg.solver.get_iterate(0)[0].copy()
        for r, at in enumerate(atlases):
            d = np.linalg.norm((dg.solver.get_iterate(r) - do.solver.get_iterate(r)).reshape(-1, 20), axis=1).max()
            assert d <= 1e-6, (r, d)
            stamps = np.array(at.kf_stamp, np.float64) * 1e-9
            files = {}
            for side, drv in (("gpu", dg), ("cpu", do)):
                T = drv.solver.trajectory(r, anchor)  # submap poses in the anchor frame [n_sub, 12]
                Rk, tk = at.keyframe_trajectory(T[:, :9].reshape(-1, 3, 3), T[:, 9:])
                files[side] = tmp_path / side / f"kimera_distributed_poses_tum_{r}.tum"
                write_tum(files[side], stamps, np.concatenate([Rk.reshape(-1, 9), tk], axis=1))
            a = _ReaderContract.read_groundtruth_tum(str(files["gpu"]))
            b = _ReaderContract.read_groundtruth_tum(str(files["cpu"]))
            assert len(a) == len(b) == len(at.kf_submap)
            assert np.array_equal(a["timestamp"].values, b["timestamp"].values)
            assert np.abs(a[["tx", "ty", "tz", "qx", "qy", "qz", "qw"]].values
                          - b[["tx", "ty", "tz", "qx", "qy", "qz", "qw"]].values).max() <= 1e-6
            la = read_dpgo_log(tmp_path / "gpu" / f"dpgo_log_{r}.csv")
            lb = read_dpgo_log(tmp_path / "cpu" / f"dpgo_log_{r}.csv")
            assert len(la) == len(lb) == 25
            for x, y in zip(la, lb):
                assert {k: v for k, v in x.items() if k != "rel_change"} == \
                    {k: v for k, v in y.items() if k != "rel_change"}
                assert abs(x["rel_change"] - y["rel_change"]) <= 1e-9
    finally:
        dg.solver.close()


@pytest.mark.timeout(300)
def test_lcd_outputs_from_hip_read_back(gpu, tmp_path):
    from kmx.io import LoopClosureRecord, write_lcd_logs, write_loop_closures_csv
    from kmx.lcd import LcdParams, LoopClosureDetector
    from kmx.synth.lcd import make_lcd_pool
    from oracle import oracle as O
    from tests.test_eval_readers_cpu import _ReaderContract
    pool = make_lcd_pool(80, 300, seed=4)
    p = LcdParams()
    det = LoopClosureDetector(p)
    det.set_pool(pool)
    got, _ = det.verify(pool.cand_query, pool.cand_match)
    ref, _ = O.lcd_verify(p.to_c(), pool, masks=False)
    ref = [{"accepted": bool(r.accepted), "mono_inliers": r.mono_inliers, "stereo_inliers": r.stereo_inliers,
            "T_query_match": np.array(r.T_query_match[:])} for r in ref]
    stamps = 1_665_000_000_000_000_000 + np.arange(pool.n_frames, dtype=np.int64) * 100_000_000
    parsed = {}
    for side, res in (("gpu", got), ("cpu", ref)):
        d = tmp_path / side
        d.mkdir()
        write_lcd_logs(d / "output_lcd_status.csv", d / "output_lcd_result.csv", pool.cand_query, pool.cand_match,
                       res, stamps_ns=stamps)
        recs = [LoopClosureRecord(0, int(pool.cand_query[k]), 1, int(pool.cand_match[k]),
                                  np.asarray(r["T_query_match"])[:9].reshape(3, 3), np.asarray(r["T_query_match"])[9:],
                                  0.5, r["mono_inliers"], r["stereo_inliers"], int(stamps[pool.cand_query[k]]))
                for k, r in enumerate(res) if r["accepted"]]
        write_loop_closures_csv(d / "loop_closures.csv", recs)
        parsed[side] = _ReaderContract.parse_csv_files(str(d / "loop_closures.csv"), str(d / "output_lcd_status.csv"),
                                                       str(d / "output_lcd_result.csv"))
        for name in ("loop_closures.csv", "output_lcd_status.csv", "output_lcd_result.csv"):
            parsed[side + name] = (d / name).read_bytes()
    inter, intra, rejected = parsed["gpu"]
    assert len(inter) == len(intra) >= 20 and len(rejected) >= 20
    assert parsed["gpu"] == parsed["cpu"]
    for name in ("loop_closures.csv", "output_lcd_status.csv", "output_lcd_result.csv"):
        assert parsed["gpu" + name] == parsed["cpu" + name], name  # the files themselves, byte for byte
