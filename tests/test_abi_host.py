"""C-ABI library and host logic (no GPU needed)."""
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_library_exports_every_header_symbol():
    from kmx import abi
    L = abi.lib()
    hdr = (ROOT / "include" / "kmx_abi.h").read_text()
    names = sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(kmx_\w+)\s*\(", hdr, re.M)))
    assert len(names) > 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.kmx_abi_version() == abi.ABI_VERSION


def test_runtime_info_names_the_rccl_serving_kmx():
    """which librccl / libamdhip64 libkmx's own calls resolve
    to (dladdr inside the library), their versions, and every copy mapped into
    the process — torch bundles a librccl of the same SONAME, so two copies can
    end up mapped when kmx is loaded first."""
    from kmx import abi
    ri = abi.runtime_info()
    assert ri["rccl_path"].endswith((".so", ".so.1")) or "librccl" in ri["rccl_path"]
    assert ri["rccl_version"] >= 20000 and ri["rccl_header_version"] >= 20000
    assert "libamdhip64" in ri["hip_path"] and ri["hip_runtime_version"] > 0
    assert ri["rccl_path_real"] in ri["mapped_rccl"]
    assert ri["single_rccl"] == (len(ri["mapped_rccl"]) == 1)


def test_no_cpu_fallback_without_gpu():
    from kmx import abi
    if abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    from kmx.dpgo.params import PGOAgentParameters
    from kmx.dpgo.solver import BlockSolver
    with pytest.raises(abi.KmxError):
        BlockSolver(PGOAgentParameters(), 0)
    from kmx.lcd import LoopClosureDetector
    with pytest.raises(abi.KmxError):
        LoopClosureDetector()


def test_params_to_c_and_yaml(tmp_path):
    from kmx.dpgo.params import PGOAgentParameters, error_threshold_at_quantile
    c = PGOAgentParameters(r=6).to_c()
    assert (c.d, c.r, c.tcg_max_iterations, c.robust_cost) == (3, 6, 10, 1)
    assert abs(error_threshold_at_quantile(0.9, 3) - 3.26261) < 1e-4  # sqrt(chi2inv(0.9, 6) = 10.6446)
    from kmx.lcd import LcdParams
    y = tmp_path / "LcdParams.yaml"
    y.write_text("%YAML:1.0\nlowe_ratio: 0.8\nmatcher_type: 4\nransac_max_iterations: 100\n"
                 "min_nr_2d2d_inliers: 12\nransac_threshold_3d3d: 0.25\n")
    p = LcdParams.from_yaml(str(y))
    assert (p.lowe_ratio, p.norm, p.ransac_max_iterations, p.min_nr_2d2d_inliers) == (0.8, "hamming", 100, 12)
    cp = p.to_c()
    assert cp.norm == 1 and cp.ransac_threshold_3d3d == 0.25


def test_reference_lcdparams_yaml_if_present():
    """The reference config loads unmodified (refine_pose: 1 included) and
    maps onto the verification parameters, Stewenius and EPnP included; the
    refinement with PnP recovery is the one combination not built."""
    f = Path("/root/reference/params/D455/LcdParams.yaml")
    if not f.exists():
        pytest.skip("reference not mounted")
    from kmx.lcd import LcdParams
    p = LcdParams.from_yaml(str(f))
    assert p.refine_pose == 1 and p.to_c().refine_pose == 1
    with pytest.raises(ValueError, match="refine_pose"):
        LcdParams.from_yaml(str(f), pose_recovery_type=1)
    assert (p.lowe_ratio, p.norm, p.ransac_max_iterations, p.ransac_probability) == (0.7, "l1", 500, 0.995)
    assert (p.min_nr_2d2d_inliers, p.min_nr_3d3d_inliers, p.ransac_threshold_2d2d) == (10, 5, 1e-6)
    assert (p.ransac_2d2d_algorithm, p.ransac_2d3d_algorithm, p.pose_recovery_type) == (0, 3, 0)
    assert p.to_c().algorithm_2d2d == 0


def test_focal_length_from_camera_file(tmp_path):
    """The PnP threshold's focal length is the camera file's fu (Kimera-VIO's
    LCD converts the pixel threshold with the left camera's intrinsics[0]);
    the default is the D455 left camera's fu (LeftCameraParams.yaml:18)."""
    import numpy as np
    from kmx.lcd import LcdParams
    from kmx.lcd.detector import camera_focal_length
    assert LcdParams().focal_length == 377.229220831
    cam = tmp_path / "LeftCameraParams.yaml"
    cam.write_text("%YAML:1.0\ncamera_id: left_cam\nintrinsics: [400.5, 401.0, 320.0, 240.0]  # [fu, fv, cu, cv]\n")
    y = tmp_path / "LcdParams.yaml"
    y.write_text("%YAML:1.0\nransac_threshold_2d3d: 2\n")
    p = LcdParams.from_yaml(str(y), camera_yaml=str(cam))
    assert p.focal_length == 400.5
    assert p.to_c().ransac_threshold_2d3d == 1.0 - np.cos(np.arctan(2.0 / 400.5))
    bad = tmp_path / "bad.yaml"
    bad.write_text("%YAML:1.0\ncamera_id: x\n")
    with pytest.raises(ValueError, match="intrinsics"):
        camera_focal_length(str(bad))
    ref = Path("/root/reference/params/D455/LeftCameraParams.yaml")
    if ref.exists():
        assert camera_focal_length(str(ref)) == LcdParams().focal_length


@pytest.mark.parametrize("line,msg", [
    ("ransac_2d2d_algorithm: 2", "ransac_2d2d_algorithm"),      # SEVENPT
    ("ransac_2d3d_algorithm: 1", "ransac_2d3d_algorithm"),      # KNEIP
    ("matcher_type: 1", "matcher_type"),                        # FLANN
    ("ransac_use_2point_2d2d: 1", "ransac_use_2point_2d2d"),
    ("optimize_3d3d_pose_from_inliers: 1", "optimize_3d3d"),
    ("no_such_key: 3", "unknown"),
])
def test_lcdparams_yaml_rejects_unbuilt(tmp_path, line, msg):
    from kmx.lcd import LcdParams
    y = tmp_path / "LcdParams.yaml"
    y.write_text("%YAML:1.0\nlowe_ratio: 0.7\n" + line + "\n")
    with pytest.raises(ValueError, match=msg):
        LcdParams.from_yaml(str(y))
    y.write_text("%YAML:1.0\nnfeatures: 700\ngnc_alpha: 0.9\nransac_2d2d_algorithm: 1\nmatcher_type: 5\n")
    p = LcdParams.from_yaml(str(y))  # out-of-path keys are ignored by name
    assert (p.ransac_2d2d_algorithm, p.norm) == (1, "hamming")


def test_synthetic_generators_are_deterministic():
    from kmx.synth import make_pose_graph
    from kmx.synth.lcd import make_lcd_pool
    a, b = make_pose_graph(3, 300, 900, seed=5), make_pose_graph(3, 300, 900, seed=5)
    for f in ("r1", "p1", "r2", "p2", "R", "t", "fixed"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    assert a.m == 900 and a.n_total == 300
    sh = a.r1 != a.r2
    assert 0 < sh.sum() < a.m
    # measurements are rotations
    assert np.abs(np.einsum("nji,njk->nik", a.R, a.R) - np.eye(3)).max() < 1e-12
    p, q = make_lcd_pool(8, 64, seed=1), make_lcd_pool(8, 64, seed=1)
    assert np.array_equal(p.desc, q.desc) and np.array_equal(p.bearings, q.bearings)
    assert np.allclose(np.linalg.norm(p.bearings, axis=-1), 1.0)


def test_robot_ranges_and_lifting():
    from kmx.dpgo.driver import robot_ranges
    from kmx.synth import lifting_matrix
    assert robot_ranges(8, 3) == [(0, 2), (2, 5), (5, 8)]
    assert robot_ranges(8, 8)[7] == (7, 8)
    Y = lifting_matrix(5)
    assert np.abs(Y.T @ Y - np.eye(3)).max() < 1e-14
