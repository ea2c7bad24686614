"""LoopClosureDetector — Kimera-Multi-LCD verification API on MI355X.

Mirrors the verification half of Kimera-Multi-LCD's LoopClosureDetector
(drawio:2550-2609) as called by Kimera-Distributed's verifyLoopSpin
(drawio:2638-2657): computeMatchedIndices -> geometricVerificationNister ->
recoverPose, batched over candidates on the GPU through kmx_lcd_* (C ABI).
Parameters are read with the keys of params/D455/LcdParams.yaml.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .. import abi
from ..abi import check


@dataclass
class LcdParams:
    """LcdParams (params/D455/LcdParams.yaml). matcher_type 3 is BruteForce-L1
    in the reference build (docker/copy/kimera_multi_lcd.patch:33-35); the
    north_star's Hamming matcher is `norm="hamming"`."""
    lowe_ratio: float = 0.7
    norm: str = "l1"
    min_nr_2d2d_inliers: int = 10
    min_nr_3d3d_inliers: int = 5
    ransac_threshold_2d2d: float = 1e-6
    ransac_threshold_3d3d: float = 0.3
    ransac_max_iterations: int = 500
    ransac_probability: float = 0.995
    ransac_randomize: int = 0
    ransac_seed: int = 12345
    rng_variant: str = "gcc9"           # libstdc++ of ROS Noetic (SURVEY.md §0 finding 5)
    ransac_use_1point_3d3d: int = 1     # 1: translation given the 2D-2D rotation; 0: Arun 3-point RANSAC
    # opengv CentralRelativePoseSacProblem::algorithm_t (LcdParams.yaml:73):
    # 0 STEWENIUS (the reference config), 1 NISTER
    ransac_2d2d_algorithm: int = 0
    # opengv AbsolutePoseSacProblem::algorithm_t (LcdParams.yaml:74): 3 EPNP
    ransac_2d3d_algorithm: int = 3
    # PnP pose recovery (pose_recovery_type 1: EPnP RANSAC, LcdParams.yaml:53,57,63,74)
    pose_recovery_type: int = 0
    min_nr_2d3d_inliers: int = 20
    ransac_threshold_2d3d: float = 1.0   # pixels
    focal_length: float = 380.0          # px, converts the 2D-3D threshold to (1 - cos) [U: D455 intrinsics]
    # BoW detection (LcdParams.yaml:3-12)
    use_nss: int = 1
    alpha: float = 0.4
    min_temporal_matches: int = 1
    recent_frames_window: int = 100
    max_db_results: int = 50
    min_nss_factor: float = 0.05
    min_matches_per_island: int = 1
    max_intraisland_gap: int = 3
    max_nrFrames_between_islands: int = 3
    max_nrFrames_between_queries: int = 2
    # stereo pose refinement after an accepted 3D-3D recovery (LcdParams.yaml:14):
    # least-squares T over the 3D-3D inliers (include/kmx_abi.h refine_pose) [U]
    refine_pose: int = 1

    @classmethod
    def from_yaml(cls, path: str, **overrides) -> "LcdParams":
        """Read an OpenCV-FileStorage LcdParams.yaml (the %YAML:1.0 header is
        skipped). `overrides` replace yaml keys (by yaml name) or dataclass
        fields before validation. Every key is accounted for: verification
        and BoW keys map onto fields, keys of stages outside the hot path
        (ORB extraction, the PGO back end, the tracker) are ignored by name,
        and anything else, or a value that selects an algorithm this build
        does not have, raises ValueError (no silent fallback)."""
        import yaml
        text = open(path).read()
        if text.startswith("%YAML"):
            text = text.split("\n", 1)[1] if "\n" in text else ""
        y = dict(yaml.safe_load(text) or {})
        y.update(overrides)
        p = cls()
        for k, v in y.items():
            if k in _YAML_FIELDS:
                setattr(p, k, type(getattr(p, k))(v))
            elif k == "matcher_type":
                # OpenCV DescriptorMatcher::MatcherType; 3 is built as BruteForce-L1
                # (docker/copy/kimera_multi_lcd.patch:33-35)
                mt = int(v)
                if mt not in _MATCHER_NORM:
                    raise ValueError(f"matcher_type {mt} is not built (3: L1, 4/5: Hamming)")
                p.norm = _MATCHER_NORM[mt]
            elif k in _YAML_SELECTORS:
                allowed, field = _YAML_SELECTORS[k]
                if int(v) not in allowed:
                    raise ValueError(f"{k}: {v} is not built (supported: {sorted(allowed)})")
                if field:
                    setattr(p, field, int(v))
            elif k in _YAML_IGNORED:
                continue
            elif k in cls.__dataclass_fields__:
                setattr(p, k, v)
            else:
                raise ValueError(f"unknown LcdParams key {k!r}")
        p.validate()
        return p

    def validate(self):
        if self.norm not in ("l1", "hamming"):
            raise ValueError(f"norm {self.norm!r}")
        if self.ransac_2d2d_algorithm not in (ALGO_STEWENIUS, ALGO_NISTER):
            raise ValueError(f"ransac_2d2d_algorithm {self.ransac_2d2d_algorithm} is not built (0 Stewenius, 1 Nister)")
        if self.ransac_2d3d_algorithm != 3:
            raise ValueError("ransac_2d3d_algorithm: only 3 (EPnP) is built")
        if self.pose_recovery_type not in (0, 1):
            raise ValueError(f"pose_recovery_type {self.pose_recovery_type}")
        if self.ransac_use_1point_3d3d not in (0, 1):
            raise ValueError("ransac_use_1point_3d3d is 0 (Arun 3-point) or 1 (given rotation)")
        if self.rng_variant not in ("gcc9", "gcc11"):
            raise ValueError(f"rng_variant {self.rng_variant!r}")
        if self.refine_pose not in (0, 1):
            raise ValueError(f"refine_pose {self.refine_pose}")
        if self.refine_pose and self.pose_recovery_type == 1:
            raise ValueError("refine_pose: 1 with pose_recovery_type 1 (PnP) is not built (refinement follows the "
                             "3D-3D recovery); set refine_pose 0")

    def to_c(self) -> abi.LcdParams:
        self.validate()
        c = abi.LcdParams()
        c.norm = abi.KMX_NORM_HAMMING if self.norm == "hamming" else abi.KMX_NORM_L1
        c.lowe_ratio = float(self.lowe_ratio)
        c.min_2d2d_inliers = int(self.min_nr_2d2d_inliers)
        c.min_3d3d_inliers = int(self.min_nr_3d3d_inliers)
        c.ransac_threshold_2d2d = float(self.ransac_threshold_2d2d)
        c.ransac_threshold_3d3d = float(self.ransac_threshold_3d3d)
        c.ransac_max_iterations = int(self.ransac_max_iterations)
        c.ransac_probability = float(self.ransac_probability)
        c.ransac_randomize = int(self.ransac_randomize)
        c.ransac_seed = int(self.ransac_seed)
        c.rng_variant = abi.KMX_RNG_GCC11 if self.rng_variant == "gcc11" else abi.KMX_RNG_GCC9
        c.use_1point_3d3d = int(self.ransac_use_1point_3d3d)
        c.algorithm_2d2d = int(self.ransac_2d2d_algorithm)
        c.refine_pose = int(self.refine_pose)
        c.pose_recovery_type = int(self.pose_recovery_type)
        c.min_2d3d_inliers = int(self.min_nr_2d3d_inliers)
        c.ransac_threshold_2d3d = 1.0 - np.cos(np.arctan(float(self.ransac_threshold_2d3d) / float(self.focal_length)))
        return c


ALGO_STEWENIUS = 0
ALGO_NISTER = 1

# yaml keys that are dataclass fields of the same name
_YAML_FIELDS = (
    "lowe_ratio", "min_nr_2d2d_inliers", "min_nr_3d3d_inliers", "ransac_threshold_2d2d",
    "ransac_threshold_3d3d", "ransac_max_iterations", "ransac_probability", "ransac_randomize",
    "ransac_use_1point_3d3d", "pose_recovery_type", "min_nr_2d3d_inliers", "ransac_threshold_2d3d",
    "ransac_2d2d_algorithm", "ransac_2d3d_algorithm",
    "use_nss", "alpha", "min_temporal_matches", "recent_frames_window", "max_db_results",
    "min_nss_factor", "min_matches_per_island", "max_intraisland_gap",
    "max_nrFrames_between_islands", "max_nrFrames_between_queries")
_MATCHER_NORM = {3: "l1", 4: "hamming", 5: "hamming"}
# switches of verification stages: yaml key -> (built values, field or None)
_YAML_SELECTORS = {
    "refine_pose": ({0, 1}, "refine_pose"),           # stereo pose refinement (LcdParams.yaml:14)
    "ransac_use_2point_2d2d": ({0}, None),            # 2-point 2D-2D given rotation (:59)
    "optimize_2d2d_pose_from_inliers": ({0}, None),   # nonlinear refits (:67-69)
    "optimize_3d3d_pose_from_inliers": ({0}, None),
    "optimize_2d3d_pose_from_inliers": ({0}, None),
}
# keys of stages outside the verification hot path (SURVEY.md §8 out of scope):
# ORB extraction (:19-27), the PGO back end (:29-37), the stereo tracker (:48)
_YAML_IGNORED = frozenset((
    "nfeatures", "scale_factor", "nlevels", "edge_threshold", "first_level", "WTA_K", "score_type_id",
    "patch_sze", "fast_threshold", "betweenRotationPrecision", "betweenTranslationPrecision",
    "odom_rot_threshold", "odom_trans_threshold", "pcm_rot_threshold", "pcm_trans_threshold", "gnc_alpha",
    "max_lc_cached_before_optimize", "disparity_threshold"))


class _BatchDesc(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32), ("max_feats", C.c_int32), ("n_feats", C.POINTER(C.c_int32)),
        ("desc", C.POINTER(C.c_uint8)), ("bearings", C.POINTER(C.c_double)), ("points", C.POINTER(C.c_double)),
        ("n_cand", C.c_int32), ("cand_query", C.POINTER(C.c_int32)), ("cand_match", C.POINTER(C.c_int32)),
    ]


class LoopClosureDetector:
    """GPU verification of loop-closure candidates over a resident frame pool
    (the VLC frames Kimera-Distributed holds, drawio:441-505)."""

    def __init__(self, params: LcdParams | None = None, device: int = 0):
        self.params = params or LcdParams()
        L = abi.lib()
        if abi.device_count() <= device:
            raise abi.KmxError(f"no HIP device {device} visible (kmx has no CPU fallback)")
        self._c = self.params.to_c()
        h = C.c_void_p()
        check(L.kmx_lcd_create(C.byref(self._c), device, C.byref(h)), "kmx_lcd_create")
        self.h, self.L = h, L
        self.max_feats = 0

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.kmx_lcd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream: int):
        check(self.L.kmx_lcd_set_stream(self.h, C.c_void_p(hip_stream)), "kmx_lcd_set_stream")

    def set_frames(self, n_feats, desc, bearings, points):
        """Upload the frame pool: desc uint8 [F, N, 32], bearings / points float64 [F, N, 3]."""
        nf = np.ascontiguousarray(n_feats, dtype=np.int32)
        de = np.ascontiguousarray(desc, dtype=np.uint8)
        be = np.ascontiguousarray(bearings, dtype=np.float64)
        pt = np.ascontiguousarray(points, dtype=np.float64)
        F, N = de.shape[0], de.shape[1]
        if de.shape != (F, N, 32) or be.shape != (F, N, 3) or pt.shape != (F, N, 3) or nf.shape != (F,):
            raise ValueError("frame pool shapes must be desc [F,N,32], bearings/points [F,N,3], n_feats [F]")
        d = _BatchDesc()
        d.n_frames, d.max_feats = F, N
        d.n_feats = nf.ctypes.data_as(C.POINTER(C.c_int32))
        d.desc = de.ctypes.data_as(C.POINTER(C.c_uint8))
        d.bearings = be.ctypes.data_as(C.POINTER(C.c_double))
        d.points = pt.ctypes.data_as(C.POINTER(C.c_double))
        check(self.L.kmx_lcd_set_frames(self.h, C.byref(d)), "kmx_lcd_set_frames")
        self.max_feats = N

    def set_pool(self, pool):
        self.set_frames(pool.n_feats, pool.desc, pool.bearings, pool.points)

    def verify(self, cand_query, cand_match, with_masks: bool = False):
        """Verify candidates; returns (list of result dicts, masks or None).
        masks[c, j]: bit0 = 2D-2D inlier, bit1 = 3D-3D inlier, j = position in
        the candidate's match list (computeMatchedIndices order)."""
        cq = np.ascontiguousarray(cand_query, dtype=np.int32)
        cm = np.ascontiguousarray(cand_match, dtype=np.int32)
        n = cq.shape[0]
        res = (abi.LcdResult * max(n, 1))()
        masks = np.zeros((n, self.max_feats), np.uint8) if with_masks else None
        check(self.L.kmx_lcd_verify(self.h, n, cq.ctypes.data_as(C.POINTER(C.c_int32)),
                                    cm.ctypes.data_as(C.POINTER(C.c_int32)), res,
                                    masks.ctypes.data_as(C.POINTER(C.c_uint8)) if with_masks else None),
              "kmx_lcd_verify")
        out = []
        for i in range(n):
            r = res[i]
            out.append({"n_matches": r.n_matches, "mono_inliers": r.mono_inliers,
                        "stereo_inliers": r.stereo_inliers, "pnp_inliers": r.pnp_inliers,
                        "accepted": bool(r.accepted),
                        "iterations_2d2d": r.iterations_2d2d, "T_query_match": np.array(r.T_query_match[:])})
        return out, masks

    def verify_async(self, cand_query, cand_match):
        cq = np.ascontiguousarray(cand_query, dtype=np.int32)
        cm = np.ascontiguousarray(cand_match, dtype=np.int32)
        check(self.L.kmx_lcd_verify_async(self.h, cq.shape[0], cq.ctypes.data_as(C.POINTER(C.c_int32)),
                                          cm.ctypes.data_as(C.POINTER(C.c_int32))), "kmx_lcd_verify_async")

    def sync(self):
        check(self.L.kmx_lcd_sync(self.h), "kmx_lcd_sync")

    def enable_timing(self, on: bool = True):
        check(self.L.kmx_lcd_enable_timing(self.h, 1 if on else 0), "kmx_lcd_enable_timing")

    def read_timing(self) -> dict:
        """Device times (ms) of the kNN2 and RANSAC launches of the last evented
        verification."""
        a, b = C.c_double(), C.c_double()
        check(self.L.kmx_lcd_read_timing(self.h, C.byref(a), C.byref(b)), "kmx_lcd_read_timing")
        return {"knn_ms": a.value, "ransac_ms": b.value}

    # computeMatchedIndices on two descriptor sets (single pair)
    @staticmethod
    def compute_matched_indices(desc_query, desc_match, lowe_ratio: float = 0.7, norm: str = "l1"):
        q = np.ascontiguousarray(desc_query, dtype=np.uint8)
        m = np.ascontiguousarray(desc_match, dtype=np.uint8)
        pairs = np.empty((max(q.shape[0], 1), 2), np.int32)
        k = C.c_int32()
        nrm = abi.KMX_NORM_HAMMING if norm == "hamming" else abi.KMX_NORM_L1
        check(abi.lib().kmx_lcd_knn2(nrm, float(lowe_ratio), q.ctypes.data_as(C.POINTER(C.c_uint8)), q.shape[0],
                                     m.ctypes.data_as(C.POINTER(C.c_uint8)), m.shape[0],
                                     pairs.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(k)),
              "kmx_lcd_knn2")
        return pairs[: k.value, 0].copy(), pairs[: k.value, 1].copy()
