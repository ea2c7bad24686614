"""ctypes binding of include/kmx_abi.h (the drop-in C ABI).

The product path has exactly one backend: the in-tree HIP library
``kmx/libkmx.so`` built for gfx950 by ``csrc/Makefile``. There is no CPU
fallback: if the library is missing or no HIP device is visible, the handles
raise ``KmxError`` (the CPU restatement in ``oracle/`` is test infrastructure
and is never reached from here).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_LIB_PATH = Path(__file__).resolve().parent / "libkmx.so"

KMX_OK = 0
KMX_ETIMEOUT = -6
ABI_VERSION = 8  # include/kmx_abi.h KMX_ABI_VERSION this binding is written for
KMX_COST_L2 = 0
KMX_COMM_ID_BYTES = 128  # include/kmx_abi.h (ncclUniqueId)
KMX_COST_GNC_TLS = 1
KMX_SCHEDULE_SEQUENTIAL = 0
KMX_SCHEDULE_CONCURRENT = 1
KMX_EVAL_COST_EGRAD = 0
KMX_EVAL_EHESS = 1
KMX_EVAL_RGRAD = 2
KMX_EVAL_RHESS = 3
KMX_EVAL_PRECON = 4
KMX_EVAL_RETRACT = 5
KMX_NORM_L1 = 0
KMX_NORM_HAMMING = 1
KMX_RNG_GCC9 = 0
KMX_RNG_GCC11 = 1
KMX_LCD_STAGE_2D2D = 1
KMX_LCD_STAGE_RECOVER = 2

TCG_STOP_NAMES = {0: "none", 1: "negative_curvature", 2: "exceeded_trust_region",
                  3: "linear", 4: "superlinear", 5: "max_iterations", 6: "skipped"}


class KmxError(RuntimeError):
    pass


class PgoParams(C.Structure):
    _fields_ = [
        ("d", C.c_int), ("r", C.c_int), ("rtr_iterations", C.c_int),
        ("tcg_max_iterations", C.c_int), ("tcg_kappa", C.c_double),
        ("tcg_theta", C.c_double), ("rtr_initial_radius", C.c_double),
        ("rtr_max_radius", C.c_double), ("rtr_accept_rho", C.c_double),
        ("gradnorm_tol", C.c_double), ("use_preconditioner", C.c_int),
        ("precond_shift", C.c_double), ("robust_cost", C.c_int),
        ("gnc_barc", C.c_double), ("gnc_mu_init", C.c_double),
        ("gnc_mu_step", C.c_double), ("acceleration", C.c_int), ("restart_interval", C.c_int),
        ("method", C.c_int), ("tcg_form", C.c_int), ("rgd_stepsize", C.c_double), ("tile_incidences", C.c_int),
        ("reserved", C.c_int),
    ]


class IterStats(C.Structure):
    _fields_ = [
        ("updated", C.c_int), ("tcg_iterations", C.c_int), ("tcg_stop", C.c_int),
        ("accepted", C.c_int), ("f_init", C.c_double), ("gradnorm_init", C.c_double),
        ("f_final", C.c_double), ("rho", C.c_double), ("radius", C.c_double),
        ("rel_change", C.c_double), ("edges", C.c_int64), ("hessvecs", C.c_int64),
    ]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_}
        d["tcg_stop"] = TCG_STOP_NAMES.get(self.tcg_stop, str(self.tcg_stop))
        return d


class PgoCounters(C.Structure):
    _fields_ = [
        ("hessvec_ms_total", C.c_double), ("hessvec_launches", C.c_int64),
        ("hessvec_alg_bytes", C.c_double), ("edges_iters", C.c_int64),
        ("block_updates", C.c_int64), ("hessvecs", C.c_int64), ("gnc_updates", C.c_int64),
    ]


class GncState(C.Structure):
    _fields_ = [
        ("inner_iter", C.c_int32), ("updates", C.c_int32), ("last_fired", C.c_int32),
        ("rounds", C.c_int32), ("mu", C.c_double), ("reserved", C.c_double * 3),
    ]

    def as_dict(self) -> dict:
        return {"inner_iter": self.inner_iter, "updates": self.updates, "last_fired": bool(self.last_fired),
                "rounds": self.rounds, "mu": self.mu}


class LcdParams(C.Structure):
    _fields_ = [
        ("norm", C.c_int), ("lowe_ratio", C.c_double), ("min_2d2d_inliers", C.c_int),
        ("min_3d3d_inliers", C.c_int), ("ransac_threshold_2d2d", C.c_double),
        ("ransac_threshold_3d3d", C.c_double), ("ransac_max_iterations", C.c_int),
        ("ransac_probability", C.c_double), ("ransac_randomize", C.c_int),
        ("ransac_seed", C.c_uint32), ("rng_variant", C.c_int),
        ("use_1point_3d3d", C.c_int), ("pose_recovery_type", C.c_int), ("min_2d3d_inliers", C.c_int),
        ("ransac_threshold_2d3d", C.c_double), ("algorithm_2d2d", C.c_int), ("refine_pose", C.c_int),
        ("rng_stream", C.c_int), ("reserved", C.c_int * 1),
    ]


class LcdResult(C.Structure):
    _fields_ = [
        ("n_matches", C.c_int32), ("mono_inliers", C.c_int32),
        ("stereo_inliers", C.c_int32), ("accepted", C.c_int32),
        ("iterations_2d2d", C.c_int32), ("pnp_inliers", C.c_int32),
        ("T_query_match", C.c_double * 12),
    ]


_lib = None


def lib() -> C.CDLL:
    """Load libkmx.so (once). Raises KmxError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("KMX_LIB", _LIB_PATH))
    if not path.exists():
        raise KmxError(
            f"HIP library {path} not found: build it with `make -C kimera-multi_amd/csrc` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    L = C.CDLL(str(path))
    P, i32, i64, f64, u8 = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_uint8
    pi32, pf64, pu8, pi64 = C.POINTER(i32), C.POINTER(f64), C.POINTER(u8), C.POINTER(i64)
    sig = {
        "kmx_last_error": ([], C.c_char_p),
        "kmx_abi_version": ([], C.c_int),
        "kmx_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "kmx_pgo_create": ([C.POINTER(PgoParams), C.c_int, C.POINTER(P)], C.c_int),
        "kmx_pgo_destroy": ([P], C.c_int),
        "kmx_pgo_set_stream": ([P, P], C.c_int),
        "kmx_pgo_set_tcg_poll": ([P, C.c_int], C.c_int),
        "kmx_comm_unique_id": ([P, i64], C.c_int),
        "kmx_runtime_info": ([C.c_char_p, i64], C.c_int),
        "kmx_pgo_comm_init": ([P, P, C.c_int, C.c_int, f64], C.c_int),
        "kmx_pgo_comm_destroy": ([P], C.c_int),
        "kmx_pgo_get_public": ([P, pf64, pf64], C.c_int),
        "kmx_pgo_set_exchange": ([P, pi32, pi64, pi32, pi64], C.c_int),
        "kmx_pgo_exchange": ([P], C.c_int),
        "kmx_pgo_set_graph": ([P, C.c_int, pi32, pu8, i64, pi32, pi32, pi32, pi32,
                               pf64, pf64, pf64, pf64, pf64, pu8], C.c_int),
        "kmx_pgo_set_iterate": ([P, C.c_int, pf64], C.c_int),
        "kmx_pgo_get_iterate": ([P, C.c_int, pf64], C.c_int),
        "kmx_pgo_public_count": ([P, pi64, pi64, pi64], C.c_int),
        "kmx_pgo_pack_public": ([P, P], C.c_int),
        "kmx_pgo_unpack_public": ([P, P], C.c_int),
        "kmx_pgo_refresh_local": ([P], C.c_int),
        "kmx_pgo_gather_public_rows": ([P, P, i64, P], C.c_int),
        "kmx_pgo_scatter_public_rows": ([P, P, i64, P], C.c_int),
        "kmx_pgo_exchange_pack": ([P, P, i64, P, C.c_int, P], C.c_int),
        "kmx_pgo_exchange_unpack": ([P, P, i64, P, C.c_int, P], C.c_int),
        "kmx_pgo_set_neighbor_poses": ([P, i64, pi32, pi32, pf64], C.c_int),
        "kmx_pgo_iterate": ([P, pu8, C.POINTER(IterStats)], C.c_int),
        "kmx_pgo_iterate_async": ([P, C.c_int, C.c_int], C.c_int),
        "kmx_pgo_sync": ([P], C.c_int),
        "kmx_pgo_sync_timeout": ([P, f64], C.c_int),
        "kmx_pgo_debug_step_stamps": ([P, i64], C.c_int),
        "kmx_pgo_update_weights": ([P, pf64], C.c_int),
        "kmx_pgo_get_mu": ([P, pf64], C.c_int),
        "kmx_pgo_set_mu": ([P, f64], C.c_int),
        "kmx_pgo_set_gnc_schedule": ([P, C.c_int, C.c_int, C.c_int, f64], C.c_int),
        "kmx_pgo_get_gnc_state": ([P, C.POINTER(GncState)], C.c_int),
        "kmx_pgo_set_gnc_state": ([P, C.POINTER(GncState)], C.c_int),
        "kmx_pgo_get_status": ([P, pf64], C.c_int),
        "kmx_pgo_set_status": ([P, pf64], C.c_int),
        "kmx_pgo_memory": ([P, pi64, C.POINTER(C.c_int)], C.c_int),
        "kmx_pgo_get_weights": ([P, pf64], C.c_int),
        "kmx_pgo_set_weights": ([P, pf64], C.c_int),
        "kmx_pgo_shared_count": ([P, pi64], C.c_int),
        "kmx_pgo_pack_shared_weights": ([P, P], C.c_int),
        "kmx_pgo_unpack_shared_weights": ([P, P], C.c_int),
        "kmx_pgo_get_trajectory": ([P, C.c_int, pf64, pf64], C.c_int),
        "kmx_pgo_eval": ([P, C.c_int, C.c_int, pf64, pf64, pf64], C.c_int),
        "kmx_pgo_local_edges": ([P, C.c_int, pi64], C.c_int),
        "kmx_pgo_enable_timing": ([P, C.c_int], C.c_int),
        "kmx_pgo_read_counters": ([P, C.POINTER(PgoCounters)], C.c_int),
    }
    pu32 = C.POINTER(C.c_uint32)
    sig.update({
        "kmx_lcd_knn2": ([C.c_int, C.c_double, pu8, i32, pu8, i32, pi32, pi32], C.c_int),
        "kmx_lcd_create": ([C.POINTER(LcdParams), C.c_int, C.POINTER(P)], C.c_int),
        "kmx_lcd_destroy": ([P], C.c_int),
        "kmx_lcd_set_stream": ([P, P], C.c_int),
        "kmx_lcd_set_frames": ([P, P], C.c_int),
        "kmx_lcd_add_frames": ([P, i32, i32, pi32, pu8, pf64, pf64, pi32], C.c_int),
        "kmx_lcd_pool_info": ([P, pi32, pi32, pi32], C.c_int),
        "kmx_lcd_match": ([P, i32, pi32, pi32, pi32, pi32], C.c_int),
        "kmx_lcd_verify": ([P, i32, pi32, pi32, C.POINTER(LcdResult), pu8], C.c_int),
        "kmx_lcd_verify_async": ([P, i32, pi32, pi32], C.c_int),
        "kmx_lcd_verify_matches": ([P, i32, pi32, pi32, pi64, pi32, pi32, C.c_int, pf64,
                                    C.POINTER(LcdResult), pu8], C.c_int),
        "kmx_lcd_sync": ([P], C.c_int),
        "kmx_lcd_enable_timing": ([P, C.c_int], C.c_int),
        "kmx_lcd_read_timing": ([P, pf64, pf64], C.c_int),
        "kmx_bow_create": ([C.c_int, C.POINTER(P)], C.c_int),
        "kmx_bow_destroy": ([P], C.c_int),
        "kmx_bow_set_stream": ([P, P], C.c_int),
        "kmx_bow_set_database": ([P, i32, i32, pi64, pu32, pf64], C.c_int),
        "kmx_bow_query": ([P, i32, pi64, pu32, pf64, pi32, i32, pi32, pi32, pf64], C.c_int),
        "kmx_bow_query_async": ([P, i32, pi64, pu32, pf64, pi32, i32], C.c_int),
        "kmx_bow_sync": ([P], C.c_int),
        "kmx_bow_score_pairs": ([P, i32, pi64, pu32, pf64, pi64, pu32, pf64, pf64], C.c_int),
    })
    for name, (argt, rest) in sig.items():
        if not hasattr(L, name):
            raise KmxError(f"{path} lacks the entry point {name}: rebuild it")
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    if L.kmx_abi_version() != ABI_VERSION:
        raise KmxError(f"{path} implements ABI {L.kmx_abi_version()}, this binding needs {ABI_VERSION}: rebuild it")
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != KMX_OK:
        msg = lib().kmx_last_error().decode(errors="replace")
        raise KmxError(f"{what} failed ({rc}): {msg}")


def device_count() -> int:
    n = C.c_int(0)
    check(lib().kmx_device_count(C.byref(n)), "kmx_device_count")
    return n.value


def fptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous, (a.dtype, a.flags)
    return a.ctypes.data_as(C.POINTER(C.c_double))


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def i64ptr(a: np.ndarray):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def u32ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def u8ptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def runtime_info() -> dict:
    """Where libkmx's RCCL / HIP calls resolve in this process, with versions
    (kmx_runtime_info), plus every librccl / libamdhip64 mapped into the
    process (/proc/self/maps): torch ships a librccl.so.1 of the same SONAME,
    so which copy serves kmx depends on load order."""
    import json
    buf = C.create_string_buffer(4096)
    check(lib().kmx_runtime_info(buf, 4096), "kmx_runtime_info")
    info = json.loads(buf.value.decode())
    import re
    mapped = {"librccl": set(), "libamdhip64": set()}
    # the core libraries only, by basename (librccl.so, librccl.so.1, ...): an
    # RCCL plugin such as librccl-net.so is not a second copy of RCCL
    core = {k: re.compile(rf"^{k}\.so(\.\d+)*$") for k in mapped}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6:
                    path = parts[-1]
                    for k in mapped:
                        if core[k].match(os.path.basename(path)):
                            mapped[k].add(os.path.realpath(path))
    except OSError:
        pass
    info["mapped_rccl"] = sorted(mapped["librccl"])
    info["mapped_hip"] = sorted(mapped["libamdhip64"])
    info["rccl_path_real"] = os.path.realpath(info["rccl_path"]) if info["rccl_path"] != "?" else "?"
    info["single_rccl"] = len(info["mapped_rccl"]) <= 1 and (
        not info["mapped_rccl"] or info["rccl_path_real"] in info["mapped_rccl"])
    return info
