"""BlockSolver: the device handle that holds a set of robot blocks on one GPU.

Thin Python owner of a ``kmx_pgo`` handle (include/kmx_abi.h). Several dpgo
agents (kmx.dpgo.agent.PGOAgent) placed on the same GPU share one BlockSolver,
so their block updates run batched in the same kernel launches.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import abi
from ..abi import check, fptr, i64ptr, iptr, u8ptr
from .params import PGOAgentParameters


class BlockSolver:
    device_pointers = True  # pack/unpack take HIP device pointers
    # every round's k_commit republishes the committed owned public rows (and an
    # accelerated round publishes Y before its exchange), so the table needs an
    # explicit refresh_local only after set_iterate
    publishes_on_commit = True

    def __init__(self, params: PGOAgentParameters, device: int = 0):
        self.params = params
        self.r = params.r
        self.device = device
        L = abi.lib()
        if abi.device_count() <= device:
            raise abi.KmxError(f"no HIP device {device} visible (kmx has no CPU fallback)")
        self._cparams = params.to_c()
        h = C.c_void_p()
        check(L.kmx_pgo_create(C.byref(self._cparams), device, C.byref(h)), "kmx_pgo_create")
        self.h = h
        self.L = L
        self.n_robots = 0
        self.n_poses = None
        self.local = None
        self.m = 0

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.kmx_pgo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream: int):
        check(self.L.kmx_pgo_set_stream(self.h, C.c_void_p(hip_stream)), "kmx_pgo_set_stream")

    def set_tcg_poll(self, mode: int):
        """-1 adaptive (default), 0 blind, 1 polled tCG enqueueing
        (kmx_pgo_set_tcg_poll; identical results in every mode)."""
        check(self.L.kmx_pgo_set_tcg_poll(self.h, int(mode)), "kmx_pgo_set_tcg_poll")

    # ------------------------------------------------- native exchange ---
    native_exchange = True  # kmx_pgo_comm_init / kmx_pgo_set_exchange (RCCL inside the round)

    @staticmethod
    def comm_unique_id() -> bytes:
        """RCCL unique id (rank 0 creates it; every rank passes it to comm_init)."""
        buf = C.create_string_buffer(abi.KMX_COMM_ID_BYTES)
        check(abi.lib().kmx_comm_unique_id(C.cast(buf, C.c_void_p), abi.KMX_COMM_ID_BYTES), "kmx_comm_unique_id")
        return buf.raw

    def comm_init(self, unique_id: bytes, world: int, rank: int, timeout_s: float = 120.0):
        """Non-blocking communicator creation with a deadline (a rank whose
        peers never arrive gets KmxError instead of hanging)."""
        if len(unique_id) != abi.KMX_COMM_ID_BYTES:
            raise ValueError(f"unique id must be {abi.KMX_COMM_ID_BYTES} bytes")
        buf = C.create_string_buffer(bytes(unique_id), abi.KMX_COMM_ID_BYTES)
        check(self.L.kmx_pgo_comm_init(self.h, C.cast(buf, C.c_void_p), int(world), int(rank), float(timeout_s)),
              "kmx_pgo_comm_init")

    @staticmethod
    def runtime_info() -> dict:
        """abi.runtime_info(): the RCCL / HIP libraries serving libkmx."""
        return abi.runtime_info()

    def comm_destroy(self):
        """Drop the communicator and the in-round exchange."""
        check(self.L.kmx_pgo_comm_destroy(self.h), "kmx_pgo_comm_destroy")

    def get_public(self, n_ext: int = 0):
        """(public table [n_public, r, 4], the last exchange's peer status words)."""
        n_pub = self.public_count()[0]
        tab = np.zeros((max(n_pub, 1), self.r, 4))
        ext = np.zeros(max(n_ext, 1))
        check(self.L.kmx_pgo_get_public(self.h, fptr(tab), fptr(ext) if n_ext else None), "kmx_pgo_get_public")
        return tab[:n_pub], ext[:n_ext]

    def set_exchange(self, send_slots, send_counts, recv_slots, recv_counts):
        """The per-peer slot lists (kmx.dpgo.driver.exchange_plan); from now on
        every round starts with the RCCL exchange on this handle's stream."""
        ss = np.ascontiguousarray(send_slots, dtype=np.int32)
        rs = np.ascontiguousarray(recv_slots, dtype=np.int32)
        sc = np.ascontiguousarray(send_counts, dtype=np.int64)
        rc = np.ascontiguousarray(recv_counts, dtype=np.int64)
        check(self.L.kmx_pgo_set_exchange(self.h, iptr(ss), i64ptr(sc), iptr(rs), i64ptr(rc)), "kmx_pgo_set_exchange")

    def exchange(self):
        """One native exchange now (kmx_pgo_exchange), outside a round."""
        check(self.L.kmx_pgo_exchange(self.h), "kmx_pgo_exchange")

    # ----------------------------------------------------------- graph ---
    def set_graph(self, n_poses, local, r1, p1, r2, p2, R, t, kappa, tau, weight, fixed):
        self.n_poses = np.ascontiguousarray(n_poses, dtype=np.int32)
        self.n_robots = int(self.n_poses.shape[0])
        self.local = np.ascontiguousarray(local, dtype=np.uint8)
        arrs = [np.ascontiguousarray(x, dtype=np.int32) for x in (r1, p1, r2, p2)]
        Rf = np.ascontiguousarray(np.asarray(R, dtype=np.float64).reshape(-1))
        tf = np.ascontiguousarray(np.asarray(t, dtype=np.float64).reshape(-1))
        k = np.ascontiguousarray(kappa, dtype=np.float64)
        ta = np.ascontiguousarray(tau, dtype=np.float64)
        w = np.ascontiguousarray(weight, dtype=np.float64)
        fx = np.ascontiguousarray(fixed, dtype=np.uint8)
        m = arrs[0].shape[0]
        for x in arrs[1:] + [k, ta, w, fx]:
            if x.shape[0] != m:
                raise ValueError("edge arrays must have equal length")
        if Rf.shape[0] != 9 * m or tf.shape[0] != 3 * m:
            raise ValueError("R must be [m,3,3] and t [m,3]")
        self.m = m
        check(self.L.kmx_pgo_set_graph(self.h, self.n_robots, iptr(self.n_poses), u8ptr(self.local), m,
                                       *[iptr(a) for a in arrs], fptr(Rf), fptr(tf), fptr(k), fptr(ta),
                                       fptr(w), u8ptr(fx)), "kmx_pgo_set_graph")

    def set_graph_data(self, g, local=None):
        if local is None:
            local = np.ones(g.n_robots, np.uint8)
        self.set_graph(g.n_poses, local, g.r1, g.p1, g.r2, g.p2, g.R, g.t, g.kappa, g.tau, g.weight, g.fixed)

    # --------------------------------------------------------- iterate ---
    def set_iterate(self, robot: int, X: np.ndarray):
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.size != int(self.n_poses[robot]) * 4 * self.r:
            raise ValueError("X must be [n_poses, r, 4]")
        check(self.L.kmx_pgo_set_iterate(self.h, robot, fptr(X)), "kmx_pgo_set_iterate")

    def get_iterate(self, robot: int) -> np.ndarray:
        X = np.empty((int(self.n_poses[robot]), self.r, 4))
        check(self.L.kmx_pgo_get_iterate(self.h, robot, fptr(X)), "kmx_pgo_get_iterate")
        return X

    def public_count(self):
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        check(self.L.kmx_pgo_public_count(self.h, C.byref(a), C.byref(b), C.byref(c)), "kmx_pgo_public_count")
        return a.value, b.value, c.value

    def pack_public(self, dev_ptr: int):
        check(self.L.kmx_pgo_pack_public(self.h, C.c_void_p(dev_ptr)), "kmx_pgo_pack_public")

    def unpack_public(self, dev_ptr: int):
        check(self.L.kmx_pgo_unpack_public(self.h, C.c_void_p(dev_ptr)), "kmx_pgo_unpack_public")

    def gather_public_rows(self, slots_ptr: int, n: int, out_ptr: int):
        check(self.L.kmx_pgo_gather_public_rows(self.h, C.c_void_p(slots_ptr), int(n), C.c_void_p(out_ptr)),
              "kmx_pgo_gather_public_rows")

    def scatter_public_rows(self, slots_ptr: int, n: int, rows_ptr: int):
        check(self.L.kmx_pgo_scatter_public_rows(self.h, C.c_void_p(slots_ptr), int(n), C.c_void_p(rows_ptr)),
              "kmx_pgo_scatter_public_rows")

    def exchange_pack(self, slots_ptr: int, n: int, seg_ptr: int, n_seg: int, out_ptr: int):
        """Rows of n owned slots + this handle's status after each of n_seg
        per-peer segments (kmx_pgo_exchange_pack)."""
        check(self.L.kmx_pgo_exchange_pack(self.h, C.c_void_p(slots_ptr), int(n), C.c_void_p(seg_ptr), int(n_seg),
                                           C.c_void_p(out_ptr)), "kmx_pgo_exchange_pack")

    def exchange_unpack(self, slots_ptr: int, n: int, seg_ptr: int, n_seg: int, in_ptr: int):
        check(self.L.kmx_pgo_exchange_unpack(self.h, C.c_void_p(slots_ptr), int(n), C.c_void_p(seg_ptr),
                                             int(n_seg), C.c_void_p(in_ptr)), "kmx_pgo_exchange_unpack")

    def refresh_local(self):
        check(self.L.kmx_pgo_refresh_local(self.h), "kmx_pgo_refresh_local")

    def set_neighbor_poses(self, robots, poses, X):
        robots = np.ascontiguousarray(robots, dtype=np.int32)
        poses = np.ascontiguousarray(poses, dtype=np.int32)
        X = np.ascontiguousarray(X, dtype=np.float64)
        check(self.L.kmx_pgo_set_neighbor_poses(self.h, robots.shape[0], iptr(robots), iptr(poses), fptr(X)),
              "kmx_pgo_set_neighbor_poses")

    def iterate(self, active=None) -> list[dict]:
        act = np.ones(self.n_robots, np.uint8) if active is None else np.ascontiguousarray(active, dtype=np.uint8)
        stats = (abi.IterStats * self.n_robots)()
        check(self.L.kmx_pgo_iterate(self.h, u8ptr(act), stats), "kmx_pgo_iterate")
        return [s.as_dict() for s in stats]

    def iterate_async(self, rounds: int, refresh_local: bool = True):
        check(self.L.kmx_pgo_iterate_async(self.h, rounds, 1 if refresh_local else 0), "kmx_pgo_iterate_async")

    def sync(self):
        check(self.L.kmx_pgo_sync(self.h), "kmx_pgo_sync")

    def sync_timeout(self, timeout_s: float) -> bool:
        """kmx_pgo_sync with a deadline: False when the stream has not drained
        after timeout_s (kmx_pgo_comm_destroy then aborts the exchange)."""
        rc = self.L.kmx_pgo_sync_timeout(self.h, float(timeout_s))
        if rc == abi.KMX_ETIMEOUT:
            return False
        check(rc, "kmx_pgo_sync_timeout")
        return True

    # ------------------------------------------------------------- GNC ---
    def set_gnc_schedule(self, enabled: bool, inner_iters: int = 20, max_updates: int = 2**31 - 1,
                         rel_change_tol: float = 1e-3):
        """Device-side shouldUpdateMeasurementWeights at every round begin."""
        check(self.L.kmx_pgo_set_gnc_schedule(self.h, 1 if enabled else 0, int(inner_iters),
                                              int(min(max_updates, 2**31 - 1)), float(rel_change_tol)),
              "kmx_pgo_set_gnc_schedule")

    def gnc_state(self) -> dict:
        s = abi.GncState()
        check(self.L.kmx_pgo_get_gnc_state(self.h, C.byref(s)), "kmx_pgo_get_gnc_state")
        return s.as_dict()

    def set_gnc_state(self, state: dict):
        s = abi.GncState()
        s.inner_iter, s.updates = int(state["inner_iter"]), int(state["updates"])
        s.last_fired, s.rounds, s.mu = int(state.get("last_fired", 0)), int(state.get("rounds", 0)), state["mu"]
        check(self.L.kmx_pgo_set_gnc_state(self.h, C.byref(s)), "kmx_pgo_set_gnc_state")

    def status(self) -> np.ndarray:
        """Per-robot relative change of the last block update (inf: none yet)."""
        v = np.full(self.n_robots, np.nan)
        check(self.L.kmx_pgo_get_status(self.h, fptr(v)), "kmx_pgo_get_status")
        return v

    def set_status(self, v: np.ndarray):
        v = np.ascontiguousarray(v, dtype=np.float64)
        check(self.L.kmx_pgo_set_status(self.h, fptr(v)), "kmx_pgo_set_status")

    def memory(self) -> tuple[int, int]:
        """(resident device bytes, bytes per incidence record)."""
        b, rb = C.c_int64(), C.c_int()
        check(self.L.kmx_pgo_memory(self.h, C.byref(b), C.byref(rb)), "kmx_pgo_memory")
        return b.value, rb.value

    def update_weights(self) -> float:
        mu = C.c_double()
        check(self.L.kmx_pgo_update_weights(self.h, C.byref(mu)), "kmx_pgo_update_weights")
        return mu.value

    @property
    def mu(self) -> float:
        mu = C.c_double()
        check(self.L.kmx_pgo_get_mu(self.h, C.byref(mu)), "kmx_pgo_get_mu")
        return mu.value

    @mu.setter
    def mu(self, v: float):
        check(self.L.kmx_pgo_set_mu(self.h, float(v)), "kmx_pgo_set_mu")

    def get_weights(self, base: np.ndarray | None = None) -> np.ndarray:
        w = np.zeros(self.m) if base is None else np.array(base, dtype=np.float64)
        check(self.L.kmx_pgo_get_weights(self.h, fptr(w)), "kmx_pgo_get_weights")
        return w

    def set_weights(self, w: np.ndarray):
        w = np.ascontiguousarray(w, dtype=np.float64)
        check(self.L.kmx_pgo_set_weights(self.h, fptr(w)), "kmx_pgo_set_weights")

    def shared_count(self) -> int:
        n = C.c_int64()
        check(self.L.kmx_pgo_shared_count(self.h, C.byref(n)), "kmx_pgo_shared_count")
        return n.value

    def pack_shared_weights(self, dev_ptr: int):
        check(self.L.kmx_pgo_pack_shared_weights(self.h, C.c_void_p(dev_ptr)), "kmx_pgo_pack_shared_weights")

    def unpack_shared_weights(self, dev_ptr: int):
        check(self.L.kmx_pgo_unpack_shared_weights(self.h, C.c_void_p(dev_ptr)), "kmx_pgo_unpack_shared_weights")

    # --------------------------------------------------------- outputs ---
    def trajectory(self, robot: int, anchor: np.ndarray) -> np.ndarray:
        anchor = np.ascontiguousarray(anchor, dtype=np.float64)
        out = np.empty((int(self.n_poses[robot]), 12))
        check(self.L.kmx_pgo_get_trajectory(self.h, robot, fptr(anchor), fptr(out)), "kmx_pgo_get_trajectory")
        return out

    def eval(self, robot: int, mode: int, V: np.ndarray | None = None):
        n = int(self.n_poses[robot])
        Vin = np.zeros((n, self.r, 4)) if V is None else np.ascontiguousarray(V, dtype=np.float64)
        out = np.empty((n, self.r, 4))
        s = C.c_double()
        check(self.L.kmx_pgo_eval(self.h, robot, mode, fptr(Vin), fptr(out), C.byref(s)), "kmx_pgo_eval")
        return out, s.value

    def local_edges(self, robot: int) -> int:
        m = C.c_int64()
        check(self.L.kmx_pgo_local_edges(self.h, robot, C.byref(m)), "kmx_pgo_local_edges")
        return m.value

    def enable_timing(self, on: bool = True):
        check(self.L.kmx_pgo_enable_timing(self.h, 1 if on else 0), "kmx_pgo_enable_timing")

    def read_counters(self) -> dict:
        c = abi.PgoCounters()
        check(self.L.kmx_pgo_read_counters(self.h, C.byref(c)), "kmx_pgo_read_counters")
        return {name: getattr(c, name) for name, _ in c._fields_}
