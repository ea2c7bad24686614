"""CPU stand-in for kmx.dpgo.solver.BlockSolver used ONLY by the gloo tests of
the multi-process driver path and the CPU pipeline tests: the same interface
(exchange pack / unpack through raw pointers with the status word after every
peer segment, the round-begin GNC schedule, the status of the last block
updates) on top of the CPU restatement. It is test infrastructure (imports
oracle/); the schedule is kmx.dpgo.schedule.GncSchedule, the host mirror of
the device rule in csrc/pgo.hip."""
import ctypes as C

import os

import numpy as np

from kmx.dpgo.schedule import GncSchedule
from oracle.oracle import OraclePGO


class OracleBlockSolver:
    def __init__(self, params):
        self.params = params
        self.r = params.r
        self.gnc = GncSchedule.from_params(params)
        self.gnc_on = False
        self.ext = np.zeros(0)

    def set_stream(self, s):  # pragma: no cover - CPU only
        pass

    def set_graph_data(self, g, local):
        self.g = g
        self.n_robots = g.n_robots
        self.local = np.asarray(local, np.uint8)
        self.o = OraclePGO(self.params.to_c(), g)
        sh = g.r1 != g.r2
        keys = np.unique(np.concatenate([(g.r1[sh].astype(np.int64) << 32) | g.p1[sh],
                                         (g.r2[sh].astype(np.int64) << 32) | g.p2[sh]]))
        self.pub_robot = (keys >> 32).astype(np.int32)
        self.pub_pose = (keys & 0xFFFFFFFF).astype(np.int32)
        own = self.local[self.pub_robot] == 1
        idx = np.nonzero(own)[0]
        self.first_owned = int(idx[0]) if idx.size else 0
        self.n_owned = int(idx.size)
        self.shared_edges = np.nonzero(sh)[0]
        self.relc = np.where(np.asarray(g.n_poses) > 0, np.inf, 0.0)

    def public_count(self):
        return int(self.pub_robot.shape[0]), self.first_owned, self.n_owned

    def local_edges(self, a):
        return self.o.local_edges(a)

    def set_iterate(self, a, X):
        self.o.set_iterate(a, X)

    def get_iterate(self, a):
        return self.o.get_iterate(a)

    def _rows(self):
        return 4 * self.r

    # ------------------------------------------------------- exchange ---
    @staticmethod
    def _i32(ptr, n):
        return np.frombuffer((C.c_int32 * n).from_address(ptr), dtype=np.int32).copy()

    def exchange_pack(self, slots_ptr, n, seg_ptr, n_seg, out_ptr):
        self.o.accel_pre(self.local)  # accelerated rounds exchange Y
        ps = self._rows()
        seg = self._i32(seg_ptr, n_seg + 1) if n_seg else np.array([0, n], np.int32)
        sl = self._i32(slots_ptr, n) if n else np.zeros(0, np.int32)
        X = np.ascontiguousarray(self.o.get_x_rows(self.pub_robot[sl], self.pub_pose[sl])).reshape(n, ps)
        tot = n * ps + n_seg
        buf = np.frombuffer((C.c_double * max(tot, 1)).from_address(out_ptr), dtype=np.float64)
        mine = float(np.max(self.relc[self.local == 1])) if self.local.any() else 0.0
        for k in range(max(n_seg, 1)):
            a, b = int(seg[k]), int(seg[k + 1])
            buf[a * ps + k: b * ps + k] = X[a:b].reshape(-1)
            if n_seg:
                buf[b * ps + k] = mine

    def exchange_unpack(self, slots_ptr, n, seg_ptr, n_seg, in_ptr):
        ps = self._rows()
        seg = self._i32(seg_ptr, n_seg + 1) if n_seg else np.array([0, n], np.int32)
        sl = self._i32(slots_ptr, n) if n else np.zeros(0, np.int32)
        tot = n * ps + n_seg
        buf = np.frombuffer((C.c_double * max(tot, 1)).from_address(in_ptr), dtype=np.float64).copy()
        rows = np.empty((n, ps))
        ext = []
        for k in range(max(n_seg, 1)):
            a, b = int(seg[k]), int(seg[k + 1])
            rows[a:b] = buf[a * ps + k: b * ps + k].reshape(-1, ps)
            if n_seg:
                ext.append(buf[b * ps + k])
        if n:
            self.o.set_nbr_rows(self.pub_robot[sl], self.pub_pose[sl], rows.reshape(n, self.r, 4))
            self._table()[sl] = rows.reshape(n, self.r, 4)
        self.ext = np.array(ext)

    def _table(self):
        if getattr(self, "pubtab", None) is None:
            self.pubtab = np.zeros((self.pub_robot.shape[0], self.r, 4))
        return self.pubtab

    def get_public(self, n_ext=0):
        """The neighbour table as installed by refresh_local / exchange_unpack."""
        return self._table().copy(), np.array(self.ext[:n_ext], dtype=np.float64)

    def refresh_local(self):
        self.o.accel_pre(self.local)  # accelerated rounds publish Y
        X = self.o.get_x_rows(self.pub_robot, self.pub_pose)
        own = self.local[self.pub_robot] == 1
        self.o.set_nbr_rows(self.pub_robot[own], self.pub_pose[own], X[own])
        self._table()[own] = X[own]

    # --------------------------------------------------------- rounds ---
    def set_gnc_schedule(self, enabled, inner_iters=20, max_updates=2**31 - 1, rel_change_tol=1e-3):
        self.gnc_on = bool(enabled)
        self.gnc.inner_iters, self.gnc.max_updates = int(inner_iters), int(max_updates)
        self.gnc.rel_change_tol = float(rel_change_tol)

    def gnc_state(self):
        return {"inner_iter": self.gnc.inner, "updates": self.gnc.updates, "mu": self.o.mu}

    def set_gnc_state(self, state):
        self.gnc.inner, self.gnc.updates = int(state["inner_iter"]), int(state["updates"])
        self.o.mu = float(state["mu"])

    def status(self):
        return self.relc.copy()

    def set_status(self, v):
        self.relc = np.array(v, dtype=np.float64)

    def _round(self, active):
        team = np.concatenate([self.relc[self.local == 1], self.ext])
        if self.gnc_on and self.gnc.should_update(team):
            self.update_weights()
        st = self.o.iterate_nbr(np.asarray(active, np.uint8) & self.local)
        for a, s in enumerate(st):
            if s["updated"]:
                self.relc[a] = s["rel_change"]
        self.gnc.round_done()
        return st

    def iterate(self, active):
        return self._round(active)

    def iterate_async(self, rounds, refresh_local=True):
        for _ in range(rounds):
            if refresh_local:
                self.refresh_local()
            self._round(self.local)

    def sync(self):
        pass

    def set_neighbor_poses(self, robots, poses, X):
        self.o.set_nbr_rows(np.asarray(robots, np.int32), np.asarray(poses, np.int32), np.asarray(X, np.float64))

    def get_weights(self, base=None):
        return self.o.get_weights()

    def set_weights(self, w):
        self.o.set_weights(np.asarray(w, np.float64))

    def trajectory(self, robot, anchor):
        return self.o.trajectory(robot, anchor)

    def update_weights(self):
        mu = self.o.update_weights_local(self.local)
        self.gnc.updated()
        return mu


class NativeOracleBlockSolver(OracleBlockSolver):
    """The native-exchange interface of BlockSolver (kmx_pgo_comm_init /
    set_exchange / exchange: every round of iterate / iterate_async starts with
    the exchange) on the restatement, with the default torch.distributed group
    (gloo) standing in for the handle's RCCL communicator. Lets the CPU tests run
    RBCDDriver's native branch across ranks."""
    native_exchange = True

    @staticmethod
    def comm_unique_id():
        return bytes(range(128))

    def comm_init(self, unique_id, world, rank, timeout_s=120.0):
        assert len(unique_id) == 128 and timeout_s > 0
        self.world, self.rank, self.xchg = world, rank, None
        self.comm_inits = getattr(self, "comm_inits", 0) + 1
        # KMX_MOCK_STORE: a posted (asynchronous) transport like ncclSend /
        # ncclRecv on the solver stream — exchange() posts this rank's segments
        # and returns, sync_timeout() waits for the peers' with a deadline
        path = os.environ.get("KMX_MOCK_STORE")
        self._store = None
        if path:
            import torch.distributed as dist
            self._store = dist.FileStore(path, world)
            self._pending = None
            self._nx = 0

    raise_in_destroy = False  # the abort itself fails (a stream already in error)

    def comm_destroy(self):
        self.xchg = None
        self._pending = None
        self.comm_destroys = getattr(self, "comm_destroys", 0) + 1
        if self.raise_in_destroy:
            raise RuntimeError("hipStreamSynchronize: an illegal memory access (injected in comm_destroy)")

    def set_exchange(self, send_slots, send_counts, recv_slots, recv_counts):
        sc, rc = np.asarray(send_counts, np.int64), np.asarray(recv_counts, np.int64)
        assert sc.shape == rc.shape == (self.world,) and sc[self.rank] == rc[self.rank]
        ss, rs = np.ascontiguousarray(send_slots, np.int32), np.ascontiguousarray(recv_slots, np.int32)
        sseg = np.concatenate([[0], np.cumsum(sc)]).astype(np.int32)
        rseg = np.concatenate([[0], np.cumsum(rc)]).astype(np.int32)
        ps = self._rows()
        self.xchg = (ss if ss.size else np.zeros(1, np.int32), int(ss.size), sseg,
                     rs if rs.size else np.zeros(1, np.int32), int(rs.size), rseg,
                     [int(c) * ps + 1 for c in sc], [int(c) * ps + 1 for c in rc])
        self.exchanges = 0

    corrupt = False  # a faulty transport for the start-up check's test

    raise_in_exchange = False  # this rank's exchange raises before posting (its peers have posted theirs)

    def exchange(self):
        import torch
        import torch.distributed as dist
        ss, ns, sseg, rs, nr, rseg, ssplit, rsplit = self.xchg
        sbuf, rbuf = np.zeros(sum(ssplit)), np.zeros(sum(rsplit))
        self.exchange_pack(ss.ctypes.data, ns, sseg.ctypes.data, self.world, sbuf.ctypes.data)
        if self.raise_in_exchange:
            raise RuntimeError("ncclSend: unhandled system error (injected)")
        if getattr(self, "_store", None) is not None:
            so = np.concatenate([[0], np.cumsum(ssplit)]).astype(np.int64)
            for q in range(self.world):
                self._store.set(f"x{self._nx}/{self.rank}->{q}", sbuf[so[q]:so[q + 1]].tobytes())
            self._pending = (rbuf, rsplit, self._nx)
            self._nx += 1
            self.exchanges += 1
            return
        out = torch.zeros(rbuf.shape[0], dtype=torch.float64)
        dist.all_to_all_single(out, torch.from_numpy(sbuf), rsplit, ssplit)
        rbuf[:] = out.numpy()
        if self.corrupt and rbuf.size:
            rbuf[0] += 1e-12
        self.exchange_unpack(rs.ctypes.data, nr, rseg.ctypes.data, self.world, rbuf.ctypes.data)
        self.exchanges += 1

    def sync_timeout(self, timeout_s):
        """Wait (bounded) for the posted exchange's incoming segments; False on
        a timeout, as kmx_pgo_sync_timeout."""
        import datetime
        if getattr(self, "_pending", None) is None:
            return True
        rbuf, rsplit, k = self._pending
        keys = [f"x{k}/{q}->{self.rank}" for q in range(self.world)]
        try:
            self._store.wait(keys, datetime.timedelta(seconds=timeout_s))
        except Exception:  # noqa: BLE001 - the store's timeout error
            return False
        ro = np.concatenate([[0], np.cumsum(rsplit)]).astype(np.int64)
        for q in range(self.world):
            rbuf[ro[q]:ro[q + 1]] = np.frombuffer(self._store.get(keys[q]), np.float64)
        if self.corrupt and rbuf.size:
            rbuf[0] += 1e-12
        ss, ns, sseg, rs, nr, rseg, _, _ = self.xchg
        self.exchange_unpack(rs.ctypes.data, nr, rseg.ctypes.data, self.world, rbuf.ctypes.data)
        self._pending = None
        return True

    def _native(self):  # the exchange lists are set: every round starts with the exchange
        if getattr(self, "xchg", None) is not None:
            self.exchange()
            assert self.sync_timeout(120.0)

    def iterate(self, active):
        self._native()
        return self._round(active)

    def iterate_async(self, rounds, refresh_local=True):
        self.async_calls = getattr(self, "async_calls", 0) + 1
        for _ in range(rounds):
            if refresh_local:
                self.refresh_local()
            self._native()
            self._round(self.local)
