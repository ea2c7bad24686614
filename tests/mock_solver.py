"""CPU stand-in for kmx.dpgo.solver.BlockSolver used ONLY by the gloo tests of
the multi-process driver path: the same exchange interface (pack / unpack of
the public-pose table through raw pointers, owner-packed shared weights) on
top of the CPU restatement. It is test infrastructure (imports oracle/)."""
import ctypes as C

import numpy as np

from oracle.oracle import OraclePGO


class OracleBlockSolver:
    def __init__(self, params):
        self.params = params
        self.r = params.r

    def set_stream(self, s):  # pragma: no cover - CPU only
        pass

    def set_graph_data(self, g, local):
        self.g = g
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
        owner = np.minimum(g.r1, g.r2)
        self.owned_shared = self.local[owner[self.shared_edges]] == 1

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

    def pack_public(self, ptr):
        sl = slice(self.first_owned, self.first_owned + self.n_owned)
        X = np.ascontiguousarray(self.o.get_x_rows(self.pub_robot[sl], self.pub_pose[sl]))
        C.memmove(ptr, X.ctypes.data, X.nbytes)

    def unpack_public(self, ptr):
        n = self.pub_robot.shape[0]
        buf = (C.c_double * (n * self._rows())).from_address(ptr)
        X = np.frombuffer(buf, dtype=np.float64).reshape(n, self.r, 4).copy()
        self.o.set_nbr_rows(self.pub_robot, self.pub_pose, X)

    def gather_public_rows(self, slots_ptr, n, out_ptr):
        if n == 0:
            return
        sl = np.frombuffer((C.c_int32 * n).from_address(slots_ptr), dtype=np.int32).copy()
        X = np.ascontiguousarray(self.o.get_x_rows(self.pub_robot[sl], self.pub_pose[sl]))
        C.memmove(out_ptr, X.ctypes.data, X.nbytes)

    def scatter_public_rows(self, slots_ptr, n, rows_ptr):
        if n == 0:
            return
        sl = np.frombuffer((C.c_int32 * n).from_address(slots_ptr), dtype=np.int32).copy()
        buf = (C.c_double * (n * self._rows())).from_address(rows_ptr)
        X = np.frombuffer(buf, dtype=np.float64).reshape(n, self.r, 4).copy()
        self.o.set_nbr_rows(self.pub_robot[sl], self.pub_pose[sl], X)

    def refresh_local(self):
        X = self.o.get_x_rows(self.pub_robot, self.pub_pose)
        self.o.set_nbr_rows(self.pub_robot, self.pub_pose, X)

    def iterate(self, active):
        act = np.asarray(active, np.uint8) & self.local
        return self.o.iterate_nbr(act)

    def iterate_async(self, rounds, refresh_local=True, gnc_every=0):
        # same schedule as kmx_pgo_iterate_async: GNC after every gnc_every-th round
        for _ in range(rounds):
            if refresh_local:
                self.refresh_local()
            self.o.iterate_nbr(self.local)
            self.rounds_done = getattr(self, "rounds_done", 0) + 1
            if gnc_every > 0 and int(self.params.robustCostParams.costType) != 0 and self.rounds_done % gnc_every == 0:
                if refresh_local:
                    self.refresh_local()
                self.update_weights()

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
        return self.o.update_weights_owned(self.local)

    def shared_count(self):
        return int(self.shared_edges.shape[0])

    def pack_shared_weights(self, ptr):
        w = self.o.get_weights()[self.shared_edges]
        w = np.ascontiguousarray(np.where(self.owned_shared, w, 0.0))
        C.memmove(ptr, w.ctypes.data, w.nbytes)

    def unpack_shared_weights(self, ptr):
        n = self.shared_edges.shape[0]
        tab = np.frombuffer((C.c_double * n).from_address(ptr), dtype=np.float64).copy()
        w = self.o.get_weights()
        w[self.shared_edges] = tab
        self.o.set_weights(w)
