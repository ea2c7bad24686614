"""Diagnostic: gather variants on configs[3] with every robot's poses relabelled
by reverse Cuthill-McKee over its intra-robot edges (locality experiment)."""
import ctypes as C, sys
from pathlib import Path
import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import bench
from kmx import abi
from kmx.dpgo.solver import BlockSolver
g, X0 = bench.make_workload("synth100k")
mode = sys.argv[1]
if mode != "none":
    perms = []
    for a in range(g.n_robots):
        n = int(g.n_poses[a])
        m = (g.r1 == a) & (g.r2 == a)
        A = sp.coo_matrix((np.ones(m.sum()), (g.p1[m], g.p2[m])), shape=(n, n)).tocsr()
        A = A + A.T
        if mode == "rcm":
            order = reverse_cuthill_mckee(A, symmetric_mode=True)   # new -> old
        else:
            order = np.random.default_rng(0).permutation(n)
        inv = np.empty(n, np.int64); inv[order] = np.arange(n)     # old -> new
        perms.append(inv)
        X0[a] = X0[a][order]
    p1 = g.p1.copy(); p2 = g.p2.copy()
    for a in range(g.n_robots):
        s1 = g.r1 == a; s2 = g.r2 == a
        p1[s1] = perms[a][g.p1[s1]]; p2[s2] = perms[a][g.p2[s2]]
    g.p1 = p1.astype(np.int32); g.p2 = p2.astype(np.int32)
P = bench.params()
s = BlockSolver(P, 0); s.set_graph_data(g)
for a in range(g.n_robots): s.set_iterate(a, X0[a])
s.refresh_local(); s.sync()
L = abi.lib(); fn = L.kmx_pgo_debug_gather_bench
fn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]; fn.restype = C.c_int
alg = 128.0 * sum(s.local_edges(a) for a in range(g.n_robots)) + 2 * 8 * 20 * g.n_total
for v in [int(x) for x in sys.argv[2].split(",")]:
    ms = C.c_double()
    rc = fn(s.h, v, 50, C.byref(ms))
    if rc: print(v, "rc", rc, L.kmx_last_error()); continue
    print("%s variant %2d: %8.1f us  alg %.2f TB/s" % (mode, v, ms.value * 1e3, alg / (ms.value * 1e-3) / 1e12), flush=True)
