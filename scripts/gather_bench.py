"""Time gather-primitive variants in isolation (diagnostic; kmx_pgo_debug_gather_bench).

usage: gather_bench.py [config] [variants] [cmp pairs a:b,...]
"""
import ctypes as C, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import bench
from kmx import abi
from kmx.dpgo.solver import BlockSolver
g, X0 = bench.make_workload(sys.argv[1] if len(sys.argv) > 1 else "synth100k")
P = bench.params()
s = BlockSolver(P, 0); s.set_graph_data(g)
for a in range(g.n_robots): s.set_iterate(a, X0[a])
s.refresh_local(); s.sync()
L = abi.lib(); fn = L.kmx_pgo_debug_gather_bench
fn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]; fn.restype = C.c_int
cmp = L.kmx_pgo_debug_gather_cmp
cmp.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]; cmp.restype = C.c_int
alg = 128.0 * sum(s.local_edges(a) for a in range(g.n_robots)) + 2 * 8 * 20 * g.n_total
if len(sys.argv) > 3:
    for pair in sys.argv[3].split(","):
        va, vb = (int(x) for x in pair.split(":"))
        md, ma = C.c_double(), C.c_double()
        rc = cmp(s.h, va, vb, C.byref(md), C.byref(ma))
        if rc: print(pair, "rc", rc, L.kmx_last_error()); continue
        print("cmp %2d vs %2d: max|diff| %.3e  max|out| %.3e  rel %.3e" % (va, vb, md.value, ma.value, md.value / max(ma.value, 1e-300)), flush=True)
for v in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "0,1,10,20,21".split(","))]:
    ms = C.c_double()
    rc = fn(s.h, v, 50, C.byref(ms))
    if rc: print(v, "rc", rc, L.kmx_last_error()); continue
    print("variant %2d: %8.1f us  alg %.2f TB/s" % (v, ms.value * 1e3, alg / (ms.value * 1e-3) / 1e12), flush=True)
