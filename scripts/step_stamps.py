"""Phase timeline of one one-sync tCG launch (k_step) on a 12.5k-pose block,
from a KMX_STEP_STAMPS build (`make -C kimera-multi_amd/csrc stamps`, run with
KMX_LIB=diag/libkmx_ss.so): per workgroup the wall clock (100 MHz) at entry,
after the decision, after the gather loop, after the Hessian's own part and at
exit of the last launch that formed step 2. Prints, relative to the earliest
entry, the spread of each stamp over the workgroups and the per-phase
durations; the robots' first tiles (which also write the state) separately.
usage: step_stamps.py [robots] [tile incidences]"""
import ctypes as C
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
import bench
from kmx import abi
from kmx.dpgo.solver import BlockSolver
from kmx.synth import lift, lifting_matrix, make_pose_graph
R = int(sys.argv[1]) if len(sys.argv) > 1 else 1
P = bench.params()
P.localOptimizationParams.tCG_form = "onesync"
P.tileIncidences = int(sys.argv[2]) if len(sys.argv) > 2 else 0
Y = lifting_matrix(5, seed=1)
g = make_pose_graph(R, 12_500 * R, 62_500 * R, seed=0)
s = BlockSolver(P, 0)
s.set_graph_data(g)
s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
for a in range(R):
    s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
s.iterate_async(50, refresh_local=True)
s.sync()
n = 16 * 8192
buf = np.zeros(n, np.uint64)
abi.check(s.L.kmx_pgo_debug_step_stamps(buf.ctypes.data_as(C.c_void_p), n), "stamps")
st = buf.reshape(-1, 16)
st = st[st[:, 0] > 0].astype(np.int64)
t0 = st[:, 0].min()
T = (st[:, :7] - t0) * 10.0 / 1000.0  # us
names = ["entry", "issued", "landed", "decided", "gathered", "own Hess", "exit"]
print(f"{len(st)} workgroups; poses/tile median {np.median(st[:, 8]):.0f}, incidences/tile median {np.median(st[:, 9]):.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:9s} min {T[:, i].min():6.2f}  median {np.median(T[:, i]):6.2f}  p90 {np.percentile(T[:, i], 90):6.2f}  max {T[:, i].max():6.2f} us")
for i in range(1, 7):
    d = T[:, i] - T[:, i - 1]
    print(f"  {names[i - 1]:>9s} -> {names[i]:9s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
w = st[:, 11] == 1
if w.any():
    print("  first tiles:", " ".join(f"{names[i]} {np.median(T[w, i]):.2f}" for i in range(7)))
s.close()
