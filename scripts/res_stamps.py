"""Phase timeline of the resident round (KMX_TCG_FORM_RESIDENT) from a
KMX_RES_STAMPS build (`make -C kimera-multi_amd/csrc res_stamps`, run with
KMX_LIB=diag/libkmx_rs.so): thread 0 of every workgroup stamps the wall clock
(100 MHz) at the phases of the last round (pgo.hip body_round). Prints, per
phase, the median / max over workgroups relative to the earliest entry, and
the per-pass durations: barrier wait (arrival -> release), decision, gather,
step body.
usage: res_stamps.py [N-GPU shard of configs[3]: 8] [rounds] [poses: a one-robot
synthetic block of this many poses (5 edges per pose) instead of the shard]"""
import ctypes as C
import dataclasses
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
import bench
from kmx import abi
from kmx.dpgo.driver import robot_ranges, team_tile_incidences
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 60
NP = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if NP:
    from kmx.synth import make_pose_graph
    g = make_pose_graph(1, NP, 5 * NP, seed=0)
    N = 1
else:
    g = config("synth100k", seed=0)
P = bench.params()
P.localOptimizationParams.tCG_form = "resident"
P = dataclasses.replace(P, tileIncidences=team_tile_incidences(g, N, P.r, "resident"))
Y = lifting_matrix(5, seed=1)
lo, hi = robot_ranges(g.n_robots, N)[0]
local = np.zeros(g.n_robots, np.uint8)
local[lo:hi] = 1
s = BlockSolver(P, 0)
s.set_graph_data(g, local)
s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
for a in range(lo, hi):
    s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
print("resident:", s.resident_info())
s.iterate_async(rounds, refresh_local=True)
s.sync()
n = 128 * 2048
buf = np.zeros(n, np.uint64)
abi.check(s.L.kmx_pgo_debug_step_stamps(buf.ctypes.data_as(C.c_void_p), n), "stamps")
st = buf.reshape(-1, 128).astype(np.int64)
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
T = np.where(st > 0, (st - t0) * 0.01, np.nan)  # us
T[:, 94:96] = np.nan
print(f"{len(st)} workgroups; poses/tile median {np.median(st[:, 94]):.0f}, incidences/tile median "
      f"{np.median(st[:, 95]):.0f} (max {st[:, 95].max()})")
def med(i):
    return np.nanmedian(T[:, i]), np.nanmax(T[:, i])
for i, nm in [(0, "entry"), (1, "prologue"), (2, "gradient")]:
    print(f"  {nm:10s} median {med(i)[0]:7.2f}  max {med(i)[1]:7.2f} us")
names = ["arrive", "release", "decided", "gathered", "step end"]
for jl in range(17):
    b = 4 + 5 * jl
    if np.all(np.isnan(T[:, b])):
        break
    row = " ".join(f"{names[k]} {np.nanmedian(T[:, b + k]):7.2f}/{np.nanmax(T[:, b + k]):7.2f}"
                   for k in range(5) if not np.all(np.isnan(T[:, b + k])))
    wait = np.nanmedian(T[:, b + 1] - T[:, b])
    dec = np.nanmedian(T[:, b + 2] - T[:, b + 1])
    gat = np.nanmedian(T[:, b + 3] - T[:, b + 2])
    body = np.nanmedian(T[:, b + 4] - T[:, b + 3])
    print(f"  pass {jl:2d}: {row}")
    print(f"           wait {wait:6.2f}  decide {dec:6.2f}  gather {gat:6.2f}  body {body:6.2f} us (medians)")
    if jl < 16 and not np.all(st[:, 96 + 2 * jl] == 0):
        drn = np.nanmedian(T[:, 96 + 2 * jl] - T[:, b])
        last = np.nanmax(T[:, 96 + 2 * jl])
        mt = np.nanmedian(T[:, 97 + 2 * jl])
        print(f"           barrier: drain {drn:6.2f}, last drained arrival {last:7.2f}, poll matched {mt:7.2f} "
              f"(+{mt - last:5.2f} after the last arrival)")
for i, nm in [(90, "cost start"), (91, "cost end"), (92, "final release"), (93, "exit")]:
    print(f"  {nm:13s} median {med(i)[0]:7.2f}  max {med(i)[1]:7.2f} us")
s.close()
