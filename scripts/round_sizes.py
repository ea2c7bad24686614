"""Per-round time of the concurrent RBCD round on one GPU vs problem size
(the per-GPU share of configs[3] at N = 8, 4, 2, 1 GPUs: 1/2/4/8 robot blocks
of 12.5k poses). Diagnostic for strong scaling; no exchange.
usage: round_sizes.py [robots,...] [standard|onesync] [tile incidences,...]"""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import bench
from kmx.dpgo.solver import BlockSolver
from kmx.synth import lift, lifting_matrix, make_pose_graph
P = bench.params()
P.localOptimizationParams.tCG_form = sys.argv[2] if len(sys.argv) > 2 else "standard"
TI = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0").split(",")]
Y = lifting_matrix(5, seed=1)
for R, ti in [(R, ti) for R in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")] for ti in TI]:
    P.tileIncidences = ti
    g = make_pose_graph(R, 12_500 * R, 62_500 * R, seed=0)
    s = BlockSolver(P, 0); s.set_graph_data(g)
    s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
    for a in range(R): s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    s.iterate_async(45, refresh_local=True); s.sync()  # the bench's burn-in + warmup: steady-state rounds
    s.read_counters()
    n = 40
    t0 = time.perf_counter(); s.iterate_async(n, refresh_local=True); s.sync(); el = time.perf_counter() - t0
    c = s.read_counters()
    print("tile incidences %4s " % (ti or "auto"), end="")
    print("robots %d poses %6d: %.1f us/round, %.3g edges*iters/s, hessvecs/round %.2f" %
          (R, g.n_total, 1e6 * el / n, c["edges_iters"] / el, c["hessvecs"] / n / R), flush=True)
    s.close()
