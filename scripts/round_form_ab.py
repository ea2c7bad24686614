"""Launched vs persistent round (kmx_pgo_set_round_form 0 / 1) on the per-GPU
shards of configs[3]: the rank-0 handle of an N-GPU team (the team's tile cut,
no exchange: foreign rows frozen) and single 12.5k / 25k-pose blocks.
Steady-state window as the bench (45-round burn-in). usage: round_form_ab.py [N,...]"""
import sys, time, dataclasses
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
import bench
from kmx.dpgo.driver import robot_ranges, team_tile_incidences
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix

g = config("synth100k", seed=0)
Y = lifting_matrix(5, seed=1)
for N in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,4").split(",")]:
    cap = team_tile_incidences(g, N, 5, bench.params())
    lo, hi = robot_ranges(g.n_robots, N)[0]
    local = np.zeros(g.n_robots, np.uint8); local[lo:hi] = 1
    res = {}
    # the launched form at its own best cut (180) and at the round's cut, then the round
    for form, tile in ((0, 180), (0, cap), (1, cap), (0, 180), (0, cap), (1, cap)):
        P = dataclasses.replace(bench.params(), tileIncidences=tile)
        s = BlockSolver(P, 0); s.set_round_form(form); s.set_graph_data(g, local)
        s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
        for a in range(lo, hi): s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
        s.refresh_local(); s.iterate_async(45, refresh_local=False); s.sync(); s.read_counters()
        n = 60
        t0 = time.perf_counter(); s.iterate_async(n, refresh_local=False); s.sync(); el = time.perf_counter() - t0
        c = s.read_counters(); f = s.round_form()
        X = s.get_iterate(lo)
        print(f"N={N} form={'persistent' if f['persistent'] else 'launched':10s} cut={tile} tiles={f['tiles']} cap={f['capacity']}: "
              f"{1e6 * el / n:7.1f} us/round, hessvecs/round {c['hessvecs'] / n:.2f}", flush=True)
        if tile == cap: res.setdefault(form, X)
        s.close()
    print(f"N={N} iterates bitwise equal: {np.array_equal(res[0], res[1])}", flush=True)
