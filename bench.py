#!/usr/bin/env python3
"""bench.py — dpgo edges·iters/sec (+ LC candidates verified/sec) on MI355X.

Contract (see task statement / DESIGN.md "Measurement"):
  python bench.py --gpus N --steps K --warmup W
  (N > 1 is launched by torch.distributed.run, one rank per GPU over RCCL).
A "step" is one synchronous RBCD round (dpgo_ros UPDATE -> PGOAgent::iterate of
every robot block, drawio:2058-2066) with the GNC weight update every 20 rounds
inside the timed region. At N = 1 the graph is configs[3]: 100k poses / 500k
edges, 20 % outlier loop closures, 8 robot blocks.

Multi-GPU (one process per GPU, robot blocks dealt to ranks, one all-to-all of
public poses per round over RCCL):
  --scaling weak (default): every GPU holds a configs[3]-shaped shard, i.e. the
      team graph has 8N robot blocks, N x 100k poses and N x 500k edges (same
      density, outlier and inter-robot fractions); value is the whole team's
      rate. The fixed configs[3] graph split over the N GPUs (strong scaling)
      is timed in the same run and reported under "strong".
  --scaling strong: value is the fixed configs[3] graph split over N GPUs.

value = sum over ranks of edges·iters (sum over executed block updates of the
block's local-problem edge count) / max-over-ranks wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))

PEAK_HBM = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="synth100k")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="N > 1: weak = a configs[3]-shaped shard per GPU; strong = configs[3] split over N")
    ap.add_argument("--strong-steps", type=int, default=None,
                    help="weak scaling at N > 1: rounds of the extra strong-scaling leg (default --steps; 0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-lcd", action="store_true")
    ap.add_argument("--profile", action="store_true", help="short run for rocprofv3 (no cpu / lcd)")
    ap.add_argument("--no-events", action="store_true", help="skip the HIP-event roofline pass (gap profiling)")
    ap.add_argument("--lcd-frames", type=int, default=50_000)
    ap.add_argument("--lcd-steps", type=int, default=3)
    return ap.parse_args()


def make_workload(name, world=1, scaling="strong"):
    """The named configs graph, or for weak scaling at N > 1 the N-shard team
    graph of the same shape per GPU (configs[3]: 8 robots / 100k poses / 500k
    edges per shard; identical to configs[3] at N = 1)."""
    from kmx.synth import config, lift, lifting_matrix, make_pose_graph
    if scaling == "weak" and world > 1:
        if name != "synth100k":
            raise SystemExit("--scaling weak is defined for configs[3] (synth100k)")
        g = make_pose_graph(8 * world, 100_000 * world, 500_000 * world, seed=0)
    else:
        g = config(name, seed=0)
    Y = lifting_matrix(5, seed=1)
    X0 = {a: lift(g.init_R[a], g.init_t[a], Y) for a in range(g.n_robots)}
    return g, X0


def params():
    from kmx.dpgo.params import PGOAgentParameters
    P = PGOAgentParameters(r=5)
    P.localOptimizationParams.RTR_iterations = 1
    P.localOptimizationParams.RTR_tCG_iterations = 10
    P.robustOptInnerIters = 20
    P.robustOptNumWeightUpdates = 10**9
    P.schedule = 1
    return P


def cpu_baseline(g, X0, P, seconds):
    """The C restatement (oracle/) on this host, single thread (dpgo runs one
    agent per process); bounded sample of whole rounds of the same workload."""
    sys.path.insert(0, str(ROOT))
    from oracle.oracle import OraclePGO
    o = OraclePGO(P.to_c(), g)
    for a in range(g.n_robots):
        o.set_iterate(a, X0[a])
    edges_iters, rounds = 0, 0
    t0 = time.perf_counter()
    while True:
        st = o.iterate(threads=1)
        edges_iters += sum(s["edges"] for s in st if s["updated"] and s["tcg_stop"] != "skipped")
        rounds += 1
        if rounds % P.robustOptInnerIters == 0:
            o.update_weights()
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": edges_iters / el, "unit": "edges*iters/s", "cores": 1, "kind": "port",
            "sample": f"{rounds} RBCD rounds of {P and 'configs[3]'} (8 blocks, 1 RTR step, <=10 tCG) "
                      f"from the same initial iterate, oracle/dpgo_oracle.c -O3 x86-64-v3, 1 thread, {el:.1f} s"}


def lcd_leg(args, rank, world, barrier_sync):
    """configs[2]: 50k keyframes x 500 ORB descriptors, one candidate per query
    (half planted loop closures), kNN2 + Lowe -> 2D-2D 5-point RANSAC -> 3D-3D.
    Candidates are sharded across ranks (independent; no collective)."""
    from kmx.lcd import LcdParams, LoopClosureDetector
    from kmx.synth.lcd import make_lcd_pool
    pool = make_lcd_pool(args.lcd_frames, 500, seed=0)
    det = LoopClosureDetector(LcdParams(), device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
    det.set_pool(pool)
    cq = pool.cand_query[rank::world].copy()
    cm = pool.cand_match[rank::world].copy()
    det.verify_async(cq, cm)  # warmup
    det.sync()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.lcd_steps):
        det.verify_async(cq, cm)
    det.sync()
    barrier_sync()
    el = time.perf_counter() - t0
    res, _ = det.verify(cq[:256], cm[:256])
    out = {"metric": "LC candidates verified/sec", "n_local": int(cq.shape[0]), "steps": args.lcd_steps,
           "elapsed": el, "accepted_frac_first256": sum(r["accepted"] for r in res) / max(len(res), 1),
           "workload": f"configs[2]: {args.lcd_frames} keyframes x 500 ORB descriptors (32 B), "
                       f"{pool.cand_query.shape[0]} candidates, L1 matcher, Lowe 0.7, 5-point RANSAC "
                       "(thr 1e-6, <=500 it, p 0.995, seed 12345, GCC-9 sampler), 1-point 3D-3D 0.3 m"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT))
        from oracle import oracle as O
        p = LcdParams().to_c()
        n, t0c, done = 0, time.perf_counter(), 0.0
        while done < args.cpu_seconds * 0.5:
            O.lcd_verify(p, pool, cand_query=pool.cand_query[n:n + 64], cand_match=pool.cand_match[n:n + 64],
                         masks=False)
            n += 64
            done = time.perf_counter() - t0c
        cpu = {"value": n / done, "unit": "candidates/s", "cores": 1, "kind": "port",
               "sample": f"first {n} candidates of configs[2] (half planted), oracle/lcd_oracle.c, 1 thread, "
                         f"{done:.1f} s"}
    return out, cpu


def bow_leg(args, rank, world, barrier_sync):
    """BoW candidate stage (configs[2] "BoW query", timed separately): robot 1's
    keyframes query robot 0's database (detectLoopWithRobot: DBoW2 queryL1,
    max_db_results 50) on a synthetic 100k-word vocabulary. Queries are
    sharded across ranks (independent; no collective)."""
    from kmx.lcd.bow import BowDatabase
    from kmx.synth.bow import make_bow_stream
    n = args.lcd_frames // 2
    st = make_bow_stream(2, n, n_words=100_000, seed=0)
    db = st.subset(np.nonzero(st.robot == 0)[0])
    qi = np.nonzero(st.robot == 1)[0][rank::world]
    qs = st.subset(qi)
    G = BowDatabase(st.n_words, device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
    G.set_entries(db.vptr, db.words, db.weights)
    G.query_async(qs.vptr, qs.words, qs.weights, 50)  # warmup
    G.sync()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.lcd_steps):
        G.query_async(qs.vptr, qs.words, qs.weights, 50)
    G.sync()
    barrier_sync()
    el = time.perf_counter() - t0
    postings = float(np.bincount(db.words, minlength=st.n_words)[qs.words].sum())
    out = {"metric": "BoW queries/sec", "n_local": int(qs.n), "steps": args.lcd_steps, "elapsed": el,
           "postings_per_query": postings / max(qs.n, 1),
           "workload": f"{qs.n} queries (robot 1) x {db.n}-entry database (robot 0), {st.n_words} words, "
                       f"~{st.words.shape[0] // st.n} words per BowVector, queryL1 top-50"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT))
        from oracle import oracle as O
        D = O.OracleBowDb(st.n_words, db.vptr, db.words, db.weights)
        k, t0c, done = 0, time.perf_counter(), 0.0
        while done < args.cpu_seconds * 0.25 and k < qs.n:
            sub = qs.subset(np.arange(k, min(k + 256, qs.n)))
            D.query(sub.vptr, sub.words, sub.weights, 50)
            k += sub.n
            done = time.perf_counter() - t0c
        cpu = {"value": k / done, "unit": "queries/s", "cores": 1, "kind": "port",
               "sample": f"first {k} queries, oracle/bow_oracle.c (DBoW2 queryL1 restated), 1 thread, {done:.1f} s"}
    return out, cpu


def load_traffic():
    f = ROOT / "profiles" / "hessvec_traffic.json"
    if f.exists():
        try:
            return json.loads(f.read_text())
        except Exception:
            return None
    return None


def _coll_device(dist):
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def dpgo_leg(g, X0, P, args, rank, world, local_rank, dist, steps, barrier, roofline=True):
    """Warm up, time `steps` concurrent RBCD rounds (max over ranks), then (if
    `roofline`) continue with HIP events around every k_hess launch. Returns
    the team totals."""
    import torch
    from kmx.dpgo.driver import RBCDDriver
    drv = RBCDDriver(P, g, rank=rank, world=world, device=local_rank if world > 1 else 0)
    drv.initialize(X0)

    def sync():
        drv.solver.sync()
        barrier()

    drv.run_async(args.warmup)
    sync()
    drv.solver.read_counters()  # reset device counters and event pool
    sync()
    el, edges_iters = 0.0, 0.0
    if not args.profile:  # --profile: every profiled k_hess dispatch is also in the roofline counters
        t0 = time.perf_counter()
        drv.run_async(steps)
        sync()
        el = time.perf_counter() - t0
        edges_iters = float(drv.solver.read_counters()["edges_iters"])
    # roofline pass: the same rounds continued with HIP events around every
    # k_hess launch (events add a few us per launch, so they stay out of `value`)
    rsteps = steps if args.profile else (0 if (args.no_events or not roofline) else max(1, min(steps, 20)))
    hv_ms, hv_bytes, hv_n = 0.0, 0.0, 0
    if rsteps:
        drv.solver.enable_timing(True)
        t0 = time.perf_counter()
        drv.run_async(rsteps)
        sync()
        if args.profile:
            el = time.perf_counter() - t0
        drv.solver.enable_timing(False)
        cnt = drv.solver.read_counters()
        if args.profile:
            edges_iters = float(cnt["edges_iters"])
        hv_ms, hv_bytes, hv_n = cnt["hessvec_ms_total"], cnt["hessvec_alg_bytes"], cnt["hessvec_launches"]
    xs, xr = drv.exchange_rows
    if dist is not None:
        t = torch.tensor([el, edges_iters, hv_ms, hv_bytes, float(hv_n), float(xs), float(xr)],
                         dtype=torch.float64, device=_coll_device(dist))
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        parts = torch.stack(parts).cpu().numpy()
        el = float(parts[:, 0].max())
        edges_iters = float(parts[:, 1].sum())
        hv_ms, hv_bytes, hv_n = float(parts[:, 2].sum()), float(parts[:, 3].sum()), int(parts[:, 4].sum())
        xs, xr = int(parts[:, 5].max()), int(parts[:, 6].max())
    drv.solver.close()
    return {"el": el, "edges_iters": edges_iters, "hv": (hv_ms, hv_bytes, hv_n), "rsteps": rsteps,
            "xrows": (xs, xr)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch
    # one GPU per rank; modulo the visible count only when rehearsing several ranks on one GPU
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    os.environ["KMX_BENCH_DEVICE"] = str(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        # KMX_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU
        # (exchange staged through host copies); the benchmark itself runs over RCCL
        backend = os.environ.get("KMX_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    P = params()
    weak = args.scaling == "weak" and world > 1
    t_gen = time.perf_counter()
    g, X0 = make_workload(args.config, world, args.scaling)
    gen_s = time.perf_counter() - t_gen
    leg = dpgo_leg(g, X0, P, args, rank, world, local_rank, dist, args.steps, barrier)
    el, edges_iters = leg["el"], leg["edges_iters"]
    hv_ms, hv_bytes, hv_n = leg["hv"]
    value = edges_iters / el
    achieved = hv_bytes / (hv_ms * 1e-3) if hv_ms > 0 else 0.0
    traffic = load_traffic()
    ps_bytes = 8 * 4 * P.r
    if weak:
        workload = (f"configs[3] shape per GPU (weak scaling): {g.n_total} poses / {g.m} edges, {g.n_robots} robot "
                    f"blocks over {world} GPUs ({g.n_robots // world} per GPU, 100k poses / 500k edges each), "
                    "20% outlier LCs, f_inter 0.10, GNC-TLS every 20 rounds")
    else:
        workload = (f"configs[3] {args.config}: {g.n_total} poses / {g.m} edges, {g.n_robots} robot blocks"
                    + (f" split over {world} GPUs" if world > 1 else "")
                    + ", 20% outlier LCs, f_inter 0.10, GNC-TLS every 20 rounds")
    out = {
        "metric": "dpgo edges*iters/sec (+ LC candidates verified/sec in 'lcd')",
        "value": value,
        "unit": "edges*iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded numpy PCG64; Campus bags unavailable offline)",
        "config": {
            "workload": workload,
            "robots": g.n_robots, "poses": g.n_total, "edges": g.m, "r": P.r,
            "rtr_iterations": 1, "tcg_max": 10, "schedule": "concurrent",
            "parallelism": f"robot blocks {g.n_robots} over {world} GPU(s)"
                           + (", public poses by one RCCL all_to_all per round" if world > 1 else ""),
            "exchange_rows_per_round": {"sent_max": leg["xrows"][0], "recv_max": leg["xrows"][1],
                                        "recv_bytes_max": leg["xrows"][1] * ps_bytes},
            "graph_gen_s": round(gen_s, 1),
        },
        "roofline": {
            "kernel": "k_hess (tCG Hessian-vector product)",
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": PEAK_HBM / 1e9,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM,
            # PMC bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section),
            # measured as a ratio to the algorithmic bytes of the same dispatches
            # (scripts/gpu_pmc_hess.sh -> profiles/hessvec_traffic.json) and applied to this run's launches
            "traffic": (traffic["traffic_over_alg"] * hv_bytes / max(hv_n, 1)) if traffic else None,
            "traffic_over_alg": traffic["traffic_over_alg"] if traffic else None,
            "launches": hv_n,
            "measured_over": f"{leg['rsteps']} further rounds with HIP events around each k_hess launch",
            "avg_launch_us": 1e3 * hv_ms / max(hv_n, 1),
            "alg_bytes_per_launch": hv_bytes / max(hv_n, 1),
        },
    }
    sst = args.steps if args.strong_steps is None else args.strong_steps
    if weak and sst > 0 and not args.profile:
        del g, X0
        gs, X0s = make_workload(args.config, 1, "strong")
        st = dpgo_leg(gs, X0s, P, args, rank, world, local_rank, dist, sst, barrier, roofline=False)
        out["strong"] = {"value": st["edges_iters"] / st["el"], "unit": "edges*iters/s", "steps": sst,
                         "ms_per_step": 1e3 * st["el"] / sst,
                         "workload": f"configs[3] {args.config}: {gs.n_total} poses / {gs.m} edges, "
                                     f"{gs.n_robots} robot blocks split over {world} GPUs (strong scaling)",
                         "exchange_rows_per_round": {"sent_max": st["xrows"][0], "recv_max": st["xrows"][1]}}
        g, X0 = gs, X0s
    if rank == 0 and world == 1 and not args.no_cpu and not args.profile:
        out["cpu_baseline"] = cpu_baseline(g, X0, P, args.cpu_seconds)
    if not args.no_lcd and not args.profile:
        lcd, lcd_cpu = lcd_leg(args, rank, world, barrier)
        n_local, lel = float(lcd["n_local"] * lcd["steps"]), lcd["elapsed"]
        if dist is not None:
            t = torch.tensor([n_local, lel], dtype=torch.float64, device=_coll_device(dist))
            parts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            parts = torch.stack(parts).cpu().numpy()
            n_local, lel = float(parts[:, 0].sum()), float(parts[:, 1].max())
        lcd["value"] = n_local / lel
        lcd["unit"] = "candidates/s"
        lcd["ms_per_step"] = 1e3 * lel / lcd["steps"]
        del lcd["elapsed"]
        if lcd_cpu:
            lcd["cpu_baseline"] = lcd_cpu
        bow, bow_cpu = bow_leg(args, rank, world, barrier)
        n_local, bel = float(bow["n_local"] * bow["steps"]), bow["elapsed"]
        if dist is not None:
            t = torch.tensor([n_local, bel], dtype=torch.float64, device=_coll_device(dist))
            parts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            parts = torch.stack(parts).cpu().numpy()
            n_local, bel = float(parts[:, 0].sum()), float(parts[:, 1].max())
        bow["value"] = n_local / bel
        bow["unit"] = "queries/s"
        bow["ms_per_step"] = 1e3 * bel / bow["steps"]
        del bow["elapsed"]
        if bow_cpu:
            bow["cpu_baseline"] = bow_cpu
        lcd["bow"] = bow
        out["lcd"] = lcd
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
