#!/usr/bin/env python3
"""bench.py — dpgo edges·iters/sec (+ LC candidates verified/sec) on MI355X.

Contract (see task statement / DESIGN.md §6 "Measurement"):
  python bench.py --gpus N --steps K --warmup W
  (N > 1 is launched by torch.distributed.run, one rank per GPU over RCCL).

A "step" is one synchronous RBCD round (dpgo_ros UPDATE -> PGOAgent::iterate of
every robot block, drawio:2058-2066), with GNC-TLS weight updates decided by
the schedule inside the timed region. The graph is configs[3]: 100k poses /
500k edges, 20 % outlier loop closures, 8 robot blocks.

The timed window is a fixed, stated slice of the solve:
  rounds [B, B + W)          untimed: B = --burn-in (default 40) rounds in which
                              tCG stops after 1-5 steps, then the W warmup rounds
  rounds [B + W, B + W + K)  timed (value), K = --steps
The window is replayed from a snapshot of the solver state (iterate, GNC
weights and schedule state, statuses) with HIP events around every
Hessian-vector launch: the roofline describes exactly the timed rounds (the
replay must reproduce their work counters). The CPU baseline restarts the
restatement from the same snapshot and times the same rounds.

Multi-GPU (one process per GPU, robot blocks dealt to ranks; per round the
public poses + status words go to every peer over RCCL, by default from inside
the solver's round: kmx_pgo_comm_init / kmx_pgo_set_exchange):
  --scaling strong (default): the fixed configs[3] graph split over the N GPUs
      (north_star's "further scaling at 8 GPUs"); value is the team's rate.
  --scaling weak: every GPU holds a configs[3]-shaped shard (8N robot blocks,
      N x 100k poses / N x 500k edges). Timed in the same run as an extra.

value = sum over ranks of edges·iters (sum over executed block updates of the
block's local-problem edge count) / max-over-ranks wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))

PEAK_HBM = 8.0e12      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
PEAK_VALU_OPS = 78.6e12  # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32 lane-ops/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--burn-in", type=int, default=40, help="untimed rounds before the warmup (steady-state window)")
    ap.add_argument("--config", default="synth100k", help="synth100k (configs[3]) or synth1m (the cold 1M/5M graph)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="N > 1: strong = configs[3] split over N (value); weak = a configs[3]-shaped shard per GPU")
    ap.add_argument("--extra-steps", type=int, default=None,
                    help="N > 1: rounds of the other scaling leg (default --steps; 0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample per variant")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-lcd", action="store_true")
    ap.add_argument("--no-replay", action="store_true", help="skip the evented replay (roofline)")
    ap.add_argument("--profile", action="store_true", help="short run for rocprofv3: timed rounds only")
    ap.add_argument("--tile-incidences", type=int, default=0,
                    help="incidences per workgroup tile (kmx_pgo_params.tile_incidences; 0: automatic)")
    ap.add_argument("--tcg-form", choices=["auto", "standard", "onesync"], default="auto",
                    help="tCG form (kmx_pgo_params.tcg_form): ROPTLIB's, or the one-sync form launched per step "
                         "(opt-in); auto = standard at every shard size (DESIGN.md section 10)")
    ap.add_argument("--lcd-frames", type=int, default=50_000)
    ap.add_argument("--lcd-steps", type=int, default=8,
                    help="back-to-back LCD verification calls timed (a call's kNN2 overlaps the previous call's "
                         "RANSAC tail on the detector's second candidate slot, as in a stream of queries)")
    ap.add_argument("--lcd-hard", type=int, default=4096,
                    help="candidates of the hard LCD leg (look-alikes that pass Lowe and fail geometry; 0 = skip)")
    ap.add_argument("--lcd-algo", type=int, default=0,
                    help="ransac_2d2d_algorithm: 0 Stewenius (the reference config, LcdParams.yaml:73), 1 Nister")
    return ap.parse_args()


def make_workload(name, world=1, scaling="strong"):
    """The named graph, or for weak scaling at N > 1 the N-shard team graph of
    the configs[3] shape per GPU (identical to configs[3] at N = 1)."""
    from kmx.synth import config, lift, lifting_matrix, make_pose_graph
    if scaling == "weak" and world > 1:
        if name != "synth100k":
            raise SystemExit("--scaling weak is defined for configs[3] (synth100k)")
        g = make_pose_graph(8 * world, 100_000 * world, 500_000 * world, seed=0)
    elif name == "synth1m":  # the cold config: ~1 GB working set, past the Infinity Cache
        g = make_pose_graph(8, 1_000_000, 5_000_000, seed=0)
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


# ---------------------------------------------------------------- snapshot ---
def snapshot(drv):
    s = drv.solver
    return {"X": {a: drv.iterate_of(a) for a in drv.robots}, "w": s.get_weights(), "gnc": s.gnc_state(),
            "status": s.status()}


def restore(drv, snap):
    s = drv.solver
    for a in drv.robots:
        s.set_iterate(a, snap["X"][a])
    s.set_weights(snap["w"])
    s.set_gnc_state(snap["gnc"])
    s.set_status(snap["status"])


# --------------------------------------------------------------- CPU legs ---
def _native_oracle():
    """Build the restatement for this host (-march=native) outside the repo;
    returns (path, march) or (None, prebuilt march) when gcc fails."""
    out = Path(os.environ.get("TMPDIR", "/tmp")) / f"kmx_liborc_native_{os.getpid()}.so"
    src = [str(ROOT / "oracle" / f) for f in ("dpgo_oracle.c", "lcd_oracle.c", "bow_oracle.c")]
    cmd = ["gcc", "-O3", "-march=native", "-ffp-contract=off", "-fPIC", "-fopenmp", "-shared", "-o", str(out), *src,
           "-lm"]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=120)
        return str(out), "native"
    except Exception:
        return None, "x86-64-v3"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(g, P, snap, steps, seconds, variants):
    """The C restatement (oracle/, -march=native) on this host from the
    snapshot of the timed window's first round: the same rounds as the GPU's
    timed window (GNC by the host mirror of the schedule), bounded by
    `seconds` per variant. variants: (threads, inner) — one thread per robot
    block (dpgo runs one agent per process), 1, and the all-cores form (blocks
    x `inner` threads inside each block update; equal to rounding only)."""
    from kmx.dpgo.schedule import GncSchedule
    sys.path.insert(0, str(ROOT))
    from oracle.oracle import OraclePGO
    out = {}
    for threads, inner in variants:
        o = OraclePGO(P.to_c(), g)
        for a, X in snap["X"].items():
            o.set_iterate(a, X)
        o.set_weights(snap["w"])
        o.mu = snap["gnc"]["mu"]
        sched = GncSchedule.from_params(P)
        sched.inner, sched.updates, sched.mu = snap["gnc"]["inner_iter"], snap["gnc"]["updates"], snap["gnc"]["mu"]
        relc = np.array(snap["status"], dtype=np.float64)
        edges_iters, hv, rounds = 0, 0, 0
        t0 = time.perf_counter()
        while rounds < steps:
            if sched.should_update(relc):
                o.refresh()
                o.update_weights()
                sched.updated()
            st = o.iterate(threads=threads, inner=inner)
            sched.round_done()
            relc = np.array([s["rel_change"] if s["updated"] else relc[a] for a, s in enumerate(st)])
            edges_iters += sum(s["edges"] for s in st if s["updated"] and s["tcg_stop"] != "skipped")
            hv += sum(s["hessvecs"] for s in st)
            rounds += 1
            if time.perf_counter() - t0 >= seconds:
                break
        el = time.perf_counter() - t0
        out[(threads, inner)] = {"value": edges_iters / el, "rounds": rounds, "seconds": el, "hessvecs": hv,
                        "ms_per_step": 1e3 * el / rounds, "edges_iters": edges_iters,
                        "X": {a: o.get_iterate(a) for a in range(g.n_robots)}}
    return out


def gpu_parity(drv, snap, cpu):
    """Free full-size, steady-state parity check: replay on the GPU, from the
    same snapshot, exactly the rounds the CPU leg ran, and compare the work
    counters (Hess-vecs, edges*iters) and every pose with the restatement's
    (north_star: 1e-6 Frobenius per pose)."""
    restore(drv, snap)
    drv.solver.sync()
    drv.solver.read_counters()
    drv.run_async(cpu["rounds"])
    drv.solver.sync()
    c = drv.solver.read_counters()
    worst = 0.0
    for a in drv.robots:
        d = np.linalg.norm((drv.iterate_of(a) - cpu["X"][a]).reshape(-1, 4 * drv.params.r), axis=1)
        worst = max(worst, float(d.max()) if d.size else 0.0)
    ok = int(c["hessvecs"]) == int(cpu["hessvecs"]) and int(c["edges_iters"]) == int(cpu["edges_iters"]) \
        and worst <= 1e-6
    if not ok:
        print(f"bench: GPU vs restatement parity FAILED over {cpu['rounds']} rounds: hessvecs "
              f"{c['hessvecs']} vs {cpu['hessvecs']}, edges*iters {c['edges_iters']} vs {cpu['edges_iters']}, "
              f"max pose diff {worst:.3e}", file=sys.stderr, flush=True)
    return {"parity_checked_rounds": int(cpu["rounds"]), "hessvecs_gpu": int(c["hessvecs"]),
            "hessvecs_cpu": int(cpu["hessvecs"]), "edges_iters_equal": int(c["edges_iters"]) == int(cpu["edges_iters"]),
            "max_pose_frobenius_diff": worst, "tolerance": 1e-6, "ok": bool(ok)}


# ---------------------------------------------------------------- LCD legs ---
PEAK_FP64 = 78.6e12  # 256 CU x 64 fp64 FMA lanes x 2 flops x 2.4 GHz (not in the in-container guide)


def ransac_roofline(algo, n_cand, tk, ratio="lcd_fp64_stewenius.json"):
    """The dominant LCD kernel, k_ransac_coop (95 % of the verification time):
    issued fp64 lane-flops per candidate from the PMC passes of the same
    workload shape (profiles/lcd_fp64_stewenius.json, scripts/gpu_lcd_pmc3.sh
    + scripts/lcd_pmc_summary.py: a stored ratio, not a counter of this run)
    times this step's candidates over its evented RANSAC time, against the fp64
    vector peak. `ratio`: the stored file for the workload (the hard leg's
    look-alikes run 500 hypotheses each: profiles/lcd_fp64_stewenius_hard.json,
    scripts/gpu_lcd_pmc3.sh TAG scripts/lcd_hard_timing.py N)."""
    out = {"kernel": "k_ransac_coop (2D-2D 5-point RANSAC)", "bound": "fp64 valu", "unit": "FLOP/s",
           "peak": PEAK_FP64, "ransac_ms": tk["ransac_ms"], "knn_ms": tk["knn_ms"],
           "ransac_share": tk["ransac_ms"] / max(tk["knn_ms"] + tk["ransac_ms"], 1e-12),
           "achieved": None, "frac": None}
    f = ROOT / "profiles" / ratio
    if algo != 0 or not f.exists() or tk["ransac_ms"] <= 0:
        out["note"] = "no stored fp64 counts for this solver"
        return out
    d = json.load(open(f))
    per = d["per_candidate"]
    ach = per["fp64_issued_flops"] * n_cand / (tk["ransac_ms"] * 1e-3)
    # gfx950 issues a wave64 VALU instruction over 2 SIMD cycles (SIMD-32,
    # MI355X_MICROARCH.md "Wave scheduling"; the same rate the 78.6 TF fp64
    # peak assumes): the share of the chip's VALU issue capacity this step used
    valu_issue = per["valu_insts"] * n_cand * 2.0 / (tk["ransac_ms"] * 1e-3) / (1024 * 2.4e9)
    out.update({"achieved": ach, "frac": ach / PEAK_FP64, "valu_issue_frac": valu_issue,
                "valu_issue_rule": f"{per['valu_insts']:.4g} VALU wave-instructions per candidate (stored PMC ratio) "
                                   "x 2 SIMD cycles each (SIMD-32) / (1024 SIMDs x 2.4 GHz)",
                "flops_source": f"stored PMC ratio (profiles/{ratio}, {d.get('commit', 'commit not recorded')}): "
                                f"{per['fp64_issued_flops']:.4g} issued fp64 lane-flops per candidate (64 lanes per "
                                "wave instruction, 2 per FMA, whatever the exec mask)",
                "fp64_share_of_valu_insts": d["fractions"]["fp64_share_of_valu_insts"],
                "valu_active_over_wave_cycles": d["fractions"]["valu_active_over_wave_cycles"]})
    lanes = d.get("lanes") or {}
    if lanes.get("valu_thread_util") is not None:
        # exec-mask aware: the share of lanes active in the VALU's active cycles
        # (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU) applied to the issued figure
        u = lanes["valu_thread_util"]
        out.update({"valu_thread_util": u, "achieved_useful": ach * u, "frac_useful": ach * u / PEAK_FP64,
                    "useful_rule": "issued fp64 lane-flops x VALU thread utilisation (stored PMC ratio)"})
    return out


def lcd_leg(args, rank, world, barrier_sync):
    """configs[2]: 50k keyframes x 500 ORB descriptors, one candidate per query
    (half planted loop closures), kNN2 + Lowe -> 2D-2D 5-point RANSAC -> 3D-3D.
    Candidates are sharded across ranks (independent; no collective)."""
    from kmx.lcd import LcdParams, LoopClosureDetector
    from kmx.synth.lcd import make_lcd_pool
    pool = make_lcd_pool(args.lcd_frames, 500, seed=0)
    params = LcdParams(ransac_2d2d_algorithm=args.lcd_algo)
    det = LoopClosureDetector(params, device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
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
    # evented pass: kNN2 and RANSAC kernel times of one step
    det.enable_timing(True)
    det.verify_async(cq, cm)
    det.sync()
    tk = det.read_timing()
    det.enable_timing(False)
    res, _ = det.verify(cq[:256], cm[:256])
    nf = pool.n_feats.astype(np.int64)
    pair_evals = float((nf[cq] * nf[cm]).sum())
    lane_ops = pair_evals * 8  # 32 B per pair: 8 v_sad_u8 lane-ops (L1, the reference matcher)
    out = {"metric": "LC candidates verified/sec", "n_local": int(cq.shape[0]), "steps": args.lcd_steps,
           "elapsed": el, "accepted_frac_first256": sum(r["accepted"] for r in res) / max(len(res), 1),
           "workload": f"configs[2]: {args.lcd_frames} keyframes x 500 ORB descriptors (32 B), "
                       f"{pool.cand_query.shape[0]} candidates, L1 matcher, Lowe 0.7, "
                       f"5-point {'Stewenius' if args.lcd_algo == 0 else 'Nister'} RANSAC "
                       "(thr 1e-6, <=500 it, p 0.995, seed 12345, GCC-9 sampler), 1-point 3D-3D 0.3 m",
           "roofline": ransac_roofline(args.lcd_algo, int(cq.shape[0]), tk),
           "knn2_roofline": {"kernel": "k_knn2 (kNN2 + Lowe)", "bound": "valu", "unit": "lane-op/s",
                             "achieved": lane_ops / (tk["knn_ms"] * 1e-3) if tk["knn_ms"] > 0 else 0.0,
                             "peak": PEAK_VALU_OPS,
                             "frac": (lane_ops / (tk["knn_ms"] * 1e-3)) / PEAK_VALU_OPS if tk["knn_ms"] > 0 else 0.0,
                             "algorithmic": f"{pair_evals:.3e} descriptor pairs x 8 v_sad_u8 lane-ops (32 B each)",
                             "knn_ms": tk["knn_ms"]}}
    out["stream"] = stream_leg(det, pool, cq, cm, args)
    out["hamming"] = hamming_leg(args, pool, cq, cm, barrier_sync)
    det.close()
    if args.lcd_hard > 0:
        out["hard"], hard_pool = hard_leg(args, params, rank, world, barrier_sync)
        if rank == 0 and world == 1:
            out["single"] = single_leg(args, params, pool, hard_pool)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT))
        from oracle import oracle as O
        p = params.to_c()
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


def hard_leg(args, params, rank, world, barrier_sync):
    """The expensive case of a real BoW candidate stream (VERDICT r4 items 3 /
    weak 5): false candidates whose frames share look-alike descriptors (150
    of 500 features: the match frame's descriptor with 5 % of its bits
    flipped, unrelated geometry). They pass Lowe and fail geometry, so every
    one runs the 2D-2D RANSAC to its 500-iteration cap (LcdParams.yaml:64-65).
    Same solver, parameters and batching as the configs[2] leg; the 1-thread C
    restatement on a bounded sample of the same candidates beside it."""
    from kmx.lcd import LcdParams, LoopClosureDetector
    from kmx.synth.lcd import make_lcd_pool
    C_ = args.lcd_hard
    pool = make_lcd_pool(2 * C_, 500, true_frac=0.0, false_frac=0.3, seed=3)
    det = LoopClosureDetector(params, device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
    det.set_pool(pool)
    cq = pool.cand_query[0::2][rank::world].copy()  # (2k, 2k + 1): the look-alike pairs
    cm = pool.cand_match[0::2][rank::world].copy()
    det.verify_async(cq, cm)
    det.sync()
    barrier_sync()
    steps = 2
    t0 = time.perf_counter()
    for _ in range(steps):
        det.verify_async(cq, cm)
    det.sync()
    barrier_sync()
    el = time.perf_counter() - t0
    det.enable_timing(True)
    det.verify_async(cq, cm)
    det.sync()
    tk = det.read_timing()
    res, _ = det.verify(cq[:512], cm[:512])
    det.close()
    its = np.array([r["iterations_2d2d"] for r in res])
    nm = np.array([r["n_matches"] for r in res])
    out = {"metric": "LC candidates verified/sec (hard: look-alikes that fail geometry)", "unit": "candidates/s",
           "value": steps * len(cq) / el * world, "n_local": int(len(cq)), "steps": steps, "elapsed": el,
           "ransac_ms": tk["ransac_ms"], "knn_ms": tk["knn_ms"],
           "roofline": ransac_roofline(args.lcd_algo, len(cq), tk, "lcd_fp64_stewenius_hard.json"),
           "first512": {"accepted": int(sum(r["accepted"] for r in res)), "iterations_2d2d_mean": float(its.mean()),
                        "iterations_2d2d_min": int(its.min()), "matches_after_lowe_mean": float(nm.mean())},
           "workload": f"{len(cq)} candidates of {2 * C_} synthetic frames x 500 ORB features: 150 look-alike "
                       "descriptors per pair (5 % of bits flipped), no true correspondence; "
                       + ("Stewenius" if args.lcd_algo == 0 else "Nister") + " RANSAC, reference parameters"}
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT))
        from oracle import oracle as O
        p = params.to_c()
        n, t0c, done = 0, time.perf_counter(), 0.0
        while done < args.cpu_seconds * 0.25 and n < len(cq):
            O.lcd_verify(p, pool, cand_query=cq[n:n + 8], cand_match=cm[n:n + 8], masks=False)
            n += 8
            done = time.perf_counter() - t0c
        out["cpu_baseline"] = {"value": n / done, "unit": "candidates/s", "cores": 1, "kind": "port",
                               "sample": f"first {n} hard candidates, oracle/lcd_oracle.c, 1 thread, {done:.1f} s"}
        out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    return out, pool


def single_leg(args, params, pool, hard_pool):
    """Call-for-call latency: the reference verifies ONE
    candidate per call on its verification thread (verifyLoopSpin ->
    computeMatchedIndices -> geometricVerificationNister -> recoverPose,
    drawio:2638-2657; INTEGRATION.md section 2 binds exactly that). Here the
    same three calls per candidate through the Python mirror (kmx_lcd_match,
    kmx_lcd_verify_matches STAGE_2D2D, then STAGE_RECOVER on its inliers),
    host argument handling and the device round trips included, for planted
    loop closures of configs[2] and for hard candidates; the 1-thread C
    restatement's time for the same candidates (one lcd_verify call each)
    beside it."""
    from kmx.lcd import LoopClosureDetector
    sys.path.insert(0, str(ROOT))
    from oracle import oracle as O
    out = {}
    for name, pl, idx in (("planted", pool, np.arange(0, 64, 2)), ("hard", hard_pool, np.arange(0, 16, 2))):
        det = LoopClosureDetector(params, device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
        det.set_pool(pl)
        q, m = pl.cand_query[idx], pl.cand_match[idx]
        lat, acc = [], 0
        for rep in range(2):  # the first pass warms the call path up
            lat = []
            for a, b in zip(q, m):
                t0 = time.perf_counter()
                iq, im = det.computeMatchedIndices(int(a), int(b))
                ok, iq2, im2, T = det.geometricVerificationNister(int(a), int(b), iq, im)
                if ok:
                    ok2, T2, _ = det.recoverPose(int(a), int(b), iq2, im2, T)
                    acc += int(ok2) if rep else 0
                lat.append(time.perf_counter() - t0)
        det.close()
        cpu = []
        if not args.no_cpu:
            p = params.to_c()
            for a, b in zip(q, m):
                t0 = time.perf_counter()
                O.lcd_verify(p, pl, cand_query=np.array([a], np.int32), cand_match=np.array([b], np.int32),
                             masks=False)
                cpu.append(time.perf_counter() - t0)
        lat = np.array(lat) * 1e3
        out[name] = {"candidates": int(len(q)), "accepted": acc, "gpu_ms_median": float(np.median(lat)),
                     "gpu_ms_max": float(lat.max()),
                     "cpu_ms_median": float(np.median(cpu) * 1e3) if cpu else None,
                     "gpu_over_cpu_latency": (float(np.median(lat)) / (np.median(cpu) * 1e3)) if cpu else None}
    out["note"] = ("one candidate per call chain (computeMatchedIndices, geometricVerificationNister, recoverPose), "
                   "as the reference's verification thread; a call this small takes the spread form (its hypotheses "
                   "on many waves at once, the serial loop's control replayed: lcd.hip k_rs_hyps (its last wave per candidate replays) / "
                   "k_rs_finish)")
    return out


def stream_leg(det, pool, cq, cm, args):
    """The streaming boundary on the resident configs[2] pool (VERDICT r3
    item 1): (a) addVLCFrame cost — 1,000 frames appended one call each
    (kmx_lcd_add_frames: host-to-device copy of the frame, the pool grows by
    capacity doubling; the first append doubles the 50k-frame pool with one
    device-to-device copy, included); (b) geometricVerificationNister +
    recoverPose on caller-supplied correspondences (kmx_lcd_verify_matches,
    both stages, no kNN2) over the step's candidates with the kNN2 pairs as
    input in CSR form — host argument checks and the CSR upload included, as a
    caller would pay them."""
    n_add = 1000
    src = np.arange(n_add) % pool.n_frames
    ts = []
    t0 = time.perf_counter()
    for f in src:
        a = time.perf_counter()
        det.add_frames(pool.n_feats[f:f + 1], pool.desc[f:f + 1], pool.bearings[f:f + 1], pool.points[f:f + 1])
        ts.append(time.perf_counter() - a)
    el = time.perf_counter() - t0
    ts = np.array(ts) * 1e6
    info = det.pool_info()
    out = {"frames_added": n_add, "us_per_frame": el * 1e6 / n_add, "us_per_frame_median": float(np.median(ts)),
           "us_first_append": float(ts[0]), "bytes_per_frame": int(pool.max_feats * (32 + 24 + 24) + 4),
           "pool_after": info,
           "note": "one kmx_lcd_add_frames call per frame from pageable host memory (copied into a pinned, "
                   "mapped staging area and scattered into the pool by one kernel); the first call doubles the "
                   "resident pool (device-to-device copy)"}
    pairs, k = det.match(cq, cm)
    mptr = np.zeros(len(cq) + 1, np.int64)
    mptr[1:] = np.cumsum(k)
    sel = np.arange(pairs.shape[1])[None, :] < k[:, None]
    iq, im = pairs[:, :, 0][sel], pairs[:, :, 1][sel]  # the kNN2 pairs as CSR, candidate order
    det.verify_matches_csr(cq[:64], cm[:64], mptr[:65], iq, im)  # warmup
    a = time.perf_counter()
    res, _ = det.verify_matches_csr(cq, cm, mptr, iq, im, stages=3, as_arrays=True)
    el2 = time.perf_counter() - a
    out["verify_matches"] = {"metric": "LC candidates verified/sec (caller-supplied correspondences, both stages)",
                             "value": len(cq) / el2, "n": int(len(cq)), "elapsed": el2,
                             "pairs": int(k.sum()), "accepted": int((res["accepted"] != 0).sum()),
                             "results": "one structured array (verify_matches_csr as_arrays)"}
    return out


def hamming_leg(args, pool, cq, cm, barrier_sync):
    """configs[2] with the Hamming matcher north_star names (BruteForce-Hamming
    over 256 bits, `norm: hamming`), same pool and candidates as the L1 leg
    (the reference build's matcher, kimera_multi_lcd.patch:33-35)."""
    from kmx.lcd import LcdParams, LoopClosureDetector
    det = LoopClosureDetector(LcdParams(ransac_2d2d_algorithm=args.lcd_algo, norm="hamming"),
                              device=int(os.environ.get("KMX_BENCH_DEVICE", "0")))
    det.set_pool(pool)
    det.verify_async(cq, cm)
    det.sync()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.lcd_steps):
        det.verify_async(cq, cm)
    det.sync()
    barrier_sync()
    el = time.perf_counter() - t0
    det.enable_timing(True)
    det.verify_async(cq, cm)
    det.sync()
    tk = det.read_timing()
    res, _ = det.verify(cq[:256], cm[:256])
    det.close()
    nf = pool.n_feats.astype(np.int64)
    pair_evals = float((nf[cq] * nf[cm]).sum())
    lane_ops = pair_evals * 16  # 8 words per pair, v_xor_b32 + v_bcnt_u32_b32 (accumulating) each
    return {"metric": "LC candidates verified/sec (Hamming matcher)", "unit": "candidates/s", "elapsed": el, "steps": args.lcd_steps,
            "accepted_frac_first256": sum(r["accepted"] for r in res) / max(len(res), 1),
            "ransac_ms": tk["ransac_ms"], "knn_ms": tk["knn_ms"],
            "knn2_roofline": {"kernel": "k_knn2 (kNN2 + Lowe, Hamming)", "bound": "valu", "unit": "lane-op/s",
                              "achieved": lane_ops / (tk["knn_ms"] * 1e-3) if tk["knn_ms"] > 0 else 0.0,
                              "peak": PEAK_VALU_OPS,
                              "frac": (lane_ops / (tk["knn_ms"] * 1e-3)) / PEAK_VALU_OPS if tk["knn_ms"] > 0 else 0.0,
                              "algorithmic": f"{pair_evals:.3e} descriptor pairs x (8 v_xor_b32 + 8 v_bcnt_u32_b32) "
                                             "lane-ops (256 bits each)"}}


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


def load_traffic(config="synth100k"):
    """PMC traffic of k_hess measured for this config (scripts/gpu_pmc_hess.sh ->
    scripts/hess_traffic.py); None when that config was not profiled."""
    f = ROOT / "profiles" / f"hessvec_traffic_{config}.json"
    if not f.exists() and config == "synth100k":
        f = ROOT / "profiles" / "hessvec_traffic.json"
    if f.exists():
        try:
            return json.loads(f.read_text())
        except Exception:
            return None
    return None


def _coll_device(dist):
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def _gather(dist, world, vals, ops):
    """Combine per-rank scalars across ranks: ops[i] in {"max", "sum"}."""
    if dist is None:
        return vals
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=_coll_device(dist))
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    a = torch.stack(parts).cpu().numpy()
    return [float(a[:, i].max() if op == "max" else a[:, i].sum()) for i, op in enumerate(ops)]


def _runtime():
    """Which librccl / libamdhip64 serve libkmx in this process (torch bundles
    copies of the same SONAME; load order decides), with versions."""
    try:
        from kmx import abi
        return abi.runtime_info()
    except Exception as e:  # noqa: BLE001 - reported, never fatal to the measurement
        return {"error": str(e)}


def _gather_each(dist, world, vals):
    """Every rank's scalars, in rank order (a list of lists)."""
    if dist is None:
        return [list(vals)]
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=_coll_device(dist))
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def dpgo_leg(g, X0, P, args, rank, world, local_rank, dist, steps, barrier, replay=True, want_snapshot=False):
    """Burn-in + warmup, snapshot, time `steps` rounds (max over ranks), then
    replay the same rounds from the snapshot with HIP events around every
    Hess-vec launch. Returns the team totals."""
    from kmx.dpgo.driver import RBCDDriver
    drv = RBCDDriver(P, g, rank=rank, world=world, device=local_rank if world > 1 else 0)
    drv.initialize(X0)

    def sync():
        drv.solver.sync()
        barrier()

    hv_ms, hv_bytes, hv_n, same, snap = 0.0, 0.0, 0, None, None
    el_local = None
    if args.profile:  # every round evented and counted (the rocprofv3 / PMC passes divide by these)
        drv.solver.read_counters()
        drv.solver.enable_timing(True)
        t0 = time.perf_counter()
        drv.run_async(args.burn_in + args.warmup + steps)
        sync()
        el = time.perf_counter() - t0
        c = drv.solver.read_counters()
        hv_ms, hv_bytes, hv_n = c["hessvec_ms_total"], c["hessvec_alg_bytes"], c["hessvec_launches"]
    else:
        drv.run_async(args.burn_in + args.warmup)
        sync()
        snap = snapshot(drv) if (replay or want_snapshot) else None
        drv.solver.read_counters()  # reset device counters and event pool
        sync()
        t0 = time.perf_counter()
        drv.run_async(steps)
        drv.solver.sync()
        el_local = time.perf_counter() - t0  # this rank's own rounds, before waiting for its peers
        barrier()
        el = time.perf_counter() - t0
        c = drv.solver.read_counters()
    if snap is not None and replay:
        restore(drv, snap)
        sync()
        drv.solver.enable_timing(True)
        drv.run_async(steps)
        sync()
        drv.solver.enable_timing(False)
        r = drv.solver.read_counters()
        hv_ms, hv_bytes, hv_n = r["hessvec_ms_total"], r["hessvec_alg_bytes"], r["hessvec_launches"]
        same = all(r[k] == c[k] for k in ("edges_iters", "hessvecs", "block_updates", "gnc_updates"))
    xs, xr = drv.exchange_rows
    native = bool(drv.native)
    mode = drv.exchange_mode
    mem = drv.solver.memory()[0]
    tot = _gather(dist, world, [el, float(c["edges_iters"]), float(c["hessvecs"]), float(c["block_updates"]),
                                float(c["gnc_updates"]), hv_ms, hv_bytes, float(hv_n), float(xs), float(xr),
                                float(mem), 1.0 if same in (None, True) else 0.0],
                  ["max", "sum", "sum", "sum", "max", "sum", "sum", "sum", "max", "max", "max", "sum"])
    per_rank = _gather_each(dist, world, [el_local if el_local is not None else el, float(c["edges_iters"])])
    if not want_snapshot:
        drv.solver.close()
        drv = None
    return {"per_rank": [{"rank": r, "ms_per_step": 1e3 * v[0] / steps, "edges_iters": int(v[1])}
                         for r, v in enumerate(per_rank)],
            "el": tot[0], "edges_iters": tot[1], "hessvecs": tot[2], "block_updates": tot[3],
            "gnc_updates": int(tot[4]), "hv": (tot[5], tot[6], int(tot[7])), "xrows": (int(tot[8]), int(tot[9])),
            "mem_max": int(tot[10]), "replay_identical": (tot[11] == world) if replay and snap is not None else None,
            "snap": snap, "native": native, "exchange": mode, "drv": drv}


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
    P.tileIncidences = args.tile_incidences
    headline = args.scaling if world > 1 else "strong"
    t_gen = time.perf_counter()
    g, X0 = make_workload(args.config, world, headline)
    gen_s = time.perf_counter() - t_gen
    if args.tcg_form == "auto":
        args.tcg_form = "standard"
    P.localOptimizationParams.tCG_form = args.tcg_form
    want_cpu = rank == 0 and world == 1 and not args.no_cpu and not args.profile
    leg = dpgo_leg(g, X0, P, args, rank, world, local_rank, dist, args.steps, barrier,
                   replay=not args.no_replay and not args.profile, want_snapshot=want_cpu)
    if args.profile:
        args.steps += args.burn_in + args.warmup  # the profile run counts every round
    el, edges_iters = leg["el"], leg["edges_iters"]
    hv_ms, hv_bytes, hv_n = leg["hv"]
    value = edges_iters / el
    achieved = hv_bytes / (hv_ms * 1e-3) if hv_ms > 0 else 0.0
    traffic = load_traffic(args.config)
    ps_bytes = 8 * 4 * P.r
    w0 = args.burn_in + args.warmup
    if headline == "weak" and world > 1:
        workload = (f"configs[3] shape per GPU (weak scaling): {g.n_total} poses / {g.m} edges, {g.n_robots} robot "
                    f"blocks over {world} GPUs ({g.n_robots // world} per GPU, 100k poses / 500k edges each), "
                    "20% outlier LCs, f_inter 0.10, GNC-TLS (inner iterations 20)")
    else:
        name = "configs[3] synth100k" if args.config == "synth100k" else f"{args.config} (cold config)"
        workload = (f"{name}: {g.n_total} poses / {g.m} edges, {g.n_robots} robot blocks"
                    + (f" split over {world} GPUs (strong scaling)" if world > 1 else "")
                    + ", 20% outlier LCs, f_inter 0.10, GNC-TLS (inner iterations 20)")
    nr = max(args.steps, 1)
    out = {
        "metric": "dpgo edges*iters/sec (+ LC candidates verified/sec in 'lcd')",
        "value": value,
        "unit": "edges*iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el / nr,
        "higher_is_better": True,
        "scaling": headline,
        "vs_baseline": None,
        "exchange": leg["exchange"],
        "per_rank": leg["per_rank"],
        "runtime": _runtime(),
        "dtype": "f64",
        "data": "synthetic (seeded numpy PCG64; Campus bags unavailable offline)",
        "config": {
            "workload": workload,
            "robots": g.n_robots, "poses": g.n_total, "edges": g.m, "r": P.r,
            "rtr_iterations": 1, "tcg_max": 10, "schedule": "concurrent", "tcg_form": args.tcg_form,
            "timed_rounds": [w0, w0 + args.steps] if not args.profile else [0, args.steps],
            "burn_in_rounds": 0 if args.profile else args.burn_in,
            "parallelism": f"robot blocks {g.n_robots} over {world} GPU(s)"
                           + ((", public poses + status exchanged "
                               + ("over RCCL (ncclSend/ncclRecv group inside each round, on the solver's stream)"
                                  if leg["native"] else
                                  f"by torch.distributed all_to_all_single ({dist.get_backend()}) per round"))
                              if world > 1 else ""),
            "exchange_rows_per_round": {"sent_max": leg["xrows"][0], "recv_max": leg["xrows"][1],
                                        "recv_bytes_max": leg["xrows"][1] * ps_bytes},
            "graph_gen_s": round(gen_s, 1),
            "device_bytes_per_gpu": leg["mem_max"],
        },
        "work": {
            "hessvecs_per_round": leg["hessvecs"] / nr,
            "hessvecs_per_block_update": leg["hessvecs"] / max(leg["block_updates"], 1),
            "edges_hessvecs_per_s": None,
            "gnc_updates_in_window": leg["gnc_updates"],
        },
    }
    # edges x Hess-vecs: every Hess-vec of a block update touches its block's edges
    out["work"]["edges_hessvecs_per_s"] = value * out["work"]["hessvecs_per_block_update"]
    if hv_n:
        out["roofline"] = {
            "kernel": ("k_hess (tCG Hessian-vector product)" if args.tcg_form == "standard" else
                       "k_step (one-sync tCG step: update + Hessian-vector product)"),
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": PEAK_HBM / 1e9,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM,
            # NOT a counter read in this run: the PMC bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
            # MI355X_MICROARCH.md HBM section) of a separate rocprofv3 --pmc pass, stored as a ratio to
            # the algorithmic bytes of the same dispatches (scripts/gpu_pmc_hess.sh ->
            # profiles/hessvec_traffic_<config>.json) and multiplied by this run's algorithmic bytes
            "traffic": (traffic["traffic_over_alg"] * hv_bytes / max(hv_n, 1)) if traffic else None,
            "traffic_over_alg": traffic["traffic_over_alg"] if traffic else None,
            "traffic_source": (f"stored PMC ratio from profiles/hessvec_traffic_{args.config}.json "
                               "(separate rocprofv3 --pmc pass) x this run's algorithmic bytes") if traffic else None,
            "launches": hv_n,
            "measured_over": (f"replay of the timed rounds {w0}..{w0 + args.steps} from their snapshot, HIP events "
                              "of each k_hess launch that ran a Hess-vec") if not args.profile else
                             f"rounds 0..{args.steps} (profile run), HIP events of each k_hess launch that ran "
                             "a Hess-vec",
            "event_form": "hipExtLaunchKernelGGL start / stop events: the dispatch's own timestamps (no event "
                          "packets between launches)",
            "replay_identical": leg["replay_identical"],
            "avg_launch_us": 1e3 * hv_ms / max(hv_n, 1),
            "hess_ms_per_round": hv_ms / nr,
            "alg_bytes_per_launch": hv_bytes / max(hv_n, 1),
            "alg_bytes_rule": "128 B per local edge + 2 x 160 B per pose of every robot in tCG (SURVEY.md §8d)",
        }
    xst = args.steps if args.extra_steps is None else args.extra_steps
    if world > 1 and xst > 0 and not args.profile:
        other = "weak" if headline == "strong" else "strong"
        del g, X0
        go, X0o = make_workload(args.config, world, other)
        st = dpgo_leg(go, X0o, P, args, rank, world, local_rank, dist, xst, barrier, replay=False)
        out[other] = {"value": st["edges_iters"] / st["el"], "unit": "edges*iters/s", "steps": xst,
                      "ms_per_step": 1e3 * st["el"] / max(xst, 1),
                      "workload": f"{go.n_total} poses / {go.m} edges, {go.n_robots} robot blocks over {world} GPUs "
                                  f"({other} scaling)",
                      "exchange_rows_per_round": {"sent_max": st["xrows"][0], "recv_max": st["xrows"][1]}}
        g, X0 = go, X0o
    if want_cpu and leg["snap"] is not None:
        lib, march = _native_oracle()
        if lib:
            os.environ["ORC_LIB"] = lib
        # the host share for the all-cores form: OMP_NUM_THREADS where set (the
        # GPU box sets it to the job's CPU share), else the affinity mask
        share = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
        inner = max(1, share // g.n_robots)
        variants = [(g.n_robots, 1), (1, 1)] + ([(g.n_robots, inner)] if inner > 1 else [])
        cpu = cpu_baseline(g, P, leg["snap"], args.steps, args.cpu_seconds, variants)
        team, one = cpu[(g.n_robots, 1)], cpu[(1, 1)]
        out["parity"] = gpu_parity(leg["drv"], leg["snap"], team)
        leg["drv"].solver.close()
        out["cpu_baseline"] = {
            "value": team["value"], "unit": "edges*iters/s", "cores": g.n_robots, "kind": "port",
            "sample": f"rounds {w0}..{w0 + team['rounds']} of the timed window (the GPU's snapshot), "
                      f"oracle/dpgo_oracle.c -O3 -march={march}, one OpenMP thread per robot block "
                      f"({g.n_robots}), {team['seconds']:.1f} s",
            "ms_per_step": team["ms_per_step"], "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "cores_note": "one thread per robot block, the reference's execution model: dpgo runs one "
                          "single-threaded PGOAgent per robot (one process per robot in 1014-example.yaml), so "
                          "the reference CPU path of this 8-block team uses 8 cores whatever the host has; the "
                          "restatement's per-block loops sum in a fixed edge order (the frozen fixtures pin it). "
                          "all_cores spends the job's whole CPU share by adding threads inside each block update; "
                          "it is slower than one thread per block (its gather form evaluates every edge at both "
                          "endpoints, and the per-block loops are too short for nested teams), so the "
                          "one-thread-per-block figure is the fastest CPU number this restatement has",
            "edge_count_rule": "same as the GPU counter: a block update counts its local edges when its "
                               "gradient norm passed gradnorm_tol (csrc/pgo.hip control_on RED_GRAD)",
            "single_thread": {"value": one["value"], "cores": 1, "rounds": one["rounds"],
                              "ms_per_step": one["ms_per_step"]},
        }
        if inner > 1:
            ac = cpu[(g.n_robots, inner)]
            out["cpu_baseline"]["all_cores"] = {
                "value": ac["value"], "cores": g.n_robots * inner, "share": share, "rounds": ac["rounds"],
                "ms_per_step": ac["ms_per_step"],
                "form": f"{g.n_robots} blocks x {inner} threads inside each block update (oracle "
                        "orc_pgo_round_mt2: edge terms gathered per pose, per-pose loops and dot products "
                        "split; equal to the serial restatement to rounding)"}
    if not args.no_lcd and not args.profile:
        lcd, lcd_cpu = lcd_leg(args, rank, world, barrier)
        n_local, lel = _gather(dist, world, [float(lcd["n_local"] * lcd["steps"]), lcd["elapsed"]], ["sum", "max"])
        lcd["value"] = n_local / lel
        lcd["unit"] = "candidates/s"
        lcd["ms_per_step"] = 1e3 * lel / lcd["steps"]
        del lcd["elapsed"]
        hm = lcd["hamming"]
        n_h, hel = _gather(dist, world, [float(lcd["n_local"] * hm["steps"]), hm["elapsed"]], ["sum", "max"])
        hm["value"] = n_h / hel
        hm["ms_per_step"] = 1e3 * hel / hm["steps"]
        del hm["elapsed"]
        if lcd_cpu:
            lcd["cpu_baseline"] = lcd_cpu
        bow, bow_cpu = bow_leg(args, rank, world, barrier)
        n_local, bel = _gather(dist, world, [float(bow["n_local"] * bow["steps"]), bow["elapsed"]], ["sum", "max"])
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
