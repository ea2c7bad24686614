"""k_ransac_coop wave stamps (diagnostic; KMX_RS_PROF=2): per-candidate wave
latency under load vs nearly alone, and the resident waves over the launch.
usage: python scripts/lcd_stamps.py [n_candidates] [algo]"""
import ctypes as C, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
os.environ["KMX_RS_PROF"] = "2"
import numpy as np
from kmx import abi
from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
algo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
pool = make_lcd_pool(n, 500, seed=0)
det = LoopClosureDetector(LcdParams(ransac_2d2d_algorithm=algo))
det.set_pool(pool)
fn = abi.lib().kmx_lcd_debug_wave_stamps
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]


only_true = os.environ.get("STAMPS_ONLY_TRUE") == "1"  # every candidate with RANSAC work


def run(k):
    cq, cm = pool.cand_query, pool.cand_match
    if only_true:
        cq, cm = cq[0::2], cm[0::2]
        k = min(k, len(cq))
    res, _ = det.verify(cq[:k], cm[:k])
    buf = (C.c_ulonglong * (2 * k))()
    fn(buf, k)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(k, 2).astype(np.int64)
    K = np.array([r["n_matches"] for r in res])
    it = np.array([r["iterations_2d2d"] for r in res])
    return st, K, it


for k in (64, 512, n):
    run(min(k, n))  # warm
    st, K, it = run(min(k, n))
    k = len(K)
    t0 = st[:, 0].min()
    s, e = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # us
    live = K >= 5
    dur = (e - s)[live]
    span = e.max()
    # resident planted waves over time (sampled every 10 us)
    ts = np.arange(0.0, span, 10.0)
    res = np.array([np.sum((s[live] <= t) & (e[live] > t)) for t in ts])
    allres = np.array([np.sum((s <= t) & (e > t)) for t in ts])
    print(f"   all waves resident: mean {allres.mean():.1f}, max {allres.max()}; latency of waves without RANSAC "
          f"{(e - s)[~live].mean() if (~live).any() else 0:.1f} us", flush=True)
    print(f"{k:6d} candidates ({live.sum()} with RANSAC, mean {it[live].mean():.1f} hypotheses): span {span:8.0f} us, "
          f"{live.sum() / span * 1e6:9.0f} planted/s; wave latency mean {dur.mean():7.0f} us, p50 {np.median(dur):7.0f}, "
          f"p90 {np.percentile(dur, 90):7.0f}, per hypothesis {np.sum(dur) / max(it[live].sum(), 1):6.1f} us; "
          f"resident planted waves mean {res.mean():7.1f}, max {res.max()}", flush=True)
    if k == n:
        # first dispatch wave of the launch vs the rest
        order = np.argsort(s[live])
        q = max(1, len(order) // 10)
        print(f"   first 10% started: latency {dur[order[:q]].mean():.0f} us; last 10%: {dur[order[-q:]].mean():.0f} us; "
              f"start of last planted {s[live].max():.0f} us", flush=True)
