"""Quick LCD throughput probe (diagnostic)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
import numpy as np
from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
t = time.time(); pool = make_lcd_pool(n, 500, seed=0); print("gen", time.time() - t, flush=True)
det = LoopClosureDetector(LcdParams()); det.set_pool(pool)
det.verify(pool.cand_query[:64], pool.cand_match[:64])
for rep in range(2):
    t = time.time(); det.verify_async(pool.cand_query, pool.cand_match); det.sync(); el_gpu = time.time() - t
    print(f"verify_async: {n} candidates in {el_gpu*1e3:.1f} ms -> {n/el_gpu:.0f} cand/s", flush=True)
    t = time.time(); res, _ = det.verify(pool.cand_query, pool.cand_match); el = time.time() - t
    acc = sum(r["accepted"] for r in res)
    print(f"{n} candidates in {el*1e3:.1f} ms -> {n/el:.0f} cand/s, accepted {acc}, mean iters "
          f"{np.mean([r['iterations_2d2d'] for r in res[0::2]]):.1f} (true) "
          f"{np.mean([r['iterations_2d2d'] for r in res[1::2]]):.1f} (false), mean K "
          f"{np.mean([r['n_matches'] for r in res[0::2]]):.0f} / {np.mean([r['n_matches'] for r in res[1::2]]):.0f}",
          flush=True)
# back-to-back calls (the bench's LCD steps): a call's kNN2 can fill the
# previous call's RANSAC tail
t = time.time()
for _ in range(4):
    det.verify_async(pool.cand_query, pool.cand_match)
det.sync()
el4 = time.time() - t
print(f"back-to-back x4: {4 * n / el4:.0f} cand/s ({el4 * 1e3 / 4:.1f} ms per call)", flush=True)
# a longer stream of calls (the detector keeps several calls in flight)
t = time.time()
for _ in range(16):
    det.verify_async(pool.cand_query, pool.cand_match)
det.sync()
el16 = time.time() - t
print(f"back-to-back x16: {16 * n / el16:.0f} cand/s ({el16 * 1e3 / 16:.1f} ms per call)", flush=True)
