"""The hard LCD workload of bench.py's hard_leg (look-alike candidates that
pass Lowe and run the 2D-2D RANSAC to its 500-iteration cap), for PMC passes
(scripts/gpu_lcd_pmc3.sh TAG scripts/lcd_hard_timing.py N): one warm-up call
of 64 candidates, then 4 single calls of N candidates, each synchronised, so
every timed k_ransac_coop dispatch is one call's."""
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pool = make_lcd_pool(2 * n, 500, true_frac=0.0, false_frac=0.3, seed=3)
cq, cm = pool.cand_query[0::2].copy(), pool.cand_match[0::2].copy()
det = LoopClosureDetector(LcdParams())
det.set_pool(pool)
det.verify(cq[:64], cm[:64])
for rep in range(4):
    t = time.time()
    det.verify_async(cq, cm)
    det.sync()
    el = time.time() - t
    print(f"hard: {len(cq)} candidates in {el * 1e3:.1f} ms -> {len(cq) / el:.0f} cand/s", flush=True)
det.close()
