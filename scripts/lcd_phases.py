"""k_ransac_coop phase timers (diagnostic; KMX_RS_PROF=1): wall-clock time per
hypothesis phase summed over the first 64 candidates."""
import ctypes as C, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
os.environ["KMX_RS_PROF"] = "1"
import numpy as np
from kmx import abi
from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool
pool = make_lcd_pool(2000, 500, seed=0)
algo = int(sys.argv[1]) if len(sys.argv) > 1 else 0
det = LoopClosureDetector(LcdParams(ransac_2d2d_algorithm=algo)); det.set_pool(pool)
L = abi.lib()
fn = L.kmx_lcd_debug_phase_times
fn.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 16)()
res, _ = det.verify(pool.cand_query[:128], pool.cand_match[:128])
fn(buf)
res, _ = det.verify(pool.cand_query[:128], pool.cand_match[:128])
fn(buf)
hyp = sum(r["iterations_2d2d"] for r in res[:64])
names = ["sample", "nullspace", "system", "gj", "roots", "models", "scoring"]
tot = sum(buf[i] for i in range(7))
print(f"hypotheses (first 64 candidates): {hyp}")
for i, n in enumerate(names):
    print(f"{n:10s} {buf[i] / 100.0 / max(hyp, 1):9.2f} us/hypothesis  {100.0 * buf[i] / max(tot, 1):5.1f} %")
sub = (["  hessenb", "  hqr", "  eigvec", "  decomp"] if algo == 0 else ["  poly", "  sturm", "  isolate", "  refine"])
for i, n in zip(range(7, 11), sub):
    print(f"{n:10s} {buf[i] / 100.0 / max(hyp, 1):9.2f} us/hypothesis (within {'models' if algo == 0 else 'roots'})")
