"""Call-for-call LCD latency, call by call (bench.py single_leg's chain):
kmx_lcd_match, kmx_lcd_verify_matches(STAGE_2D2D), (STAGE_RECOVER) for one
candidate at a time, each timed on the host; run under rocprofv3
--kernel-trace --memory-copy-trace to see the device side of each call.
usage: lcd_single.py [planted|hard] [candidates]"""
import os
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
from kmx.lcd import LcdParams, LoopClosureDetector
from kmx.synth.lcd import make_lcd_pool

kind = sys.argv[1] if len(sys.argv) > 1 else "planted"
nc = int(sys.argv[2]) if len(sys.argv) > 2 else 16
p = LcdParams()
if kind == "planted":
    pool = make_lcd_pool(256, 500, seed=3)
    idx = np.arange(0, 2 * nc, 2)
else:
    pool = make_lcd_pool(512, 500, true_frac=0.0, false_frac=0.3, seed=3)  # bench.py hard_leg's look-alikes
    idx = np.arange(0, 2 * nc, 2)
det = LoopClosureDetector(p)
det.set_pool(pool)
q, m = pool.cand_query[idx], pool.cand_match[idx]
for rep in range(3):
    t = np.zeros((len(q), 3))
    for i, (a, b) in enumerate(zip(q, m)):
        t0 = time.perf_counter()
        iq, im = det.computeMatchedIndices(int(a), int(b))
        t1 = time.perf_counter()
        ok, iq2, im2, T = det.geometricVerificationNister(int(a), int(b), iq, im)
        t2 = time.perf_counter()
        if ok:
            det.recoverPose(int(a), int(b), iq2, im2, T)
        t3 = time.perf_counter()
        t[i] = (t1 - t0, t2 - t1, t3 - t2)
    med = np.median(t, axis=0) * 1e3
    print(f"pass {rep}: match {med[0]:.3f} ms, 2d2d {med[1]:.3f} ms, recover {med[2]:.3f} ms, "
          f"chain {np.median(t.sum(1)) * 1e3:.3f} ms")
det.close()
if os.environ.get("KMX_RS_PROF") == "3":  # the recovery tail's phase timers (lcd.hip ransac_tail<true>)
    import ctypes as C
    from kmx import abi
    fn = abi.lib().kmx_lcd_debug_phase_times
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 16)()
    fn(buf)
    calls = max(buf[15], 1)
    print(f"recovery tail: {buf[15]} calls, n3 mean {buf[14] / calls:.1f}; per call: count {buf[11] / 100 / calls:.1f} us, "
          f"final pass {buf[12] / 100 / calls:.1f} us, refit {buf[13] / 100 / calls:.1f} us")
if os.environ.get("KMX_RS_PROF") == "1":  # the spread form's hypothesis waves (lcd.hip k_rs_hyps)
    import ctypes as C
    from kmx import abi
    fn = abi.lib().kmx_lcd_debug_phase_times
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 16)()
    fn(buf)
    w = max(buf[15], 1)
    names = {0: "sample", 1: "nullspace", 2: "system", 7: "hessenberg", 8: "hqr", 9: "eigvec", 10: "decomp",
             12: "compaction", 13: "scoring", 11: "whole wave"}
    print(f"{buf[15]} hypothesis waves; per wave (us): " +
          ", ".join(f"{n} {buf[i] / 100 / w:.1f}" for i, n in names.items()))
