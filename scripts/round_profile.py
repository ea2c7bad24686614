"""Per-round work of the configs[3] bench run: Hess-vecs, tCG steps and GNC
updates per round, over `rounds` rounds from the bench's initial iterate
(the stats path: one synchronised round at a time)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from kmx.dpgo.driver import RBCDDriver  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
g, X0 = bench.make_workload("synth100k")
P = bench.params()
drv = RBCDDriver(P, g, device=0)
drv.initialize(X0)
out = []
for k in range(rounds):
    t0 = time.perf_counter()
    st = drv.step(with_stats=True)
    dt = time.perf_counter() - t0
    hv = [s["hessvecs"] for s in st]
    out.append({"round": k, "hessvecs": int(sum(hv)), "tcg_max": int(max(s["tcg_iterations"] for s in st)),
                "accepted": int(sum(s["accepted"] for s in st)), "gnc_updates": drv.weight_updates,
                "ms": 1e3 * dt})
print(json.dumps(out))
