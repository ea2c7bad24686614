"""Per-launch HBM traffic of k_hess from the PMC passes of scripts/gpu_pmc_hess.sh.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. MI355X_MICROARCH.md (HBM):
FETCH_SIZE on gfx950 reports 1/2 of the bytes of wide coalesced reads -> x2;
WRITE_SIZE is taken as is. Each pass is normalised by its own bench JSON
(launch count and algorithmic bytes of exactly the profiled dispatches).
usage: python scripts/hess_traffic.py gpurun_out/<tag> [profiles/hessvec_traffic.json]"""
import csv, glob, json, sys
from pathlib import Path

d = Path(sys.argv[1])
out = {"kernel": "k_hess", "source": str(d), "fetch_correction": 2.0}
for i, ctr in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE"), (3, None)):
    js = json.loads((d / f"p{i}.json").read_text().strip().splitlines()[-1])
    n, alg = js["roofline"]["launches"], js["roofline"]["alg_bytes_per_launch"]
    tot = {}
    cnt = 0
    for f in glob.glob(str(d / f"p{i}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_hess" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            cnt += 1
    if ctr == "FETCH_SIZE":
        out["fetch_bytes_per_launch"] = 2.0 * 1024 * tot[ctr] / n
        out["alg_bytes_per_launch"] = alg
        out["launches_profiled"] = n
        out["dispatch_rows"] = cnt
    elif ctr == "WRITE_SIZE":
        out["write_bytes_per_launch"] = 1024 * tot[ctr] / n
    else:
        out["l2_hit_rate"] = tot["TCC_HIT_sum"] / max(tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"], 1.0)
out["bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
out["traffic_over_alg"] = out["bytes_per_launch"] / out["alg_bytes_per_launch"]
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(out, indent=1) + "\n")
