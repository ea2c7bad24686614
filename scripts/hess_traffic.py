"""Per-launch HBM traffic of k_hess from the PMC passes of scripts/gpu_pmc_hess.sh
or scripts/gpu_hess_probe.sh.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. MI355X_MICROARCH.md (HBM):
FETCH_SIZE on gfx950 reports 1/2 of the bytes of wide coalesced reads -> x2
(confirmed for k_hess's own access patterns by scripts/probe/traffic_calib.py,
profiles/r04/calib/); WRITE_SIZE is taken as is.

Dispatches are split by their duration (the counter rows carry the dispatch's
timestamps): a dispatch longer than --min-us ran Hess-vecs; a shorter one is a
launch every robot skipped (out of tCG: a blind step past a robot's end). The
two kinds are reported separately. Up to round 3 the sum over ALL dispatches
was divided by the Hess-vec launch count, which charged the skipped launches'
traffic (each one still fetches its first record chunk, ~44 MB at 100k poses)
to the real ones. The count of long dispatches is checked against the bench's
own launch count.
usage: python scripts/hess_traffic.py DIR [OUT.json] [--min-us 15]"""
import csv, glob, json, sys
from pathlib import Path

args = [a for a in sys.argv[1:] if not a.startswith("--")]
min_us = 15.0
if "--min-us" in sys.argv:
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1])
    args = [a for a in args if a != sys.argv[sys.argv.index("--min-us") + 1]]
d = Path(args[0])
out = {"kernel": "k_hess", "source": str(d), "fetch_correction": 2.0, "min_us": min_us}


def rows(i):
    """{dispatch: (duration_us, {counter: value})} of k_hess in pass i."""
    by = {}
    for f in glob.glob(str(d / f"p{i}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_hess" not in r["Kernel_Name"]:
                continue
            key = (r.get("Process_Id"), int(r["Dispatch_Id"]))
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            e = by.setdefault(key, [us, {}])
            e[1][r["Counter_Name"]] = e[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return by


def split(by, ctr, scale):
    full = [v[ctr] * scale for us, v in by.values() if us > min_us]
    empty = [v[ctr] * scale for us, v in by.values() if us <= min_us]
    return full, empty


for i, ctr in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE"), (3, None)):
    p = d / f"p{i}.json"
    if not p.exists():
        continue
    js = json.loads(p.read_text().strip().splitlines()[-1])
    n, alg = js["roofline"]["launches"], js["roofline"]["alg_bytes_per_launch"]
    by = rows(i)
    if ctr is None:
        h = sum(v.get("TCC_HIT_sum", 0.0) for us, v in by.values() if us > min_us)
        m = sum(v.get("TCC_MISS_sum", 0.0) for us, v in by.values() if us > min_us)
        out["l2_hit_rate"] = h / max(h + m, 1.0)
        continue
    scale = (2.0 if ctr == "FETCH_SIZE" else 1.0) * 1024
    full, empty = split(by, ctr, scale)
    key = "fetch" if ctr == "FETCH_SIZE" else "write"
    out[f"{key}_bytes_per_launch"] = sum(full) / max(len(full), 1)
    out[f"{key}_bytes_per_skipped_launch"] = sum(empty) / max(len(empty), 1) if empty else 0.0
    out[f"{key}_pass_launches"] = {"bench": n, "long_dispatches": len(full), "short_dispatches": len(empty)}
    if len(full) != n:
        out.setdefault("warnings", []).append(f"{ctr}: {len(full)} long dispatches vs {n} bench launches")
    if ctr == "FETCH_SIZE":
        out["alg_bytes_per_launch"] = alg
        out["launches_profiled"] = n
        # the round-3 figure (all dispatches over the Hess-vec launches), for comparison
        out["fetch_bytes_per_launch_r3_method"] = (sum(full) + sum(empty)) / n
out["bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
out["traffic_over_alg"] = out["bytes_per_launch"] / out["alg_bytes_per_launch"]
# the duration split must find the bench's Hess-vec launches: more long dispatches than
# launches means skipped launches ran past --min-us and are averaged in (round 5's 1M file)
out["split_ok"] = all(v["long_dispatches"] <= v["bench"] + 1 for k, v in out.items() if k.endswith("_pass_launches"))
if not out["split_ok"]:
    print("warning: more long dispatches than Hess-vec launches; raise --min-us", file=sys.stderr)
print(json.dumps(out, indent=1))
if len(args) > 1:
    Path(args[1]).write_text(json.dumps(out, indent=1) + "\n")
