"""Per-dispatch means of arbitrary PMC counters for one kernel, from the pass
directories of scripts/gpu_pmc_hess.sh (PASSES=...), with the kernel's mean
duration and the counters per CU-cycle (÷ 256 CUs ÷ duration × clock).
usage: python scripts/pmc_units.py DIR [kernel=k_hess] [--min-us 15] [--mhz 2400]"""
import csv, glob, sys
from collections import defaultdict
from pathlib import Path

args = [a for a in sys.argv[1:] if not a.startswith("--")]
d = Path(args[0])
kern = args[1] if len(args) > 1 else "k_hess"
min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 15.0
mhz = float(sys.argv[sys.argv.index("--mhz") + 1]) if "--mhz" in sys.argv else 2400.0
if "--min-us" in sys.argv:
    args = [a for a in args if a != sys.argv[sys.argv.index("--min-us") + 1]]
for pdir in sorted(d.glob("p*/")):
    f = glob.glob(str(pdir / "**" / "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f[0])):
        if kern not in r.get("Kernel_Name", ""):
            continue
        did = r["Dispatch_Id"]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            dur[did] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    keep = [k for k in per if dur.get(k, 1e9) >= min_us]
    if not keep:
        continue
    mean_us = sum(dur.get(k, 0.0) for k in keep) / len(keep)
    names = sorted({c for k in keep for c in per[k]})
    print(f"{pdir.name}: {len(keep)} dispatches >= {min_us} us, mean {mean_us:.1f} us")
    for c in names:
        v = sum(per[k][c] for k in keep) / len(keep)
        print(f"  {c:40s} {v:16.1f} per dispatch  {v / (256 * mean_us * mhz):8.3f} per CU-cycle")
