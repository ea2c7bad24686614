"""Summarize rocprofv3 --pmc passes: per kernel, mean counter value per dispatch."""
import csv, glob, re, sys, collections
d = sys.argv[1]
kern_filter = sys.argv[2] if len(sys.argv) > 2 else None
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+)(<[^>]*>)?", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:30]
        res[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in res.items():
    if kern_filter and kern_filter not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        # only dispatches with meaningful work: take the max-dispatch and the mean
        print("   %-26s n=%4d mean=%14.1f max=%14.1f" % (c, len(v), sum(v) / len(v), max(v)))
