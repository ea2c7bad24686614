"""Mean PMC counter per k_gbench dispatch, per variant (scripts/gpu_pmc_gather.sh output)."""
import collections, csv, glob, os, re, sys
d = sys.argv[1]
for vdir in sorted(set(re.sub(r"_p\d+$", "", os.path.basename(p)) for p in glob.glob(f"{d}/v*_p*") if os.path.isdir(p))):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{vdir}_p*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_gbench" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(vdir)
    for c, v in sorted(acc.items()):
        print("   %-30s n=%4d mean=%16.1f" % (c, len(v), sum(v) / len(v)))
