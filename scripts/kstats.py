"""Per-kernel averages of the dpgo round kernels from a rocprofv3 kernel_stats.csv
(the prof / prof:ARGS steps of scripts/gpu.sh): python scripts/kstats.py TAG [TAG ...]"""
import csv
import glob
import sys

KS = ("k_hess", "k_update", "k_reduce", "k_grad", "k_cost", "k_retract", "k_commit", "k_begin", "k_step")
for tag in sys.argv[1:]:
    fs = sorted(glob.glob(f"gpurun_out/{tag}/**/*kernel_stats.csv", recursive=True))
    if not fs:
        print(tag, "no kernel_stats.csv")
        continue
    rows = list(csv.DictReader(open(fs[0])))
    rounds = max((int(r["Calls"]) for r in rows if "k_grad<" in r["Name"]), default=0)
    print(f"{tag}  ({fs[0]}; {rounds} rounds)")
    tot = 0.0
    for r in rows:
        for k in KS:
            if k + "<" in r["Name"] or k + "(" in r["Name"]:
                per = float(r["TotalDurationNs"]) / 1e3 / max(rounds, 1)
                tot += per
                print(f"  {k:10s} calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1e3:7.2f} us  {per:7.1f} us/round")
    print(f"  {'sum':10s} {tot:7.1f} us/round")
