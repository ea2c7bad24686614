"""k_hess launch durations from a rocprofv3 kernel trace, split into launches
that ran Hess-vecs and early exits (no robot in tCG), next to the bench JSON's
evented figure (bench.py roofline.avg_launch_us).
usage: python scripts/hess_launch_stats.py <run_kernel_trace.csv> [bench.json]"""
import csv
import json
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_hess<" in r["Kernel_Name"])
full = [x for x in d if x > 20.0]
print(f"k_hess dispatches {len(d)}: mean {statistics.mean(d):.2f} us (rocprofv3 --stats average)")
print(f"  ran Hess-vecs (> 20 us) {len(full)}: mean {statistics.mean(full):.2f} us, median {statistics.median(full):.2f} us")
print(f"  early exits {len(d) - len(full)}: mean {statistics.mean([x for x in d if x <= 20.0] or [0]):.2f} us")
if len(sys.argv) > 2:
    js = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    r = js["roofline"]
    print(f"bench evented replay of the timed rounds: {r['avg_launch_us']:.2f} us per Hess-vec launch "
          f"(HIP events around each launch), frac {r['frac']:.3f}; with the trace's mean "
          f"{r['alg_bytes_per_launch'] / statistics.mean(full) / 1e3 / r['peak']:.3f}")
