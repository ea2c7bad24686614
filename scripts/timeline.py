"""Print per-kernel stats and one round's timeline from a rocprofv3 csv dir."""
import csv, re, sys
d = sys.argv[1]
rnd = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:14]:
    print("%-40s %5s %10.1f us avg %6.2f%%" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
def nm(s):
    m = re.search(r"(k_[a-z_]+)", s)
    return m.group(1) if m else s[:14]
seq = [(nm(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, int(r["Start_Timestamp"])) for r in rows]
seq.sort(key=lambda x: x[2])
starts = [i for i, s in enumerate(seq) if s[0] == "k_round_begin"]
if len(starts) > rnd + 1:
    i0, i1 = starts[rnd], starts[rnd + 1]
    t0 = seq[i0][2]
    for s in seq[i0:i1]:
        print("%-14s %8.1f us  @%8.1f" % (s[0], s[1], (s[2] - t0) / 1000))
    print("round total %.1f us" % ((seq[i1][2] - t0) / 1000))
