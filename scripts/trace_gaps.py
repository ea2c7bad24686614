"""Per-round wall time, busy time and inter-kernel gaps from a rocprofv3
kernel trace (last 10 complete rounds, rounds delimited by k_grad)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
g = [t for t in ts if "k_grad" in t[2]]
s0, s1 = g[-11][0], g[-1][0]
seq = [t for t in ts if t[0] >= s0 and t[1] <= s1]
busy = sum(b - a for a, b, _ in seq)
print(f"wall {(s1 - s0) / 10e3:.1f} us/round, busy {busy / 10e3:.1f} us/round, kernels/round {len(seq) / 10:.1f}")


def nm(n):
    for k in ("k_step", "k_hess", "k_update", "k_reduce", "k_grad", "k_cost", "k_retract", "k_commit", "k_begin", "k_precond",
              "k_publish", "k_accel"):
        if k in n:
            return k
    return n[:16]


gap = defaultdict(list)
for i in range(len(seq) - 1):
    gap[(nm(seq[i][2]), nm(seq[i + 1][2]))].append((seq[i + 1][0] - seq[i][1]) / 1e3)
for k, v in sorted(gap.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:>10s} -> {k[1]:10s} n={len(v):4d} mean gap {sum(v) / len(v):6.2f} us, total/round {sum(v) / 10:7.1f} us")

kt = defaultdict(list)
for a, b, n in seq:
    kt[nm(n)].append((b - a) / 1e3)
for k, v in sorted(kt.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:>10s} n/round={len(v) / 10:5.1f} mean {sum(v) / len(v):6.2f} us, total/round {sum(v) / 10:7.1f} us")
