"""k_hess occupancy / wait / latency counters from scripts/gpu_cold_diag.sh's
PMC passes (bench.py --profile on synth1m): averages per dispatch that ran
Hess-vecs, and the derived figures (waves resident, VMEM instructions in
flight, mean EA read latency by Little's law).
usage: hess_diag.py DIAG_DIR [OUT_JSON]"""
import csv, glob, json, os, sys
from collections import defaultdict

d = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
dur = {}
for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        if "k_hess<" not in r["Kernel_Name"]:
            continue
        key = (p, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
full = {k: v for k, v in per.items() if dur[k] > 100.0}  # cold config: a Hess-vec launch is ~450 us
agg = defaultdict(list)
for k, v in full.items():
    for c, x in v.items():
        agg[c].append(x)
    agg["duration_us"].append(dur[k])
m = {c: sum(v) / len(v) for c, v in agg.items()}
out = {"source": d, "dispatches": {c: len(v) for c, v in agg.items()}, "mean_per_dispatch": m}
g = lambda c: m.get(c, float("nan"))
out["derived"] = {
    "waves_resident_avg (SQ_LEVEL_WAVES / SQ_BUSY_CYCLES)": g("SQ_LEVEL_WAVES") / g("SQ_BUSY_CYCLES"),
    "wave_cycles_waiting_any": g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
    "wave_cycles_waiting_inst_any": g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
    "wave_cycles_issuing_any": g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES"),
    "vmem_insts_in_flight_avg (SQ_INST_LEVEL_VMEM / SQ_BUSY_CYCLES)": g("SQ_INST_LEVEL_VMEM") / g("SQ_BUSY_CYCLES"),
    "ea_read_latency_tcc_cycles (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ)": g("TCC_EA0_RDREQ_LEVEL_sum") / g("TCC_EA0_RDREQ_sum"),
    "ea_read_requests_per_us": g("TCC_EA0_RDREQ_sum") / g("duration_us"),
}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
