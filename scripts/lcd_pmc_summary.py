"""Summarise the k_ransac_coop PMC passes of scripts/gpu_lcd_pmc3.sh (run
over scripts/lcd_timing.py N: one warm-up launch of 64 candidates, then 4
launches of N) into the per-candidate counts bench.py's LCD roofline uses.
usage: lcd_pmc_summary.py PMC_DIR OUT_JSON [N] [LAUNCHES]
N (the candidates per timed launch, scripts/lcd_timing.py's argument): the
work-queue k_ransac_coop's grid is its resident waves, not its candidates,
so the candidates counted are N per timed launch; without N the grid rule of
the one-workgroup-per-candidate kernel is used. LAUNCHES (default 4): only
the first LAUNCHES timed dispatches of each pass count — lcd_timing.py's
single calls; its back-to-back calls run the next call's kNN2 on a side
stream concurrently, and the SQ counters of a dispatch then include the
kNN2 kernel's instructions."""
import csv, glob, json, os, sys
from collections import defaultdict

d, out = sys.argv[1], sys.argv[2]
vals = defaultdict(float)
disp = set()
cand = 0
LAUNCHES = int(sys.argv[4]) if len(sys.argv) > 4 else 4
for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")),
                key=lambda x: int(os.path.basename(os.path.dirname(x))[1:])):
    rows = [r for r in csv.DictReader(open(p))
            if "k_ransac_coop" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 64 * 1000]  # timed launches only
    keep = sorted({int(r["Dispatch_Id"]) for r in rows})[:LAUNCHES]
    here = defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            here[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in here.items():  # a counter collected in two passes counts once (its first pass)
        if k not in vals:
            vals[k] = v
    disp |= {len(keep)}
# candidates per pass: grid / 64 per launch, 4 launches
grids = []
for r in csv.DictReader(open(glob.glob(os.path.join(d, "p1", "run_counter_collection.csv"))[0])):
    if "k_ransac_coop" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 64 * 1000 and r["Counter_Name"] == "SQ_WAVES":
        grids.append(int(r["Grid_Size"]) // 64)
grids = grids[:LAUNCHES]
cand = len(grids) * int(sys.argv[3]) if len(sys.argv) > 3 else sum(grids)
kern = [float(r["TotalDurationNs"]) for r in csv.DictReader(open(os.path.join(d, "stats", "run_kernel_stats.csv")))
        if "k_ransac_coop" in r["Name"]]
f64 = {k: vals[k] for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                            "SQ_INSTS_VALU_TRANS_F64")}
# issued fp64 lane-flops: 64 lanes per wave instruction, 2 for an FMA (the
# counters count wave instructions whatever the exec mask)
flops = 64.0 * (f64["SQ_INSTS_VALU_ADD_F64"] + f64["SQ_INSTS_VALU_MUL_F64"] + 2.0 * f64["SQ_INSTS_VALU_FMA_F64"]
                + f64["SQ_INSTS_VALU_TRANS_F64"])
res = {
    "source": d, "kernel": "k_ransac_coop (Stewenius, 2D-2D RANSAC)", "candidates_counted": cand,
    "per_candidate": {
        "valu_insts": vals["SQ_INSTS_VALU"] / cand,
        "fp64_insts": sum(f64.values()) / cand,
        "fp64_issued_flops": flops / cand,
        "lds_insts": vals["SQ_INSTS_LDS"] / cand,
        "salu_insts": vals["SQ_INSTS_SALU"] / cand,
        "vmem_rd_insts": vals["SQ_INSTS_VMEM_RD"] / cand,
    },
    # exec-mask-aware: SQ_THREAD_CYCLES_VALU counts active
    # lanes per VALU cycle; over 64 x SQ_ACTIVE_INST_VALU it is the share of
    # lanes doing work in the VALU's active cycles. SQ_INSTS_VALU_FLOPS_FP64
    # is the hardware's own fp64 FLOP count (compared with the issued figure
    # above: equal means it ignores the exec mask, lower means it counts lanes)
    "lanes": {
        "valu_thread_util": vals["SQ_THREAD_CYCLES_VALU"] / max(64.0 * vals["SQ_ACTIVE_INST_VALU"], 1.0)
        if "SQ_THREAD_CYCLES_VALU" in vals else None,
        "fp64_flops_counter_per_candidate": (vals["SQ_INSTS_VALU_FLOPS_FP64"] + vals.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0))
        / cand if "SQ_INSTS_VALU_FLOPS_FP64" in vals else None,
    },
    "fractions": {
        "fp64_share_of_valu_insts": sum(f64.values()) / max(vals["SQ_INSTS_VALU"], 1.0),
        "valu_active_over_wave_cycles": vals["SQ_ACTIVE_INST_VALU"] / max(vals["SQ_WAVE_CYCLES"], 1.0),
        "any_active_over_wave_cycles": vals["SQ_ACTIVE_INST_ANY"] / max(vals["SQ_WAVE_CYCLES"], 1.0),
        "wait_inst_any_over_wave_cycles": vals["SQ_WAIT_INST_ANY"] / max(vals["SQ_WAVE_CYCLES"], 1.0),
        "wait_inst_lds_over_wave_cycles": vals["SQ_WAIT_INST_LDS"] / max(vals["SQ_WAVE_CYCLES"], 1.0),
    },
    "raw": dict(vals),
    "kernel_time_ns_stats_pass": kern,
    "note": "half of the candidates are planted (RANSAC runs ~32 hypotheses), half have no match (K = 0, no RANSAC); "
            "bench.py multiplies fp64_issued_flops per candidate by its live candidates/s and divides by the "
            "78.6 TFLOP/s fp64 vector peak (a stored PMC ratio, labelled as such in the JSON)",
}
json.dump(res, open(out, "w"), indent=1)
if res["lanes"]["valu_thread_util"] is not None:
    res["per_candidate"]["fp64_useful_flops"] = res["per_candidate"]["fp64_issued_flops"] * res["lanes"]["valu_thread_util"]
print(json.dumps({k: res[k] for k in ("candidates_counted", "per_candidate", "lanes", "fractions")}, indent=1))
