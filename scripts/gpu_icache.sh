# Instruction-cache behaviour of the small-shard round (one 12.5k-pose block):
# per-kernel SQC_ICACHE_MISSES / HITS and wave cycles, one rocprofv3 --pmc
# pass per counter group (kernel trace only). usage: bash scripts/gpu_icache.sh TAG [form]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-icache}; F=${2:-standard}
mkdir -p gpurun_out/$T
i=0
for C in "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$T/p$i -o run --output-format csv -- python3 scripts/round_sizes.py 1 $F > gpurun_out/$T/p$i.log 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/$T/p$i.log; exit 1; }
done
python3 - "$T" <<'PY'
import csv, glob, sys
from collections import defaultdict
t = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in glob.glob(f"gpurun_out/{t}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    d = max(len(n[k]), 1)
    h, m = v.get("SQC_ICACHE_HITS", 0), v.get("SQC_ICACHE_MISSES", 0)
    print(f"{k:16s} dispatches {d:6d} icache misses/disp {m / d:9.1f} hit rate {h / max(h + m, 1):.3f} "
          f"wave-cycles/disp {v.get('SQ_WAVE_CYCLES', 0) / d:10.0f} wait_inst/wave-cycles {v.get('SQ_WAIT_INST_ANY', 0) / max(v.get('SQ_WAVE_CYCLES', 0), 1):.3f} "
          f"ifetch/disp {v.get('SQ_IFETCH', 0) / d:9.0f}")
PY
