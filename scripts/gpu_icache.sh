# usage: bash scripts/gpu_icache.sh tag [tests] — the -m gpu suite (optional),
# then instruction-cache counters of the LCD RANSAC kernel (4000-candidate
# Stewenius run): is the 134 KB k_ransac_coop<3, true> fetch-bound?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-icache}
mkdir -p gpurun_out/$TAG
if [ "${2:-}" = tests ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -ne 0 ] && exit 1
fi
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/$TAG/list_avail.txt 2>&1
grep -oE "SQC_[A-Z0-9_]+|SQ_IFETCH[A-Z0-9_]*|SQ_WAIT_INST[A-Z0-9_]*" gpurun_out/$TAG/list_avail.txt | sort -u > gpurun_out/$TAG/sqc_counters.txt
cat gpurun_out/$TAG/sqc_counters.txt | tr '\n' ' '; echo
i=0
for C in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
         "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  ok=1
  for c in $C; do grep -qx "$c" gpurun_out/$TAG/sqc_counters.txt || case $c in SQ_WAVE_CYCLES|SQ_INSTS_VALU|SQ_INSTS_SALU) ;; *) ok=0;; esac; done
  [ $ok -eq 0 ] && { echo "pass $i skipped (counter missing): $C"; continue; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 scripts/lcd_timing.py 4000 > gpurun_out/$TAG/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && tail -3 gpurun_out/$TAG/p$i.log
  [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
done
exit 0
