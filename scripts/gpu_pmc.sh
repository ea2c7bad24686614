# PMC passes (one counter group per pass, --kernel-trace only) on a short bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1; echo "list rc=$?"; fi
i=0
for C in ${PMC_SETS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --profile > gpurun_out/$TAG/p$i.log 2>&1
  echo "pass $i ($C) rc=$?"
done
exit 0
