# usage: bash scripts/gpu_pmc_gather.sh TAG "60 70" — PMC passes (kernel trace only,
# one rocprofv3 run per counter group and variant) over scripts/gather_bench.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-gpmc}
VARS=${2:-"60 70"}
mkdir -p gpurun_out/$TAG
for V in $VARS; do
  i=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY" \
           "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/v${V}_p$i -o run --output-format csv -- python3 scripts/gather_bench.py synth100k $V > gpurun_out/$TAG/v${V}_p$i.log 2>&1
    rc=$?; echo "variant $V pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
