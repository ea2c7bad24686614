# usage: bash scripts/gpu_lcd_pmc3.sh tag [workload script] [N] — the counters behind the LCD
# roofline: VALU / LDS activity and fp64 instruction
# counts of k_ransac_coop over a 4000-candidate Stewenius run, one rocprofv3
# --pmc pass per counter group (kernel trace only), then a --stats pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lcdpmc3}
WL=${2:-scripts/lcd_timing.py}  # or scripts/lcd_hard_timing.py (bench.py's hard leg)
NC=${3:-4000}
mkdir -p gpurun_out/$TAG
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/$TAG/list_avail.txt 2>&1
grep -oE "SQ_[A-Z0-9_]+|GRBM_[A-Z_]+" gpurun_out/$TAG/list_avail.txt | sort -u > gpurun_out/$TAG/sq_counters.txt
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
         "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
         "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 $WL $NC > gpurun_out/$TAG/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && tail -3 gpurun_out/$TAG/p$i.log
  [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/stats -o run --output-format csv -- python3 $WL $NC > gpurun_out/$TAG/stats.log 2>&1; echo "stats rc=$?"
exit 0
