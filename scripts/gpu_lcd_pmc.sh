# usage: bash scripts/gpu_lcd_pmc.sh tag — SQ / TCC counters of the LCD kernels
# (separate rocprofv3 --pmc passes, kernel trace only) over scripts/lcd_timing.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lcdpmc}
mkdir -p gpurun_out/$TAG
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 scripts/lcd_timing.py 20000 > gpurun_out/$TAG/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/p$i.log; exit $rc; }
done
exit 0
