# round 3: why the cold-config k_hess streams at ~3.9 TB/s:
# occupancy / wait / latency counters over bench.py --profile on synth1m, one
# rocprofv3 --pmc pass per group; then the N = 2, 4 bench path over gloo on one
# GPU (the multi-rank driver after this round's start-up changes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-colddiag}
mkdir -p gpurun_out/$T
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_CYCLE_sum" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$T/p$i -o run --output-format csv -- python3 bench.py --config synth1m --burn-in 40 --steps 10 --warmup 0 --profile --no-cpu --no-lcd > gpurun_out/$T/p$i.json 2> gpurun_out/$T/p$i.err
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/$T/p$i.err; exit 1; }
done
bash scripts/gpu_multirank_rehearsal.sh ${T}_mg 2 4 || exit 1
exit 0
