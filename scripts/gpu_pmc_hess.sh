# usage: bash scripts/gpu_pmc_hess.sh [tag] [config] — HBM traffic of the dpgo kernels:
# separate rocprofv3 --pmc passes (kernel trace only) over `bench.py --profile` (burn-in 40 +
# 10 rounds, every round evented), so every profiled k_hess dispatch is also counted in the
# bench JSON of that pass (empty dispatches read ~0 bytes and are not counted as launches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
CFG=${2:-synth100k}
mkdir -p gpurun_out/$TAG
i=0
# PASSES (optional): ";"-separated counter sets replacing the three traffic passes
IFS=';' read -ra SETS <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum}"
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 bench.py --config $CFG --burn-in ${BURN:-40} --steps ${STEPS:-10} --warmup 0 --profile --no-cpu --no-lcd > gpurun_out/$TAG/p$i.json 2> gpurun_out/$TAG/p$i.err
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
