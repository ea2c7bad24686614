# Reduction form (KMX_RED=0 launch, 2 consumer) on the configs[3] rank handles at N = 8 / 4 / 2
# (scripts/host_seam.py batch and native rows), same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-redrank}
mkdir -p gpurun_out/$T
for n in 8 4 2; do
  for r in 0 2; do
    echo "== N=$n KMX_RED=$r" | tee -a gpurun_out/$T/ab.log
    KMX_RED=$r timeout -k 10 200 python scripts/host_seam.py $n 60 2>&1 | grep -E "batch|native" | tee -a gpurun_out/$T/ab.log || exit 1
  done
done
