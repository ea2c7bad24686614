# lane-per-incidence gather prototype vs G5 (timing + output comparison)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/hinc
KMX_RECT=0 timeout -k 10 200 python scripts/gather_bench.py synth100k ${1:-60,91,92,93,60,91,92,93} ${2:-60:92,60:93} > gpurun_out/hinc/rect0.log 2>&1
rc=$?; cat gpurun_out/hinc/rect0.log; exit $rc
