# round 3: the long-horizon parity tests (configs[0] to termination, configs[1]
# converged, configs[3] bench window)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-long}
mkdir -p gpurun_out/$T
timeout -k 10 1100 python -u -m pytest tests/test_parity_long_gpu.py -x -v --timeout 900 --timeout-method thread -m gpu > gpurun_out/$T/pytest_long.log 2>&1
rc=$?; echo "long rc=$rc"; tail -8 gpurun_out/$T/pytest_long.log; exit $rc
