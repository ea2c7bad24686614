# usage: bash scripts/gpu_subset.sh TAG test_files... — a pytest -m gpu subset
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/$T/pytest.log | tail -40; tail -3 gpurun_out/$T/pytest.log; exit $rc
