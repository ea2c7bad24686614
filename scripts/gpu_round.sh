# persistent round: bitwise tests vs the launched form, then the A/B timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-round}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_round_kernel_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/pytest_round.log 2>&1
rc=$?; echo "round tests rc=$rc"; tail -15 gpurun_out/$T/pytest_round.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/round_form_ab.py 8,4 > gpurun_out/$T/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/$T/ab.log
