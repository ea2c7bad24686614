# round-2 check: GPU parity at every BASELINE config size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 900 --timeout-method thread > gpurun_out/configs_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/configs_gpu.log
exit $rc
