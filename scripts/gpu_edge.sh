set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/edge
timeout -k 10 300 python -u -m pytest tests/test_dpgo_edge_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/edge/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/edge/pytest.log; exit $rc
