set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_dpgo_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" 
tail -30 gpurun_out/pytest_gpu.log
