# GPU check: pytest -m gpu, smoke, a short dpgo bench (round 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-chk}
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit $?
cat gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-lcd > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
