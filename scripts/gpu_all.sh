# usage: bash scripts/gpu_all.sh [tag]  — GPU tests, bench, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 40 --warmup 5 ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG/bench.json; tail -3 gpurun_out/$TAG/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --profile > gpurun_out/$TAG/prof.log 2>&1
echo "prof rc=$?"
