# usage: bash scripts/gpu_iter.sh tag — GPU tests, gather microbench, quick dpgo bench, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-iter}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/gather_bench.py synth100k ${GB_VARIANTS:-20,21,40,41,42,45} > gpurun_out/$TAG/gbench.log 2>&1
rc=$?; echo "gbench rc=$rc"; cat gpurun_out/$TAG/gbench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu ${BENCH_ARGS:---no-lcd} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG/bench.json; tail -3 gpurun_out/$TAG/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --profile > gpurun_out/$TAG/prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_noev -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-lcd --no-events > gpurun_out/$TAG/prof_noev.log 2>&1
echo "prof_noev rc=$?"
