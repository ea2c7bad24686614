# dpgo parity subset + short bench + rocprofv3 kernel stats of the bench's profile mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-prof}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_dpgo_gpu.py tests/test_distributed_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-lcd > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp -o run --output-format csv -- python3 bench.py --steps 10 --warmup 0 --profile --no-cpu --no-lcd > gpurun_out/$T/prof.log 2>&1 || { tail gpurun_out/$T/prof.log; exit 1; }
f=$(find gpurun_out/$T/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats.csv; head -20 gpurun_out/$T/kernel_stats.csv | cut -c1-160
