# round-3 evidence: -m gpu suite (long file included), default bench + 20/40
# windows, rocprofv3 kernel stats of the default bench command, k_hess launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-final3}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
bash scripts/gpu_bench.sh $T || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp -o run --output-format csv -- python3 bench.py > gpurun_out/$T/prof_default.json 2> gpurun_out/$T/prof_default.err || { tail gpurun_out/$T/prof_default.err; exit 1; }
f=$(find gpurun_out/$T/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats.csv; head -14 gpurun_out/$T/kernel_stats.csv | cut -c1-150
f=$(find gpurun_out/$T/rp -name '*kernel_trace.csv' | head -1); python3 scripts/hess_launch_stats.py "$f" gpurun_out/$T/prof_default.json > gpurun_out/$T/k_hess_launch_stats.txt; cat gpurun_out/$T/k_hess_launch_stats.txt
