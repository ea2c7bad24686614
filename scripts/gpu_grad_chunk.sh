# k_grad chunk-size check: dpgo parity tests, round time vs size, and the
# rocprof kernel averages of the 100k-pose rounds (bash scripts/gpu_grad_chunk.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-gchunk}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_dpgo_gpu.py tests/test_configs_gpu.py tests/test_golden_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$T/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/round_sizes.py 1,8 2>&1 | grep robots || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp -o run --output-format csv -- python3 scripts/round_sizes.py 8 > gpurun_out/$T/sizes.log 2>&1 || exit 1
f=$(find gpurun_out/$T/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$T/kernel_stats.csv')):
    n=r['Name']
    if any(k in n for k in ('k_grad','k_hess','k_cost','k_update')): print(n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
