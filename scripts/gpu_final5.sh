# round-3 closing evidence: -m gpu suite + smoke, default bench + 20 / 40-round
# windows, rocprofv3 kernel stats of the default bench command, the N = 8 / 4
# rank-handle emulation (strong-scaling estimate), the cold 1M-pose config.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-final5}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/$T/smoke.log
bash scripts/gpu_bench.sh $T || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp -o run --output-format csv -- python3 bench.py > gpurun_out/$T/prof_default.json 2> gpurun_out/$T/prof_default.err || { tail gpurun_out/$T/prof_default.err; exit 1; }
f=$(find gpurun_out/$T/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats.csv; head -8 gpurun_out/$T/kernel_stats.csv | cut -c1-120
f=$(find gpurun_out/$T/rp -name '*kernel_trace.csv' | head -1); python3 scripts/hess_launch_stats.py "$f" gpurun_out/$T/prof_default.json > gpurun_out/$T/k_hess_launch_stats.txt; cat gpurun_out/$T/k_hess_launch_stats.txt
rm -rf gpurun_out/$T/rp
for n in 8 4; do timeout -k 10 300 python -u scripts/host_seam.py $n 40 > gpurun_out/$T/host_seam_n$n.log 2>&1; echo "host_seam $n rc=$?"; grep -v Warn gpurun_out/$T/host_seam_n$n.log | tail -4; done
timeout -k 10 400 python bench.py --config synth1m --no-cpu --no-lcd --steps 20 > gpurun_out/$T/cold_1m.json 2> gpurun_out/$T/cold_1m.err; echo "cold rc=$?"
python -c "import json; d=json.load(open('gpurun_out/$T/cold_1m.json')); r=d['roofline']; print('cold 1m', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
