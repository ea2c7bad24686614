# G = 9 Hessian gather: GPU parity tests, then bench A/B (KMX_HINC=1 vs 0) and kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-hab}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/$TAG/pytest.log; exit $rc; }
for H in 1 0; do
  KMX_HINC=$H timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/$TAG/bench_h$H.json 2> gpurun_out/$TAG/bench_h$H.err
  rc=$?; echo "hinc=$H bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/$TAG/bench_h$H.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_h$H.json'));print('hinc=$H', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms', d['roofline']['avg_launch_us'], round(d['roofline']['frac'],3))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --profile > gpurun_out/$TAG/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
