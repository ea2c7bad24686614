# LCD check: LCD GPU tests (both 5-point solvers) + the LCD bench leg per solver
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcd}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_lcd_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_lcd.log 2>&1
rc=$?; tail -5 gpurun_out/$T/pytest_lcd.log; [ $rc -eq 0 ] || exit $rc
for a in 0 1; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --burn-in 0 --no-cpu --no-replay --lcd-algo $a > gpurun_out/$T/bench_a$a.json 2> gpurun_out/$T/bench_a$a.err || { tail gpurun_out/$T/bench_a$a.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/$T/bench_a$a.json')); print($a, json.dumps(d.get('lcd')))"
done
