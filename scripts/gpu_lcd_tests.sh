# LCD parity tests (incl. the Stewenius batch stopping cases) + bench LCD leg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcdt}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_lcd_gpu.py tests/test_golden_gpu.py tests/test_outputs_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/pytest_lcd.log 2>&1 || { echo "lcd tests failed"; tail -30 gpurun_out/$T/pytest_lcd.log; exit 1; }
tail -2 gpurun_out/$T/pytest_lcd.log
timeout -k 10 300 python -u bench.py --no-cpu --no-replay --steps 5 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -5 gpurun_out/$T/bench.err; exit 1; }
T=$T python - <<'PY'
import json, os
d = json.load(open(f"gpurun_out/{os.environ['T']}/bench.json"))
print("lcd", d["lcd"]["value"], d["lcd"]["roofline"]["frac"], d["lcd"]["roofline"]["ransac_share"])
PY
