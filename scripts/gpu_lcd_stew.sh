# round 3: batched Stewenius eigenvalues — LCD parity tests, then throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-stew}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_lcd_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "lcd or golden or configs2" > gpurun_out/$T/pytest_lcd.log 2>&1 || { echo "lcd tests failed"; tail -30 gpurun_out/$T/pytest_lcd.log; exit 1; }
tail -2 gpurun_out/$T/pytest_lcd.log
timeout -k 10 200 python -u scripts/lcd_timing.py 4000 > gpurun_out/$T/timing4k.log 2>&1; echo "timing rc=$?"; cat gpurun_out/$T/timing4k.log
timeout -k 10 300 python -u bench.py --no-cpu --no-replay --steps 5 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -5 gpurun_out/$T/bench.err; exit 1; }
T=$T python - <<'PY'
import json, os
d = json.load(open(f"gpurun_out/{os.environ['T']}/bench.json"))
print("lcd", d["lcd"]["value"], d["lcd"].get("ransac_share"), d["lcd"].get("nister_value"))
PY
