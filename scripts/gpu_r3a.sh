# round 3: the -m gpu suite (minus the long-horizon parity file), then the
# default bench (with the CPU-leg parity replay)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3a}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu --deselect tests/test_parity_long_gpu.py > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$T/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -20 gpurun_out/$T/bench.err; exit 1; }
T=$T python - <<'PY'
import json, os
d = json.load(open(f"gpurun_out/{os.environ['T']}/bench.json"))
print({k: d[k] for k in ("value", "ms_per_step", "exchange")}, d.get("parity"), d["roofline"]["frac"], d["cpu_baseline"]["value"], d["lcd"]["value"])
PY
