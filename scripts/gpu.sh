# One parameterised GPU-box driver (replaces the per-session gpu_*.sh scripts).
# Usage (from gpurun):  bash scripts/gpu.sh TAG STEP [STEP ...]
# Steps, each under its own time limit, stopping at the first failure:
#   tests        pytest -m gpu (whole suite)          -> TAG/pytest_gpu.log
#   tests:EXPR   pytest -m gpu -k EXPR (commas = spaces) -> TAG/pytest_k<n>.log
#   smoke        __graft_entry__.smoke()               -> TAG/smoke.log
#   bench        python bench.py (defaults)            -> TAG/default.json
#   bench:ARGS   python bench.py ARGS (commas = spaces)-> TAG/bench_<n>.json
#   prof         rocprofv3 --kernel-trace --stats of the default bench -> TAG/prof/
#   prof:ARGS    the same of bench.py ARGS (commas = spaces) -> TAG/prof_<n>/
#   py:SCRIPT    python SCRIPT (commas = spaces)       -> TAG/py_<n>.log
#   env:VAR=VAL:ARGS  bench.py ARGS under VAR=VAL       -> TAG/bench_<n>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T
mkdir -p "$O"
n=0
for step in "$@"; do
  n=$((n + 1))
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu \
        > "$O/pytest_gpu.log" 2>&1 || { echo "gpu suite failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
      tail -2 "$O/pytest_gpu.log" ;;
    tests:*)
      kx=${step#tests:}
      timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "${kx//,/ }" \
        > "$O/pytest_k$n.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_k$n.log"; exit 1; }
      tail -2 "$O/pytest_k$n.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python bench.py > "$O/default.json" 2> "$O/default.err" \
        || { echo "bench failed"; tail -20 "$O/default.err"; exit 1; }
      python scripts/bench_summary.py "$O/default.json" ;;
    bench:*)
      args=${step#bench:}
      timeout -k 10 600 python bench.py ${args//,/ } > "$O/bench_$n.json" 2> "$O/bench_$n.err" \
        || { echo "bench $args failed"; tail -20 "$O/bench_$n.err"; exit 1; }
      python scripts/bench_summary.py "$O/bench_$n.json" ;;
    env:*)  # env:VAR=VAL:bench-args (commas = spaces): bench.py under one environment setting
      rest=${step#env:}; kv=${rest%%:*}; args=${rest#*:}
      env "$kv" timeout -k 10 600 python bench.py ${args//,/ } > "$O/bench_$n.json" 2> "$O/bench_$n.err" \
        || { echo "bench $kv $args failed"; tail -20 "$O/bench_$n.err"; exit 1; }
      echo -n "$kv: "; python scripts/bench_summary.py "$O/bench_$n.json" ;;
    prof)
      mkdir -p "$O/prof"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 bench.py \
        > "$O/prof/bench.json" 2> "$O/prof/rocprof.err" || { echo "prof failed"; tail -20 "$O/prof/rocprof.err"; exit 1; }
      find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats.csv"
      head -12 "$O/kernel_stats.csv" | cut -c1-160 ;;
    prof:*)
      args=${step#prof:}
      mkdir -p "$O/prof_$n"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run --output-format csv -- python3 bench.py ${args//,/ } \
        > "$O/prof_$n/bench.json" 2> "$O/prof_$n/rocprof.err" || { echo "prof $args failed"; tail -20 "$O/prof_$n/rocprof.err"; exit 1; }
      find "$O/prof_$n" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats_$n.csv"
      head -12 "$O/kernel_stats_$n.csv" | cut -c1-160 ;;
    py:*)
      args=${step#py:}
      timeout -k 10 600 python -u ${args//,/ } > "$O/py_$n.log" 2>&1 \
        || { echo "py $args failed"; tail -30 "$O/py_$n.log"; exit 1; }
      tail -15 "$O/py_$n.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
