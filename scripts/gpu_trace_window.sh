# kernel trace of the timed bench window (no evented replay): bash scripts/gpu_trace_window.sh TAG [env...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
for E in "$@"; do export $E; done
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/rp -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-replay --no-cpu --no-lcd > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail gpurun_out/$T/bench.err; exit 1; }
f=$(find gpurun_out/$T/rp -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/$T/kernel_trace.csv
python3 scripts/trace_gaps.py gpurun_out/$T/kernel_trace.csv
