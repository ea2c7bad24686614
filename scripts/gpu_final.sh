# round-end evidence: default bench, the 20 / 40-step windows, and the rocprofv3
# kernel stats of the default bench command (bash scripts/gpu_final.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-final}
mkdir -p gpurun_out/$T
bash scripts/gpu_bench.sh $T || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp -o run --output-format csv -- python3 bench.py > gpurun_out/$T/prof_default.json 2> gpurun_out/$T/prof_default.err || { tail gpurun_out/$T/prof_default.err; exit 1; }
f=$(find gpurun_out/$T/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats.csv; head -12 gpurun_out/$T/kernel_stats.csv | cut -c1-150
