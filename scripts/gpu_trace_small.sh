# kernel trace of the strong-scaling floor (one 12.5k-pose robot block per GPU):
# bash scripts/gpu_trace_small.sh TAG [robots] [form] [env...]   (form: standard | onesync)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; R=${2:-1}; F=${3:-standard}; shift; shift; shift
for E in "$@"; do export $E; done
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/rp -o run --output-format csv -- python3 scripts/round_sizes.py $R $F > gpurun_out/$T/sizes.log 2> gpurun_out/$T/sizes.err || { tail gpurun_out/$T/sizes.err; exit 1; }
cat gpurun_out/$T/sizes.log
f=$(find gpurun_out/$T/rp -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/$T/kernel_trace.csv
python3 scripts/trace_gaps.py gpurun_out/$T/kernel_trace.csv | tee gpurun_out/$T/gaps.txt
