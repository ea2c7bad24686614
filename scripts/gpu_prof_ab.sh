# rocprofv3 kernel stats of the bench's profile mode under env settings: bash scripts/gpu_prof_ab.sh TAG "VAR=a" "VAR=b"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
i=0
for E in "$@"; do
  i=$((i+1))
  export $E
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp$i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 0 --profile --no-cpu --no-lcd > gpurun_out/$T/prof$i.log 2>&1 || { tail gpurun_out/$T/prof$i.log; exit 1; }
  f=$(find gpurun_out/$T/rp$i -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T/kernel_stats_$i.csv
  echo "== $E"; cut -d, -f1-5 gpurun_out/$T/kernel_stats_$i.csv | cut -c1-150 | head -12
done
