# A/B of env settings on the steady-state bench window: bash scripts/gpu_ab.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-lcd > gpurun_out/$T/b$i.json 2> gpurun_out/$T/b$i.err || { tail gpurun_out/$T/b$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/b$i.json')); r=d['roofline']; print('$E', round(d['value']/1e6,1), 'Me*i/s', round(d['ms_per_step'],4), 'ms/round', round(r['avg_launch_us'],2), 'us k_hess', round(r['frac'],4))"
done
