# LCD verification throughput vs k_ransac_coop's register budget (KMX_COOP_LB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcd_lb}; shift
mkdir -p gpurun_out/$T
for lb in "$@"; do
  KMX_COOP_LB=$lb timeout -k 10 300 python bench.py --steps 2 --warmup 1 --burn-in 0 --no-cpu --no-replay --lcd-algo ${ALGO:-0} > gpurun_out/$T/lb$lb.json 2> gpurun_out/$T/lb$lb.err || { tail gpurun_out/$T/lb$lb.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/lb$lb.json'))['lcd']; print('lb $lb', d['value'], d['ms_per_step'])" | tee -a gpurun_out/$T/ab.log
done
