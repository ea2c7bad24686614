# reduction form at configs[3] 100k (one GPU): launch (KMX_RED=0) vs consumer
# with the stop test after the gather (KMX_RED=2 KMX_EARLY=0) and before it
# (KMX_EARLY=1), alternating, no CPU/LCD legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-redab}
mkdir -p gpurun_out/$T
for k in 1 2; do
  for v in "KMX_RED=0" "KMX_RED=2 KMX_EARLY=0" "KMX_RED=2 KMX_EARLY=1"; do
    n=$(echo $v | tr ' =' '__')
    env $v timeout -k 10 200 python bench.py --steps 100 --no-cpu --no-lcd --no-replay > gpurun_out/$T/${n}_$k.json 2> gpurun_out/$T/${n}_$k.err || { echo "$v failed"; tail -3 gpurun_out/$T/${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$T/${n}_$k.json')); print('$v', round(d['value']/1e8,3), 'e8', round(d['ms_per_step']*1e3,1), 'us/round')"
  done
done
