# k_grad epilogue ablation (KMX_PGO_DBG bits: 1 no precon, 2 no symYtG) — timing only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gabl
for D in 0 1 2 3; do
  KMX_PGO_DBG=$D timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/gabl/d$D -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --profile > gpurun_out/gabl/d$D.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/gabl/d$D.log; exit $rc; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/gabl/d$D/run_kernel_stats.csv')):
    if 'k_grad' in r['Name'] or 'k_cost' in r['Name']: print('dbg=$D', r['Name'][28:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
