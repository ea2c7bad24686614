# same-box A/B of two builds (KMX_LIB): round time and kernel averages at 100k poses
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-gchunkab}; ALT=$2
mkdir -p gpurun_out/$T
for V in base alt base alt; do
  if [ $V = alt ]; then export KMX_LIB=$PWD/$ALT; else unset KMX_LIB; fi
  echo "== $V" | tee -a gpurun_out/$T/ab.log
  timeout -k 10 200 python scripts/round_sizes.py 1,8 2>&1 | grep robots | tee -a gpurun_out/$T/ab.log || exit 1
done
for V in base alt; do
  if [ $V = alt ]; then export KMX_LIB=$PWD/$ALT; else unset KMX_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/rp_$V -o run --output-format csv -- python3 scripts/round_sizes.py 8 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/$T/rp_$V -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('k_grad','k_cost')): print('$V', n[:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))
" | tee -a gpurun_out/$T/ab.log
done
