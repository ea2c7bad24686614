# Stewenius launch bound A/B (KMX_COOP_LB 3 default vs 4), 20k candidates, twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcdlb}
mkdir -p gpurun_out/$T
for k in 1 2; do for lb in 3 4; do
  KMX_COOP_LB=$lb timeout -k 10 200 python -u scripts/lcd_timing.py 20000 > gpurun_out/$T/lb${lb}_$k.log 2>&1; echo "lb$lb rc=$?"; grep verify_async gpurun_out/$T/lb${lb}_$k.log | tail -1
done; done
