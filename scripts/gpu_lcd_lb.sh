# usage: bash scripts/gpu_lcd_lb.sh tag "1 2 4" — LCD verify rate per KMX_RS_LB value
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-lcdlb}
mkdir -p gpurun_out/$TAG
for LB in ${2:-1 2 4}; do
  KMX_RS_LB=$LB timeout -k 10 300 python scripts/lcd_timing.py 20000 > gpurun_out/$TAG/lb$LB.log 2>&1
  rc=$?; echo "LB=$LB rc=$rc"; tail -3 gpurun_out/$TAG/lb$LB.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
