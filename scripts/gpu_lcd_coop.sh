# usage: bash scripts/gpu_lcd_coop.sh tag — LCD GPU tests, then verify rate and
# phase times per k_ransac_coop bound (LBS="4 8"), then a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-coop}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -m pytest tests/test_lcd_gpu.py -x -q --timeout 300 > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "lcd tests rc=$rc"; tail -15 gpurun_out/$TAG/pytest.log
[ $rc -ne 0 ] && exit $rc
for LB in ${LBS:-4}; do
  KMX_COOP_LB=$LB timeout -k 10 300 python scripts/lcd_timing.py 20000 > gpurun_out/$TAG/lb$LB.log 2>&1
  rc=$?; echo "KMX_COOP_LB=$LB rc=$rc"; tail -2 gpurun_out/$TAG/lb$LB.log
  [ $rc -ne 0 ] && exit $rc
  KMX_COOP_LB=$LB timeout -k 10 300 python scripts/lcd_phases.py > gpurun_out/$TAG/ph$LB.log 2>&1
  cat gpurun_out/$TAG/ph$LB.log
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 scripts/lcd_timing.py 20000 > gpurun_out/$TAG/prof.log 2>&1
  echo "prof rc=$?"; cut -d, -f1-4 gpurun_out/$TAG/prof/*/run_kernel_stats.csv 2>/dev/null | head -8
fi
exit 0
