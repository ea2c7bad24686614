# usage: bash scripts/gpu_r3g.sh tag — LCD work-queue kernel: LCD / configs /
# pipeline GPU tests, wave stamps at launch bounds 3 and 2, throughput at 20k.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3g}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_lcd_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py tests/test_outputs_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_lcd.log 2>&1; rc=$?; echo "lcd tests rc=$rc"; tail -3 gpurun_out/$T/pytest_lcd.log
[ $rc -ne 0 -a $rc -ne 1 ] && exit 1
for lb in 3 2; do
  KMX_COOP_LB=$lb timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps_lb$lb.log 2>&1; echo "stamps lb$lb rc=$?"
  grep -v Warn gpurun_out/$T/stamps_lb$lb.log | tail -3
  KMX_COOP_LB=$lb timeout -k 10 200 python3 -u scripts/lcd_timing.py 20000 > gpurun_out/$T/timing_lb$lb.log 2>&1; echo "timing lb$lb rc=$?"; grep -E 'verify_async|accepted' gpurun_out/$T/timing_lb$lb.log
done
