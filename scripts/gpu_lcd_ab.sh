# A/B of LCD builds: in-tree vs alt/ libraries (throughput at 20k candidates),
# then the in-tree build's LCD parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcdab}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/lcd_timing.py 20000 > gpurun_out/$T/timing_$name.log 2>&1; echo "timing $name rc=$?"; grep verify_async gpurun_out/$T/timing_$name.log | tail -1
}
for k in 1 2; do
  run intree_$k KMX_DUMMY=1
  for f in alt/*.so; do b=$(basename $f .so); run ${b}_$k KMX_LIB=$PWD/$f; done
done
timeout -k 10 120 python -u scripts/lcd_phases.py 0 > gpurun_out/$T/phases.log 2>&1; echo "phases rc=$?"; cat gpurun_out/$T/phases.log
timeout -k 10 400 python -u -m pytest tests/test_lcd_gpu.py tests/test_golden_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "lcd or golden or configs2" > gpurun_out/$T/pytest_lcd.log 2>&1; echo "lcd tests rc=$?"; tail -2 gpurun_out/$T/pytest_lcd.log
