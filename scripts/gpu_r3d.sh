# usage: bash scripts/gpu_r3d.sh tag — occupancy probe (1-wave workgroups vs
# LDS / VGPR budget), the LCD tests and wave stamps of the in-tree build at
# launch bounds 3 and 2, then k_hess roofline of dpgo builds (bench replay).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3d}
mkdir -p gpurun_out/$T
timeout -k 10 60 ./scripts/probe/occ_probe > gpurun_out/$T/occ.log 2>&1; echo "occ rc=$?"; cat gpurun_out/$T/occ.log
timeout -k 10 300 python -u -m pytest tests/test_lcd_gpu.py tests/test_configs_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_lcd.log 2>&1; echo "lcd tests rc=$?"; tail -2 gpurun_out/$T/pytest_lcd.log
for lb in 3 2; do
  KMX_COOP_LB=$lb timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps_lb$lb.log 2>&1; echo "stamps lb$lb rc=$?"
  grep -v Warn gpurun_out/$T/stamps_lb$lb.log | tail -2
done
for v in intree dh2 head; do
  if [ $v = intree ]; then E=KMX_DUMMY=1; else E=KMX_LIB=$PWD/alt/$v.so; fi
  env $E timeout -k 10 200 python bench.py --steps 100 --no-cpu --no-lcd > gpurun_out/$T/bench_$v.json 2> gpurun_out/$T/bench_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/$T/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/bench_$v.json')); r=d['roofline']; print('$v', round(d['value']/1e8,3), 'e8', round(d['ms_per_step']*1e3,1), 'us/round, k_hess', round(r['avg_launch_us'],2), 'us', round(r['frac'],4))"
done
