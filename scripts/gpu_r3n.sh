# usage: bash scripts/gpu_r3n.sh tag — LCD tests, then the LCD bench leg
# in-tree vs alt/prev.so alternating twice, and the wave stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3n}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_lcd_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py tests/test_outputs_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_lcd.log 2>&1; rc=$?; echo "lcd tests rc=$rc"; tail -3 gpurun_out/$T/pytest_lcd.log
[ $rc -ne 0 ] && exit 1
for k in 1 2; do
  for v in intree prev; do
    if [ $v = intree ]; then E=KMX_DUMMY=1; else E=KMX_LIB=$PWD/alt/prev.so; fi
    env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --burn-in 1 --no-cpu --no-replay > gpurun_out/$T/bench_${v}_$k.json 2> gpurun_out/$T/bench_${v}_$k.err || { tail -3 gpurun_out/$T/bench_${v}_$k.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$T/bench_${v}_$k.json')); l=d['lcd']; r=l['roofline']; print('$v $k lcd', round(l['value']), 'ransac ms', round(r['ransac_ms'],2), 'knn ms', round(r['knn_ms'],2))"
  done
done
timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps.log 2>&1; echo "stamps rc=$?"; grep -v Warn gpurun_out/$T/stamps.log | tail -3
