# usage: bash scripts/gpu_r3h.sh tag — LCD tests after the kNN2 key rewrite,
# the LCD bench leg alone (knn_ms / ransac_ms), then the PMC ratios.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3h}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_lcd_gpu.py tests/test_configs_gpu.py tests/test_bow_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_lcd.log 2>&1; rc=$?; echo "lcd tests rc=$rc"; tail -3 gpurun_out/$T/pytest_lcd.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu --no-replay > gpurun_out/$T/bench_lcd.json 2> gpurun_out/$T/bench_lcd.err || { tail -3 gpurun_out/$T/bench_lcd.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$T/bench_lcd.json')); l=d['lcd']; r=l['roofline']; print('lcd', l['value'], 'knn_ms', r['knn_ms'], 'ransac_ms', r['ransac_ms'], 'knn frac', l['knn2_roofline']['frac'])"
bash scripts/gpu_pmc_r3.sh $T/pmc
