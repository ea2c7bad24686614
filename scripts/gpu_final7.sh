# round-3 last evidence: -m gpu suite + smoke, the default bench, the LCD PMC
# ratios of the current kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-final7}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/default.json 2> gpurun_out/$T/default.err || { tail gpurun_out/$T/default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$T/default.json')); l=d['lcd']; print('dpgo', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['ok'], 'lcd', l['value'], 'bow', l['bow']['value'])"
bash scripts/gpu_lcd_pmc3.sh $T/lcd || exit 1
python3 scripts/lcd_pmc_summary.py gpurun_out/$T/lcd gpurun_out/$T/lcd_fp64_stewenius.json 4000 | tail -12
