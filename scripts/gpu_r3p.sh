# usage: bash scripts/gpu_r3p.sh tag — the LCD PMC ratios of the current
# kernel (scripts/gpu_lcd_pmc3.sh) and the LCD leg with the Nister solver.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3p}
mkdir -p gpurun_out/$T
bash scripts/gpu_lcd_pmc3.sh $T/lcd || exit 1
python3 scripts/lcd_pmc_summary.py gpurun_out/$T/lcd gpurun_out/$T/lcd_fp64_stewenius.json 4000 | tail -14
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --burn-in 1 --no-cpu --no-replay --lcd-algo 1 > gpurun_out/$T/bench_nister.json 2> gpurun_out/$T/bench_nister.err || { tail -3 gpurun_out/$T/bench_nister.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$T/bench_nister.json')); l=d['lcd']; print('nister lcd', round(l['value']), 'ransac ms', round(l['roofline']['ransac_ms'],2))"
