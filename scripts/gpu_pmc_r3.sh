# usage: bash scripts/gpu_pmc_r3.sh tag — the stored PMC ratios bench.py reads:
# k_hess traffic at configs[3] (scripts/gpu_pmc_hess.sh) and the LCD
# Stewenius per-candidate instruction counts (scripts/gpu_lcd_pmc3.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pmcr3}
mkdir -p gpurun_out/$T
bash scripts/gpu_pmc_hess.sh $T/hess synth100k || exit 1
python3 scripts/hess_traffic.py gpurun_out/$T/hess gpurun_out/$T/hessvec_traffic_synth100k.json | tail -3
bash scripts/gpu_lcd_pmc3.sh $T/lcd || exit 1
python3 scripts/lcd_pmc_summary.py gpurun_out/$T/lcd gpurun_out/$T/lcd_fp64_stewenius.json 4000 | tail -12
