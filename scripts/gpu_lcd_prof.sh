# usage: bash scripts/gpu_lcd_prof.sh tag — kernel stats of the LCD legs (verification + BoW)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lcdprof}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --lcd-steps 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
echo "lcd prof rc=$?"
