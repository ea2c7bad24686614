set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ph
for a in 0 1; do timeout -k 10 300 python scripts/lcd_phases.py $a > gpurun_out/ph/a$a.log 2>&1 || exit 1; cat gpurun_out/ph/a$a.log; done
