# usage: bash scripts/gpu_ab_r3b.sh tag — LCD occupancy probe (wave stamps at the
# Stewenius launch bounds 3 and 2: resident waves, loaded latency), then the
# dpgo builds in-tree vs alt/*.so (scripts/gpu_pgo_ab.sh) and the dpgo parity
# tests on alt/dh2.so (the fold-every-2-steps variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abr3b}
mkdir -p gpurun_out/$T
for lb in 3 2; do
  KMX_COOP_LB=$lb timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps_lb$lb.log 2>&1; echo "stamps lb$lb rc=$?"
  grep -v Warn gpurun_out/$T/stamps_lb$lb.log | tail -4
done
bash scripts/gpu_pgo_ab.sh $T/pgo || exit 1
KMX_LIB=$PWD/alt/dh2.so timeout -k 10 600 python -u -m pytest tests/test_dpgo_gpu.py tests/test_parity_long_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/pytest_dh2.log 2>&1; echo "dh2 tests rc=$?"; tail -2 gpurun_out/$T/pytest_dh2.log
