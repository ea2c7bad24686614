# usage: bash scripts/gpu_r3f.sh tag — LCD wave residency: the alternating
# true / false pool vs true candidates only (launch bounds 3).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3f}
mkdir -p gpurun_out/$T
timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps_mixed.log 2>&1; echo "mixed rc=$?"; grep -v Warn gpurun_out/$T/stamps_mixed.log | tail -3
STAMPS_ONLY_TRUE=1 timeout -k 10 200 python3 -u scripts/lcd_stamps.py 40000 > gpurun_out/$T/stamps_true.log 2>&1; echo "true rc=$?"; grep -v Warn gpurun_out/$T/stamps_true.log | tail -3
