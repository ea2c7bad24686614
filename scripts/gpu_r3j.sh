# usage: bash scripts/gpu_r3j.sh tag — dpgo GPU tests, then in-tree vs
# alt/prev.so (scripts/gpu_pgo_ab.sh: 12.5k / 25k rounds + configs[3] window,
# alternating twice).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3j}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_dpgo_gpu.py tests/test_dpgo_edge_gpu.py tests/test_parity_long_gpu.py tests/test_distributed_gpu.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_dpgo.log 2>&1; rc=$?; echo "dpgo tests rc=$rc"; tail -3 gpurun_out/$T/pytest_dpgo.log
[ $rc -ne 0 ] && exit 1
bash scripts/gpu_pgo_ab.sh $T/ab
timeout -k 10 300 python -u scripts/host_seam.py 8 40 > gpurun_out/$T/host_seam_n8.log 2>&1; echo "host_seam rc=$?"; grep -v Warn gpurun_out/$T/host_seam_n8.log | tail -3
KMX_LIB=$PWD/alt/prev.so timeout -k 10 300 python -u scripts/host_seam.py 8 40 > gpurun_out/$T/host_seam_n8_prev.log 2>&1; echo "host_seam prev rc=$?"; grep -v Warn gpurun_out/$T/host_seam_n8_prev.log | tail -3
