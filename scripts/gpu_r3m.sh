# usage: bash scripts/gpu_r3m.sh tag — dpgo GPU tests, then three arms
# alternating twice: in-tree (k_hess_epi + k_grad prefetch), in-tree with
# KMX_HESS_EPI=0, alt/prev.so; round sizes 12.5k / 25k, configs[3] window and
# the N = 8 rank handle (host_seam).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3m}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_dpgo_gpu.py tests/test_dpgo_edge_gpu.py tests/test_parity_long_gpu.py tests/test_distributed_gpu.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_dpgo.log 2>&1; rc=$?; echo "dpgo tests rc=$rc"; tail -3 gpurun_out/$T/pytest_dpgo.log
[ $rc -ne 0 ] && exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 -u scripts/round_sizes.py 1,2 > gpurun_out/$T/sizes_$name.log 2>&1 || { echo "sizes $name failed"; tail -3 gpurun_out/$T/sizes_$name.log; exit 1; }
  sed "s/^/$name /" gpurun_out/$T/sizes_$name.log
  env "$@" timeout -k 10 240 python3 bench.py --steps 100 --no-cpu --no-lcd --no-replay > gpurun_out/$T/bench_$name.json 2> gpurun_out/$T/bench_$name.err || { echo "bench $name failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_$name.json')); print('$name bench', round(d['value']/1e8,3), 'e8', round(d['ms_per_step']*1e3,1), 'us/round')"
  env "$@" timeout -k 10 300 python -u scripts/host_seam.py 8 40 > gpurun_out/$T/seam_$name.log 2>&1 || { echo "seam $name failed"; exit 1; }
  grep -E 'batch|native' gpurun_out/$T/seam_$name.log | sed "s/^/$name /"
}
for k in 1 2; do
  run both_$k KMX_DUMMY=1 || exit 1
  run gradonly_$k KMX_HESS_EPI=0 || exit 1
  run prev_$k KMX_LIB=$PWD/alt/prev.so || exit 1
done
