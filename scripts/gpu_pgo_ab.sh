# A/B of dpgo builds: in-tree vs alt/*.so (KMX_LIB), alternating twice:
# round time at 12.5k / 25k poses (round_sizes.py) and the configs[3] bench
# (no CPU / LCD legs); then the in-tree build's dpgo parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pgoab}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 -u scripts/round_sizes.py 1,2 > gpurun_out/$T/sizes_$name.log 2>&1 || { echo "sizes $name failed"; tail -3 gpurun_out/$T/sizes_$name.log; exit 1; }
  sed "s/^/$name /" gpurun_out/$T/sizes_$name.log
  env "$@" timeout -k 10 240 python3 bench.py --steps 100 --no-cpu --no-lcd --no-replay > gpurun_out/$T/bench_$name.json 2> gpurun_out/$T/bench_$name.err || { echo "bench $name failed"; tail -3 gpurun_out/$T/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_$name.json')); print('$name bench', round(d['value']/1e8,3), 'e8', round(d['ms_per_step']*1e3,1), 'us/round')"
}
for k in 1 2; do
  run intree_$k KMX_DUMMY=1 || exit 1
  for f in alt/*.so; do b=$(basename $f .so); run ${b}_$k KMX_LIB=$PWD/$f || exit 1; done
done
timeout -k 10 600 python -u -m pytest tests/test_dpgo_gpu.py tests/test_dpgo_edge_gpu.py tests/test_parity_long_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/pytest_dpgo.log 2>&1; echo "dpgo tests rc=$?"; tail -3 gpurun_out/$T/pytest_dpgo.log
