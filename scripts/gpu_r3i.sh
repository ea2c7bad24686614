# usage: bash scripts/gpu_r3i.sh tag — BoW query work queue: BoW / LCD tests,
# then the bench's LCD + BoW legs, in-tree vs alt/head.so, alternating twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3i}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_bow_gpu.py tests/test_configs_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_bow.log 2>&1; rc=$?; echo "bow tests rc=$rc"; tail -3 gpurun_out/$T/pytest_bow.log
[ $rc -ne 0 ] && exit 1
for k in 1 2; do
  for v in intree head; do
    if [ $v = intree ]; then E=KMX_DUMMY=1; else E=KMX_LIB=$PWD/alt/head.so; fi
    env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --burn-in 1 --no-cpu --no-replay > gpurun_out/$T/bench_${v}_$k.json 2> gpurun_out/$T/bench_${v}_$k.err || { tail -3 gpurun_out/$T/bench_${v}_$k.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$T/bench_${v}_$k.json')); l=d['lcd']; print('$v $k lcd', round(l['value']), 'bow', round(l['bow']['value']), 'bow ms', round(l['bow']['ms_per_step'],2))"
  done
done
