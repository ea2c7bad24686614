# usage: bash scripts/gpu_r3c.sh tag — the -m gpu suite, a dpgo bench (CPU
# leg replaying the timed window for parity), then the LCD instruction-cache
# counters (scripts/gpu_icache.sh without its test step).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3c}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
[ $rc -ne 0 -a $rc -ne 1 ] && exit 1  # 1: failed tests (listed above); go on to the measurements
timeout -k 10 300 python bench.py --no-lcd > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity'))"
bash scripts/gpu_icache.sh $TAG/icache
