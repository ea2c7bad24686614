# usage: bash scripts/gpu_r3e.sh tag — the -m gpu suite, LCD wave stamps and
# throughput after the XCD-balanced candidate mapping, then the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3e}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/$T/pytest_gpu.log
[ $rc -ne 0 -a $rc -ne 1 ] && exit 1
for lb in 3 2; do
  KMX_COOP_LB=$lb timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps_lb$lb.log 2>&1; echo "stamps lb$lb rc=$?"
  grep -v Warn gpurun_out/$T/stamps_lb$lb.log | tail -2
done
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && { tail -5 gpurun_out/$T/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); r=d['roofline']; l=d['lcd']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d.get('parity',{}).get('ok'), 'lcd', l['value'], l['roofline']['frac'], 'bow', l['bow']['value'])"
