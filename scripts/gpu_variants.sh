# A/B the kernel variants: parity tests + bench + profile per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-var}
mkdir -p gpurun_out/$TAG
for V in ${VARIANTS:-21 20 01}; do
  export KMX_GATHER=${V:0:1} KMX_FUSED=${V:1:1}
  N=g${V:0:1}f${V:1:1}
  timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_$N.log 2>&1
  rc=$?; echo "$N pytest rc=$rc $(tail -1 gpurun_out/$TAG/pytest_$N.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/$TAG/pytest_$N.log; exit $rc; }
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/$TAG/bench_$N.json 2> gpurun_out/$TAG/bench_$N.err
  rc=$?; echo "$N bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$N.json'));print('$N', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms', d['roofline']['avg_launch_us'], round(d['roofline']['frac'],3))"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$N -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --profile > gpurun_out/$TAG/prof_$N.log 2>&1
  rc=$?; echo "$N prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
