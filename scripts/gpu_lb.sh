# usage: bash scripts/gpu_lb.sh tag "5 6 7" — dpgo bench + kernel stats per
# launch-bounds build (libkmx_lb<N>.so built with -DKMX_LB_GATHER=N; 5 = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lb}
mkdir -p gpurun_out/$TAG
for LB in ${2:-5 6 7}; do
  if [ "$LB" = 5 ]; then export KMX_LIB=$PWD/kimera-multi_amd/kmx/libkmx.so; else export KMX_LIB=$PWD/kimera-multi_amd/kmx/libkmx_lb$LB.so; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/$TAG/bench_lb$LB.json 2> gpurun_out/$TAG/bench_lb$LB.err
  rc=$?; echo "lb$LB bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/$TAG/bench_lb$LB.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_lb$LB.json'));print('lb$LB', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms', d['roofline']['avg_launch_us'], round(d['roofline']['frac'],3))"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_lb$LB -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --profile > gpurun_out/$TAG/prof_lb$LB.log 2>&1
  rc=$?; echo "lb$LB prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
