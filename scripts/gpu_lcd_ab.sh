# LCD verification throughput, current library vs ab_libs/libkmx_prev.so (per solver)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcd_ab}; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do for lib in cur prev; do for a in 0 1; do
  if [ $lib = prev ]; then export KMX_LIB=ab_libs/libkmx_prev.so; else unset KMX_LIB; fi
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --burn-in 0 --no-cpu --no-replay --lcd-algo $a > gpurun_out/$T/$lib$a.json 2> gpurun_out/$T/$lib$a.err || { tail gpurun_out/$T/$lib$a.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/$lib$a.json'))['lcd']; print('$lib algo $a', round(d['value']), round(d['ms_per_step'],2))" | tee -a gpurun_out/$T/ab.log
done; done; done
