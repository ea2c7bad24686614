# KMX_TILECAP sweep: G = 9 gathers alone + bench (30 rounds). "def" = the
# handle's default cap (two chunks for G = 9), 0 = no cap, N = cap at N.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tcap
for C in ${1:-def 0 480 384}; do
  if [ "$C" = def ]; then unset KMX_TILECAP; else export KMX_TILECAP=$C; fi
  timeout -k 10 200 python scripts/gather_bench.py synth100k 92,93,92,93 > gpurun_out/tcap/g$C.log 2>&1
  rc=$?; echo "cap=$C"; cat gpurun_out/tcap/g$C.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-lcd > gpurun_out/tcap/b$C.json 2> gpurun_out/tcap/b$C.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/tcap/b$C.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/tcap/b$C.json'));print('cap=$C bench', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms', round(d['roofline']['avg_launch_us'],1))"
done
