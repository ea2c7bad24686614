# smoke() + KMX_FUSED A/B with the G = 9 kernels (30 rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fz
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fz/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/fz/smoke.log; [ $rc -ne 0 ] && exit $rc
for F in 0 1; do
  KMX_FUSED=$F timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-lcd > gpurun_out/fz/b$F.json 2> gpurun_out/fz/b$F.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/fz/b$F.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/fz/b$F.json'));print('fused=$F bench', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms', round(d['roofline']['avg_launch_us'],1))"
done
