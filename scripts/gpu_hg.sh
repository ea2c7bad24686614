# k_grad chunk size A/B: libkmx.so (192) vs libkmx_hg240.so (240)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/hg
for V in 192 240; do
  if [ $V = 192 ]; then export KMX_LIB=$PWD/kimera-multi_amd/kmx/libkmx.so; else export KMX_LIB=$PWD/kimera-multi_amd/kmx/libkmx_hg$V.so; fi
  timeout -k 10 200 python scripts/gather_bench.py synth100k 93,93 > gpurun_out/hg/g$V.log 2>&1
  rc=$?; echo "ch=$V"; cat gpurun_out/hg/g$V.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-lcd > gpurun_out/hg/b$V.json 2> gpurun_out/hg/b$V.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/hg/b$V.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/hg/b$V.json'));print('ch=$V bench', round(d['value']/1e6,1),'M', round(d['ms_per_step'],3),'ms')"
done
