# default bench + the driver's window (20 / 40 steps) for the stability check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-bench}
mkdir -p gpurun_out/$T
timeout -k 10 400 python bench.py > gpurun_out/$T/default.json 2> gpurun_out/$T/default.err || { tail gpurun_out/$T/default.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-lcd > gpurun_out/$T/s20.json 2> gpurun_out/$T/s20.err || exit 1
timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-lcd > gpurun_out/$T/s40.json 2> gpurun_out/$T/s40.err || exit 1
for f in default s20 s40; do python -c "import json,sys; d=json.load(open('gpurun_out/$T/$f.json')); print('$f', d['value'], d['ms_per_step'], d['work'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('replay_identical'))"; done
