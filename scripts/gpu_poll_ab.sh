# Same-box A/B of the tCG enqueue modes (KMX_POLL=1 polled, 0 blind, unset adaptive):
# round time vs size, the emulated multi-rank seam (N = 8, 4) and the bench window.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pollab}
mkdir -p gpurun_out/$T
for M in 1 0 a; do
  if [ $M = a ]; then unset KMX_POLL; else export KMX_POLL=$M; fi
  echo "== mode $M" | tee -a gpurun_out/$T/ab.log
  timeout -k 10 200 python scripts/round_sizes.py 1,8 2>&1 | tee -a gpurun_out/$T/ab.log || exit 1
  for n in 8 4; do timeout -k 10 150 python scripts/host_seam.py $n 60 2>&1 | grep -E "batch|seam" | sed "s/^/N=$n /" | tee -a gpurun_out/$T/ab.log || exit 1; done
  timeout -k 10 200 python bench.py --steps 40 --no-cpu --no-lcd > gpurun_out/$T/b$M.json 2>gpurun_out/$T/b$M.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/b$M.json')); print('bench', d['value'], d['ms_per_step'])" | tee -a gpurun_out/$T/ab.log
done
