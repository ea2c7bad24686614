# A/B of the round time vs per-GPU size under env settings:
# bash scripts/gpu_ab_sizes.sh TAG "sizes|ENV=.. ENV=.." ...   (one case per argument)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
for C in "$@"; do
  S=${C%%|*}; E=${C#*|}
  echo "== sizes $S env [$E]" | tee -a gpurun_out/$T/ab.log
  env $E timeout -k 10 240 python3 scripts/round_sizes.py $S 2>&1 | tee -a gpurun_out/$T/ab.log || exit 1
done
