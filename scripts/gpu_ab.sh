# Same-box A/B of one command under several settings, alternating REPS times.
# usage: bash scripts/gpu_ab.sh TAG REPS "command args" SETTING [SETTING ...]
# SETTING: "-" (as is) or comma-separated VAR=VAL pairs (KMX_LIB=diag/x.so
# is made absolute). Each run's output goes to gpurun_out/TAG/<i>_<rep>.log and
# its last 3 lines are echoed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=$1; REPS=$2; CMD=$3; shift 3
mkdir -p gpurun_out/$T
for rep in $(seq 1 "$REPS"); do
  i=0
  for S in "$@"; do
    i=$((i + 1))
    envs=()
    if [ "$S" != "-" ]; then
      IFS=',' read -ra kv <<< "$S"
      for e in "${kv[@]}"; do
        case "$e" in KMX_LIB=*) e="KMX_LIB=$PWD/${e#KMX_LIB=}" ;; esac
        envs+=("$e")
      done
    fi
    env "${envs[@]}" timeout -k 10 400 $CMD > gpurun_out/$T/${i}_$rep.log 2>&1 \
      || { echo "[$S] failed"; tail -20 gpurun_out/$T/${i}_$rep.log; exit 1; }
    echo "[$S] rep $rep: $(tail -3 gpurun_out/$T/${i}_$rep.log | tr '\n' ' ')"
  done
done
echo "ab done"
