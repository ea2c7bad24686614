# round 3: persistent round kernel tests + A/B, then the rest of the -m gpu
# suite and the bench (scripts/gpu_r3a.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round.sh r3b_round || exit 1
bash scripts/gpu_r3a.sh r3b
