# round 3: the -m gpu suite (minus the long-horizon file) and the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r3a.sh r3b
