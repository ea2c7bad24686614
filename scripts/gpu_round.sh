# usage: bash scripts/gpu_round.sh tag — GPU tests, bench, kernel stats, PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-round}
bash scripts/gpu_all.sh $TAG && bash scripts/gpu_pmc_hess.sh $TAG/pmc
