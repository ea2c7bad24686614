set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5u/seam8 -o run --output-format csv -- python3 scripts/host_seam.py 8 40 standard > gpurun_out/r5u/seam8.txt 2>&1
