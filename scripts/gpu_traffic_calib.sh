# FETCH_SIZE / WRITE_SIZE calibration of k_hess's access patterns (one --pmc
# pass per counter over scripts/probe/traffic_probe, built in-tree beforehand).
# usage: bash scripts/gpu_traffic_calib.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-calib}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 60 ./scripts/probe/traffic_probe > $O/probe.txt || { echo "probe failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- ./scripts/probe/traffic_probe > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail $O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- ./scripts/probe/traffic_probe > $O/write.log 2>&1 || { echo "write pass failed"; tail $O/write.log; exit 1; }
python3 scripts/probe/traffic_calib.py $O $O/calib.json | head -80
