# Rehearsal of the N > 1 bench path on one MI355X: N ranks share the GPU and
# exchange through gloo (KMX_DIST_BACKEND=gloo). Exercises the multi-rank driver,
# exchange and bench plumbing end to end; not a scaling measurement.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp KMX_DIST_BACKEND=gloo
T=${1:-mg}; shift
mkdir -p gpurun_out/$T
port=29531
for n in "$@"; do
  port=$((port + 1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 10 --warmup 2 --no-cpu --no-lcd > gpurun_out/$T/n$n.json 2> gpurun_out/$T/n$n.err || { tail gpurun_out/$T/n$n.err; exit 1; }
  python3 - "$T" "$n" <<'PY' | tee -a gpurun_out/$T/summary.txt
import json, sys
t, n = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/{t}/n{n}.json").read().strip().splitlines()[-1])
print(n, d["value"], d["ms_per_step"], d["scaling"], d["config"]["parallelism"], d["roofline"]["replay_identical"],
      d["config"]["exchange_rows_per_round"])
PY
done
