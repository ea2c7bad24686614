# Round time and k_hess roofline against the tile cut (bench.py --tile-incidences:
# incidences per workgroup tile; the default cut gives 2,084 tiles at configs[3], i.e. two
# generations of the 1,024 resident k_hess workgroups plus 36 tiles).
# usage: bash scripts/gpu_tile_sweep.sh TAG cap...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-tiles}; shift
mkdir -p gpurun_out/$T
for cap in "$@"; do
  if [ "$cap" = default ]; then ti=0; else ti=$cap; fi
  timeout -k 10 300 python bench.py --no-cpu --no-lcd --steps 200 --tile-incidences $ti > gpurun_out/$T/cap_$cap.json 2> gpurun_out/$T/cap_$cap.err \
    || { echo "cap $cap failed"; tail -5 gpurun_out/$T/cap_$cap.err; exit 1; }
  python3 - "$T" "$cap" <<'PY' | tee -a gpurun_out/$T/summary.txt
import json, sys
t, cap = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/{t}/cap_{cap}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"cap {cap}: {d['value']:.4g} edges*iters/s, {d['ms_per_step']*1e3:.1f} us/round, k_hess {r['avg_launch_us']:.1f} us frac {r['frac']:.3f}, hessvecs/round {d['work']['hessvecs_per_round']:.2f}, parity {d.get('parity', {}).get('ok')}")
PY
done
