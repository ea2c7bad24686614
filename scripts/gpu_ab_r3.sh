# usage: bash scripts/gpu_ab_r3.sh tag — in-tree build vs alt/head.so (KMX_LIB),
# alternating: dpgo configs[3] bench window + the 12.5k / 25k round sizes
# (scripts/gpu_pgo_ab.sh's runs), then LCD Stewenius throughput at 20k
# candidates (scripts/lcd_timing.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abr3}
mkdir -p gpurun_out/$T
lcd() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 -u scripts/lcd_timing.py 20000 > gpurun_out/$T/lcd_$name.log 2>&1 || { echo "lcd $name failed"; tail -3 gpurun_out/$T/lcd_$name.log; exit 1; }
  grep verify_async gpurun_out/$T/lcd_$name.log | sed "s/^/$name /"
}
for k in 1 2; do
  lcd intree_$k KMX_DUMMY=1 || exit 1
  lcd head_$k KMX_LIB=$PWD/alt/head.so || exit 1
done
bash scripts/gpu_pgo_ab.sh $T/pgo
timeout -k 10 200 python3 -u scripts/lcd_stamps.py 20000 > gpurun_out/$T/stamps.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/$T/stamps.log | grep -v Warn | tail -5
