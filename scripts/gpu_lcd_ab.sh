# A/B of LCD variants: in-tree build under KMX_COOP_LB settings vs alt/libkmx_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-lcdab}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/lcd_timing.py 20000 > gpurun_out/$T/timing_$name.log 2>&1; echo "timing $name rc=$?"; grep verify_async gpurun_out/$T/timing_$name.log | tail -1
}
run lb3 KMX_DUMMY=1
run lb4 KMX_COOP_LB=4
run lb5 KMX_COOP_LB=5
run old KMX_LIB=$PWD/alt/libkmx_old.so
timeout -k 10 120 python -u scripts/lcd_phases.py 0 > gpurun_out/$T/phases_lb3.log 2>&1; echo "phases rc=$?"; cat gpurun_out/$T/phases_lb3.log
