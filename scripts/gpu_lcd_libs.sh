# Same-box LCD A/B of library variants (configs[2] shape, Stewenius,
# scripts/lcd_timing.py): the in-tree library and each alt/ library named,
# alternating twice. usage: bash scripts/gpu_lcd_libs.sh TAG N lib1 [lib2 ...]
# (lib: a file name under diag/, e.g. libkmx_sg4.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-lcdlibs}; N=${2:-20000}; shift; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do
  timeout -k 10 300 python scripts/lcd_timing.py $N > gpurun_out/$T/intree_$rep.log 2>&1 || { tail gpurun_out/$T/intree_$rep.log; exit 1; }
  echo "intree $rep: $(grep -E "verify_async|back-to-back" gpurun_out/$T/intree_$rep.log | tail -2 | tr "\n" " ")"
  for L in "$@"; do
    KMX_LIB=$PWD/diag/$L timeout -k 10 300 python scripts/lcd_timing.py $N > gpurun_out/$T/${L}_$rep.log 2>&1 || { tail gpurun_out/$T/${L}_$rep.log; exit 1; }
    echo "$L $rep: $(grep -E "verify_async|back-to-back" gpurun_out/$T/${L}_$rep.log | tail -2 | tr "\n" " ")"
  done
done
