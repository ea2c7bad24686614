# Same-box LCD A/B (configs[2] shape, Stewenius): the in-tree library against
# alt/libkmx_r3.so (the round-3 library, built from its commit), alternating
# twice, plus the longest-first queue order (KMX_LCD_ORDER=1) on the in-tree one.
# usage: bash scripts/gpu_lcd_ab2.sh TAG [candidates]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-lcdab}; N=${2:-20000}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  timeout -k 10 300 python scripts/lcd_timing.py $N > gpurun_out/$T/intree_$rep.log 2>&1 || { tail gpurun_out/$T/intree_$rep.log; exit 1; }
  echo "intree $rep: $(grep -E "verify_async|back-to-back" gpurun_out/$T/intree_$rep.log | tail -2 | tr "\n" " ")"
  KMX_LIB=$PWD/alt/libkmx_r3.so KMX_AB_OLDLIB=1 timeout -k 10 300 python scripts/lcd_timing.py $N > gpurun_out/$T/r3_$rep.log 2>&1 || { tail gpurun_out/$T/r3_$rep.log; exit 1; }
  echo "r3     $rep: $(grep -E "verify_async|back-to-back" gpurun_out/$T/r3_$rep.log | tail -2 | tr "\n" " ")"
  KMX_LCD_ORDER=1 timeout -k 10 300 python scripts/lcd_timing.py $N > gpurun_out/$T/order_$rep.log 2>&1 || { tail gpurun_out/$T/order_$rep.log; exit 1; }
  echo "order  $rep: $(grep -E "verify_async|back-to-back" gpurun_out/$T/order_$rep.log | tail -2 | tr "\n" " ")"
done
