# rocprofv3 kernel + memory-copy trace of the call-for-call LCD chain
# (scripts/lcd_single.py) -> gpurun_out/$1/lcd_single_{planted,hard}/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for k in planted hard; do
  O=gpurun_out/$1/lcd_single_$k
  mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O -o run --output-format csv \
    -- python3 scripts/lcd_single.py $k 16 > $O/out.txt 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  cat $O/out.txt
done
