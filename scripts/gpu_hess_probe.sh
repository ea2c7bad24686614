# k_hess traffic attribution: FETCH_SIZE and WRITE_SIZE per
# k_hess launch for the product build and for KMX_HESS_PROBE builds that each
# drop one stream (1 neighbour rows, 2 own rows + D_i, 4 delta_old / Hdelta_old,
# 8 the delta / Hdelta stores, 15 all: records + CSR only), built beforehand by
# `make -C kimera-multi_amd/csrc probe PROBE=n` into diag/.
# usage: [BURN=40] bash scripts/gpu_hess_probe.sh TAG [variants...]  (BURN: rounds before the window;
# 10 = first tCG steps, 40 = the bench steady-state window with delta_old / Hdelta_old in play)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-hprobe}; shift
V=${@:-0 1 2 4 8 15}
mkdir -p gpurun_out/$T
for v in $V; do
  if [ "$v" = 0 ]; then lib=$PWD/kimera-multi_amd/kmx/libkmx.so; else lib=$PWD/diag/libkmx_hp$v.so; fi
  O=gpurun_out/$T/v$v
  mkdir -p $O
  i=0
  for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    KMX_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d $O/p$i -o run --output-format csv -- python3 bench.py --burn-in ${BURN:-40} --steps 10 --warmup 0 --profile --no-cpu --no-lcd > $O/p$i.json 2> $O/p$i.err
    rc=$?; echo "variant $v pass $i ($C) rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/p$i.err; exit $rc; }
  done
  python3 scripts/hess_traffic.py $O $O/traffic.json | tr -d '\n' | cut -c1-400; echo
done
exit 0
