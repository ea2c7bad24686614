# Same-box A/B of library builds by rocprofv3 kernel stats of the dpgo bench: bash scripts/gpu_ab_prof.sh TAG lib1.so [lib2.so ...] (diag/ names; two reps each, alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for L in "" "$@"; do
    tag=${L:-intree}_$rep
    if [ -n "$L" ]; then export KMX_LIB=$PWD/diag/$L; else unset KMX_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/$tag -o run --output-format csv -- python3 bench.py --no-cpu --no-lcd --steps 10 > gpurun_out/$T/$tag.json 2> gpurun_out/$T/$tag.err || { tail gpurun_out/$T/$tag.err; exit 1; }
    echo "$tag done"
  done
done
