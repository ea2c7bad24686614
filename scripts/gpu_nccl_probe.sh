# Probe: can two ranks share one GPU over RCCL (nccl backend)? Exercises the
# driver's device-pointer exchange on torch's stream when RCCL allows it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-nccl}
mkdir -p gpurun_out/$T
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --burn-in 5 --no-cpu --no-lcd --extra-steps 0 \
  > gpurun_out/$T/n2.json 2> gpurun_out/$T/n2.err
echo "nccl n2 rc=$?"; tail -c 1500 gpurun_out/$T/n2.json; grep -iE "error|duplicate|invalid" gpurun_out/$T/n2.err | head -5
