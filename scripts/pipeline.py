"""configs[4] end to end (kmx.pipeline): inter-robot LCD stream -> shared loop
closures -> distributed initialisation -> RBCD + GNC rounds.

  python scripts/pipeline.py [--robots 8 --poses 20000 ...]            # one GPU
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      scripts/pipeline.py ...                                          # N GPUs
Rank 0 prints one JSON line."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=8)
    ap.add_argument("--poses", type=int, default=20_000, help="poses per robot")
    ap.add_argument("--edges-per-pose", type=float, default=5.0)
    ap.add_argument("--true-per-robot", type=int, default=1000)
    ap.add_argument("--false-per-robot", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=500)
    ap.add_argument("--sigma-r", type=float, default=0.002, help="odometry rotation noise per keyframe (rad)")
    ap.add_argument("--sigma-t", type=float, default=0.02, help="odometry translation noise per keyframe (m)")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import bench
    from kmx import pipeline as PL
    from kmx.lcd import LcdParams
    from kmx.synth import make_pose_graph
    t0 = time.perf_counter()
    n = a.robots * a.poses
    g0 = make_pose_graph(a.robots, n, int(a.edges_per_pose * n), f_inter=0.0, outlier_scope="robot",
                         sigma_R=a.sigma_r, sigma_t=a.sigma_t, seed=a.seed)
    stream = PL.make_lc_stream(g0, a.robots * a.true_per_robot, a.robots * a.false_per_robot, seed=a.seed + 1)
    gen = time.perf_counter() - t0
    out = PL.run_pipeline(g0, stream, bench.params(), LcdParams(), rank=rank, world=world, device=local_rank,
                          rounds=a.rounds)
    out["config"] = {"workload": f"configs[4]: {a.robots} robots x {a.poses} poses, {g0.m} base edges "
                                 f"(intra-robot loop closures, 20% intra outliers, odometry noise "
                                 f"{a.sigma_r} rad / {a.sigma_t} m), LC stream "
                                 f"{stream.truth.shape[0]} candidates ({int(stream.truth.sum())} planted)",
                     "n_gpus": world, "generation_s": round(gen, 1)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
