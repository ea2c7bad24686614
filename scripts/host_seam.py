"""Host seam of the multi-rank round, emulated on one GPU.

A rank of the N-GPU strong-scaling bench runs, per round: exchange_pack ->
all_to_all (RCCL) -> exchange_unpack -> one round (kmx_pgo_iterate_async(1)).
With host-polled tCG the host is inside the round's tCG loop until the GPU
reports the stop, so the next round's exchange is enqueued only then. This
script builds the rank-`k` handle of configs[3] split over N ranks (the real
per-rank graph and exchange plan), replaces the peers by a frozen neighbour
table (rows gathered once) and times rounds under:
  batch  iterate_async(n)   (single-GPU path: no exchange)
  seam   per-round pack + all_to_all_single (RCCL, world 1: the c10d/RCCL host
         path and a GPU copy of the receive size) + unpack + iterate_async(1)
  native the exchange inside the round (kmx_pgo_comm_init / set_exchange on a
         world-1 communicator, the segment sent to self by ncclSend / ncclRecv:
         min(sent, received) rows, so the rows are the rank's own, not its
         peers' — timing only), all rounds from one iterate_async call
The handle's tCG enqueueing is the default adaptive mode
(kmx_pgo_set_tcg_poll(-1)); KMX_SEAM_POLL=0 / 1 sets blind / polled.
usage: python scripts/host_seam.py N [rounds] [standard|onesync]  (the tCG form)
"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import torch.distributed as dist

import bench
from kmx.dpgo.driver import exchange_plan, robot_ranges, team_tile_incidences
from kmx.dpgo.solver import BlockSolver
from kmx.synth import config, lift, lifting_matrix
import dataclasses

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n_rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 40
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29655")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))

g = config("synth100k", seed=0)
P = bench.params()
P.localOptimizationParams.tCG_form = sys.argv[3] if len(sys.argv) > 3 else "standard"
P = dataclasses.replace(P, tileIncidences=team_tile_incidences(g, N, P.r))
Y = lifting_matrix(5, seed=1)
lo, hi = robot_ranges(g.n_robots, N)[0]
local = np.zeros(g.n_robots, np.uint8)
local[lo:hi] = 1
ss, sc, rs, rc = exchange_plan(g, N, 0)
ps = 4 * P.r
dev = torch.device("cuda", 0)


def make():
    s = BlockSolver(P, 0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    if os.environ.get("KMX_SEAM_POLL"):  # tCG enqueue mode: -1 adaptive (default), 0 blind, 1 polled
        s.set_tcg_poll(int(os.environ["KMX_SEAM_POLL"]))
    s.set_graph_data(g, local)
    s.set_gnc_schedule(True, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol)
    for a in range(lo, hi):
        s.set_iterate(a, lift(g.init_R[a], g.init_t[a], Y))
    s.refresh_local()
    return s


def t(x):
    return torch.as_tensor(np.asarray(x, np.int32), device=dev)


sslots, rslots = t(ss if ss.size else [0]), t(rs if rs.size else [0])
sseg, rseg = t(np.concatenate([[0], np.cumsum(sc)])), t(np.concatenate([[0], np.cumsum(rc)]))
n_send, n_recv = int(ss.size), int(rs.size)
sbuf = torch.zeros(n_send * ps + N, dtype=torch.float64, device=dev)
rbuf = torch.zeros(n_recv * ps + N, dtype=torch.float64, device=dev)
wire_in = torch.zeros(n_recv * ps + N, dtype=torch.float64, device=dev)
wire_out = torch.zeros_like(wire_in)
print(f"N={N}: rank 0 holds robots {lo}..{hi - 1}, {int(g.n_poses[lo:hi].sum())} poses; "
      f"sends {n_send} rows, receives {n_recv} rows ({n_recv * ps * 8 / 1e6:.2f} MB) per round; "
      f"adaptive tCG enqueueing, {P.localOptimizationParams.tCG_form} tCG", flush=True)

modes = ("batch", "seam", "native", "lagged") if os.environ.get("KMX_SEAM_LAG") else ("batch", "seam", "native")
for mode in modes:
    s = make()
    if mode in ("native", "lagged"):
        os.environ["KMX_XCHG_SELF_P2P"] = "1"
        # lagged: the one-round-stale exchange (KMX_XCHG_LAG, pgo.hip enqueue_exchange_lag) on its own stream
        os.environ["KMX_XCHG_LAG"] = "1" if mode == "lagged" else "0"
        k = min(n_send, n_recv)
        s.comm_init(s.comm_unique_id(), 1, 0)
        s.set_exchange(ss[:k], [k], rs[:k], [k])
    if mode == "seam":  # the frozen neighbour table: the initial rows of the foreign slots
        s.gather_public_rows(rslots.data_ptr(), n_recv, rbuf.data_ptr())
        torch.cuda.synchronize()
        rows = rbuf[:n_recv * ps].cpu().numpy().reshape(n_recv, ps)
        segs, off = [], np.concatenate([[0], np.cumsum(rc)])
        for k in range(N):  # each peer's rows, then its status word (not converged)
            segs += [rows[off[k]:off[k + 1]].reshape(-1), np.array([1.0])]
        wire_in.copy_(torch.as_tensor(np.concatenate(segs)))
    burn = 45
    s.iterate_async(burn, refresh_local=True)
    s.sync()
    s.read_counters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode in ("batch", "native", "lagged"):
        s.iterate_async(n_rounds, refresh_local=False)
    else:
        for _ in range(n_rounds):
            s.exchange_pack(sslots.data_ptr(), n_send, sseg.data_ptr(), N, sbuf.data_ptr())
            dist.all_to_all_single(wire_out, wire_in)  # RCCL host path + a receive-sized GPU copy
            s.exchange_unpack(rslots.data_ptr(), n_recv, rseg.data_ptr(), N, wire_out.data_ptr())
            s.iterate_async(1, refresh_local=False)
    s.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    c = s.read_counters()
    print(f"  {mode:5s}: {1e6 * el / n_rounds:7.1f} us/round, hessvecs/round {c['hessvecs'] / n_rounds:.2f}, "
          f"{c['edges_iters'] / el:.3g} edges*iters/s", flush=True)
    s.close()
dist.destroy_process_group()
