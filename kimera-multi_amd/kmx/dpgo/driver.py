"""RBCDDriver — the dpgo_ros synchronous scheduler on MI355X.

Reference control flow (drawio:1954-2066, 2071, 2466-2481):
  * every round the executing robots run PGOAgent::iterate(doOptimization)
    against the neighbour poses they last received (publishPublicPoses ->
    updateNeighborPoses, drawio:2340-2355);
  * every ``robustOptInnerIters`` rounds the leader sends UPDATE_WEIGHT and every
    agent runs updateMeasurementWeights (drawio:2212-2215); the owner of a
    shared loop closure (lower robot id) sends its weight to the peer
    (publishMeasurementWeights, drawio:2195-2198);
  * schedule: dpgo_ros lets ONE robot iterate per round (``sequential``,
    drawio:2478-2481); the MI355X layout updates every block each round
    (``concurrent``, SURVEY.md §0 finding 6, §8e).

Placement: robot blocks are dealt to ranks in contiguous ranges (one process
per GPU). ROS topics become collectives over RCCL/xGMI:
  public_poses          -> one all_to_all per round carrying, to every peer,
                           only the public-pose rows its shared loop closures
                           reference (``exchange="alltoall"``, default); or one
                           all_gather of every owned public row (``"allgather"``)
  measurement_weights   -> all_reduce(SUM) of the owner-packed shared weights
  lifting_matrix/anchor -> injected at initialisation (identical on all ranks)
"""
from __future__ import annotations

import numpy as np

from .params import PGOAgentParameters
from .solver import BlockSolver


def robot_ranges(n_robots: int, world: int) -> list[tuple[int, int]]:
    out = []
    for k in range(world):
        out.append((k * n_robots // world, (k + 1) * n_robots // world))
    return out


def exchange_plan(graph, world: int, rank: int):
    """Slot lists of the sparse public-pose exchange for `rank`.

    The public table holds every endpoint of a shared loop closure, sorted by
    (robot, pose) (the order kmx_pgo_set_graph uses), so the slots a rank owns
    are one contiguous range. A rank needs the rows of the foreign endpoints
    of its shared loop closures; it sends to every peer the rows that peer
    needs from the robots it owns. Returns (send_slots, send_counts[world],
    recv_slots, recv_counts[world]): send slots grouped by destination rank,
    receive slots grouped by source rank, every group in increasing slot order
    on both sides (so the sender's and the receiver's row orders agree)."""
    g = graph
    sh = g.r1 != g.r2
    k1 = (g.r1[sh].astype(np.int64) << 32) | g.p1[sh].astype(np.int64)
    k2 = (g.r2[sh].astype(np.int64) << 32) | g.p2[sh].astype(np.int64)
    keys = np.unique(np.concatenate([k1, k2]))
    nk = max(int(keys.shape[0]), 1)
    s1, s2 = np.searchsorted(keys, k1), np.searchsorted(keys, k2)
    rank_of = np.empty(g.n_robots, np.int64)
    for k, (lo, hi) in enumerate(robot_ranges(g.n_robots, world)):
        rank_of[lo:hi] = k
    q1, q2 = rank_of[g.r1[sh]], rank_of[g.r2[sh]]
    x = q1 != q2
    # (needing rank, slot) pairs, sorted by rank then slot
    pair = np.unique(np.concatenate([q1[x] * nk + s2[x], q2[x] * nk + s1[x]]))
    need_rank, need_slot = pair // nk, pair % nk
    owner = rank_of[keys[need_slot] >> 32] if need_slot.size else need_slot
    sm = owner == rank
    rm = need_rank == rank
    return (need_slot[sm], np.bincount(need_rank[sm], minlength=world)[:world],
            need_slot[rm], np.bincount(owner[rm], minlength=world)[:world])


class RBCDDriver:
    def __init__(self, params: PGOAgentParameters, graph, *, rank: int = 0, world: int = 1,
                 device: int = 0, seed: int = 0, solver=None, exchange_device: str | None = None,
                 exchange: str = "alltoall"):
        """`solver` defaults to a BlockSolver on HIP device `device`; any object
        with the same exchange interface can be injected (the CPU gloo tests do).
        `exchange_device` is where the collective runs ("cuda" for RCCL, "cpu"
        for gloo). A GPU solver under gloo packs into device buffers and stages
        them through host copies (used to test N ranks on one GPU).
        `exchange` selects the public-pose collective ("alltoall" or
        "allgather"); both give bitwise identical iterates."""
        if world > graph.n_robots:
            raise ValueError("need at least one robot block per rank")
        if exchange not in ("alltoall", "allgather"):
            raise ValueError("exchange must be 'alltoall' or 'allgather'")
        self.params = params
        self.graph = graph
        self.rank, self.world = rank, world
        self.exchange = exchange
        lo, hi = robot_ranges(graph.n_robots, world)[rank]
        self.robots = list(range(lo, hi))
        local = np.zeros(graph.n_robots, np.uint8)
        local[lo:hi] = 1
        self.local = local
        self.solver = solver if solver is not None else BlockSolver(params, device)
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.round_index = 0
        self.weight_updates = 0
        self._torch = None
        self._xdev = exchange_device
        if world > 1:
            import torch
            import torch.distributed as dist
            self._torch, self._dist = torch, dist
            if self._xdev is None:
                self._xdev = "cuda" if dist.get_backend() == "nccl" else "cpu"
            if getattr(self.solver, "device_pointers", False):  # order kmx work with torch's copies
                self.solver.set_stream(torch.cuda.current_stream().cuda_stream)
        self.solver.set_graph_data(graph, local)
        self.n_pub, self.first_owned, self.n_owned = self.solver.public_count()
        self.m_local = {a: self.solver.local_edges(a) for a in self.robots}
        self.exchange_rows = (0, 0)  # (rows sent, rows received) per round
        if world > 1:
            self._setup_exchange()

    # ------------------------------------------------------ collectives ---
    def _setup_exchange(self):
        torch, dist = self._torch, self._dist
        ps = 4 * self.params.r
        on_gpu = bool(getattr(self.solver, "device_pointers", False))
        self._stage = on_gpu and self._xdev != "cuda"
        dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
        self.n_shared = self.solver.shared_count()
        self._wshared = torch.zeros(max(self.n_shared, 1), dtype=torch.float64, device=dev)
        if self.exchange == "alltoall":
            send_slots, send_counts, recv_slots, recv_counts = exchange_plan(self.graph, self.world, self.rank)
            self._n_send, self._n_recv = int(send_slots.shape[0]), int(recv_slots.shape[0])
            self._send_splits = [int(c) * ps for c in send_counts]
            self._recv_splits = [int(c) * ps for c in recv_counts]
            one = np.zeros(1, np.int32)
            self._sslots = torch.as_tensor(send_slots.astype(np.int32) if self._n_send else one, device=dev)
            self._rslots = torch.as_tensor(recv_slots.astype(np.int32) if self._n_recv else one, device=dev)
            self._sbuf = torch.zeros(max(self._n_send, 1) * ps, dtype=torch.float64, device=dev)
            self._rbuf = torch.zeros(max(self._n_recv, 1) * ps, dtype=torch.float64, device=dev)
            self.exchange_rows = (self._n_send, self._n_recv)
            return
        counts = [None] * self.world
        dist.all_gather_object(counts, (self.first_owned, self.n_owned))
        self.max_owned = max(max(c[1] for c in counts), 1)
        self._send = torch.zeros(self.max_owned * ps, dtype=torch.float64, device=dev)
        self._recv = torch.zeros(self.world * self.max_owned * ps, dtype=torch.float64, device=dev)
        # rows of the gathered buffer in public-table order
        idx = np.full(max(self.n_pub, 1), 0, dtype=np.int64)
        for k, (first, n) in enumerate(counts):
            idx[first:first + n] = k * self.max_owned + np.arange(n)
        self._row_index = torch.as_tensor(idx[: max(self.n_pub, 1)], device=dev)
        self._table = torch.zeros(max(self.n_pub, 1) * ps, dtype=torch.float64, device=dev)
        self.exchange_rows = (self.n_owned * (self.world - 1), self.n_pub - self.n_owned)

    def _all_gather(self, out, inp):
        """One all-gather of equal-size chunks (RCCL: into one tensor; gloo has
        no all_gather_into_tensor, so gather a list of views)."""
        if self._xdev == "cuda":
            self._dist.all_gather_into_tensor(out, inp)
        elif self._stage:
            self.solver.sync()
            ho, hi = out.cpu(), inp.cpu()
            self._dist.all_gather(list(ho.chunk(self.world)), hi)
            out.copy_(ho)
        else:
            self._dist.all_gather(list(out.chunk(self.world)), inp)

    def _all_to_all(self, out, inp):
        """One all-to-all with per-peer row counts (RCCL directly; a GPU solver
        under gloo stages through host copies)."""
        o, i = out[: sum(self._recv_splits)], inp[: sum(self._send_splits)]
        if self._stage:
            self.solver.sync()
            ho, hi = o.cpu(), i.cpu()
            self._dist.all_to_all_single(ho, hi, self._recv_splits, self._send_splits)
            o.copy_(ho)
        else:
            self._dist.all_to_all_single(o, i, self._recv_splits, self._send_splits)

    def exchange_public(self):
        """publishPublicPoses -> updateNeighborPoses for the whole team."""
        if self.world == 1:
            self.solver.refresh_local()
            return
        ps = 4 * self.params.r
        if self.exchange == "alltoall":
            self.solver.refresh_local()  # the owned slots of the table
            self.solver.gather_public_rows(self._sslots.data_ptr(), self._n_send, self._sbuf.data_ptr())
            self._all_to_all(self._rbuf, self._sbuf)
            self.solver.scatter_public_rows(self._rslots.data_ptr(), self._n_recv, self._rbuf.data_ptr())
            return
        self.solver.pack_public(self._send.data_ptr())
        self._all_gather(self._recv, self._send)
        if self.n_pub:
            rows = self._recv.view(-1, ps).index_select(0, self._row_index)
            self._table.view(-1, ps).copy_(rows)
            self.solver.unpack_public(self._table.data_ptr())

    def update_weights(self) -> float:
        """UPDATE_WEIGHT: every agent re-weights the loop closures it owns, then
        owners send shared-edge weights to their peers."""
        self.exchange_public()
        mu = self.solver.update_weights()
        if self.world > 1 and self.n_shared:
            self.solver.pack_shared_weights(self._wshared.data_ptr())
            if self._stage:
                self.solver.sync()
                hw = self._wshared.cpu()
                self._dist.all_reduce(hw)
                self._wshared.copy_(hw)
            else:
                self._dist.all_reduce(self._wshared)
            self.solver.unpack_shared_weights(self._wshared.data_ptr())
        self.weight_updates += 1
        return mu

    # ------------------------------------------------------------ rounds ---
    def initialize(self, X_by_robot: dict):
        for a in self.robots:
            self.solver.set_iterate(a, X_by_robot[a])

    def should_update_weights(self) -> bool:
        """shouldUpdateMeasurementWeights (drawio:2466-2469), iteration-count form."""
        rc = self.params.robustCostParams
        if int(rc.costType) == 0:
            return False
        if self.weight_updates >= self.params.robustOptNumWeightUpdates:
            return False
        return self.round_index > 0 and self.round_index % self.params.robustOptInnerIters == 0

    def active_mask(self) -> np.ndarray:
        act = np.zeros(self.graph.n_robots, np.uint8)
        if self.params.schedule == 0:  # sequential: leader picks one executing robot
            act[self.round_index % self.graph.n_robots] = 1
        else:
            act[:] = 1
        return act

    def step(self, with_stats: bool = True):
        """One synchronous round. Returns per-robot stats (team-indexed)."""
        self.exchange_public()
        stats = None
        if with_stats or self.params.schedule == 0:
            stats = self.solver.iterate(self.active_mask())
        else:
            self.solver.iterate_async(1, refresh_local=False, gnc_every=0)
        self.round_index += 1
        if self.should_update_weights():
            self.update_weights()
        return stats

    def run_async(self, rounds: int):
        """Benchmark path: enqueue `rounds` concurrent rounds with no host sync
        (single GPU: one C call; multi-GPU: collectives between rounds)."""
        if self.world == 1 and self.params.schedule == 1:
            gnc = self.params.robustOptInnerIters if int(self.params.robustCostParams.costType) != 0 else 0
            self.solver.iterate_async(rounds, refresh_local=True, gnc_every=gnc)
            self.round_index += rounds
            return
        for _ in range(rounds):
            self.step(with_stats=False)

    def iterate_of(self, robot: int) -> np.ndarray:
        return self.solver.get_iterate(robot)
