"""RBCDDriver — the dpgo_ros synchronous scheduler on MI355X.

Reference control flow (drawio:1954-2066, 2071, 2466-2481):
  * every round the executing robots run PGOAgent::iterate(doOptimization)
    against the neighbour poses they last received (publishPublicPoses ->
    updateNeighborPoses, drawio:2340-2355);
  * the leader sends UPDATE_WEIGHT when shouldUpdateMeasurementWeights holds
    (drawio:2466-2469: more than robustOptInnerIters rounds since the last
    update, or every agent converged; at most robustOptNumWeightUpdates
    updates) and every agent runs updateMeasurementWeights (drawio:2212-2215);
  * schedule: dpgo_ros lets ONE robot iterate per round (``sequential``,
    drawio:2478-2481; the leader picks it round-robin or uniformly at random,
    kmx.dpgo.schedule.ExecutingRobot); the MI355X layout updates every block
    each round (``concurrent``, SURVEY.md §0 finding 6, §8e);
  * the leader terminates the team once every agent is ready or maxNumIters
    rounds ran (shouldTerminate, drawio:2027-2030).

Placement: robot blocks are dealt to ranks in contiguous ranges (one process
per GPU). ROS topics become collectives over RCCL/xGMI:
  public_poses + status -> ONE all_to_all per round carrying, to every peer,
                           only the public-pose rows its shared loop closures
                           reference, plus this rank's status word (its largest
                           relative change) at the end of every segment
  measurement_weights   -> none: both ranks of a shared loop closure evaluate
                           its GNC weight from the same two rows on the device
                           (bitwise the owner's value, drawio:2195-2198)
  lifting_matrix/anchor -> injected at initialisation (identical on all ranks)
  UPDATE_WEIGHT         -> decided on the device at the start of each round
                           from the schedule state and the team status
  TERMINATE             -> all_reduce(MAX) of the ranks' largest relative change
  commands / timeout    -> handle_command applies the dpgo_ros command set on
                           every rank (TERMINATE, HARD_TERMINATE = reset,
                           RECOVER, SET_ACTIVE_ROBOTS, UPDATE, UPDATE_WEIGHT,
                           INITIALIZE, NOOP); check_timeout is the leader's
                           checkTimeout (kmx.dpgo.command), rank 0's decision
                           broadcast so every rank applies the same command
"""
from __future__ import annotations

import os
import time

import numpy as np

from .command import TimeoutMonitor, TimeoutParameters
from .messages import Command, CommandType, PGOAgentState
from .params import PGOAgentParameters
from .schedule import ExecutingRobot
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


TILES_TARGET = 736  # csrc/pgo.hip: the tile count the cut of small problems aims at


def team_tile_incidences(graph, world: int, r: int) -> int:
    """The tile cut (incidences per workgroup tile) kmx_pgo_set_graph picks
    automatically for a handle holding 1/world of the team's incidences; the
    multi-rank driver passes it to every rank, so all ranks cut their robots
    alike whatever their share (csrc/pgo.hip set_graph)."""
    tp = 4 * (64 // r)
    inc = 2 * int(graph.m) // max(world, 1)
    return min(2 * tp * r, max(180, -(-inc // TILES_TARGET)))


class RBCDDriver:
    def __init__(self, params: PGOAgentParameters, graph, *, rank: int = 0, world: int = 1,
                 device: int = 0, solver=None, exchange_device: str | None = None, log_dir: str | None = None,
                 timeout: TimeoutParameters | None = None):
        """`solver` defaults to a BlockSolver on HIP device `device`; any object
        with the same interface can be injected (the CPU gloo tests inject the
        restatement). `exchange_device` is where the collective runs ("cuda"
        for RCCL, "cpu" for gloo). A GPU solver under gloo packs into device
        buffers and stages them through host copies (N ranks on one GPU).
        `log_dir`: write dpgo_log_<robot>.csv for the robots of this rank
        (one row per round in which the robot updated, kmx.io.DpgoIterationLog).
        `timeout`: the checkTimeout parameters (kmx.dpgo.command)."""
        if world > graph.n_robots:
            raise ValueError("need at least one robot block per rank")
        self.params = params
        self.graph = graph
        self.rank, self.world = rank, world
        lo, hi = robot_ranges(graph.n_robots, world)[rank]
        self.robots = list(range(lo, hi))
        local = np.zeros(graph.n_robots, np.uint8)
        local[lo:hi] = 1
        self.local = local
        if solver is None and world > 1 and params.tileIncidences == 0:
            import dataclasses
            params = dataclasses.replace(params, tileIncidences=team_tile_incidences(
                graph, world, params.r))
            self.params = params
        self.solver = solver if solver is not None else BlockSolver(params, device)
        self.executing = ExecutingRobot(params.updateRule, params.randomSeed)
        self.round_index = 0
        self._torch = None
        self._xdev = exchange_device
        self.native = False  # RCCL exchange inside the solver's rounds (_setup_native)
        self._native_verified = True
        self.exchange_mode = "none (one rank)" if world == 1 else ""
        if world > 1:
            import torch
            import torch.distributed as dist
            self._torch, self._dist = torch, dist
            if self._xdev is None:
                self._xdev = "cuda" if dist.get_backend() == "nccl" else "cpu"
            if getattr(self.solver, "device_pointers", False):  # order kmx work with torch's copies
                self.solver.set_stream(torch.cuda.current_stream().cuda_stream)
        self.solver.set_graph_data(graph, local)
        P = params
        self.solver.set_gnc_schedule(int(P.robustCostParams.costType) != 0, P.robustOptInnerIters,
                                     P.robustOptNumWeightUpdates, P.relChangeTol)
        self.n_pub, self.first_owned, self.n_owned = self.solver.public_count()
        self.m_local = {a: self.solver.local_edges(a) for a in self.robots}
        self.exchange_rows = (0, 0)  # (rows sent, rows received) per round
        if world > 1:
            self._setup_exchange()
        self.logs = {}
        if log_dir is not None:
            from ..io import DpgoIterationLog
            self.logs = {a: DpgoIterationLog(log_dir, a) for a in self.robots}
        # the command channel's state (dpgo_ros PGOAgentROS; kmx.dpgo.command)
        self.state = PGOAgentState.WAIT_FOR_INITIALIZATION  # the graph is bound at construction
        self.instance = 0
        self.terminated = False
        self.active_robots = set(range(graph.n_robots))
        self.monitor = TimeoutMonitor(timeout, now=time.monotonic())
        self._X0 = None
        self._pub_fresh = False  # owned public rows current (see exchange_public)

    # ------------------------------------------------------ collectives ---
    def _setup_exchange(self):
        torch = self._torch
        ps = 4 * self.params.r
        on_gpu = bool(getattr(self.solver, "device_pointers", False))
        self._stage = on_gpu and self._xdev != "cuda"
        dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
        send_slots, send_counts, recv_slots, recv_counts = exchange_plan(self.graph, self.world, self.rank)
        self._n_send, self._n_recv = int(send_slots.shape[0]), int(recv_slots.shape[0])
        # one status double closes every per-peer segment
        self._send_splits = [int(c) * ps + 1 for c in send_counts]
        self._recv_splits = [int(c) * ps + 1 for c in recv_counts]
        one = np.zeros(1, np.int32)
        self._sslots = torch.as_tensor(send_slots.astype(np.int32) if self._n_send else one, device=dev)
        self._rslots = torch.as_tensor(recv_slots.astype(np.int32) if self._n_recv else one, device=dev)
        self._sseg = torch.as_tensor(np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int32), device=dev)
        self._rseg = torch.as_tensor(np.concatenate([[0], np.cumsum(recv_counts)]).astype(np.int32), device=dev)
        self._sbuf = torch.zeros(sum(self._send_splits), dtype=torch.float64, device=dev)
        self._rbuf = torch.zeros(sum(self._recv_splits), dtype=torch.float64, device=dev)
        self.exchange_rows = (self._n_send, self._n_recv)
        # RCCL inside the round (kmx_pgo_comm_init / kmx_pgo_set_exchange): the
        # exchange runs on the solver's stream, enqueued by the same C call as
        # the round, so a batch of rounds is one host call with no Python or
        # cross-stream hop between exchange and round. KMX_NATIVE_XCHG=0 keeps
        # the torch.distributed all_to_all of exchange_public.
        self._plan = (send_slots, send_counts, recv_slots, recv_counts)
        self.native = self._setup_native()
        self._native_verified = not self.native

    def _agree(self, ok: bool) -> bool:
        """True on every rank iff ok on every rank (one MIN all-reduce)."""
        t = self._torch.tensor([1 if ok else 0], dtype=self._torch.int32,
                               device="cuda" if self._dist.get_backend() == "nccl" else "cpu")
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MIN)
        return bool(t.item())

    def _setup_native(self) -> bool:
        """The in-round RCCL exchange, set up in steps every rank passes
        together, so a failure on one rank never leaves its peers waiting in a
        collective or a rendezvous:
          1. local checks (solver capable, backend nccl, not disabled); rank 0
             creates the unique id; the id slot is broadcast ALWAYS (None when
             rank 0 failed), then one MIN all-reduce agrees on going ahead;
          2. every rank creates its communicator non-blocking with a deadline
             (kmx_pgo_comm_init), then one MIN all-reduce agrees on success;
             on any failure every rank drops its communicator;
          3. at the first round the native exchange is checked bit for bit
             against the torch.distributed all_to_all (_verify_native).
        self.exchange_mode says which exchange runs and why."""
        self.exchange_mode = "torch.distributed all_to_all_single"
        capable = (self._xdev == "cuda" and bool(getattr(self.solver, "native_exchange", False))
                   and os.environ.get("KMX_NATIVE_XCHG", "1") != "0")
        uid = None
        if self.rank == 0 and capable:
            try:
                uid = self.solver.comm_unique_id()
            except Exception as e:  # noqa: BLE001 - reported, then every rank falls back
                self._native_error = f"rank 0 unique id: {e}"
        box = [uid]
        self._dist.broadcast_object_list(box, src=0)  # always, so every rank stays in step
        if not self._agree(capable and box[0] is not None):
            if capable:
                self.exchange_mode += " (fallback: the RCCL exchange could not start on every rank)"
            return False
        ok = True
        try:
            self.solver.comm_init(box[0], self.world, self.rank,
                                  float(os.environ.get("KMX_COMM_TIMEOUT", "120")))
        except Exception as e:  # noqa: BLE001
            import warnings
            warnings.warn(f"native RCCL exchange unavailable on rank {self.rank} ({e})")
            ok = False
        if not self._agree(ok):
            if ok:
                self._destroy_comm()
            self.exchange_mode += " (fallback: a rank could not create its RCCL communicator)"
            return False
        self.solver.set_exchange(*self._plan)
        self.exchange_mode = "RCCL ncclSend/ncclRecv group inside each round (solver stream)"
        info = getattr(self.solver, "runtime_info", None)
        refuse = None
        if info is not None:
            # torch bundles a librccl of the same SONAME as the one kmx links: one
            # copy must serve both, or kmx's communicator runs on a different RCCL
            # (and HIP runtime) than torch's process group
            ri = info()
            self.runtime = ri
            self.exchange_mode += f" [kmx RCCL {ri.get('rccl_version')} at {ri.get('rccl_path_real')}]"
            if not ri.get("single_rccl", True):
                self.exchange_mode += f" (WARNING: {len(ri.get('mapped_rccl', []))} RCCL copies mapped)"
                if os.environ.get("KMX_REQUIRE_NATIVE", "0") == "1":
                    refuse = ("KMX_REQUIRE_NATIVE=1: libkmx's RCCL symbols resolve to "
                              f"{ri.get('rccl_path_real')} but the process maps {ri.get('mapped_rccl')}")
        # the refusal is agreed, so every rank raises together (a per-rank raise
        # would leave the peers waiting in their first exchange)
        if not self._agree(refuse is None):
            self._destroy_comm()
            raise RuntimeError(refuse or "KMX_REQUIRE_NATIVE=1: a peer rank maps more than one RCCL copy")
        return True

    def _destroy_comm(self):
        """Abort the native communicator; an error from it (a stream already in
        error, a timeout) is recorded, never raised, so the caller still reaches
        the agreement its peers wait in."""
        try:
            self.solver.comm_destroy()
        except Exception as e:  # noqa: BLE001 - reported through exchange_mode
            prev = getattr(self, "_native_error", None)
            msg = f"comm_destroy on rank {self.rank}: {type(e).__name__}: {e}"
            self._native_error = f"{prev}; {msg}" if prev else msg

    def _torch_exchange(self):
        s = self.solver
        s.exchange_pack(self._sslots.data_ptr(), self._n_send, self._sseg.data_ptr(), self.world,
                        self._sbuf.data_ptr())
        self._all_to_all(self._rbuf, self._sbuf)
        s.exchange_unpack(self._rslots.data_ptr(), self._n_recv, self._rseg.data_ptr(), self.world,
                          self._rbuf.data_ptr())

    def _verify_native(self):
        """First round only: the in-round RCCL exchange and the torch.distributed
        all_to_all must install the same public table and peer statuses bit for
        bit; otherwise every rank drops the native exchange (exchange_mode says
        so). KMX_REQUIRE_NATIVE=1 makes a mismatch or fallback an error."""
        if self._native_verified:
            return
        self._native_verified = True
        s = self.solver
        alive = True
        # Bounded: a rank whose exchange raises after its peers have posted
        # their ncclSend / ncclRecv leaves those peers waiting on the stream;
        # they wait at most KMX_XCHG_TIMEOUT s (kmx_pgo_sync_timeout), then
        # abort their communicator (kmx_pgo_comm_destroy), which releases the
        # stream, and every rank reaches the agreement below.
        deadline = float(os.environ.get("KMX_XCHG_TIMEOUT", "60"))
        try:  # an error here must still reach the agreement below on every rank
            s.exchange()
            if hasattr(s, "sync_timeout") and not s.sync_timeout(deadline):
                raise TimeoutError(f"the first native exchange did not complete within {deadline:g} s")
            tab_n, ext_n = s.get_public(self.world)
        except Exception as e:  # noqa: BLE001 - reported through exchange_mode
            tab_n = ext_n = None
            self._native_error = f"first native exchange on rank {self.rank}: {type(e).__name__}: {e}"
            self._destroy_comm()  # abort: the stream drains even if a peer's half never comes
            alive = False
        self._torch_exchange()
        tab_t, ext_t = s.get_public(self.world)
        same = tab_n is not None and np.array_equal(tab_n, tab_t) and np.array_equal(ext_n, ext_t)
        if self._agree(same):
            self.exchange_mode += ", checked bitwise against all_to_all at the first round"
            return
        errs = [None] * self.world
        self._dist.all_gather_object(errs, getattr(self, "_native_error", None))
        if alive:
            self._destroy_comm()
        self.native = False
        failed = [e for e in errs if e]
        if failed:  # an exception (a timeout included) is not a bitwise mismatch: say which
            self.exchange_mode = ("torch.distributed all_to_all_single (fallback: the RCCL exchange failed: "
                                  + "; ".join(failed) + ")")
        else:
            self.exchange_mode = "torch.distributed all_to_all_single (fallback: the RCCL exchange differed from it)"
        if os.environ.get("KMX_REQUIRE_NATIVE", "0") == "1":
            raise RuntimeError(self.exchange_mode)

    def _all_to_all(self, out, inp):
        """One all-to-all with per-peer sizes (RCCL directly; a GPU solver under
        gloo stages through host copies)."""
        if self._stage:
            self.solver.sync()
            ho, hi = out.cpu(), inp.cpu()
            self._dist.all_to_all_single(ho, hi, self._recv_splits, self._send_splits)
            out.copy_(ho)
        else:
            self._dist.all_to_all_single(out, inp, self._recv_splits, self._send_splits)

    def _refresh_owned(self):
        if not (self._pub_fresh and getattr(self.solver, "publishes_on_commit", False)):
            self.solver.refresh_local()  # the owned slots of the table
            self._pub_fresh = True

    def exchange_public(self):
        """publishPublicPoses -> updateNeighborPoses (+ publishStatus) for the
        whole team."""
        self._refresh_owned()
        if self.world == 1:
            return
        if self.native:  # every round starts with it; this is an extra one (UPDATE_WEIGHT)
            self._verify_native()
            if self.native:
                self.solver.exchange()
                return
        self._torch_exchange()

    def update_weights(self) -> float:
        """An explicit UPDATE_WEIGHT (outside the schedule): fresh neighbour rows,
        then every handle re-weights the loop closures it holds."""
        self.exchange_public()
        return self.solver.update_weights()

    @property
    def weight_updates(self) -> int:
        return int(self.solver.gnc_state()["updates"])

    # ------------------------------------------------------------ rounds ---
    def initialize(self, X_by_robot: dict):
        self._X0 = {a: np.array(X_by_robot[a], dtype=np.float64) for a in self.robots}
        for a in self.robots:
            self.solver.set_iterate(a, self._X0[a])
        self._pub_fresh = False
        self.state = PGOAgentState.INITIALIZED
        self.terminated = False

    def active_mask(self) -> np.ndarray:
        act = np.zeros(self.graph.n_robots, np.uint8)
        if self.params.schedule == 0:  # sequential: the leader picks one executing robot
            act[self.executing.next(sorted(self.active_robots))] = 1
        else:
            act[sorted(self.active_robots)] = 1
        return act

    def _all_active(self) -> bool:
        return len(self.active_robots) == self.graph.n_robots

    def _check_running(self):
        if self.state != PGOAgentState.INITIALIZED:
            raise ValueError("round before initialize (or after HARD_TERMINATE)")
        if self.terminated:
            raise ValueError("round after TERMINATE")

    def step(self, with_stats: bool = True):
        """One synchronous round (its GNC decision runs on the device first).
        Returns per-robot stats (team-indexed) when with_stats."""
        self._check_running()
        if self.native:  # the round starts with the exchange itself
            self._refresh_owned()
            self._verify_native()
        if not self.native:
            self.exchange_public()
        stats = None
        if with_stats or self.params.schedule == 0 or self.logs or not self._all_active():
            act = self.active_mask()
            stats = self.solver.iterate(act)
            if self.logs:
                nbytes = self.exchange_rows[1] * 4 * self.params.r * 8
                for a, log in self.logs.items():
                    if stats[a]["updated"]:
                        log.log_iteration(self.round_index, int(act.sum()), int(self.graph.n_poses[a]), nbytes,
                                          stats[a])
        else:
            self.solver.iterate_async(1, refresh_local=False)
        self.round_index += 1
        return stats

    def run_async(self, rounds: int):
        """Benchmark path: enqueue `rounds` concurrent rounds with no host sync
        (single GPU: one C call; multi-GPU: one all-to-all between rounds)."""
        self._check_running()
        if self.native:
            self._refresh_owned()
            self._verify_native()
        if (self.world == 1 or self.native) and self.params.schedule == 1 and self._all_active():
            self.solver.iterate_async(rounds, refresh_local=True)
            self.round_index += rounds
            return
        for _ in range(rounds):
            self.step(with_stats=False)

    def team_max_rel_change(self) -> float:
        """Largest relative change of the team's last block updates (one
        all_reduce(MAX) of the ranks' status; synchronises)."""
        v = self.solver.status()
        local = float(np.max(v[self.robots])) if self.robots else 0.0
        if self.world == 1:
            return local
        t = self._torch.tensor([local], dtype=self._torch.float64,
                               device="cuda" if self._xdev == "cuda" else "cpu")
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX)
        return float(t.item())

    def _team_sum(self, vals):
        if self.world == 1:
            return [float(v) for v in vals]
        t = self._torch.tensor([float(v) for v in vals], dtype=self._torch.float64,
                               device="cuda" if self._xdev == "cuda" else "cpu")
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu().tolist()]

    def converged_weight_ratio(self) -> float:
        """Fraction of the team's loop closures (non-fixed measurements) whose
        GNC weight has converged to 0 or 1 (dpgo's robust-optimisation
        convergence statistic [U: dpgo not vendored; |w| or |1 - w| <= 1e-8]).
        Each measurement is counted once, on the rank owning its lower robot
        id (drawio:2198). One all_reduce(SUM) when world > 1."""
        g = self.graph
        own = self.local[np.minimum(g.r1, g.r2)] == 1
        lc = own & (np.asarray(g.fixed) == 0)
        n = int(lc.sum())
        conv = 0
        if n:
            w = np.asarray(self.solver.get_weights(), np.float64)[lc]
            conv = int(((np.abs(w) <= 1e-8) | (np.abs(1.0 - w) <= 1e-8)).sum())
        conv_t, n_t = self._team_sum([conv, n])
        return 1.0 if n_t == 0 else conv_t / n_t

    def should_terminate(self) -> bool:
        """shouldTerminate (drawio:2027-2030): maxNumIters rounds ran, or every
        agent's relative change is below relChangeTol — and, for a robust cost,
        GNC is done: robustOptNumWeightUpdates weight updates ran, or at least
        robustOptMinConvergenceRatio of the loop-closure weights converged to
        0 / 1 (dpgo keeps iterating while GNC still moves the weights; an
        agent converged on the current weights is exactly what fires the next
        update, drawio:2466-2469)."""
        P = self.params
        if self.round_index >= P.maxNumIters:
            return True
        if not self.team_max_rel_change() < P.relChangeTol:
            return False
        if int(P.robustCostParams.costType) == 0:  # L2
            return True
        if self.weight_updates >= P.robustOptNumWeightUpdates:
            return True
        return self.converged_weight_ratio() >= P.robustOptMinConvergenceRatio

    def run(self, max_rounds: int | None = None, check_every: int = 10) -> int:
        """Rounds until shouldTerminate (checked every `check_every` rounds and
        at the end); returns the rounds run."""
        limit = self.params.maxNumIters if max_rounds is None else max_rounds
        done = 0
        while done < limit and not self.terminated:
            k = min(check_every, limit - done)
            self.run_async(k)
            done += k
            if self.should_terminate():
                break
        return done

    def iterate_of(self, robot: int) -> np.ndarray:
        return self.solver.get_iterate(robot)

    # ---------------------------------------------------------- commands ---
    def reset(self):
        """PGOAgent::reset as HARD_TERMINATE runs it (drawio:2433-2436): next
        instance, iteration number 0, GNC weights / mu / schedule and the team
        status back to their initial values; the graph stays bound, so the
        team resumes with INITIALIZE (or initialize(X))."""
        P, g = self.params, self.graph
        self.instance += 1
        self.round_index = 0
        self.state = PGOAgentState.WAIT_FOR_INITIALIZATION
        self.terminated = False
        self.active_robots = set(range(g.n_robots))
        self.executing = ExecutingRobot(P.updateRule, P.randomSeed)
        self.solver.set_weights(np.asarray(g.weight, np.float64))
        self.solver.set_gnc_state({"inner_iter": 0, "updates": 0, "mu": P.robustCostParams.GNCInitMu})
        self.solver.set_status(np.where(np.asarray(g.n_poses) > 0, np.inf, 0.0))

    def handle_command(self, cmd: Command, now: float | None = None):
        """commandCallback of dpgo_ros (drawio:2124-2481) on this rank; every
        rank receives the same command. Returns the stats of an UPDATE round
        (None otherwise).
          TERMINATE          stop; the iterate stays readable (drawio:2180)
          HARD_TERMINATE     reset() (drawio:2433-2436)
          RECOVER            iteration number := executing_iteration, active
                             robots := the message's (if it names any), resume
                             (drawio:2448, 2472-2481)
          SET_ACTIVE_ROBOTS  the robots that update in later rounds (drawio:2405)
          UPDATE             one round; executing_robot >= 0 runs that robot
                             alone (drawio:2369, 2478-2481)
          UPDATE_WEIGHT      GNC weight update now (drawio:2212-2215)
          INITIALIZE         re-apply the last initial iterate after a reset
          REQUEST_POSE_GRAPH the graph was bound at construction: no-op
          NOOP               refreshes the command clock only (drawio:2402)"""
        now = time.monotonic() if now is None else float(now)
        self.monitor.note_command(now)
        c = CommandType(cmd.command)
        if c == CommandType.TERMINATE:
            self.terminated = True
        elif c == CommandType.HARD_TERMINATE:
            self.reset()
        elif c == CommandType.RECOVER:
            # the leader's iteration number (check_timeout sends rank 0's), so
            # ranks whose counters drifted resume in step; its robot list is
            # validated as SET_ACTIVE_ROBOTS's
            if cmd.active_robots:
                self.active_robots = self._valid_robots(cmd.active_robots, "RECOVER")
            self.round_index = int(cmd.executing_iteration)
            self.terminated = False
        elif c == CommandType.SET_ACTIVE_ROBOTS:
            self.active_robots = self._valid_robots(cmd.active_robots, "SET_ACTIVE_ROBOTS")
        elif c == CommandType.UPDATE:
            keep = self.active_robots
            if cmd.executing_robot >= 0:
                if cmd.executing_robot not in keep:
                    raise ValueError(f"UPDATE: robot {cmd.executing_robot} is not active")
                self.active_robots = {int(cmd.executing_robot)}
            try:
                st = self.step(with_stats=True)
            finally:
                self.active_robots = keep
            self.monitor.note_update(now)
            return st
        elif c == CommandType.UPDATE_WEIGHT:
            self._check_running()
            self.update_weights()
        elif c == CommandType.INITIALIZE:
            if self.state != PGOAgentState.INITIALIZED:
                if self._X0 is None:
                    raise ValueError("INITIALIZE: no initial iterate; call initialize(X) first")
                self.initialize(self._X0)
        return None

    def _valid_robots(self, robots, what: str) -> set:
        act = {int(a) for a in robots}
        if not act or not act <= set(range(self.graph.n_robots)):
            raise ValueError(f"{what}: robots must be a non-empty subset of the team, got {sorted(act)}")
        return act

    def check_timeout(self, now: float | None = None) -> Command | None:
        """The leader's checkTimeout (kmx.dpgo.command.TimeoutMonitor): rank 0
        decides, every rank applies the same HARD_TERMINATE or RECOVER (one
        broadcast when world > 1). Returns the command applied, or None."""
        now = time.monotonic() if now is None else float(now)
        c = self.monitor.check(now, self.state, self.round_index, len(self.active_robots))
        it = self.round_index
        if self.world > 1:  # the leader's decision and iteration number reach every rank
            t = self._torch.tensor([-1 if c is None else int(c), it], dtype=self._torch.int64,
                                   device="cuda" if self._xdev == "cuda" else "cpu")
            self._dist.broadcast(t, src=0)
            v, it = (int(x) for x in t.cpu().tolist())
            c = None if v < 0 else CommandType(v)
        if c is None:
            return None
        cmd = Command(0, c, executing_iteration=it, active_robots=sorted(self.active_robots))
        self.handle_command(cmd, now)
        return cmd
