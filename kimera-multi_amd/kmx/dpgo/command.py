"""The dpgo_ros command channel's failure handling: the leader's timeout check
and the TERMINATE / HARD_TERMINATE / RECOVER transitions.

Reference (drawio:2417-2451; dpgo_ros is not vendored, so the exact ROS
parameter names and defaults are [U]):

  checkTimeout()   when now - mLastCommandTime > timeoutThreshold:
                     HARD_TERMINATE -> reset(); publishHardTerminateCommand()
                       if 1) numActiveRobots() == 0, or 2) !enableRecovery, or
                          3) state != INITIALIZED || iteration_number() == 0, or
                          4) now - mLastUpdateTime > 3 * timeoutThreshold
                     otherwise (enableRecovery)
                     RECOVER -> publishRecoverCommand()          (drawio:2425, 2448)
  RECOVER          "1 reset iteration number", updateActiveRobots(msg),
                   publishUpdateCommand()                        (drawio:2472-2481)

TimeoutMonitor is the decision alone (clock-agnostic: the caller passes
`now`); RBCDDriver.handle_command / check_timeout apply it to the device state.
"""
from __future__ import annotations

from dataclasses import dataclass

from .messages import CommandType, PGOAgentState


@dataclass
class TimeoutParameters:
    timeoutThreshold: float = 15.0   # seconds without a command before checkTimeout acts [U default]
    enableRecovery: bool = True      # RECOVER instead of HARD_TERMINATE when the team can resume [U default]


class TimeoutMonitor:
    """mLastCommandTime / mLastUpdateTime bookkeeping and the checkTimeout rule."""

    def __init__(self, params: TimeoutParameters | None = None, now: float = 0.0):
        self.params = params if params is not None else TimeoutParameters()
        self.last_command = float(now)
        self.last_update = float(now)

    def note_command(self, now: float):
        self.last_command = float(now)

    def note_update(self, now: float):
        self.last_update = float(now)

    def check(self, now: float, state: PGOAgentState, iteration: int, n_active: int) -> CommandType | None:
        """None while commands keep arriving; otherwise the command checkTimeout
        publishes (drawio:2417 conditions 1-4 -> HARD_TERMINATE, else RECOVER)."""
        thr = self.params.timeoutThreshold
        if now - self.last_command <= thr:
            return None
        if (n_active == 0 or not self.params.enableRecovery
                or state != PGOAgentState.INITIALIZED or iteration == 0
                or now - self.last_update > 3.0 * thr):
            return CommandType.HARD_TERMINATE
        return CommandType.RECOVER
