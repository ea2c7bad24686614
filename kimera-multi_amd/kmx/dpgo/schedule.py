"""dpgo / dpgo_ros scheduling rules shared by the agent API, the driver and
the CPU test stand-ins (the HIP path evaluates the GNC rule on the device,
csrc/pgo.hip gnc_should_update, and is tested against this mirror).

  GncSchedule            PGOAgent::shouldUpdateMeasurementWeights (drawio:2466-2469):
                         never for the L2 cost or after robustOptNumWeightUpdates
                         updates; otherwise when the inner-iteration counter
                         exceeds robustOptInnerIters, or when every agent of the
                         team has converged (relative change of its last block
                         update <= relChangeTol). updateMeasurementWeights resets
                         the counter (drawio:2215); every round (iterate) counts.
  ExecutingRobot         dpgo_ros synchronous mode: the leader designates the next
                         executing robot (publishUpdateCommand, drawio:2478-2481):
                         round-robin over the active robots, or uniformly at
                         random from a seeded std::mt19937 (the distribution is
                         restated per libstdc++ release, SURVEY.md §0 finding 5).
"""
from __future__ import annotations

ROUND_ROBIN = 0
UNIFORM = 1
RNG_GCC9 = 0
RNG_GCC11 = 1


class MT19937:
    """std::mt19937 (the 32-bit Mersenne Twister, default seeding)."""

    def __init__(self, seed: int = 5489):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __call__(self) -> int:
        if self.i >= 624:
            mt = self.mt
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7FFFFFFF)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def uniform_int(gen: MT19937, a: int, b: int, variant: int = RNG_GCC11) -> int:
    """std::uniform_int_distribution<int>(a, b)(gen) with b - a < 2^32 - 1:
    GCC >= 11 downscales by Lemire's nearly divisionless method with a 64-bit
    product (bits/uniform_int_dist.h _S_nd); GCC 9 by rejection with two
    divisions."""
    uerange = (b - a) + 1
    if variant == RNG_GCC11:
        product = gen() * uerange
        low = product & 0xFFFFFFFF
        if low < uerange:
            threshold = ((1 << 32) - uerange) % uerange
            while low < threshold:
                product = gen() * uerange
                low = product & 0xFFFFFFFF
        return a + (product >> 32)
    scaling = 0xFFFFFFFF // uerange
    past = uerange * scaling
    ret = gen()
    while ret >= past:
        ret = gen()
    return a + ret // scaling


class GncSchedule:
    """Host mirror of the GNC schedule (see module doc)."""

    def __init__(self, robust: bool, inner_iters: int, max_updates: int, rel_change_tol: float, mu_init: float,
                 mu_step: float):
        self.robust = bool(robust)
        self.inner_iters = int(inner_iters)
        self.max_updates = int(max_updates)
        self.rel_change_tol = float(rel_change_tol)
        self.mu = float(mu_init)
        self.mu_step = float(mu_step)
        self.inner = 0
        self.updates = 0

    @classmethod
    def from_params(cls, P) -> "GncSchedule":
        rc = P.robustCostParams
        return cls(int(rc.costType) != 0, P.robustOptInnerIters, P.robustOptNumWeightUpdates, P.relChangeTol,
                   rc.GNCInitMu, rc.GNCMuStep)

    def round_done(self):
        self.inner += 1

    def should_update(self, rel_changes) -> bool:
        """rel_changes: the team's statuses (relative change of each agent's last
        block update; inf before its first)."""
        if not self.robust or self.updates >= self.max_updates:
            return False
        if self.inner > self.inner_iters:
            return True
        return all(float(v) <= self.rel_change_tol for v in rel_changes)

    def updated(self) -> float:
        """Book-keeping of one updateMeasurementWeights; returns the mu used."""
        mu = self.mu
        self.inner = 0
        self.updates += 1
        self.mu *= self.mu_step
        return mu


class ExecutingRobot:
    """The leader's choice of the next executing robot (sequential schedule)."""

    def __init__(self, rule: int = ROUND_ROBIN, seed: int = 0, variant: int = RNG_GCC11):
        if rule not in (ROUND_ROBIN, UNIFORM):
            raise ValueError(f"unknown update rule {rule}")
        self.rule = rule
        self.variant = variant
        self.gen = MT19937(seed)
        self.last = -1

    def next(self, active_robots) -> int:
        act = sorted(int(a) for a in active_robots)
        if not act:
            raise ValueError("no active robot")
        if self.rule == ROUND_ROBIN:
            later = [a for a in act if a > self.last]
            self.last = later[0] if later else act[0]
        else:
            self.last = act[uniform_int(self.gen, 0, len(act) - 1, self.variant)]
        return self.last
