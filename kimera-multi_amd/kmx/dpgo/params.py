"""dpgo parameter structs (PGOAgentParameters, ROptParameters,
RobustCostParameters) as dataclasses, convertible to the C ABI struct.

Defaults follow dpgo as recalled in SURVEY.md §9.2 ([U] items: r = 5,
GNC mu0 = 1e-5, mu step = 1.4, c-bar = 5; RTR initial radius 100; tCG kappa
0.1 / theta 1) and SURVEY.md §8d for the benchmark (1 RTR iteration with at
most 10 tCG steps per block update, GNC weight update every 20 rounds).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import IntEnum

from ..abi import KMX_COST_GNC_TLS, KMX_COST_L2, PgoParams


class RobustCostType(IntEnum):
    L2 = KMX_COST_L2
    GNC_TLS = KMX_COST_GNC_TLS


def error_threshold_at_quantile(quantile: float, dimension: int = 3) -> float:
    """c-bar = sqrt(chi2inv(quantile, dof)) with dof = d(d+1)/2 (the SE(d)
    residual's degrees of freedom); the dpgo_ros GNC_quantile parameter."""
    from scipy.stats import chi2
    dof = dimension * (dimension + 1) // 2
    return math.sqrt(float(chi2.ppf(quantile, dof)))


@dataclass
class RobustCostParameters:
    costType: RobustCostType = RobustCostType.GNC_TLS
    GNCBarc: float = 5.0
    GNCMuStep: float = 1.4
    GNCInitMu: float = 1e-5


class ROptMethod(IntEnum):
    RTR = 0
    RGD = 1


@dataclass
class ROptParameters:
    method: ROptMethod = ROptMethod.RTR     # dpgo ROptParameters::method
    RGD_stepsize: float = 1e-3              # [U] dpgo default
    RTR_iterations: int = 1
    RTR_tCG_iterations: int = 10
    RTR_initial_radius: float = 100.0
    RTR_max_radius: float = 1e4
    RTR_accept_rho: float = 0.1
    tCG_kappa: float = 0.1
    tCG_theta: float = 1.0
    gradnorm_tol: float = 1e-2
    use_preconditioner: bool = True
    precond_shift: float = 1e-1
    # kmx opt-in: "standard" (ROPTLIB's tCG) or "onesync" (one reduction and
    # one kernel per tCG step, KMX_TCG_FORM_ONESYNC; parity at convergence only)
    tCG_form: str = "standard"


@dataclass
class PGOAgentParameters:
    d: int = 3
    r: int = 5
    num_robots: int = 1
    localOptimizationParams: ROptParameters = field(default_factory=ROptParameters)
    robustCostParams: RobustCostParameters = field(default_factory=RobustCostParameters)
    maxNumIters: int = 1000
    relChangeTol: float = 1e-3
    robustOptInnerIters: int = 20          # rounds between GNC weight updates
    robustOptNumWeightUpdates: int = 50    # after this many updates weights freeze
    # shouldTerminate's "GNC done" gate (RBCDDriver.should_terminate) [U: a
    # restated substitute for dpgo's rule, which is not vendored; drawio:2030
    # shows only iteration_number() > maxNumIters]: a robust run stops on
    # relChangeTol only once this fraction of the loop-closure weights sits
    # within 1e-8 of 0 or 1 (team-wide) or robustOptNumWeightUpdates ran.
    # 0 restores the plain relChangeTol / maxNumIters stop.
    robustOptMinConvergenceRatio: float = 0.8
    schedule: int = 1                      # 0 sequential (dpgo_ros sync), 1 concurrent
    updateRule: int = 0                    # sequential: 0 round-robin, 1 uniform (dpgo_ros update rule)
    randomSeed: int = 0                    # seed of the uniform rule's std::mt19937 (dpgo_ros random_seed)
    acceleration: bool = False             # Nesterov-accelerated RBCD (dpgo acceleration; concurrent schedule)
    restartInterval: int = 30              # acceleration restart period in rounds (dpgo restartInterval [U])
    tileIncidences: int = 0                # kmx: incidences per workgroup tile (0: from the handle's problem)
    localInitializationMethod: str = "odometry"  # dpgo local initialisation: "odometry" or "chordal" [U default]

    def to_c(self) -> PgoParams:
        lo, rc = self.localOptimizationParams, self.robustCostParams
        p = PgoParams()
        p.d, p.r = self.d, self.r
        p.rtr_iterations = lo.RTR_iterations
        p.tcg_max_iterations = lo.RTR_tCG_iterations
        p.tcg_kappa, p.tcg_theta = lo.tCG_kappa, lo.tCG_theta
        p.rtr_initial_radius, p.rtr_max_radius = lo.RTR_initial_radius, lo.RTR_max_radius
        p.rtr_accept_rho, p.gradnorm_tol = lo.RTR_accept_rho, lo.gradnorm_tol
        p.use_preconditioner = 1 if lo.use_preconditioner else 0
        p.precond_shift = lo.precond_shift
        p.robust_cost = int(rc.costType)
        p.gnc_barc, p.gnc_mu_init, p.gnc_mu_step = rc.GNCBarc, rc.GNCInitMu, rc.GNCMuStep
        p.method = int(lo.method)
        p.rgd_stepsize = float(lo.RGD_stepsize)
        p.acceleration = 1 if self.acceleration else 0
        p.restart_interval = int(self.restartInterval)
        p.tile_incidences = int(self.tileIncidences)
        forms = {"standard": 0, "onesync": 1}
        if lo.tCG_form not in forms:
            raise ValueError(f"tCG_form must be one of {sorted(forms)}, got {lo.tCG_form!r}")
        p.tcg_form = forms[lo.tCG_form]
        return p
