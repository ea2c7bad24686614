"""configs[4] end to end on MI355X: the HIP LCD + RBCD pipeline equals the
same pipeline run on the CPU restatement (accepted loop-closure set bit-exact,
so the team graph and initialisation are identical; final trajectory error
within 1e-6 m)."""
import pytest

from kmx import pipeline as PL
from kmx.synth import make_pose_graph

pytestmark = pytest.mark.gpu


def _setup():
    from kmx.dpgo.params import PGOAgentParameters
    g0 = make_pose_graph(3, 3000, 12000, f_inter=0.0, outlier_scope="robot", seed=4)
    st = PL.make_lc_stream(g0, 60, 30, n_feats=200, seed=2)
    P = PGOAgentParameters(r=5)
    P.robustOptInnerIters = 10
    P.schedule = 1
    return g0, st, P


@pytest.mark.timeout(300)
def test_pipeline_gpu_matches_oracle(gpu):
    from kmx.lcd import LcdParams
    from tests.mock_solver import OracleBlockSolver
    from tests.test_pipeline_cpu import _oracle_verifier
    g0, st, P = _setup()
    gpu_out = PL.run_pipeline(g0, st, P, LcdParams(), rounds=40, device=0)
    cpu_out = PL.run_pipeline(g0, st, P, LcdParams(), rounds=40, verifier=_oracle_verifier(st),
                              solver=OracleBlockSolver(P))
    for k in ("verified", "accepted", "true_positives"):
        assert gpu_out["lcd"][k] == cpu_out["lcd"][k], k
    assert gpu_out["init"]["ate_m"] == cpu_out["init"]["ate_m"]
    assert abs(gpu_out["dpgo"]["ate_m"] - cpu_out["dpgo"]["ate_m"]) < 1e-6
    assert gpu_out["dpgo"]["ate_m"] < gpu_out["init"]["ate_m"]
    assert gpu_out["dpgo"]["edges_iters_per_s"] > 0
