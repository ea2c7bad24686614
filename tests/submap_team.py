"""Test helper: a keyframe-level team graph taken through the callers either
side of dpgo: Kimera-Distributed's submap coarsening (f1:
odometry keyframes -> submaps, keyframe loop closures -> submap edges, the
request_pose_graph message round trip) and the distributed initialisation
(f4: each robot's odometry starts in its own frame; robots 1.. are aligned to
robot 0's frame by GNC-TLS robust single-pose averaging over the shared submap
loop closures). Used by tests/test_frontend_submaps.py (restatement solver) and
tests/test_outputs_gpu.py (the HIP solver)."""
import numpy as np

from kmx.dpgo.init import align_to_world, transform_trajectory
from kmx.dpgo.messages import RelativeSEMeasurement
from kmx.frontend import SubmapAtlas, graph_data, measurements_from_pose_graph, pose_graph_from_measurements
from kmx.synth import lift, lifting_matrix, make_pose_graph


def submap_team(seed=5, n_robots=2, n_kf=1600, m=2600, noise_free=False):
    g = make_pose_graph(n_robots, n_kf, m, outlier_frac=0.2, f_inter=0.3, noise_free=noise_free, sigma_R=0.002,
                        sigma_t=0.02, seed=seed)
    atlases = []
    for a in range(n_robots):
        # each robot's VIO odometry in its own frame (first keyframe at the origin)
        R0, t0 = g.init_R[a][0], g.init_t[a][0]
        R_loc = np.einsum("ji,njk->nik", R0, g.init_R[a])
        t_loc = (g.init_t[a] - t0) @ R0
        at = SubmapAtlas(a, max_distance=4.0, max_keyframes=8)
        for k in range(int(g.n_poses[a])):
            at.add_keyframe(k, 1_600_000_000_000_000_000 + 200_000_000 * k, R_loc[k], t_loc[k])
        atlases.append(at)
    ms = []
    for at in atlases:
        ms += at.odometry_edges(1e4, 1e2)
    for e in np.nonzero(g.fixed == 0)[0]:
        m_ = SubmapAtlas.submap_loop_closure(atlases[g.r1[e]], int(g.p1[e]), atlases[g.r2[e]], int(g.p2[e]),
                                             g.R[e], g.t[e], float(g.kappa[e]), float(g.tau[e]))
        if m_ is not None:  # both keyframes in one submap: no submap edge
            ms.append(m_)
    # what dpgo receives: the request_pose_graph reply (pose_graph_tools message)
    ms = measurements_from_pose_graph(pose_graph_from_measurements(ms))
    sg = graph_data(ms, [at.n_submaps for at in atlases])
    # f4: robot 0's frame is the world; the others are aligned to it
    R_sub = [np.array([p[0] for p in at.submap_pose]) for at in atlases]
    t_sub = [np.array([p[1] for p in at.submap_pose]) for at in atlases]
    world = {(0, i): (R_sub[0][i], t_sub[0][i]) for i in range(atlases[0].n_submaps)}
    align = {}
    for a in range(1, n_robots):
        shared = [x for x in ms if x.r1 != x.r2 and a in (x.r1, x.r2) and 0 in (x.r1, x.r2)]
        out = align_to_world(shared, a, R_sub[a], t_sub[a], world)
        assert out is not None
        R_WA, t_WA, w = out
        align[a] = (R_WA, t_WA, w)
        R_sub[a], t_sub[a] = transform_trajectory(R_WA, t_WA, R_sub[a], t_sub[a])
    Y = lifting_matrix(5, seed=1)
    X0 = {a: lift(R_sub[a], t_sub[a], Y) for a in range(n_robots)}
    return g, atlases, sg, X0, align


def planted_alignment(g, a):
    """The frame change that maps robot a's odometry frame to robot 0's:
    T_W0_A = T_0^-1 T_A (both odometry chains anchored at their first pose)."""
    R0, t0 = g.init_R[0][0], g.init_t[0][0]
    Ra, ta = g.init_R[a][0], g.init_t[a][0]
    R = R0.T @ Ra
    t = R0.T @ (ta - t0)
    return R, t
