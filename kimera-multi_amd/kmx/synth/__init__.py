from .pose_graph import PoseGraphData, make_pose_graph, lifting_matrix, lift, config  # noqa: F401
