"""Callers either side of the dpgo path: Kimera-Distributed's submap
coarsening and the pose_graph_tools PoseGraph message."""
from .submaps import (PoseGraph, PoseGraphEdge, PoseGraphNode, SubmapAtlas, graph_data,  # noqa: F401
                      measurements_from_pose_graph, pose_graph_from_measurements)
