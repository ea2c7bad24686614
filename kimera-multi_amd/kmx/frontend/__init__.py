"""Callers either side of the dpgo path: Kimera-Distributed's submap
coarsening and the pose_graph_tools PoseGraph message."""
from .submaps import (PoseGraph, PoseGraphEdge, PoseGraphNode, SubmapAtlas, measurements_from_pose_graph,  # noqa: F401
                      pose_graph_from_measurements)
