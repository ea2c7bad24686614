"""File formats either side of the hot path: TUM
trajectories, the loop-closure / keyframe CSV logs read by the reference's
evaluation scripts, and g2o pose graphs as an input format."""
from .formats import (DpgoIterationLog, LoopClosureRecord, lcd_status_name, quat_to_rot, read_dpgo_log,  # noqa: F401
                      read_g2o, read_loop_closures_csv, read_tum, rot_to_quat, write_g2o, write_keyframes_csv,
                      write_lcd_logs, write_loop_closures_csv, write_tum)
