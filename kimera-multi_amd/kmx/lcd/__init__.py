from .detector import LcdParams, LoopClosureDetector  # noqa: F401
