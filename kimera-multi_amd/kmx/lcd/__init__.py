from .detector import LcdParams, LoopClosureDetector, VLCFrame  # noqa: F401
from .bow import BowDatabase, BowDetector  # noqa: F401
