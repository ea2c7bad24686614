from .detector import LcdParams, LoopClosureDetector  # noqa: F401
from .bow import BowDatabase, BowDetector  # noqa: F401
