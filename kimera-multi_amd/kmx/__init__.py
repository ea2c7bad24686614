"""kmx — MI355X-native drop-in for Kimera-Multi's dpgo + LCD verification hot path.

Subpackages:
  kmx.dpgo   PGOAgent / PGOAgentParameters / RBCD driver (dpgo + dpgo_ros API)
  kmx.lcd    LoopClosureDetector verification (Kimera-Multi-LCD API)
  kmx.synth  seeded synthetic workloads of the BASELINE.json configs
The compute path is libkmx.so (HIP, gfx950) through kmx.abi; no CPU fallback.
"""
__version__ = "0.1.0"
