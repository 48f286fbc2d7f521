"""mqhip -- MI355X-native 2D->3D macaque pose hot path (ViTPose-H top-down + anipose lift).

Host side of libmq_hip.so (include/mq_hip.h).  See DESIGN.md at the repo root.
"""
__version__ = "0.1.0"
