"""fu — MI355X-native Flow Updating engine (drop-in for the SimGrid actor scripts of
AvilaAndre/simgrid-flow-updating-implementation).

Host side in Python, compute in libfu.so (hand-written HIP for gfx950, C ABI in
include/fu.h) loaded with ctypes. There is no CPU fallback: importing this package fails
if libfu.so has not been built.
"""
from ._lib import FuError, copy_bandwidth, device_count, mem_info  # noqa: F401
from .engine import CollectAll, Replay, Trace  # noqa: F401
from .graph import Graph, component_means, uniform_values  # noqa: F401
from .platform import load_deployment, load_platform  # noqa: F401
from .sim import CollectAllPeer, Engine, PairwisePeer, run_reference_main  # noqa: F401

__all__ = ["FuError", "copy_bandwidth", "device_count", "mem_info", "CollectAll", "Replay", "Trace", "Graph",
           "component_means", "uniform_values", "load_deployment", "load_platform",
           "CollectAllPeer", "PairwisePeer", "Engine", "run_reference_main"]
