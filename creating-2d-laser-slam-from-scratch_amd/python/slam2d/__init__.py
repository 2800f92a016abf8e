"""slam2d: MI355X-native Hector scan-matching + occupancy-grid hot path (and the GMapping particle
grid path) of tonglf/Creating-2D-laser-slam-from-scratch, behind the C-ABI in include/slam2d/*.h.

Import is cheap; the HIP library is loaded on first use (slam2d._lib.lib()).
"""
from ._lib import LIB_PATH, Slam2dError, build, lib  # noqa: F401

__all__ = ["LIB_PATH", "Slam2dError", "build", "lib"]
