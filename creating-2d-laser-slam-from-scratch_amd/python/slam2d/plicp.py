"""PL-ICP scan matching over the MI355X C-ABI (include/slam2d/plicp.h).

Reference: lesson3's ScanMatchPLICP (lesson3/src/plicp_odometry.cc) -- LaserScanToLDP (:285-322)
and CSM `sm_icp` (:391) with the node's parameters (:58-186).  `PLICP.icp` mirrors one sm_icp call;
`PLICP.icp_batch_device` runs many independent scan pairs in one launch.  CSM is absent from the
image: the results are checked against oracle/plicp_oracle.c (parity unpinned against CSM).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import Slam2dError


class PlParams(C.Structure):
    _fields_ = [("max_angular_correction_deg", C.c_double), ("max_linear_correction", C.c_double),
                ("epsilon_xy", C.c_double), ("epsilon_theta", C.c_double),
                ("max_correspondence_dist", C.c_double), ("outliers_maxPerc", C.c_double),
                ("outliers_adaptive_order", C.c_double), ("outliers_adaptive_mult", C.c_double),
                ("max_iterations", C.c_int), ("use_point_to_line_distance", C.c_int),
                ("outliers_remove_doubles", C.c_int), ("pad_", C.c_int)]


class PlResult(C.Structure):
    _fields_ = [("x", C.c_double * 3), ("error", C.c_double), ("valid", C.c_int), ("iterations", C.c_int),
                ("nvalid", C.c_int), ("pad_", C.c_int)]


def _declare(L):
    if getattr(L, "_pl_declared", False):
        return
    L.pl_version.restype = C.c_char_p
    L.pl_last_error.restype = C.c_char_p
    L.pl_default_params.argtypes = [C.POINTER(PlParams)]
    L.pl_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.POINTER(PlParams)]
    L.pl_destroy.argtypes = [C.c_void_p]
    L.pl_icp.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.POINTER(PlResult)]
    L.pl_icp_batch_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.pl_set_timing.argtypes = [C.c_void_p, C.c_int]
    L.pl_get_kernel_times.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L._pl_declared = True


def default_params() -> PlParams:
    L = _lib.lib()
    _declare(L)
    p = PlParams()
    L.pl_default_params(C.byref(p))
    return p


def laser_scan_to_readings(ranges, range_min, range_max) -> np.ndarray:
    """LaserScanToLDP (lesson3/src/plicp_odometry.cc:292-305): r if range_min < r < range_max else -1."""
    r = np.asarray(ranges, np.float64)
    return np.where((r > range_min) & (r < range_max), r, -1.0)


class PLICP:
    def __init__(self, max_pairs: int = 1, max_rays: int = 1081, params: PlParams | None = None):
        self.L = _lib.lib()
        _declare(self.L)
        self.h = C.c_void_p()
        self.params = params or default_params()
        self._check(self.L.pl_create(C.byref(self.h), max_pairs, max_rays, C.byref(self.params)), "pl_create")

    def _check(self, rc, what):
        if rc != 0:
            raise Slam2dError(f"{what} failed with code {rc}: {self.L.pl_last_error().decode(errors='replace')}")

    def close(self):
        if self.h:
            self.L.pl_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def icp(self, ref, sens, angle_min, angle_inc, first_guess=(0.0, 0.0, 0.0)) -> dict:
        """One sm_icp call (lesson3/src/plicp_odometry.cc:391)."""
        ref = np.ascontiguousarray(ref, np.float64)
        sens = np.ascontiguousarray(sens, np.float64)
        g = np.ascontiguousarray(first_guess, np.float64)
        r = PlResult()
        self._check(self.L.pl_icp(self.h, ref.shape[0], float(angle_min), float(angle_inc),
                                  ref.ctypes.data_as(C.c_void_p), sens.ctypes.data_as(C.c_void_p),
                                  g.ctypes.data_as(C.c_void_p), C.byref(r)), "pl_icp")
        return dict(x=np.array(r.x[:]), valid=bool(r.valid), iterations=r.iterations, nvalid=r.nvalid, error=r.error)

    def icp_batch_device(self, count, n, angle_min, angle_inc, d_ref, d_sens, d_guess, d_results, hip_stream=0):
        self._check(self.L.pl_icp_batch_device(self.h, count, n, float(angle_min), float(angle_inc),
                                               C.c_void_p(d_ref), C.c_void_p(d_sens), C.c_void_p(d_guess or None),
                                               C.c_void_p(d_results), C.c_void_p(hip_stream or None)),
                    "pl_icp_batch_device")

    def set_timing(self, on: bool):
        self._check(self.L.pl_set_timing(self.h, 1 if on else 0), "pl_set_timing")

    def kernel_times(self, reset=True):
        ms = C.c_double()
        n = C.c_int64()
        self._check(self.L.pl_get_kernel_times(self.h, C.byref(ms), C.byref(n), 1 if reset else 0), "pl_get_kernel_times")
        return ms.value, n.value
