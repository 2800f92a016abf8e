"""Karto correlative scan matching over the MI355X C-ABI (include/slam2d/karto.h).

Reference: open_karto's ScanMatcher (lesson6/lib/open_karto/src/Mapper.cpp).  `ScanMatcher.Create`
mirrors ScanMatcher::Create (:126-171) and `ScanMatcher.MatchScan` one MatchScan call (:184-300);
`match_batch_device` runs many independent MatchScan calls (a loop-closure candidate batch) on
pooled scans.  open_karto needs boost and is not built here: results are checked against
oracle/karto_oracle.c (parity unpinned against open_karto itself).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import Slam2dError


class KtLaser(C.Structure):
    """The LaserRangeFinder fields LocalizedRangeScan::Update reads (Karto.h:5362-5404)."""
    _fields_ = [("minimum_angle", C.c_double), ("angular_resolution", C.c_double),
                ("minimum_range", C.c_double), ("range_threshold", C.c_double),
                ("n_readings", C.c_int), ("pad_", C.c_int)]


class KtParams(C.Structure):
    _fields_ = [("search_size", C.c_double), ("resolution", C.c_double), ("smear_deviation", C.c_double),
                ("distance_variance_penalty", C.c_double), ("angle_variance_penalty", C.c_double),
                ("fine_search_angle_offset", C.c_double), ("coarse_search_angle_offset", C.c_double),
                ("coarse_angle_resolution", C.c_double), ("minimum_angle_penalty", C.c_double),
                ("minimum_distance_penalty", C.c_double), ("use_response_expansion", C.c_int),
                ("pad_", C.c_int)]


class KtResult(C.Structure):
    _fields_ = [("mean", C.c_double * 3), ("covariance", C.c_double * 9), ("response", C.c_double),
                ("status", C.c_int), ("pad_", C.c_int)]


RESULT_DTYPE = np.dtype([("mean", np.float64, 3), ("covariance", np.float64, 9), ("response", np.float64),
                         ("status", np.int32), ("pad_", np.int32)])
assert RESULT_DTYPE.itemsize == C.sizeof(KtResult)


def _declare(L):
    if getattr(L, "_kt_declared", False):
        return
    vp, i, d = C.c_void_p, C.c_int, C.c_double
    L.kt_version.restype = C.c_char_p
    L.kt_last_error.restype = C.c_char_p
    L.kt_default_params.argtypes = [C.POINTER(KtParams)]
    L.kt_default_loop_params.argtypes = [C.POINTER(KtParams)]
    L.kt_create.argtypes = [C.POINTER(vp), C.POINTER(KtLaser), C.POINTER(KtParams), i, i, i]
    L.kt_destroy.argtypes = [vp]
    L.kt_get_grid_info.argtypes = [vp, vp]
    L.kt_set_scans.argtypes = [vp, i, i, vp, vp]
    L.kt_set_scans_device.argtypes = [vp, i, i, vp, vp, vp]
    L.kt_match_scan.argtypes = [vp, vp, vp, i, vp, vp, i, i, C.POINTER(KtResult)]
    L.kt_match_batch_device.argtypes = [vp, i, vp, vp, vp, i, i, vp, vp]
    L.kt_window_exchange_words.restype = C.c_size_t
    L.kt_window_exchange_words.argtypes = [vp]
    L.kt_match_sharded_begin_device.argtypes = [vp, i, vp, vp, vp, i, i, i, vp, vp]
    L.kt_match_sharded_end_device.argtypes = [vp, i, vp, vp, i, i, vp, vp, vp]
    L.kt_set_timing.argtypes = [vp, i]
    L.kt_kernel_name.restype = C.c_char_p
    L.kt_kernel_name.argtypes = [i]
    L.kt_get_kernel_times.argtypes = [vp, vp, vp, i]
    L._kt_declared = True


def default_params(loop: bool = False) -> KtParams:
    """Mapper::InitializeParameters defaults (Mapper.cpp:1569-1660)."""
    L = _lib.lib()
    _declare(L)
    p = KtParams()
    (L.kt_default_loop_params if loop else L.kt_default_params)(C.byref(p))
    return p


def laser(n_readings: int, minimum_angle: float, angular_resolution: float, minimum_range: float = 0.0,
          range_threshold: float = 12.0) -> KtLaser:
    return KtLaser(float(minimum_angle), float(angular_resolution), float(minimum_range), float(range_threshold),
                   int(n_readings), 0)


class ScanMatcher:
    """ScanMatcher::Create(mapper, searchSize, resolution, smearDeviation, rangeThreshold) for a batch of
    `max_matches` concurrent matches over a pool of `max_scans` scans."""

    def __init__(self, laser: KtLaser, params: KtParams | None = None, max_matches: int = 1, max_scans: int = 64,
                 max_base: int = 63):
        self.L = _lib.lib()
        _declare(self.L)
        self.laser = laser
        self.params = params or default_params()
        self.h = C.c_void_p()
        self._check(self.L.kt_create(C.byref(self.h), C.byref(laser), C.byref(self.params), max_matches, max_scans,
                                     max_base), "kt_create")
        info = np.zeros(10, np.int32)
        self._check(self.L.kt_get_grid_info(self.h, info.ctypes.data_as(C.c_void_p)), "kt_get_grid_info")
        keys = ["grid_size", "border", "width", "ws", "data_size", "side", "probs_ws", "half", "ksize", "max_poses"]
        self.info = {k: int(v) for k, v in zip(keys, info)}

    @classmethod
    def Create(cls, laser: KtLaser, searchSize: float, resolution: float, smearDeviation: float,
               params: KtParams | None = None, **kw) -> "ScanMatcher":
        p = params or default_params()
        p.search_size, p.resolution, p.smear_deviation = float(searchSize), float(resolution), float(smearDeviation)
        return cls(laser, p, **kw)

    def _check(self, rc, what):
        if rc != 0:
            raise Slam2dError(f"{what} failed with code {rc}: {self.L.kt_last_error().decode(errors='replace')}")

    def close(self):
        if self.h:
            self.L.kt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def MatchScan(self, ranges, pose, base_ranges, base_poses, doPenalize: bool = True,
                  doRefineMatch: bool = True):
        """ScanMatcher::MatchScan (Mapper.cpp:184-300): returns (mean[3], covariance[3,3], response)."""
        n = self.laser.n_readings
        q = np.ascontiguousarray(ranges, np.float64).reshape(n)
        qp = np.ascontiguousarray(pose, np.float64).reshape(3)
        b = np.ascontiguousarray(base_ranges, np.float64).reshape(-1, n)
        bp = np.ascontiguousarray(base_poses, np.float64).reshape(-1, 3)
        r = KtResult()
        self._check(self.L.kt_match_scan(self.h, q.ctypes.data_as(C.c_void_p), qp.ctypes.data_as(C.c_void_p),
                                         b.shape[0], b.ctypes.data_as(C.c_void_p), bp.ctypes.data_as(C.c_void_p),
                                         int(doPenalize), int(doRefineMatch), C.byref(r)), "kt_match_scan")
        if r.status != 0:
            raise Slam2dError(f"MatchScan: status {r.status} (an index the reference throws on)")
        return np.array(r.mean[:]), np.array(r.covariance[:]).reshape(3, 3), r.response

    def set_scans(self, first: int, ranges, poses):
        n = self.laser.n_readings
        r = np.ascontiguousarray(ranges, np.float64).reshape(-1, n)
        p = np.ascontiguousarray(poses, np.float64).reshape(-1, 3)
        self._check(self.L.kt_set_scans(self.h, first, r.shape[0], r.ctypes.data_as(C.c_void_p),
                                        p.ctypes.data_as(C.c_void_p)), "kt_set_scans")

    def set_scans_device(self, first: int, count: int, d_ranges: int, d_poses: int, hip_stream: int = 0):
        self._check(self.L.kt_set_scans_device(self.h, first, count, C.c_void_p(d_ranges), C.c_void_p(d_poses),
                                               C.c_void_p(hip_stream or None)), "kt_set_scans_device")

    def match_batch_device(self, count: int, d_query: int, d_base_begin: int, d_base_index: int, d_results: int,
                           doPenalize: bool = True, doRefineMatch: bool = True, hip_stream: int = 0):
        self._check(self.L.kt_match_batch_device(self.h, count, C.c_void_p(d_query), C.c_void_p(d_base_begin),
                                                 C.c_void_p(d_base_index), int(doPenalize), int(doRefineMatch),
                                                 C.c_void_p(d_results), C.c_void_p(hip_stream or None)),
                    "kt_match_batch_device")

    # ---- one window sharded over GPUs ----
    def exchange_words(self) -> int:
        """int64 words one match exports in a sharded window (kt_window_exchange_words)."""
        return int(self.L.kt_window_exchange_words(self.h))

    def match_sharded_begin_device(self, count: int, d_query: int, d_base_begin: int, d_base_index: int,
                                   shard: int, nshards: int, d_exchange: int, doPenalize: bool = True,
                                   hip_stream: int = 0):
        self._check(self.L.kt_match_sharded_begin_device(self.h, count, C.c_void_p(d_query), C.c_void_p(d_base_begin),
                                                         C.c_void_p(d_base_index), int(doPenalize), shard, nshards,
                                                         C.c_void_p(d_exchange), C.c_void_p(hip_stream or None)),
                    "kt_match_sharded_begin_device")

    def match_sharded_end_device(self, count: int, d_base_begin: int, d_base_index: int, d_exchange: int,
                                 d_results: int, doPenalize: bool = True, doRefineMatch: bool = True,
                                 hip_stream: int = 0):
        self._check(self.L.kt_match_sharded_end_device(self.h, count, C.c_void_p(d_base_begin),
                                                       C.c_void_p(d_base_index), int(doPenalize), int(doRefineMatch),
                                                       C.c_void_p(d_exchange), C.c_void_p(d_results),
                                                       C.c_void_p(hip_stream or None)),
                    "kt_match_sharded_end_device")

    def match_sharded(self, count: int, d_query: int, d_base_begin: int, d_base_index: int, d_results: int,
                      doPenalize: bool = True, doRefineMatch: bool = True, group=None):
        """MatchScan batch with the coarse window split over the ranks of `group` (one GPU each): every
        rank evaluates the angles a = rank (mod world), ONE all-reduce (MAX) of the exchange words over
        RCCL, then every rank finishes the identical result (equal to match_batch_device)."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        hs = torch.cuda.current_stream().cuda_stream
        x = torch.empty((count, self.exchange_words()), dtype=torch.int64, device="cuda")
        self.match_sharded_begin_device(count, d_query, d_base_begin, d_base_index, rank, world, x.data_ptr(),
                                        doPenalize, hs)
        allreduce_window(x, group)
        self.match_sharded_end_device(count, d_base_begin, d_base_index, x.data_ptr(), d_results, doPenalize,
                                      doRefineMatch, hs)

    def set_timing(self, on: bool):
        self._check(self.L.kt_set_timing(self.h, 1 if on else 0), "kt_set_timing")

    def kernel_times(self, reset: bool = True) -> dict:
        k = self.L.kt_num_kernels()
        ms = np.zeros(k, np.float64)
        n = np.zeros(k, np.int64)
        self._check(self.L.kt_get_kernel_times(self.h, ms.ctypes.data_as(C.c_void_p), n.ctypes.data_as(C.c_void_p),
                                               1 if reset else 0), "kt_get_kernel_times")
        return {self.L.kt_kernel_name(i).decode(): (float(ms[i]), int(n[i])) for i in range(k)}


def shard_owns_angle(a: int, shard: int, nshards: int) -> bool:
    """The coarse angle ownership rule of a sharded window (kt_coarse_kernel)."""
    return a % nshards == shard


def allreduce_window(x, group=None):
    """The one exchange step of a sharded window: element-wise MAX over the ranks of the int64 export
    words.  Every word is the bit pattern of a non-negative double (or a 0/1 flag), where signed-integer
    order equals numeric order, so MAX of one owner's value and the others' +0.0 is that value."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(x, op=dist.ReduceOp.MAX, group=group)
    return x


def results_from_bytes(buf: np.ndarray) -> np.ndarray:
    """View a uint8 buffer of kt_result records as a structured array."""
    return np.frombuffer(np.ascontiguousarray(buf).tobytes(), dtype=RESULT_DTYPE)


DEG = math.pi / 180.0
