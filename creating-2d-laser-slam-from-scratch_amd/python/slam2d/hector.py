"""Host-side mirror of the reference's Hector interface over the MI355X C-ABI (include/slam2d/hector.h).

Reference classes mirrored (lesson4/include/lesson4/hector_mapping/):
  * DataContainer          scan/DataPointContainer.h:37-95   (points in map scale + origo)
  * HectorSlamProcessor    slam_main/HectorSlamProcessor.h:54-149
  * MapRepresentationInterface (slam_main/MapRepresentationInterface.h:44-69) is the seam the
    device backend implements; `HectorFleet` exposes it for B independent streams at once.

Method names follow the reference (camelCase) so parity tests read like the reference's API.
Every compute call goes to the HIP library; there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check

_f = C.c_float


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class DataContainer:
    """hectorslam::DataContainer (scan/DataPointContainer.h:37-95)."""

    def __init__(self, size: int = 1000):
        self._pts: list = []
        self._arr = None
        self.origo = np.zeros(2, np.float32)

    def setFrom(self, other: "DataContainer", factor: float) -> None:  # :46-58
        f = np.float32(factor)
        self.origo = (other.getOrigo() * f).astype(np.float32)
        self._arr = (other.points() * f).astype(np.float32)
        self._pts = []

    def add(self, p) -> None:  # :60-63
        self._flush()
        self._pts.append(np.asarray(p, np.float32))

    def clear(self) -> None:
        self._pts = []
        self._arr = np.zeros((0, 2), np.float32)

    def getSize(self) -> int:
        return int(self.points().shape[0])

    def getVecEntry(self, i: int) -> np.ndarray:
        return self.points()[i]

    def getOrigo(self) -> np.ndarray:
        return self.origo.copy()

    def setOrigo(self, o) -> None:
        self.origo = np.asarray(o, np.float32).reshape(2)

    # helpers
    def _flush(self):
        if self._arr is not None and len(self._arr):
            self._pts = list(self._arr)
        self._arr = None

    def points(self) -> np.ndarray:
        if self._arr is None:
            self._arr = np.asarray(self._pts, np.float32).reshape(-1, 2) if self._pts else np.zeros((0, 2), np.float32)
        return self._arr

    @staticmethod
    def from_points(pts, origo=(0.0, 0.0)) -> "DataContainer":
        d = DataContainer()
        d._arr = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        d.setOrigo(origo)
        return d


class HsLaser(C.Structure):
    """include/slam2d/hector.h hs_laser (the node's scan geometry and filter parameters)."""
    _fields_ = [("n_beams", C.c_int), ("angle_min", C.c_float), ("angle_increment", C.c_float),
                ("range_min", C.c_float), ("range_cutoff", C.c_double), ("basis", C.c_double * 9),
                ("origin", C.c_double * 3), ("sqr_laser_min_dist", C.c_float), ("sqr_laser_max_dist", C.c_float),
                ("use_max_scan_range", C.c_double), ("laser_z_min_value", C.c_float),
                ("laser_z_max_value", C.c_float)]

    @classmethod
    def defaults(cls, n_beams: int, angle_min: float, angle_increment: float) -> "HsLaser":
        L = cls()
        _lib.lib().hs_default_laser(C.byref(L), n_beams, angle_min, angle_increment)
        return L

    def as_oracle_dict(self) -> dict:
        """The same parameters in the form oracle.ingest takes (tests only)."""
        return {"range_cutoff": self.range_cutoff, "range_min": self.range_min,
                "tf": list(self.basis) + list(self.origin), "sqr_min": self.sqr_laser_min_dist,
                "sqr_max": self.sqr_laser_max_dist, "use_max": self.use_max_scan_range,
                "z_min": self.laser_z_min_value, "z_max": self.laser_z_max_value}


class HectorFleet:
    """B independent Hector SLAM streams resident in HBM (one MapRepMultiMap pyramid each)."""

    def __init__(self, num_streams=1, map_resolution=0.05, map_size=2048, map_start=(0.5, 0.5), levels=3,
                 max_points=1081, map_size_y=None):
        self.L = _lib.lib()
        self.B = int(num_streams)
        self.levels = int(levels)
        self.max_points = int(max_points)
        h = C.c_void_p()
        sy = map_size if map_size_y is None else map_size_y
        check(self.L.hs_create(C.byref(h), self.B, _f(map_resolution), int(map_size), int(sy), _f(map_start[0]),
                               _f(map_start[1]), self.levels, self.max_points), "hs_create")
        self.h = h

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "h", None):
            self.L.hs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(self.L.hs_reset(self.h), "hs_reset")

    def set_update_factors(self, free_factor: float, occupied_factor: float):
        check(self.L.hs_set_update_factors(self.h, _f(free_factor), _f(occupied_factor)), "hs_set_update_factors")

    def set_thresholds(self, min_dist: float, min_angle: float):
        check(self.L.hs_set_map_update_thresholds(self.h, _f(min_dist), _f(min_angle)), "hs_set_map_update_thresholds")

    ORDER_REFERENCE = 0   # H / b summed in point order, as OccGridMapUtil.h:94-126 (default)
    ORDER_TREE256 = 256   # 256-thread tree (faster; the oracle's reduce_threads=256)

    def set_reduction_order(self, order: int):
        check(self.L.hs_set_reduction_order(self.h, int(order)), "hs_set_reduction_order")

    def reduction_order(self) -> int:
        o = C.c_int()
        check(self.L.hs_get_reduction_order(self.h, C.byref(o)), "hs_get_reduction_order")
        return o.value

    # ---------------------------------------------------------------- single-stream (host buffers)
    def update(self, stream: int, pts, origo=(0.0, 0.0), hint=None, map_without_matching=False):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        did = C.c_int()
        hp = None
        if hint is not None:
            hint = np.ascontiguousarray(hint, np.float32)
            hp = _fp(hint)
        check(self.L.hs_update(self.h, stream, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]), hp,
                               1 if map_without_matching else 0, _fp(pose), _fp(cov), C.byref(did)), "hs_update")
        return pose, cov.reshape(3, 3), bool(did.value)

    def match(self, stream: int, pts, hint, origo=(0.0, 0.0)):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        hint = np.ascontiguousarray(hint, np.float32)
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        check(self.L.hs_match(self.h, stream, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]), _fp(hint),
                              _fp(pose), _fp(cov)), "hs_match")
        return pose, cov.reshape(3, 3)

    def update_by_scan(self, stream: int, pts, pose, origo=(0.0, 0.0)):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        pose = np.ascontiguousarray(pose, np.float32)
        check(self.L.hs_update_by_scan(self.h, stream, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]),
                                       _fp(pose)), "hs_update_by_scan")

    def last_pose(self, stream: int = 0):
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        check(self.L.hs_get_last_pose(self.h, stream, _fp(pose), _fp(cov)), "hs_get_last_pose")
        return pose, cov.reshape(3, 3)

    def map_info(self, level: int = 0):
        sx, sy, cl = C.c_int(), C.c_int(), C.c_float()
        org = np.zeros(2, np.float32)
        check(self.L.hs_get_map_info(self.h, level, C.byref(sx), C.byref(sy), C.byref(cl), _fp(org)), "hs_get_map_info")
        return sx.value, sy.value, cl.value, org

    def scale_to_map(self) -> float:
        s = C.c_float()
        check(self.L.hs_get_scale_to_map(self.h, C.byref(s)), "hs_get_scale_to_map")
        return s.value

    def get_map(self, stream: int = 0, level: int = 0, want_occ=True, want_raw=True):
        sx, sy, _, _ = self.map_info(level)
        occ = np.empty(sx * sy, np.int8) if want_occ else None
        l = np.empty(sx * sy, np.float32) if want_raw else None
        u = np.empty(sx * sy, np.int32) if want_raw else None
        ui = C.c_int()
        check(self.L.hs_get_map(self.h, stream, level, _fp(occ) if want_occ else None, _fp(l) if want_raw else None,
                                _fp(u) if want_raw else None, C.byref(ui)), "hs_get_map")
        r = {"update_index": ui.value}
        if want_occ:
            r["occ"] = occ.reshape(sy, sx)
        if want_raw:
            r["logodds"] = l.reshape(sy, sx)
            r["upd"] = u.reshape(sy, sx)
        return r

    def flush_ordinals(self, hip_stream: int = 0):
        """hs_flush_ordinals: every stream's 16-bit update ordinals into the int32 updateIndex plane now (zero-copy
        readers of hs_get_device_buffers; replayed graph captures of *_device calls, at least every 32000 steps)."""
        check(self.L.hs_flush_ordinals(self.h, C.c_void_p(hip_stream or None)), "hs_flush_ordinals")

    def device_cells(self):
        """(device pointer, bytes, stream_words) of the tiled cell storage (hs_get_device_buffers)."""
        p, nb, sw = C.c_void_p(), C.c_size_t(), C.c_size_t()
        check(self.L.hs_get_device_buffers(self.h, C.byref(p), C.byref(nb), C.byref(sw)), "hs_get_device_buffers")
        return p.value, nb.value, sw.value

    def set_map(self, stream: int, level: int, logodds, upd):
        l = np.ascontiguousarray(logodds, np.float32)
        u = np.ascontiguousarray(upd, np.int32)
        check(self.L.hs_set_map(self.h, stream, level, _fp(l), _fp(u)), "hs_set_map")

    # ---------------------------------------------------------------- batched device path
    def step_device(self, d_xy: int, xy_stride: int, d_n: int, d_origo: int = 0, d_hints: int = 0,
                    stream_begin: int = 0, count: int | None = None, hip_stream: int = 0):
        """One HectorSlamProcessor::update for every stream; pointers are device addresses (ints)."""
        count = self.B - stream_begin if count is None else count
        check(self.L.hs_step_batch_device(self.h, stream_begin, count, C.c_void_p(d_xy), int(xy_stride),
                                          C.c_void_p(d_n), C.c_void_p(d_origo or None), C.c_void_p(d_hints or None),
                                          C.c_void_p(hip_stream or None)), "hs_step_batch_device")

    # ---- scan ingest (LaserScan -> DataContainer on the device), hector_slam.cc:186-198, 320-362 ----
    def set_laser(self, laser: "HsLaser", unit_vectors=None):
        """HectorMappingRos's scan geometry + filters (hs_set_laser); unit_vectors [n, 2] double or None
        (computed with the host libm as laser_geometry's getUnitVectors_)."""
        uv = None
        if unit_vectors is not None:
            uv = np.ascontiguousarray(unit_vectors, np.float64).reshape(-1)
        check(self.L.hs_set_laser(self.h, C.byref(laser), _fp(uv) if uv is not None else None), "hs_set_laser")

    def ingest_device(self, count: int, d_ranges: int, range_stride: int, d_xy: int, xy_stride: int, d_n: int,
                      d_origo: int = 0, hip_stream: int = 0):
        check(self.L.hs_ingest_batch_device(self.h, count, C.c_void_p(d_ranges), int(range_stride), C.c_void_p(d_xy),
                                            int(xy_stride), C.c_void_p(d_n), C.c_void_p(d_origo or None),
                                            C.c_void_p(hip_stream or None)), "hs_ingest_batch_device")

    def step_ranges_device(self, d_ranges: int, range_stride: int, d_hints: int = 0, stream_begin: int = 0,
                           count: int | None = None, hip_stream: int = 0):
        """scanCallback for every stream: ingest + HectorSlamProcessor::update (device pointers)."""
        count = self.B - stream_begin if count is None else count
        check(self.L.hs_step_ranges_batch_device(self.h, stream_begin, count, C.c_void_p(d_ranges), int(range_stride),
                                                 C.c_void_p(d_hints or None), C.c_void_p(hip_stream or None)),
              "hs_step_ranges_batch_device")

    def run_ranges_device(self, steps: int, d_ranges: int, range_stride: int, step_stride: int, hip_stream: int = 0):
        """scanCallback for `steps` consecutive scans of every stream (step k at d_ranges + k * step_stride
        floats); two fleet halves pipelined on two HIP streams, joined on hip_stream."""
        check(self.L.hs_run_ranges_device(self.h, int(steps), C.c_void_p(d_ranges), int(range_stride),
                                          int(step_stride), C.c_void_p(hip_stream or None)), "hs_run_ranges_device")

    def update_ranges(self, stream: int, ranges):
        """scanCallback for one stream from host ranges (float32 [n_beams])."""
        r = np.ascontiguousarray(ranges, np.float32)
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        did = C.c_int()
        check(self.L.hs_update_ranges(self.h, stream, _fp(r), _fp(pose), _fp(cov), C.byref(did)), "hs_update_ranges")
        return pose, cov.reshape(3, 3), bool(did.value)

    def poses(self):
        p = np.zeros((self.B, 3), np.float32)
        cv = np.zeros((self.B, 9), np.float32)
        d = np.zeros(self.B, np.int32)
        cells = np.zeros(self.B, np.int64)
        check(self.L.hs_get_poses(self.h, _fp(p), _fp(cv), _fp(d), _fp(cells)), "hs_get_poses")
        return p, cv.reshape(self.B, 3, 3), d.astype(bool), cells

    def counters(self, reset=True):
        o = np.zeros(6, np.int64)
        check(self.L.hs_get_counters(self.h, _fp(o), 1 if reset else 0), "hs_get_counters")
        return {"cells": int(o[0]), "rays": int(o[1]), "gn_points": int(o[2]), "updates": int(o[3]), "steps": int(o[4]),
                "touched": int(o[5])}

    def set_pose_log(self, d_buf: int, streams: int, capacity: int):
        """Device pose log (float32 [capacity][streams][3]) filled by every step; d_buf = 0 disables."""
        check(self.L.hs_set_pose_log(self.h, C.c_void_p(d_buf or None), int(streams), int(capacity)), "hs_set_pose_log")

    def set_pose_log_slots(self, d_buf: int, d_slot_of_stream: int, slots: int, capacity: int):
        """Device pose log of any subset of streams: stream s -> slot d_slot_of_stream[s] (< 0: not logged)."""
        check(self.L.hs_set_pose_log_slots(self.h, C.c_void_p(d_buf or None), C.c_void_p(d_slot_of_stream or None),
                                           int(slots), int(capacity)), "hs_set_pose_log_slots")

    def queue_stats(self, reset_stamps=True):
        o = np.zeros(8, np.int64)
        check(self.L.hs_get_queue_stats(self.h, _fp(o), 1 if reset_stamps else 0), "hs_get_queue_stats")
        return {"items": int(o[0]), "segments": int(o[1]), "whole": int(o[2]), "overflow": int(o[3]),
                "cyc_setup": int(o[4]), "cyc_raster": int(o[5]), "cyc_apply": int(o[6]), "tiles": int(o[7])}

    def diag_stamps(self, reset=True):
        """hs_get_diag_stamps: the 8 cycle sums a diagnostic build accumulates (tools/build_diag.py)."""
        o = np.zeros(8, np.int64)
        check(self.L.hs_get_diag_stamps(self.h, _fp(o), 1 if reset else 0), "hs_get_diag_stamps")
        return o

    def stream_handle(self) -> int:
        return int(self.L.hs_get_stream(self.h) or 0)

    def set_timing(self, enable: bool):
        check(self.L.hs_set_timing(self.h, 1 if enable else 0), "hs_set_timing")

    def kernel_times(self, reset=True):
        ms = np.zeros(3, np.float64)
        n = np.zeros(3, np.int64)
        check(self.L.hs_get_kernel_times(self.h, _fp(ms), _fp(n), 1 if reset else 0), "hs_get_kernel_times")
        names = ("match", "bin", "update")  # slot 2: hs_update_kernel (default) or hs_tile_kernel (binned)
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(names)}

    def set_clock_probe(self, enable: bool):
        check(self.L.hs_set_clock_probe(self.h, 1 if enable else 0), "hs_set_clock_probe")

    def clock_probe(self, reset=True):
        """Effective shader clock (MHz) of the match and update kernels over the sampled workgroups'
        lifetimes since the last reset (s_memtime / s_memrealtime x 100 MHz), with the raw sums."""
        o = np.zeros(6, np.float64)
        check(self.L.hs_get_clock_probe(self.h, _fp(o), 1 if reset else 0), "hs_get_clock_probe")
        out = {}
        for i, k in enumerate(("match", "update")):
            cyc, ticks, wgs = o[3 * i: 3 * i + 3]
            out[k] = {"sclk_mhz": round(cyc / ticks * 100.0, 1) if ticks > 0 else None,
                      "cycles": int(cyc), "ticks_100mhz": int(ticks), "workgroups_sampled": int(wgs),
                      "cycles_per_workgroup": round(cyc / wgs, 1) if wgs else None}
        return out


class HectorSlamProcessor:
    """hectorslam::HectorSlamProcessor (slam_main/HectorSlamProcessor.h:54-149), device-backed."""

    def __init__(self, mapResolution=0.05, mapSizeX=2048, mapSizeY=2048, startCoords=(0.5, 0.5), multi_res_size=3,
                 max_points=4096):
        self.fleet = HectorFleet(1, mapResolution, mapSizeX, startCoords, multi_res_size, max_points,
                                 map_size_y=mapSizeY)
        self._cov = np.zeros((3, 3), np.float32)

    def update(self, dataContainer: DataContainer, poseHintWorld, map_without_matching=False):  # :81-108
        pose, cov, _ = self.fleet.update(0, dataContainer.points(), dataContainer.getOrigo(), poseHintWorld,
                                         map_without_matching)
        return pose

    def reset(self):  # :111-117
        self.fleet.reset()

    def getLastScanMatchPose(self):
        return self.fleet.last_pose(0)[0]

    def getLastScanMatchCovariance(self):
        return self.fleet.last_pose(0)[1]

    def getScaleToMap(self) -> float:
        return self.fleet.scale_to_map()

    def getMapLevels(self) -> int:
        return self.fleet.levels

    def getGridMap(self, mapLevel=0):
        return self.fleet.get_map(0, mapLevel)

    def setUpdateFactorFree(self, free_factor):
        self._free = free_factor
        self.fleet.set_update_factors(free_factor, getattr(self, "_occ", 0.6))

    def setUpdateFactorOccupied(self, occupied_factor):
        self._occ = occupied_factor
        self.fleet.set_update_factors(getattr(self, "_free", 0.4), occupied_factor)

    def setMapUpdateMinDistDiff(self, minDist):
        self._dist = minDist
        self.fleet.set_thresholds(minDist, getattr(self, "_ang", 0.13))

    def setMapUpdateMinAngleDiff(self, angleChange):
        self._ang = angleChange
        self.fleet.set_thresholds(getattr(self, "_dist", 0.4), angleChange)
