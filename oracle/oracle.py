"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes bindings of the CPU checkers.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.

* HectorOracle   : oracle/build/libhector_oracle.so  (C restatement, parity unpinned -- see hector_oracle.c)
* gmapping_oracle: oracle/build/libgmapping_oracle.so (C restatement)
* gmapping_ref   : oracle/_ref/libgmapping_ref.so    (reference GMapping headers compiled unmodified)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")
REF = os.path.join(HERE, "_ref")

_f = C.c_float
_i = C.c_int
_p = C.c_void_p


def build(ref: bool | None = None) -> None:
    """Compile the oracle libraries (and oracle/_ref when /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])
    if ref is None:
        ref = os.path.isdir("/root/reference/lesson4/include")
    if ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def _lib(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
    return C.CDLL(path)


def _fp(a):
    return a.ctypes.data_as(C.c_void_p)


_HL = {}


def hector_lib(variant: str = "") -> C.CDLL:
    """variant "" = -O3 build, "O0" = the -O0 build (CPU-baseline comparison only)."""
    if variant not in _HL:
        L = _lib(os.path.join(BUILD, f"libhector_oracle{'_' + variant if variant else ''}.so"))
        L.ho_create.restype = _p
        L.ho_create.argtypes = [_f, _i, _i, _f, _f, _i]
        L.ho_destroy.argtypes = [_p]
        L.ho_reset.argtypes = [_p]
        L.ho_set_update_factors.argtypes = [_p, _f, _f]
        L.ho_set_thresholds.argtypes = [_p, _f, _f]
        L.ho_set_mode.argtypes = [_p, _i, _i]
        L.ho_enable_trace.argtypes = [_p, _i]
        L.ho_trace_len.argtypes = [_p]
        L.ho_get_trace.argtypes = [_p, _p]
        L.ho_match.argtypes = [_p, _p, _i, _f, _f, _p, _p, _p]
        L.ho_update_by_scan.argtypes = [_p, _p, _i, _f, _f, _p]
        L.ho_process.restype = _i
        L.ho_process.argtypes = [_p, _p, _i, _f, _f, _p, _i, _p, _p]
        L.ho_get_last_pose.argtypes = [_p, _p]
        L.ho_get_last_cov.argtypes = [_p, _p]
        L.ho_level_dims.argtypes = [_p, _i, C.POINTER(_i), C.POINTER(_i)]
        L.ho_get_level.argtypes = [_p, _i, _p, _p]
        L.ho_set_level.argtypes = [_p, _i, _p, _p]
        L.ho_update_index.argtypes = [_p, _i]
        L.ho_cur_update_index.argtypes = [_p, _i]
        L.ho_sum_L.restype = C.c_ulonglong
        L.ho_sum_L.argtypes = [_p]
        L.ho_sum_free.restype = C.c_ulonglong
        L.ho_sum_free.argtypes = [_p]
        L.ho_valid_rays.argtypes = [_p]
        L.ho_clamp_count.argtypes = [_p]
        L.ho_get_factors.argtypes = [_p, C.POINTER(_f), C.POINTER(_f)]
        L.ho_get_transform.argtypes = [_p, _i, _p]
        L.ho_publish_level.argtypes = [_p, _i, _p]
        L.ho_ray_cells.restype = _i
        L.ho_ray_cells.argtypes = [_i, _i, _i, _i, _i, _i, _p, _i]
        L.ho_unit_vectors.argtypes = [_i, _f, _f, _p]
        L.ho_ingest.restype = _i
        L.ho_ingest.argtypes = [_i, _p, _p, C.c_double, _f, _p, _f, _f, C.c_double, _f, _f, _f, _p, _p]
        for n in ("ho_det_sinf", "ho_det_cosf", "ho_det_expf", "ho_det_prob", "ho_det_prob_to_logodds"):
            getattr(L, n).restype = _f
            getattr(L, n).argtypes = [_f]
        _HL[variant] = L
    return _HL[variant]


class HectorOracle:
    """CPU restatement of HectorSlamProcessor + MapRepMultiMap (H/slam_main/*).

    reduce_threads: 0 = reference (sequential) Hessian sums; T = the HIP kernel's tree order.
    use_libm: evaluate sin/cos/exp with libm instead of the deterministic detmath.h.
    """

    def __init__(self, map_resolution=0.05, map_size=1024, start=(0.5, 0.5), levels=1, reduce_threads=0,
                 use_libm=False, map_size_y=None, lib_variant=""):
        self.L = hector_lib(lib_variant)
        sy = map_size if map_size_y is None else map_size_y
        self.h = self.L.ho_create(_f(map_resolution), map_size, sy, _f(start[0]), _f(start[1]), levels)
        if not self.h:
            raise ValueError("ho_create failed")
        self.levels = levels
        self.L.ho_set_mode(self.h, reduce_threads, 1 if use_libm else 0)

    def close(self):
        if self.h:
            self.L.ho_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_update_factors(self, free_f, occ_f):
        self.L.ho_set_update_factors(self.h, _f(free_f), _f(occ_f))

    def set_thresholds(self, dist, ang):
        self.L.ho_set_thresholds(self.h, _f(dist), _f(ang))

    def reset(self):
        self.L.ho_reset(self.h)

    def process(self, pts, origo=(0.0, 0.0), hint=None, map_without_matching=False):
        pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 2)
        if hint is None:
            hint = self.last_pose()
        hint = np.asarray(hint, np.float32)
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        did = self.L.ho_process(self.h, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]), _fp(hint),
                                1 if map_without_matching else 0, _fp(pose), _fp(cov))
        return pose, cov.reshape(3, 3), bool(did)

    def match(self, pts, hint, origo=(0.0, 0.0)):
        """MapRepMultiMap::matchData: pose + cov; keeps the container for levels >= 1 (:161)."""
        pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 2)
        hint = np.asarray(hint, np.float32)
        pose = np.zeros(3, np.float32)
        cov = np.zeros(9, np.float32)
        self.L.ho_match(self.h, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]), _fp(hint), _fp(pose), _fp(cov))
        return pose, cov.reshape(3, 3)

    def update_by_scan(self, pts, pose, origo=(0.0, 0.0)):
        pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 2)
        pose = np.asarray(pose, np.float32)
        self.L.ho_update_by_scan(self.h, _fp(pts), pts.shape[0], _f(origo[0]), _f(origo[1]), _fp(pose))

    def last_pose(self):
        p = np.zeros(3, np.float32)
        self.L.ho_get_last_pose(self.h, _fp(p))
        return p

    def last_cov(self):
        """HectorSlamProcessor::getLastScanMatchCovariance (HectorSlamProcessor.h:122)."""
        cv = np.zeros(9, np.float32)
        self.L.ho_get_last_cov(self.h, _fp(cv))
        return cv.reshape(3, 3)

    def dims(self, lvl):
        sx, sy = _i(), _i()
        self.L.ho_level_dims(self.h, lvl, C.byref(sx), C.byref(sy))
        return sx.value, sy.value

    def level(self, lvl):
        sx, sy = self.dims(lvl)
        l = np.empty(sx * sy, np.float32)
        u = np.empty(sx * sy, np.int32)
        self.L.ho_get_level(self.h, lvl, _fp(l), _fp(u))
        return l.reshape(sy, sx), u.reshape(sy, sx)

    def set_level(self, lvl, l, u):
        l = np.ascontiguousarray(l, np.float32)
        u = np.ascontiguousarray(u, np.int32)
        self.L.ho_set_level(self.h, lvl, _fp(l), _fp(u))

    def publish(self, lvl=0):
        sx, sy = self.dims(lvl)
        o = np.empty(sx * sy, np.int8)
        self.L.ho_publish_level(self.h, lvl, _fp(o))
        return o.reshape(sy, sx)

    def update_index(self, lvl=0):
        return self.L.ho_update_index(self.h, lvl)

    def cur_update_index(self, lvl=0):
        return self.L.ho_cur_update_index(self.h, lvl)

    def sum_L(self):
        return int(self.L.ho_sum_L(self.h))

    def sum_free(self):
        return int(self.L.ho_sum_free(self.h))

    def valid_rays(self):
        return int(self.L.ho_valid_rays(self.h))

    def factors(self):
        a, b = _f(), _f()
        self.L.ho_get_factors(self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def transform(self, lvl):
        o = np.zeros(8, np.float32)
        self.L.ho_get_transform(self.h, lvl, _fp(o))
        return o

    def enable_trace(self, cap):
        self.L.ho_enable_trace(self.h, cap)

    def trace(self):
        n = self.L.ho_trace_len(self.h)
        o = np.zeros((n, 16), np.float32)
        self.L.ho_get_trace(self.h, _fp(o))
        return o


def unit_vectors(n, angle_min, angle_increment):
    """laser_geometry getUnitVectors_ restated (ho_unit_vectors): [n, 2] double (cos, sin)."""
    out = np.zeros((n, 2), dtype=np.float64)
    hector_lib().ho_unit_vectors(n, angle_min, angle_increment, _fp(out))
    return out


def ingest(ranges, cs, laser: dict, scale_to_map: float):
    """projectLaser + rosPointCloudToDataContainer restated (ho_ingest, hector_slam.cc:193, 320-362).
    laser: range_cutoff, range_min, tf (12 doubles: basis row-major + origin), sqr_min, sqr_max,
    use_max, z_min, z_max.  Returns (points float32 [m, 2], origo float32 [2])."""
    r = np.ascontiguousarray(ranges, dtype=np.float32)
    cs = np.ascontiguousarray(cs, dtype=np.float64)
    tf = np.ascontiguousarray(laser["tf"], dtype=np.float64)
    xy = np.zeros((r.shape[0], 2), dtype=np.float32)
    org = np.zeros(2, dtype=np.float32)
    m = hector_lib().ho_ingest(r.shape[0], _fp(r), _fp(cs), laser["range_cutoff"], laser["range_min"], _fp(tf),
                               laser["sqr_min"], laser["sqr_max"], laser["use_max"], laser["z_min"], laser["z_max"],
                               scale_to_map, _fp(xy), _fp(org))
    return xy[:m].copy(), org


def ray_cells(sx, sy, x0, y0, x1, y1):
    L = hector_lib()
    cap = 2 * (sx + sy) + 8
    o = np.zeros(cap, np.uint32)
    k = L.ho_ray_cells(sx, sy, x0, y0, x1, y1, _fp(o), cap)
    return o[:k]


# ---------------------------------------------------------------------------------------------- GMapping
_GO = None
_GR = None

_GM_ARGS = [C.c_double, C.c_double, C.c_double, C.c_double, _p, _i, _p, _p, C.c_double, C.c_double,
            C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, _p, _p, _p, C.POINTER(_i)]


def gmapping_oracle_lib():
    global _GO
    if _GO is None:
        L = _lib(os.path.join(BUILD, "libgmapping_oracle.so"))
        L.gmo_compute_map.restype = C.c_longlong
        L.gmo_compute_map.argtypes = _GM_ARGS + [C.POINTER(_i)]
        L.gmo_map_geometry.argtypes = [C.c_double] * 5 + [C.POINTER(_i)] * 4 + [C.POINTER(C.c_double)] * 2
        L.gmo_grid_line.restype = _i
        L.gmo_grid_line.argtypes = [_i, _i, _i, _i, _p]
        L.gmo_publish.argtypes = [_p, _p, _i, _i, C.c_double, _p]
        _GO = L
    return _GO


def gmapping_ref_lib():
    global _GR
    if _GR is None:
        L = _lib(os.path.join(REF, "libgmapping_ref.so"))
        L.gmr_compute_map.restype = C.c_longlong
        L.gmr_compute_map.argtypes = _GM_ARGS
        L.gmr_map_size.argtypes = [C.c_double] * 5 + [C.POINTER(_i)] * 2
        L.gmr_grid_line.restype = _i
        L.gmr_grid_line.argtypes = [_i, _i, _i, _i, _p, _i]
        L.gmr_world2map.argtypes = [C.c_double] * 7 + [C.POINTER(_i)] * 2
        _GR = L
    return _GR


GM_DEFAULTS = dict(max_range=30 - 0.01, max_urange=25.0, xmin=-40.0, ymin=-40.0, xmax=40.0, ymax=40.0, delta=0.05)


def gm_geometry(p=GM_DEFAULTS):
    L = gmapping_oracle_lib()
    sx, sy, sx2, sy2 = _i(), _i(), _i(), _i()
    cx, cy = C.c_double(), C.c_double()
    L.gmo_map_geometry(p["xmin"], p["ymin"], p["xmax"], p["ymax"], p["delta"], C.byref(sx), C.byref(sy),
                       C.byref(sx2), C.byref(sy2), C.byref(cx), C.byref(cy))
    return sx.value, sy.value, sx2.value, sy2.value


def gm_compute(ranges, a_cos, a_sin, pose=(0.0, 0.0, 1.0, 0.0), which="oracle", p=GM_DEFAULTS):
    """pose = (x, y, cos theta, sin theta). Returns (n, visits, acc, nfree, nhits) dense row-major."""
    sx, sy, _, _ = gm_geometry(p)
    ranges = np.ascontiguousarray(ranges, np.float32)
    a_cos = np.ascontiguousarray(a_cos, np.float64)
    a_sin = np.ascontiguousarray(a_sin, np.float64)
    n = np.zeros(sx * sy, np.int32)
    v = np.zeros(sx * sy, np.int32)
    acc = np.zeros(2 * sx * sy, np.float32)
    nh = _i()
    args = [pose[0], pose[1], pose[2], pose[3], _fp(ranges), ranges.shape[0], _fp(a_cos), _fp(a_sin),
            p["max_range"], p["max_urange"], p["xmin"], p["ymin"], p["xmax"], p["ymax"], p["delta"],
            _fp(n), _fp(v), _fp(acc), C.byref(nh)]
    if which == "oracle":
        oob = _i()
        nfree = gmapping_oracle_lib().gmo_compute_map(*args, C.byref(oob))
    else:
        nfree = gmapping_ref_lib().gmr_compute_map(*args)
    return n.reshape(sy, sx), v.reshape(sy, sx), acc.reshape(sy, sx, 2), int(nfree), nh.value


# ---------------------------------------------------------------------------------------------- PL-ICP
class PlParams(C.Structure):
    """plo_params / pl_params (lesson3/src/plicp_odometry.cc:74-186 defaults)."""
    _fields_ = [("max_angular_correction_deg", C.c_double), ("max_linear_correction", C.c_double),
                ("epsilon_xy", C.c_double), ("epsilon_theta", C.c_double),
                ("max_correspondence_dist", C.c_double), ("outliers_maxPerc", C.c_double),
                ("outliers_adaptive_order", C.c_double), ("outliers_adaptive_mult", C.c_double),
                ("max_iterations", C.c_int), ("use_point_to_line_distance", C.c_int),
                ("outliers_remove_doubles", C.c_int), ("pad_", C.c_int)]


_PL = None


def plicp_lib():
    global _PL
    if _PL is None:
        L = _lib(os.path.join(BUILD, "libplicp_oracle.so"))
        L.plo_default_params.argtypes = [C.POINTER(PlParams)]
        L.plo_icp.restype = _i
        L.plo_icp.argtypes = [C.POINTER(PlParams), _i, C.c_double, C.c_double, _p, _p, _p, _i, _p,
                              C.POINTER(_i), C.POINTER(_i), C.POINTER(C.c_double), _p]
        _PL = L
    return _PL


def pl_default_params() -> PlParams:
    p = PlParams()
    plicp_lib().plo_default_params(C.byref(p))
    return p


def plicp(ref, sens, angle_min, angle_inc, first_guess=(0.0, 0.0, 0.0), params=None, reduce_threads=0):
    """CPU restatement of CSM sm_icp (parity unpinned).  Returns dict(x, valid, iterations, nvalid, error)."""
    L = plicp_lib()
    p = params or pl_default_params()
    ref = np.ascontiguousarray(ref, np.float64)
    sens = np.ascontiguousarray(sens, np.float64)
    g = np.ascontiguousarray(first_guess, np.float64)
    x = np.zeros(3, np.float64)
    it, nv, err = _i(), _i(), C.c_double()
    hashes = np.zeros(64, np.int32)
    ok = L.plo_icp(C.byref(p), ref.shape[0], float(angle_min), float(angle_inc), _fp(ref), _fp(sens), _fp(g),
                   reduce_threads, _fp(x), C.byref(it), C.byref(nv), C.byref(err), _fp(hashes))
    return dict(x=x, valid=bool(ok), iterations=it.value, nvalid=nv.value, error=err.value)


# ---------------------------------------------------------------------------------------------- Karto
class KtLaser(C.Structure):
    """ko_laser / kt_laser: the LaserRangeFinder fields LocalizedRangeScan::Update reads."""
    _fields_ = [("minimum_angle", C.c_double), ("angular_resolution", C.c_double),
                ("minimum_range", C.c_double), ("range_threshold", C.c_double),
                ("n_readings", C.c_int), ("pad_", C.c_int)]


class KtParams(C.Structure):
    """ko_params / kt_params: one ScanMatcher's parameters (Mapper.cpp:1569-1660 names)."""
    _fields_ = [("search_size", C.c_double), ("resolution", C.c_double), ("smear_deviation", C.c_double),
                ("distance_variance_penalty", C.c_double), ("angle_variance_penalty", C.c_double),
                ("fine_search_angle_offset", C.c_double), ("coarse_search_angle_offset", C.c_double),
                ("coarse_angle_resolution", C.c_double), ("minimum_angle_penalty", C.c_double),
                ("minimum_distance_penalty", C.c_double), ("use_response_expansion", C.c_int),
                ("pad_", C.c_int)]


_KO = None


def karto_lib():
    global _KO
    if _KO is None:
        L = _lib(os.path.join(BUILD, "libkarto_oracle.so"))
        L.ko_match_scan.restype = _i
        L.ko_match_scan.argtypes = [C.POINTER(KtLaser), C.POINTER(KtParams), _p, _p, _i, _p, _p, _i, _i, _p, _p,
                                    C.POINTER(C.c_double)]
        L.ko_grid_info.restype = _i
        L.ko_grid_info.argtypes = [C.POINTER(KtParams), C.POINTER(KtLaser), _p]
        L.ko_kernel.restype = _i
        L.ko_kernel.argtypes = [C.POINTER(KtParams), C.POINTER(KtLaser), _p, _i]
        L.ko_coarse_responses.restype = _i
        L.ko_coarse_responses.argtypes = [C.POINTER(KtLaser), C.POINTER(KtParams), _p, _p, _i, _p, _p, _i, _p]
        L.ko_build_grid.restype = _i
        L.ko_build_grid.argtypes = [C.POINTER(KtLaser), C.POINTER(KtParams), _p, _i, _p, _p, _p]
        _KO = L
    return _KO


def karto_grid_info(params: KtParams, laser: KtLaser) -> dict:
    out = np.zeros(10, np.int32)
    rc = karto_lib().ko_grid_info(C.byref(params), C.byref(laser), _fp(out))
    if rc:
        raise ValueError(f"ko_grid_info: {rc}")
    keys = ["grid_size", "border", "width", "ws", "data_size", "side", "probs_ws", "half", "ksize"]
    return {k: int(v) for k, v in zip(keys, out)}


def karto_match(laser: KtLaser, params: KtParams, q_ranges, q_pose, b_ranges, b_poses, penalize=True,
                refine=True):
    """CPU restatement of ScanMatcher::MatchScan (parity unpinned).  Returns (mean[3], cov[3,3], response)."""
    q = np.ascontiguousarray(q_ranges, np.float64)
    qp = np.ascontiguousarray(q_pose, np.float64)
    b = np.ascontiguousarray(b_ranges, np.float64).reshape(-1, laser.n_readings)
    bp = np.ascontiguousarray(b_poses, np.float64).reshape(-1, 3)
    mean = np.zeros(3, np.float64)
    cov = np.zeros(9, np.float64)
    r = C.c_double()
    rc = karto_lib().ko_match_scan(C.byref(laser), C.byref(params), _fp(q), _fp(qp), b.shape[0], _fp(b), _fp(bp),
                                   int(penalize), int(refine), _fp(mean), _fp(cov), C.byref(r))
    if rc:
        raise RuntimeError(f"ko_match_scan: {rc}")
    return mean, cov.reshape(3, 3), r.value


def karto_coarse_responses(laser: KtLaser, params: KtParams, q_ranges, q_pose, b_ranges, b_poses, n_xy: int,
                           n_angles: int, penalize=True) -> np.ndarray:
    """The first coarse CorrelateScan's responses [n_xy, n_xy, n_angles] in pose order (test hook)."""
    q = np.ascontiguousarray(q_ranges, np.float64)
    qp = np.ascontiguousarray(q_pose, np.float64)
    b = np.ascontiguousarray(b_ranges, np.float64).reshape(-1, laser.n_readings)
    bp = np.ascontiguousarray(b_poses, np.float64).reshape(-1, 3)
    out = np.full(n_xy * n_xy * n_angles, np.nan, np.float64)
    rc = karto_lib().ko_coarse_responses(C.byref(laser), C.byref(params), _fp(q), _fp(qp), b.shape[0], _fp(b),
                                         _fp(bp), int(penalize), _fp(out))
    if rc:
        raise RuntimeError(f"ko_coarse_responses: {rc}")
    return out.reshape(n_xy, n_xy, n_angles)


def karto_build_grid(laser: KtLaser, params: KtParams, q_pose, b_ranges, b_poses) -> np.ndarray:
    info = karto_grid_info(params, laser)
    out = np.zeros(info["data_size"], np.uint8)
    b = np.ascontiguousarray(b_ranges, np.float64).reshape(-1, laser.n_readings)
    bp = np.ascontiguousarray(b_poses, np.float64).reshape(-1, 3)
    qp = np.ascontiguousarray(q_pose, np.float64)
    rc = karto_lib().ko_build_grid(C.byref(laser), C.byref(params), _fp(qp), b.shape[0], _fp(b), _fp(bp), _fp(out))
    if rc:
        raise RuntimeError(f"ko_build_grid: {rc}")
    return out.reshape(info["width"], info["ws"])
