"""Deterministic synthetic 2D laser scans (SURVEY.md §8d "Synthetic inputs").

The reference's bag files are absent (.MISSING_LARGE_BLOBS), so every input is generated here:

* sensor: 1081 beams, angle_min = -3*pi/4, increment 0.25 deg, max range 30 m, Gaussian range
  noise sigma = 0.01 m, seed 12345 + stream id (numpy PCG64);
* world: a closed 30 m x 20 m room with 6 box obstacles (exact ray/segment intersection);
* trajectory: a smooth elliptic loop, <= 0.1 m and <= 5 deg per scan, expressed in the frame of the
  first pose (the reference starts every run at pose (0,0,0): hector_slam.cc:195-201).

Scan -> Hector DataContainer follows HectorMappingRos::rosPointCloudToDataContainer
(lesson4/src/hector_mapping/hector_slam.cc:320-362) with an identity laser TF:
  keep 0.2 m < d < 30 m (laser_min/max_dist), drop x < 0 && d^2 < 0.5, drop d > 20 m
  (use_max_scan_range), point = float(xy) * scaleToMap (float), origo = (0, 0).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

N_BEAMS = 1081
ANGLE_MIN = np.float32(-3.0 * math.pi / 4.0)
ANGLE_INC = np.float32(math.radians(0.25))
RANGE_MAX = 30.0


def _box(cx, cy, w, h):
    x0, x1, y0, y1 = cx - w / 2, cx + w / 2, cy - h / 2, cy + h / 2
    return [((x0, y0), (x1, y0)), ((x1, y0), (x1, y1)), ((x1, y1), (x0, y1)), ((x0, y1), (x0, y0))]


def world_segments() -> np.ndarray:
    """30 x 20 m room centred at the origin + 6 boxes; returns [S, 2, 2] float64."""
    segs = _box(0.0, 0.0, 30.0, 20.0)
    for b in [(0.0, 0.0, 4.0, 2.0), (-11.5, 7.5, 2.0, 2.0), (11.5, -7.5, 2.0, 2.0),
              (11.5, 7.5, 1.5, 1.5), (-11.5, -7.5, 1.5, 1.5), (0.0, 8.6, 3.0, 1.0)]:
        segs += _box(*b)
    return np.asarray(segs, dtype=np.float64)


def beam_angles(n_beams: int = N_BEAMS) -> np.ndarray:
    """angle_min + i*increment in double, as GMapping::CreateCache does (gmapping.cc:118-123)."""
    return np.float64(ANGLE_MIN) + np.arange(n_beams, dtype=np.float64) * np.float64(ANGLE_INC)


def trajectory(num_scans: int, phase: float) -> np.ndarray:
    """Room-frame poses [T, 3] along the ellipse x = 8 cos t, y = 5 sin t (heading = tangent)."""
    # arc step ~0.08 m on a ~41.9 m loop
    dt = 0.08 / 6.7
    t = phase + dt * np.arange(num_scans, dtype=np.float64)
    x = 8.0 * np.cos(t)
    y = 5.0 * np.sin(t)
    th = np.arctan2(5.0 * np.cos(t), -8.0 * np.sin(t))
    return np.stack([x, y, th], axis=1)


def cast_ranges(poses: np.ndarray, segs: np.ndarray, n_beams: int = N_BEAMS) -> np.ndarray:
    """Exact ranges [T, n_beams] (inf when nothing within RANGE_MAX)."""
    ang = beam_angles(n_beams)
    a = segs[:, 0, :]
    e = segs[:, 1, :] - segs[:, 0, :]
    out = np.empty((poses.shape[0], n_beams), dtype=np.float64)
    for k, (px, py, th) in enumerate(poses):
        d = np.stack([np.cos(th + ang), np.sin(th + ang)], axis=1)  # [B, 2]
        # solve p + t d = a + u e
        den = d[:, None, 0] * e[None, :, 1] - d[:, None, 1] * e[None, :, 0]  # [B, S]
        wx = a[None, :, 0] - px
        wy = a[None, :, 1] - py
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (wx * e[None, :, 1] - wy * e[None, :, 0]) / den
            u = (wx * d[:, None, 1] - wy * d[:, None, 0]) / den
        ok = (np.abs(den) > 1e-12) & (t > 1e-9) & (u >= 0.0) & (u <= 1.0)
        t = np.where(ok, t, np.inf)
        r = t.min(axis=1)
        r[r > RANGE_MAX] = np.inf
        out[k] = r
    return out


def ranges_to_points(ranges: np.ndarray, scale_to_map: float = 20.0, laser_min: float = 0.2,
                     laser_max: float = 30.0, use_max: float = 20.0):
    """LaserScan ranges [n] -> (points float32 [m, 2] in map scale, m). hector_slam.cc:331-358."""
    ang = beam_angles(ranges.shape[0])
    x = (ranges * np.cos(ang)).astype(np.float32)
    y = (ranges * np.sin(ang)).astype(np.float32)
    xd = x.astype(np.float32)
    yd = y.astype(np.float32)
    d2 = xd * xd + yd * yd  # float: currPoint.x * currPoint.x + ... (Point32 floats)
    min2 = np.float32(laser_min * laser_min)
    max2 = np.float32(laser_max * laser_max)
    keep = np.isfinite(ranges) & (d2 > min2) & (d2 < max2)
    keep &= ~((xd < 0.0) & (d2 < np.float32(0.5)))
    keep &= ~(d2.astype(np.float64) > use_max * use_max)
    s = np.float32(scale_to_map)
    pts = np.stack([xd[keep] * s, yd[keep] * s], axis=1).astype(np.float32)
    return pts, pts.shape[0]


@dataclass
class ScanSet:
    """Per-stream scan sequences.  points: [S, T, n_max, 2] float32 (zero-padded), counts [S, T] int32,
    ranges [S, T, n_beams] float32, gt [S, T, 3] float64 (first-pose frame)."""
    points: np.ndarray
    counts: np.ndarray
    ranges: np.ndarray
    gt: np.ndarray


def make_streams(num_streams: int, num_scans: int, seed: int = 12345, n_beams: int = N_BEAMS,
                 noise_sigma: float = 0.01, distinct_paths: int = 64, scale_to_map: float = 20.0,
                 with_points: bool = True) -> ScanSet:
    """Stream s follows base path s % distinct_paths (its own phase on the loop) with its own range
    noise (seed + s), so every stream's data is distinct while ray casting stays cheap."""
    segs = world_segments()
    n_paths = min(distinct_paths, num_streams)
    base_ranges = []
    base_gt = []
    for p in range(n_paths):
        phase = 2.0 * math.pi * p / max(n_paths, 1)
        poses = trajectory(num_scans, phase)
        base_ranges.append(cast_ranges(poses, segs, n_beams))
        # express in the first pose's frame
        x0, y0, t0 = poses[0]
        c, s = math.cos(-t0), math.sin(-t0)
        dx, dy = poses[:, 0] - x0, poses[:, 1] - y0
        rel = np.stack([c * dx - s * dy, s * dx + c * dy, np.arctan2(np.sin(poses[:, 2] - t0), np.cos(poses[:, 2] - t0))], 1)
        base_gt.append(rel)
    ranges = np.empty((num_streams, num_scans, n_beams), dtype=np.float32)
    gt = np.empty((num_streams, num_scans, 3), dtype=np.float64)
    for s_ in range(num_streams):
        rng = np.random.default_rng(seed + s_)
        r = base_ranges[s_ % n_paths] + rng.normal(0.0, noise_sigma, size=(num_scans, n_beams))
        r = np.where(np.isfinite(base_ranges[s_ % n_paths]), r, np.inf)
        ranges[s_] = r.astype(np.float32)
        gt[s_] = base_gt[s_ % n_paths]
    if with_points:
        points = np.zeros((num_streams, num_scans, n_beams, 2), dtype=np.float32)
        counts = np.zeros((num_streams, num_scans), dtype=np.int32)
        for s_ in range(num_streams):
            for t in range(num_scans):
                pts, m = ranges_to_points(ranges[s_, t].astype(np.float64), scale_to_map)
                points[s_, t, :m] = pts
                counts[s_, t] = m
    else:
        points = np.zeros((0,), np.float32)
        counts = np.zeros((0,), np.int32)
    return ScanSet(points=points, counts=counts, ranges=ranges, gt=gt)


def karto_sequential(num_matches: int, num_base: int, seed: int = 777, perturb=(0.03, 0.03, 0.02),
                     noise: float = 0.01, step: int = 2, phase: float = 0.3, n_beams: int = N_BEAMS):
    """Karto sequential-matcher workload: T = num_matches + num_base scans along the
    loop, `step` trajectory samples apart; scan i >= num_base is matched against the num_base scans
    before it (the running scans, Mapper.cpp:2040).  Base scans carry their true poses (already
    corrected by the mapper), the query an odometry pose = truth + N(0, perturb).
    Returns (ranges [T, n_beams] with inf for no return, true poses [T, 3], query poses [T, 3])."""
    rng = np.random.default_rng(seed)
    T = num_matches + num_base
    poses = trajectory(T * step, phase)[::step]
    R = cast_ranges(poses, world_segments(), n_beams)
    R = R + rng.normal(0.0, noise, R.shape)
    qp = poses + rng.normal(0.0, 1.0, poses.shape) * np.asarray(perturb, np.float64)
    return R, poses, qp


def karto_loop(num_matches: int, chain: int = 10, seed: int = 778, perturb=(0.4, 0.4, 0.05), noise: float = 0.01,
               n_beams: int = N_BEAMS):
    """Loop-closure candidate batch (MapperGraph::TryCloseLoop, Mapper.cpp:976-1016): each query scan
    (second lap) is matched against a chain of `chain` scans recorded near the same place on the first
    lap; the query pose carries an accumulated drift ~ N(0, perturb).
    Returns (query ranges [M, n], query poses [M, 3], true query poses [M, 3],
             chain ranges [M, chain, n], chain poses [M, chain, 3])."""
    rng = np.random.default_rng(seed)
    segs = world_segments()
    lap = 2.0 * math.pi
    t0 = rng.uniform(0.0, lap, num_matches)
    dt = 0.08 / 6.7
    qt = t0 + lap + rng.uniform(-2 * dt, 2 * dt, num_matches)

    def pose_at(t):
        return np.stack([8.0 * np.cos(t), 5.0 * np.sin(t), np.arctan2(5.0 * np.cos(t), -8.0 * np.sin(t))], axis=-1)

    qtrue = pose_at(qt)
    ct = t0[:, None] + dt * 3 * (np.arange(chain)[None, :] - chain // 2)
    cposes = pose_at(ct)
    QR = cast_ranges(qtrue, segs, n_beams) + rng.normal(0.0, noise, (num_matches, n_beams))
    CR = cast_ranges(cposes.reshape(-1, 3), segs, n_beams).reshape(num_matches, chain, n_beams)
    CR = CR + rng.normal(0.0, noise, CR.shape)
    qpose = qtrue + rng.normal(0.0, 1.0, qtrue.shape) * np.asarray(perturb, np.float64)
    return QR, qpose, qtrue, CR, cposes
