"""GPU parity of the Hector path: HIP kernels (through the C-ABI) vs the CPU oracle.

Bar (BASELINE.json north_star):
  * integer / byte work bit-exact: every cell's updateIndex, the Bresenham cell count ΣL, the
    did-update gate, the map update index;
  * poses, covariances and log-odds floats bit-exact against the oracle in the reference's sequential
    Hessian summation order (reduce_threads=0, OccGridMapUtil.h:94-126), which is the kernel's default
    (HS_ORDER_REFERENCE): the north star's pose bar (<= 1e-4 m / rad) holds by construction;
  * the opt-in tree order (HS_ORDER_TREE256) bit-exact against the oracle's reduce_threads=256 and
    within POSE_TOL_M / POSE_TOL_RAD of the reference order.
"""
import os

import numpy as np
import pytest

import oracle as O
from slam2d import synth
from slam2d.hector import DataContainer, HectorFleet, HectorSlamProcessor

pytestmark = pytest.mark.gpu

POSE_TOL_M = 1e-4    # north_star: pose error <= 1e-4 m
POSE_TOL_RAD = 1e-4  # north_star: pose error <= 1e-4 rad
T_RED = 0            # the oracle in the reference summation order == the kernel default (HS_ORDER_REFERENCE)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def _run_pair(levels, size, scans, n_scans=25, thresholds=(0.4, 0.9), stream=0, origo=(0.0, 0.0)):
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), levels, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(*thresholds)
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), levels, reduce_threads=T_RED)
    ora.set_update_factors(0.4, 0.9)
    ora.set_thresholds(*thresholds)
    for k in range(n_scans):
        pts = scans.points[stream, k, : scans.counts[stream, k]]
        gp, gc, gd = fleet.update(0, pts, origo)
        op, oc, od = ora.process(pts, origo)
        assert gd == od, f"scan {k}: did_update {gd} vs {od}"
        np.testing.assert_array_equal(_bits(gp), _bits(op), err_msg=f"scan {k} pose")
        np.testing.assert_array_equal(_bits(gc), _bits(oc), err_msg=f"scan {k} cov")
    for lvl in range(levels):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou, err_msg=f"level {lvl} updateIndex")
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol), err_msg=f"level {lvl} log-odds bits")
        np.testing.assert_array_equal(m["occ"], ora.publish(lvl), err_msg=f"level {lvl} publish")
        assert m["update_index"] == ora.update_index(lvl)
    return fleet, ora


@pytest.fixture(scope="module")
def scans():
    return synth.make_streams(4, 40)


def test_single_level_1024_bitexact(gpu, scans):
    _run_pair(1, 1024, scans, n_scans=30)


def test_three_level_2048_bitexact(gpu, scans):
    _run_pair(3, 2048, scans, n_scans=20, stream=1)


def test_force_update_every_scan(gpu, scans):
    # benchmark mode: thresholds < 0 force a map update on every scan
    _run_pair(2, 512, scans, n_scans=20, thresholds=(-1.0, -1.0), stream=2)


def test_origo_offset(gpu, scans):
    _run_pair(2, 1024, scans, n_scans=12, origo=(3.25, -1.5), stream=3)


def test_out_of_map_beams_small_map(gpu, scans):
    # 256^2 at 5 cm = 12.8 m: many beams end outside and are cancelled (OccGridMapBase.h:226-238)
    _run_pair(1, 256, scans, n_scans=15, thresholds=(-1.0, -1.0))


@pytest.mark.parametrize("kernel", ["clip", "ring", "binned"])
@pytest.mark.parametrize("sweep,thresholds", [("1", (-1.0, -1.0)), ("3", (-1.0, -1.0)), ("2", (0.4, 0.9))])
def test_ordinal_sweep_bitexact(gpu, scans, monkeypatch, kernel, sweep, thresholds):
    """The updateIndex as a 16-bit hot ordinal + the cold int plane (hector_internal.h ORD_OFF): with an ordinal
    sweep every 1 / 2 / 3 steps (SLAM2D_ORD_SWEEP; the library's default is 32000), forced updates and the node's
    gate, every update kernel: every cell's updateIndex (decoded by hs_get_map) and log-odds stay bit-exact."""
    monkeypatch.setenv("SLAM2D_ORD_SWEEP", sweep)
    if kernel == "ring":
        monkeypatch.setenv("SLAM2D_UPD_KERNEL", "ring")
    elif kernel == "binned":
        monkeypatch.setenv("SLAM2D_UPDATE", "binned")
    _run_pair(2, 512, scans, n_scans=12, thresholds=thresholds, stream=3)


@pytest.mark.parametrize("cap_env", ["SLAM2D_SEG_CAP", "SLAM2D_ITEM_CAP"])
def test_unbinned_fallback_bitexact(gpu, scans, monkeypatch, cap_env):
    """Binned path, queue overflow -> WHOLE items (every ray against every tile of the level's bbox)."""
    monkeypatch.setenv("SLAM2D_UPDATE", "binned")
    monkeypatch.setenv(cap_env, "8")
    fleet, _ = _run_pair(2, 1024, scans, n_scans=8, thresholds=(-1.0, -1.0), stream=2)
    q = fleet.queue_stats()
    assert q["whole"] > 0 and q["overflow"] > 0, q


@pytest.mark.parametrize("parts", ["1", "2"])
def test_binned_path_bitexact(gpu, scans, monkeypatch, parts):
    """Alternative update path: hs_bin_kernel + hs_tile_kernel (SLAM2D_UPDATE=binned)."""
    monkeypatch.setenv("SLAM2D_UPDATE", "binned")
    monkeypatch.setenv("SLAM2D_PARTS", parts)
    fleet, _ = _run_pair(3, 2048, scans, n_scans=10, thresholds=(-1.0, -1.0), stream=1)
    q = fleet.queue_stats()
    assert q["whole"] == 0 and q["overflow"] == 0 and q["items"] > 0, q


def test_tree_order_opt_in(gpu, scans):
    """HS_ORDER_TREE256: bit-exact vs the oracle's tree order, within the pose tolerance of the reference
    order; switching back restores the reference order."""
    n = 30
    fleet = HectorFleet(1, 0.05, 2048, (0.5, 0.5), 3, max_points=1081)
    assert fleet.reduction_order() == HectorFleet.ORDER_REFERENCE
    fleet.set_reduction_order(HectorFleet.ORDER_TREE256)
    assert fleet.reduction_order() == HectorFleet.ORDER_TREE256
    tree = O.HectorOracle(0.05, 2048, (0.5, 0.5), 3, reduce_threads=256)
    ref = O.HectorOracle(0.05, 2048, (0.5, 0.5), 3, reduce_threads=0)
    for f in (fleet, tree, ref):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(0.4, 0.9)
    errs = []
    for k in range(n):
        pts = scans.points[0, k, : scans.counts[0, k]]
        gp, _, _ = fleet.update(0, pts)
        tp, _, _ = tree.process(pts)
        rp, _, _ = ref.process(pts)
        np.testing.assert_array_equal(_bits(gp), _bits(tp), err_msg=f"scan {k}")
        errs.append(np.abs(gp.astype(np.float64) - rp.astype(np.float64)))
    e = np.max(errs, axis=0)
    assert e[0] <= POSE_TOL_M and e[1] <= POSE_TOL_M and e[2] <= POSE_TOL_RAD, e
    with pytest.raises(Exception):
        fleet.set_reduction_order(128)


def test_match_only_and_update_by_scan(gpu, scans):
    """MapRepresentationInterface::matchData / updateByScan entry points."""
    fleet = HectorFleet(1, 0.05, 1024, (0.5, 0.5), 2, max_points=1081)
    ora = O.HectorOracle(0.05, 1024, (0.5, 0.5), 2, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
    pose = np.zeros(3, np.float32)
    for k in range(8):
        pts = scans.points[0, k, : scans.counts[0, k]]
        gp, gc = fleet.match(0, pts, pose)
        op, oc = ora.match(pts, pose)
        np.testing.assert_array_equal(_bits(gp), _bits(op))
        np.testing.assert_array_equal(_bits(gc), _bits(oc))
        fleet.update_by_scan(0, pts, gp)
        ora.update_by_scan(pts, op)
        pose = op
    for lvl in range(2):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou)
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


def test_map_without_matching_and_empty_scan(gpu, scans):
    fleet = HectorFleet(1, 0.05, 512, (0.5, 0.5), 1, max_points=1081)
    ora = O.HectorOracle(0.05, 512, (0.5, 0.5), 1, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(0.4, 0.9)
    hint = np.array([0.1, -0.05, 0.02], np.float32)
    pts = scans.points[0, 0, : scans.counts[0, 0]]
    gp, _, gd = fleet.update(0, pts, hint=hint, map_without_matching=True)
    op, _, od = ora.process(pts, hint=hint, map_without_matching=True)
    assert gd and od
    np.testing.assert_array_equal(_bits(gp), _bits(op))
    # empty scan: pose = hint, no GN step (ScanMatcher.h:65, :96)
    e = np.zeros((0, 2), np.float32)
    gp, _, gd = fleet.update(0, e, hint=hint)
    op, _, od = ora.process(e, hint=hint)
    np.testing.assert_array_equal(_bits(gp), _bits(op))
    assert gd == od
    m = fleet.get_map(0, 0)
    ol, ou = ora.level(0)
    np.testing.assert_array_equal(m["upd"], ou)
    np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


def _same_levels(fleet, ora, levels, what=""):
    for lvl in range(levels):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou, err_msg=f"{what} level {lvl} updateIndex")
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol), err_msg=f"{what} level {lvl} log-odds")
        assert m["update_index"] == ora.update_index(lvl), (what, lvl)


@pytest.mark.parametrize("levels", [2, 3])
def test_map_without_matching_stored_containers(gpu, scans, levels):
    """MapRepMultiMap keeps the container of the last matchData (setFrom, MapRepMultiMap.h:161) and
    updateByScan draws THAT into levels >= 1 (:187): HectorSlamProcessor::update(map_without_matching)
    updates level 0 with the new scan and the coarse levels with the previously matched one -- nothing at
    all before the first match.  Bit-exact vs the oracle, which keeps the same state."""
    size = 1024
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), levels, max_points=1081)
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), levels, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(0.4, 0.9)
    hint = np.array([0.1, -0.05, 0.02], np.float32)
    a = scans.points[1, 0, : scans.counts[1, 0]]
    b = scans.points[1, 5, : scans.counts[1, 5]]
    c = scans.points[2, 9, : scans.counts[2, 9]]
    # first call: no match yet, the coarse levels get an empty container (index advance only)
    gp, _, gd = fleet.update(0, a, origo=(0.5, -0.25), hint=hint, map_without_matching=True)
    op, _, od = ora.process(a, origo=(0.5, -0.25), hint=hint, map_without_matching=True)
    assert gd and od
    np.testing.assert_array_equal(_bits(gp), _bits(op))
    _same_levels(fleet, ora, levels, "first call")
    assert (fleet.get_map(0, 1)["upd"] >= 0).sum() == 0  # nothing drawn into level 1
    # a match of scan b (own origo), then map_without_matching with scan c: coarse levels draw b
    gp, gc = fleet.match(0, b, hint, origo=(-0.75, 0.3))
    op, oc = ora.match(b, hint, origo=(-0.75, 0.3))
    np.testing.assert_array_equal(_bits(gp), _bits(op))
    np.testing.assert_array_equal(_bits(gc), _bits(oc))
    pose = np.array([0.3, 0.2, -0.4], np.float32)
    for k in range(2):
        gp, _, gd = fleet.update(0, c, hint=pose, map_without_matching=True)
        op, _, od = ora.process(c, hint=pose, map_without_matching=True)
        assert gd and od
        np.testing.assert_array_equal(_bits(gp), _bits(op))
        _same_levels(fleet, ora, levels, f"after match, call {k}")
    # a full update (match + gate) re-stores its own scan
    gp, _, gd = fleet.update(0, a)
    op, _, od = ora.process(a)
    assert gd == od
    np.testing.assert_array_equal(_bits(gp), _bits(op))
    gp, _, _ = fleet.update(0, b, hint=pose, map_without_matching=True)
    op, _, _ = ora.process(b, hint=pose, map_without_matching=True)
    _same_levels(fleet, ora, levels, "after a full update")


def test_update_by_scan_after_match_of_other_scan(gpu, scans):
    """hs_update_by_scan after hs_match on different data: level 0 from the given scan, levels >= 1 from
    the matched one (MapRepMultiMap.h:174-191)."""
    levels = 3
    fleet = HectorFleet(1, 0.05, 1024, (0.5, 0.5), levels, max_points=1081)
    ora = O.HectorOracle(0.05, 1024, (0.5, 0.5), levels, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
    # before any match: coarse levels untouched
    a = scans.points[3, 2, : scans.counts[3, 2]]
    pose = np.array([0.05, 0.02, 0.1], np.float32)
    fleet.update_by_scan(0, a, pose, origo=(0.1, 0.1))
    ora.update_by_scan(a, pose, origo=(0.1, 0.1))
    _same_levels(fleet, ora, levels, "before a match")
    for k in range(4):
        m = scans.points[0, k, : scans.counts[0, k]]
        u = scans.points[3, 10 + k, : scans.counts[3, 10 + k]]
        gp, _ = fleet.match(0, m, pose, origo=(0.2 * k, -0.1))
        op, _ = ora.match(m, pose, origo=(0.2 * k, -0.1))
        np.testing.assert_array_equal(_bits(gp), _bits(op))
        fleet.update_by_scan(0, u, op, origo=(-0.3, 0.05 * k))
        ora.update_by_scan(u, op, origo=(-0.3, 0.05 * k))
        _same_levels(fleet, ora, levels, f"round {k}")


def test_degenerate_rays(gpu):
    """Zero-length beams (begin == end, skipped), 1-cell rays, rays along axes and diagonals."""
    pts = []
    for r in (0.0, 0.3, 0.6, 1.0, 1.5, 7.0, 40.0):
        for a in np.linspace(-np.pi, np.pi, 37):
            pts.append((r * np.cos(a), r * np.sin(a)))
    pts += [(5.0, 0.0), (0.0, 5.0), (-5.0, 0.0), (0.0, -5.0), (5.0, 5.0), (-5.0, 5.0), (5.0, -5.0), (-5.0, -5.0)]
    pts = np.asarray(pts, np.float32)
    fleet = HectorFleet(1, 0.05, 128, (0.5, 0.5), 2, max_points=len(pts))
    ora = O.HectorOracle(0.05, 128, (0.5, 0.5), 2, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    for k, pose in enumerate([(0.0, 0.0, 0.0), (0.013, -0.021, 0.3), (0.4, 0.2, -1.2), (-1.0, 1.0, 2.9)]):
        pose = np.asarray(pose, np.float32)
        fleet.update_by_scan(0, pts, pose, origo=(0.2 * k, -0.1 * k))
        ora.update_by_scan(pts, pose, origo=(0.2 * k, -0.1 * k))
    for lvl in range(2):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou)
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


def test_long_rays_over_16384_cells(gpu):
    """Rays longer than 16384 cells (a 16640 x 64 map, the robot near its left end): the default update
    kernel's packed walk holds the Bresenham error in 14 bits, so the host sends such maps to the binned
    kernels (upd_single_ok); the result must still equal the oracle cell for cell."""
    sx, sy = 16640, 64
    # DataContainer points are in map scale (cells of level 0, hector_slam.cc:356): 16434 cells = 821.7 m
    pts = [(16434.0, 6.0), (16434.0, -24.0), (14000.0, 18.0), (-100.0, 4.0), (60.0, 20.0), (10.0, -30.0)]
    pts = np.asarray(pts, np.float32)
    fleet = HectorFleet(1, 0.05, sx, (0.01, 0.5), 2, max_points=len(pts), map_size_y=sy)
    ora = O.HectorOracle(0.05, sx, (0.01, 0.5), 2, reduce_threads=T_RED, map_size_y=sy)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    for k, pose in enumerate([(0.0, 0.0, 0.0), (0.5, 0.3, 0.001), (-0.2, -0.1, -0.0004)]):
        pose = np.asarray(pose, np.float32)
        fleet.update_by_scan(0, pts, pose)
        ora.update_by_scan(pts, pose)
    ctr = fleet.counters(reset=False)
    assert ctr["cells"] > 3 * 16384, ctr  # the long rays were drawn
    for lvl in range(2):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou, err_msg=f"level {lvl}")
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol), err_msg=f"level {lvl}")


def test_big_level_gathers_bitexact(gpu, scans):
    """A level of more than 2^30 storage words (32768 x 13184 cells at level 0: 210944 tiles x 5120 words): the
    match's gathers would overflow their 32-bit byte offsets from the level base, so the host launches the
    64-bit-address instance (hs_match_kernel BIG).  Every matched pose, covariance and gate equals the oracle."""
    sx, sy = 32768, 13184
    fleet = HectorFleet(1, 0.05, sx, (0.5, 0.5), 2, max_points=1081, map_size_y=sy)
    ora = O.HectorOracle(0.05, sx, (0.5, 0.5), 2, reduce_threads=T_RED, map_size_y=sy)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(0.4, 0.9)
    for k in range(8):
        pts = scans.points[1, k, : scans.counts[1, k]]
        gp, gc, gd = fleet.update(0, pts, (0.0, 0.0))
        op, oc, od = ora.process(pts, (0.0, 0.0))
        assert gd == od, f"scan {k}: did_update {gd} vs {od}"
        np.testing.assert_array_equal(_bits(gp), _bits(op), err_msg=f"scan {k} pose")
        np.testing.assert_array_equal(_bits(gc), _bits(oc), err_msg=f"scan {k} cov")
    fleet.close()
    ora.close()


def test_reset(gpu, scans):
    """HectorSlamProcessor::reset (HectorSlamProcessor.h:111-117): grids cleared and poses reset; the grids'
    update indices (GridMapBase::reset clears cells only), the covariance and the stored containers stay
    -- so later updates index cells exactly as the reference does."""
    fleet = HectorFleet(1, 0.05, 256, (0.5, 0.5), 2, max_points=1081)
    ora = O.HectorOracle(0.05, 256, (0.5, 0.5), 2, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    for k in range(3):
        pts = scans.points[0, k, : scans.counts[0, k]]
        fleet.update(0, pts)
        ora.process(pts)
    fleet.reset()
    ora.reset()
    m = fleet.get_map(0, 0)
    assert np.all(m["logodds"] == 0.0) and np.all(m["upd"] == -1)
    assert m["update_index"] == ora.update_index(0) == 2
    assert np.all(fleet.last_pose(0)[0] == 0.0)
    np.testing.assert_array_equal(_bits(fleet.last_pose(0)[1]), _bits(ora.last_cov()))
    # map_without_matching right after reset: coarse level draws the container stored before it
    pts = scans.points[0, 4, : scans.counts[0, 4]]
    hint = np.array([0.02, 0.01, 0.0], np.float32)
    fleet.update(0, pts, hint=hint, map_without_matching=True)
    ora.process(pts, hint=hint, map_without_matching=True)
    for k in range(5, 8):
        pts = scans.points[0, k, : scans.counts[0, k]]
        gp, _, _ = fleet.update(0, pts)
        op, _, _ = ora.process(pts)
        np.testing.assert_array_equal(_bits(gp), _bits(op))
    _same_levels(fleet, ora, 2, "after reset")


@pytest.mark.parametrize("sweep", ["1", "2", "3"])
def test_reset_mid_run_with_sweeps(gpu, scans, monkeypatch, sweep):
    """hs_reset between ordinal sweeps: the reset keeps the stream's update index and ordinal epoch
    (GridMapBase::reset clears cells only) while the fill zeroes the hot ordinals and the cold plane, so the
    updates after it must decode to the reference's updateIndex whatever the sweep phase -- every cell of both
    levels bit-exact before and after the reset, with a sweep every 1, 2 or 3 steps."""
    monkeypatch.setenv("SLAM2D_ORD_SWEEP", sweep)
    fleet = HectorFleet(1, 0.05, 512, (0.5, 0.5), 2, max_points=1081)
    ora = O.HectorOracle(0.05, 512, (0.5, 0.5), 2, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    for k in range(4):
        pts = scans.points[1, k, : scans.counts[1, k]]
        fleet.update(0, pts)
        ora.process(pts)
    _same_levels(fleet, ora, 2, "before reset")
    fleet.reset()
    ora.reset()
    for k in range(4, 9):
        pts = scans.points[1, k, : scans.counts[1, k]]
        gp, _, _ = fleet.update(0, pts)
        op, _, _ = ora.process(pts)
        np.testing.assert_array_equal(_bits(gp), _bits(op), err_msg=f"scan {k} after reset")
    _same_levels(fleet, ora, 2, "after reset")


def _dev_bytes(ptr, nbytes):
    """nbytes of device memory at ptr, copied to the host with hipMemcpy (after a device synchronisation)."""
    import ctypes

    import torch

    torch.cuda.synchronize()
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    out = np.empty(nbytes, np.uint8)
    rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2)
    assert rc == 0, rc
    return out


def test_flush_ordinals_zero_copy(gpu, scans):
    """hs_flush_ordinals: after it every 16-bit ordinal of the device cell storage is 0 and the int32
    plane alone holds each cell's updateIndex, so a zero-copy reader of hs_get_device_buffers decodes without the
    internal epoch: level 0 read raw from the device equals hs_get_map (log-odds and updateIndex); further updates
    after the flush stay bit-exact vs the oracle."""
    fleet = HectorFleet(1, 0.05, 512, (0.5, 0.5), 2, max_points=1081)
    ora = O.HectorOracle(0.05, 512, (0.5, 0.5), 2, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    for k in range(6):
        pts = scans.points[2, k, : scans.counts[2, k]]
        fleet.update(0, pts)
        ora.process(pts)
    want = fleet.get_map(0, 0)
    fleet.flush_ordinals()
    ptr, _, _ = fleet.device_cells()
    sx, sy, _, _ = fleet.map_info(0)
    tx, ty = (sx + 63) // 64, (sy + 31) // 32
    raw = _dev_bytes(ptr, tx * ty * 20480).view(np.int32).reshape(ty, tx, 5120)  # level 0 is first in the stream
    y, x = np.mgrid[0:sy, 0:sx]
    e = ((y % 32) // 4 * 16 + (x % 64) // 4) * 16 + (y % 4) * 4 + x % 4  # element of the cell in its tile's planes
    tile = raw[y // 32, x // 64]
    logodds = np.take_along_axis(tile[..., :2048], e[..., None], -1)[..., 0]
    ords = tile[..., 2048:3072].copy().view(np.uint16)
    cold = np.take_along_axis(tile[..., 3072:], e[..., None], -1)[..., 0]
    assert not ords.any(), "hot ordinals left after hs_flush_ordinals"
    np.testing.assert_array_equal(cold, want["upd"])
    np.testing.assert_array_equal(logodds, _bits(want["logodds"]))
    for k in range(6, 9):
        pts = scans.points[2, k, : scans.counts[2, k]]
        gp, _, _ = fleet.update(0, pts)
        op, _, _ = ora.process(pts)
        np.testing.assert_array_equal(_bits(gp), _bits(op), err_msg=f"scan {k} after flush")
    _same_levels(fleet, ora, 2, "after flush")


def test_ordinal_overflow_is_refused(gpu, monkeypatch):
    """A caller that never lets the library sweep (SLAM2D_ORD_SWEEP=0: the test knob standing for replayed graph
    captures of *_device calls) drives a stream past 32767 map updates in one ordinal epoch: the device flags the
    stream and hs_get_map refuses its updateIndex (HS_ESTATE) instead of decoding wrapped 16-bit ordinals; hs_reset
    starts a fresh epoch, after which updates decode bit-exact vs the oracle again."""
    import torch

    monkeypatch.setenv("SLAM2D_ORD_SWEEP", "0")
    size, n = 64, 16
    a = np.linspace(0.0, 2 * np.pi, n, endpoint=False)
    pts = (np.stack([np.cos(a), np.sin(a)], 1) * 20.0).astype(np.float32)  # map scale: 1 m rays on a 3.2 m map
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), 1, max_points=n)
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), 1, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    d_xy = torch.from_numpy(pts[None]).cuda()
    d_n = torch.tensor([n], dtype=torch.int32).cuda()
    steps = 32768  # the update k = 32767 needs ordinal 2 k + 2 = 65536
    for _ in range(steps):
        fleet.step_device(d_xy.data_ptr(), n, d_n.data_ptr())
        ora.process(pts)
    torch.cuda.synchronize()
    with pytest.raises(Exception, match="code -5"):
        fleet.get_map(0, 0)
    fleet.reset()
    ora.reset()
    for _ in range(3):
        fleet.update(0, pts)
        ora.process(pts)
    _same_levels(fleet, ora, 1, "after overflow + reset")


@pytest.mark.parametrize("parts", ["1", "2"])
def test_ordinal_sweep_part_streams(gpu, monkeypatch, parts):
    """The ordinal sweep on the batched issue path with the fleet split over part streams (SLAM2D_PARTS=2: the
    sweep runs on the context's stream before ev_start fans the step out to the part streams), a sweep
    every 2 steps, 128 streams x 5 steps at 512^2 x 2 levels: poses of every step and every cell of sampled streams
    bit-exact vs the oracle."""
    import torch

    monkeypatch.setenv("SLAM2D_ORD_SWEEP", "2")
    monkeypatch.setenv("SLAM2D_PARTS", parts)
    B, T = 128, 5
    S = synth.make_streams(B, T, seed=71)
    fleet = HectorFleet(B, 0.05, 512, (0.5, 0.5), 2, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    check = [0, 63, 64, B - 1]  # both halves of a two-part split
    oras = {s: O.HectorOracle(0.05, 512, (0.5, 0.5), 2, reduce_threads=T_RED) for s in check}
    for o in oras.values():
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(-1.0, -1.0)
    for t in range(T):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(S.counts[:, t].astype(np.int32))
        fleet.step_device(d_xy.data_ptr(), 1081, d_n.data_ptr())
        torch.cuda.synchronize()
        gp = fleet.poses()[0]
        for s in check:
            op, _, _ = oras[s].process(S.points[s, t, : S.counts[s, t]])
            np.testing.assert_array_equal(_bits(gp[s]), _bits(op), err_msg=f"t={t} s={s}")
    for s in check:
        for lvl in range(2):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            np.testing.assert_array_equal(m["upd"], ou, err_msg=f"s={s} level {lvl} updateIndex")
            np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol), err_msg=f"s={s} level {lvl} log-odds")


def test_processor_mirror(gpu, scans):
    """HectorSlamProcessor mirror (reference API names) over DataContainer."""
    proc = HectorSlamProcessor(0.05, 1024, 1024, (0.5, 0.5), 2, max_points=1081)
    proc.setUpdateFactorFree(0.4)
    proc.setUpdateFactorOccupied(0.9)
    proc.setMapUpdateMinDistDiff(0.4)
    proc.setMapUpdateMinAngleDiff(0.9)
    ora = O.HectorOracle(0.05, 1024, (0.5, 0.5), 2, reduce_threads=T_RED)
    ora.set_update_factors(0.4, 0.9)
    ora.set_thresholds(0.4, 0.9)
    for k in range(10):
        dc = DataContainer.from_points(scans.points[1, k, : scans.counts[1, k]])
        p = proc.update(dc, proc.getLastScanMatchPose())
        op, _, _ = ora.process(dc.points())
        np.testing.assert_array_equal(_bits(p), _bits(op))
    assert proc.getMapLevels() == 2 and proc.getScaleToMap() == 20.0
    g = proc.getGridMap(0)
    np.testing.assert_array_equal(g["occ"], ora.publish(0))


def _torch_dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_batched_device_ragged(gpu):
    """hs_step_batch_device over B streams with ragged scan sizes (incl. an empty scan) == per-stream oracle."""
    import torch

    B, T = 6, 12
    S = synth.make_streams(B, T, seed=777)
    counts = S.counts.copy()
    counts[2, 5] = 0             # empty scan
    counts[4, :] = np.minimum(counts[4, :], 300)  # truncated scans
    fleet = HectorFleet(B, 0.05, 1024, (0.5, 0.5), 2, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(0.4, 0.9)
    oras = []
    for s in range(B):
        o = O.HectorOracle(0.05, 1024, (0.5, 0.5), 2, reduce_threads=T_RED)
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(0.4, 0.9)
        oras.append(o)
    stride = 1081
    for t in range(T):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(counts[:, t].astype(np.int32))
        fleet.step_device(d_xy.data_ptr(), stride, d_n.data_ptr())
        torch.cuda.synchronize()
        gp, gc, gd, cells = fleet.poses()
        for s in range(B):
            pts = S.points[s, t, : counts[s, t]]
            op, oc, od = oras[s].process(pts)
            assert gd[s] == od, (t, s)
            np.testing.assert_array_equal(_bits(gp[s]), _bits(op), err_msg=f"t={t} s={s}")
            if od:
                assert cells[s] == oras[s].sum_L(), (t, s, cells[s], oras[s].sum_L())
    for s in range(B):
        for lvl in range(2):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            np.testing.assert_array_equal(m["upd"], ou, err_msg=f"s={s} lvl={lvl}")
            np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol), err_msg=f"s={s} lvl={lvl}")


# ----------------------------------------------------------------------------- golden fixtures on the GPU
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(GOLD) if f.startswith("hector_")))
def test_golden_fixture(gpu, name):
    """Committed oracle fixtures (tests/golden, oracle/make_golden.py) replayed through the C-ABI.
    The fleet runs in the fixture's summation order (reference sequential / tree 256); everything must
    match bit for bit (NaN == NaN for the diverging case)."""
    d = np.load(os.path.join(GOLD, name))
    levels, size = int(d["levels"]), int(d["size"])
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), levels, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(*[float(v) for v in d["thresholds"]])
    # the fixture's summation order: reference (0) by default, the tree (256) opt-in
    fleet.set_reduction_order(int(d["reduce_threads"]))
    exact = True
    for k in range(len(d["counts"])):
        gp, gc, gd = fleet.update(0, d["points"][k, : d["counts"][k]])
        if exact:
            assert gd == bool(d["did_update"][k]), k
            np.testing.assert_array_equal(gp, d["poses"][k], err_msg=f"scan {k}")
            np.testing.assert_array_equal(gc, d["covs"][k], err_msg=f"scan {k}")
            if gd:
                assert fleet.poses()[3][0] == int(d["sum_L"][k]), k
        else:
            e = np.abs(gp.astype(np.float64) - d["poses"][k].astype(np.float64))
            assert e[0] <= POSE_TOL_M and e[1] <= POSE_TOL_M and e[2] <= POSE_TOL_RAD, (k, e)
    if exact:
        for lvl in range(levels):
            m = fleet.get_map(0, lvl)
            idx = np.nonzero(m["upd"].ravel() >= 0)[0]
            np.testing.assert_array_equal(idx, d[f"l{lvl}_idx"])
            np.testing.assert_array_equal(_bits(m["logodds"].ravel()[idx]), d[f"l{lvl}_logodds_bits"])
            np.testing.assert_array_equal(m["upd"].ravel()[idx], d[f"l{lvl}_upd"])
            np.testing.assert_array_equal(m["occ"].ravel()[idx], d[f"l{lvl}_publish"])
            assert m["update_index"] == int(d[f"l{lvl}_update_index"])


def _pair_small(size=64, levels=1):
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), levels, max_points=64)
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), levels, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
    return fleet, ora


def _same_level(fleet, ora, lvl=0):
    m = fleet.get_map(0, lvl)
    ol, ou = ora.level(lvl)
    np.testing.assert_array_equal(m["upd"], ou)
    np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


def test_once_per_scan_hand_built(gpu):
    """The hand-derived once-per-scan sequences of tests/test_oracle_cpu.py on the GPU."""
    fleet, ora = _pair_small()
    pose = np.zeros(3, np.float32)
    for pts in (np.array([[10.0, 0.0]], np.float32),
                np.array([[10.0, 0.0], [5.0, 0.0], [13.0, 0.0], [12.0, 0.0], [8.0, 0.0], [10.0, 0.0]], np.float32)):
        fleet.update_by_scan(0, pts, pose)
        ora.update_by_scan(pts, pose)
        _same_level(fleet, ora)


def test_occupied_clamp_at_50(gpu):
    fleet, ora = _pair_small()
    l, u = ora.level(0)
    l = l.copy()
    l[32, 40], l[32, 41], l[32, 36] = 49.9, 50.0, 1e30
    ora.set_level(0, l, u)
    fleet.set_map(0, 0, l, u)
    pose = np.zeros(3, np.float32)
    for pts in (np.array([[8.0, 0.0]], np.float32), np.array([[9.0, 0.0], [4.0, 0.0]], np.float32)):
        fleet.update_by_scan(0, pts, pose)
        ora.update_by_scan(pts, pose)
        _same_level(fleet, ora)


def test_nan_pose_is_out_of_map(gpu):
    """A diverged pose must not write any cell (GPU float->int would otherwise map NaN to cell 0)."""
    fleet, ora = _pair_small(128, 2)
    pts = np.array([[10.0, 0.0], [0.0, 7.0], [-3.0, -3.0]], np.float32)
    for pose in (np.array([np.nan, 0.0, 0.0], np.float32), np.array([0.0, 0.0, np.nan], np.float32)):
        fleet.update_by_scan(0, pts, pose)
        ora.update_by_scan(pts, pose)
    for lvl in range(2):
        _same_level(fleet, ora, lvl)
        assert (fleet.get_map(0, lvl)["upd"] >= 0).sum() == 0
    gp, _ = fleet.match(0, pts, np.array([np.nan] * 3, np.float32))
    assert np.isnan(gp).all()


# ----------------------------------------------------------------------------- scan-size edge cases
@pytest.mark.parametrize("n_beams,levels,size", [(2400, 3, 1024), (6000, 2, 1024), (16000, 2, 512)])
def test_dense_scans_bitexact(gpu, n_beams, levels, size):
    """Scans larger than the match kernel's register-resident points (> 1280: the strided loop); at 6000
    beams more than 64 fan groups, so the clip update's groups past the ballot's first 64 take its scalar
    box-test path; and at 16000 beams, larger than the single-kernel update's LDS budget (the binned update
    takes over): poses, gate and maps bit-exact vs the oracle."""
    S = synth.make_streams(1, 6, seed=4711, n_beams=n_beams)
    fleet = HectorFleet(1, 0.05, size, (0.5, 0.5), levels, max_points=n_beams)
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), levels, reduce_threads=T_RED)
    for f in (fleet, ora):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
    assert S.counts.max() > 1280
    for k in range(6):
        pts = S.points[0, k, : S.counts[0, k]]
        gp, _, gd = fleet.update(0, pts)
        op, _, od = ora.process(pts)
        assert gd == od
        np.testing.assert_array_equal(_bits(gp), _bits(op), err_msg=f"scan {k}")
    for lvl in range(levels):
        m = fleet.get_map(0, lvl)
        ol, ou = ora.level(lvl)
        np.testing.assert_array_equal(m["upd"], ou)
        np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


@pytest.mark.parametrize("B", [40, 600])
def test_batch_sizes_across_split_rules(gpu, B):
    """The update's batch-adaptive tile split (B = 40: 25 level-0 workgroups per stream; B = 600: 2) vs
    the oracle on a sample of streams, 3 steps, 3 levels: poses and maps bit-exact."""
    import torch

    T = 3
    S = synth.make_streams(B, T, seed=99)
    fleet = HectorFleet(B, 0.05, 1024, (0.5, 0.5), 3, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    check = [0, 1, B // 2, B - 1]
    oras = {s: O.HectorOracle(0.05, 1024, (0.5, 0.5), 3, reduce_threads=T_RED) for s in check}
    for o in oras.values():
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(-1.0, -1.0)
    for t in range(T):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(S.counts[:, t].astype(np.int32))
        fleet.step_device(d_xy.data_ptr(), 1081, d_n.data_ptr())
        torch.cuda.synchronize()
        gp = fleet.poses()[0]
        for s in check:
            op, _, _ = oras[s].process(S.points[s, t, : S.counts[s, t]])
            np.testing.assert_array_equal(_bits(gp[s]), _bits(op), err_msg=f"t={t} s={s}")
    for s in check:
        for lvl in range(3):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            np.testing.assert_array_equal(m["upd"], ou)
            np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))


@pytest.mark.parametrize("split", ["", "1,1,1", "6,3,2"])
def test_ring_kernel_equals_clip_kernel(gpu, monkeypatch, split):
    """The round-4 ring-ordered cursor update (opt-in, SLAM2D_UPD_KERNEL=ring) and the per-tile clipping kernel
    (default) on the same 96-stream fleet, 4 steps, 2048^2 x 3 levels: every stream's pose and
    every cell of sampled streams identical -- including ring-range parts (SLAM2D_UPD_SPLIT)."""
    import torch

    B, T = 96, 4
    S = synth.make_streams(B, T, seed=31)
    if split:
        monkeypatch.setenv("SLAM2D_UPD_SPLIT", split)
    fleets = {}
    for kern in ("ring", "clip"):
        monkeypatch.setenv("SLAM2D_UPD_KERNEL", kern)
        f = HectorFleet(B, 0.05, 2048, (0.5, 0.5), 3, max_points=1081)
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
        fleets[kern] = f
    monkeypatch.delenv("SLAM2D_UPD_KERNEL", raising=False)
    for t in range(T):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(S.counts[:, t].astype(np.int32))
        for f in fleets.values():
            f.step_device(d_xy.data_ptr(), 1081, d_n.data_ptr())
        torch.cuda.synchronize()
        pr, pc = fleets["ring"].poses()[0], fleets["clip"].poses()[0]
        np.testing.assert_array_equal(_bits(pr), _bits(pc), err_msg=f"step {t}")
    cr, cc = fleets["ring"].counters(reset=False), fleets["clip"].counters(reset=False)
    assert cr["cells"] == cc["cells"] and cr["touched"] == cc["touched"], (cr, cc)
    for s in (0, 47, B - 1):
        for lvl in range(3):
            mr, mc = fleets["ring"].get_map(s, lvl), fleets["clip"].get_map(s, lvl)
            np.testing.assert_array_equal(mr["upd"], mc["upd"], err_msg=f"s={s} lvl={lvl}")
            np.testing.assert_array_equal(_bits(mr["logodds"]), _bits(mc["logodds"]), err_msg=f"s={s} lvl={lvl}")


def test_clock_probe(gpu):
    """hs_set_clock_probe: the sampled workgroups of both kernels report a plausible shader clock."""
    import torch

    B = 64
    S = synth.make_streams(B, 3, seed=5)
    fleet = HectorFleet(B, 0.05, 1024, (0.5, 0.5), 2, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    fleet.set_clock_probe(True)
    fleet.clock_probe(reset=True)
    for t in range(3):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(S.counts[:, t].astype(np.int32))
        fleet.step_device(d_xy.data_ptr(), 1081, d_n.data_ptr())
    torch.cuda.synchronize()
    c = fleet.clock_probe(reset=True)
    fleet.set_clock_probe(False)
    for k in ("match", "update"):
        assert c[k]["workgroups_sampled"] > 0, c
        assert 300.0 < c[k]["sclk_mhz"] < 3000.0, c


@pytest.mark.parametrize("pad", ["4352", "69888"])
def test_stream_pad_layout(gpu, monkeypatch, pad):
    """SLAM2D_STREAM_PAD staggers the streams' blocks in memory: reset fills the planes per stream, and 3
    streams x 4 steps stay bit-exact vs the oracle (poses and both planes of every level)."""
    import torch

    monkeypatch.setenv("SLAM2D_STREAM_PAD", pad)
    B, T = 3, 4
    S = synth.make_streams(B, T, seed=17)
    fleet = HectorFleet(B, 0.05, 512, (0.5, 0.5), 2, max_points=1081)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    oras = [O.HectorOracle(0.05, 512, (0.5, 0.5), 2, reduce_threads=T_RED) for _ in range(B)]
    for o in oras:
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(-1.0, -1.0)
    for t in range(T):
        d_xy = _torch_dev(S.points[:, t])
        d_n = _torch_dev(S.counts[:, t].astype(np.int32))
        fleet.step_device(d_xy.data_ptr(), 1081, d_n.data_ptr())
        torch.cuda.synchronize()
        gp = fleet.poses()[0]
        for s in range(B):
            op, _, _ = oras[s].process(S.points[s, t, : S.counts[s, t]])
            np.testing.assert_array_equal(_bits(gp[s]), _bits(op), err_msg=f"t={t} s={s}")
    for s in range(B):
        for lvl in range(2):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            np.testing.assert_array_equal(m["upd"], ou)
            np.testing.assert_array_equal(_bits(m["logodds"]), _bits(ol))
