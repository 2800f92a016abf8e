"""GPU parity of the on-device scan ingest:
HectorMappingRos::scanCallback's projectLaser + rosPointCloudToDataContainer
(lesson4/src/hector_mapping/hector_slam.cc:186-198, 320-362) as hs_ingest_kernel, against the C
restatement oracle.ingest.  Bar: bit-exact (point count, every float bit of every point, origo).
laser_geometry itself is absent (third party), so the projectLaser step is parity unpinned; the
node-side filters are restated from the reference file line by line.
"""
import math

import numpy as np
import pytest

import oracle as O
from slam2d import synth
from slam2d.hector import HectorFleet, HsLaser

pytestmark = pytest.mark.gpu

N = 1081
AMIN = np.float32(-3.0 * math.pi / 4.0)
AINC = np.float32(math.radians(0.25))


def _roll_pi_laser(n=N):
    """hector_slam.launch's static TF: x y z yaw pitch roll = 0 0 0.254 0 0 3.1415926."""
    L = HsLaser.defaults(n, float(AMIN), float(AINC))
    r = 3.1415926
    c, s = math.cos(r), math.sin(r)
    basis = [1.0, 0.0, 0.0, 0.0, c, -s, 0.0, s, c]
    for i, v in enumerate(basis):
        L.basis[i] = v
    L.origin[0], L.origin[1], L.origin[2] = 0.0, 0.0, 0.254
    return L


def _tilted_laser(n=N):
    """A pitched, offset laser: z of far points leaves (-1, 1), exercising the z filter (:351-353)."""
    L = HsLaser.defaults(n, float(AMIN), float(AINC))
    p = 0.08
    c, s = math.cos(p), math.sin(p)
    basis = [c, 0.0, s, 0.0, 1.0, 0.0, -s, 0.0, c]
    for i, v in enumerate(basis):
        L.basis[i] = v
    L.origin[0], L.origin[1], L.origin[2] = 0.31, -0.07, 0.4
    L.range_min = 0.05
    return L


def _edge_ranges(rng, B, n=N):
    """Ranges hitting every branch: NaN / inf / negative, below range_min, around 0.2 m, the
    x < 0 && d^2 < 0.5 cut (rear beams under 0.707 m), around 20 m and 30 m."""
    r = rng.uniform(0.0, 32.0, size=(B, n)).astype(np.float32)
    pick = rng.integers(0, 9, size=(B, n))
    r[pick == 0] = np.nan
    r[pick == 1] = np.inf
    r[pick == 2] = rng.uniform(0.15, 0.25, size=int((pick == 2).sum())).astype(np.float32)
    r[pick == 3] = rng.uniform(0.6, 0.8, size=int((pick == 3).sum())).astype(np.float32)
    r[pick == 4] = rng.uniform(19.9, 20.1, size=int((pick == 4).sum())).astype(np.float32)
    r[pick == 5] = rng.uniform(29.9, 30.1, size=int((pick == 5).sum())).astype(np.float32)
    r[pick == 6] = -1.0
    r[:, :8] = np.float32(30.0)   # exactly the cutoff: dropped (range < cutoff)
    r[:, 8:16] = np.float32(20.0)
    return r


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.mark.parametrize("make_laser", [_roll_pi_laser, _tilted_laser, None])
def test_ingest_batch_bitexact(gpu, make_laser):
    import torch
    B = 64
    L = make_laser() if make_laser else HsLaser.defaults(N, float(AMIN), float(AINC))
    fleet = HectorFleet(B, 0.05, 256, (0.5, 0.5), 1, max_points=N)
    fleet.set_laser(L)
    rng = np.random.default_rng(4242)
    r = _edge_ranges(rng, B)
    d_r = torch.from_numpy(r).cuda()
    d_xy = torch.full((B, N, 2), -7.0, dtype=torch.float32, device="cuda")
    d_n = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    d_o = torch.zeros((B, 2), dtype=torch.float32, device="cuda")
    fleet.ingest_device(B, d_r.data_ptr(), N, d_xy.data_ptr(), N, d_n.data_ptr(), d_o.data_ptr())
    torch.cuda.synchronize()
    xy, n, org = d_xy.cpu().numpy(), d_n.cpu().numpy(), d_o.cpu().numpy()
    cs = O.unit_vectors(N, float(AMIN), float(AINC))
    scale = fleet.scale_to_map()
    total = 0
    for b in range(B):
        opts, oorg = O.ingest(r[b], cs, L.as_oracle_dict(), scale)
        assert n[b] == opts.shape[0], (b, n[b], opts.shape[0])
        assert np.array_equal(_bits(xy[b, : n[b]]), _bits(opts)), b
        assert np.array_equal(_bits(org[b]), _bits(oorg))
        assert np.all(xy[b, n[b]:] == -7.0), "ingest wrote past the stream's point count"
        total += n[b]
    assert 0 < total < B * N  # the filters dropped some beams and kept others


def test_ingest_empty_and_all_invalid(gpu):
    import torch
    L = HsLaser.defaults(N, float(AMIN), float(AINC))
    fleet = HectorFleet(2, 0.05, 256, (0.5, 0.5), 1, max_points=N)
    fleet.set_laser(L)
    r = np.full((2, N), np.nan, np.float32)
    r[1] = 0.1  # all under laser_min_dist
    d_r = torch.from_numpy(r).cuda()
    d_xy = torch.zeros((2, N, 2), dtype=torch.float32, device="cuda")
    d_n = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    fleet.ingest_device(2, d_r.data_ptr(), N, d_xy.data_ptr(), N, d_n.data_ptr())
    torch.cuda.synchronize()
    assert d_n.cpu().tolist() == [0, 0]
    # an empty DataContainer: the step returns the hint (ScanMatcher.h:65, 96) and updates the map
    pose, _, did = fleet.update_ranges(0, r[0])
    assert np.all(pose == 0.0) and did


def test_step_ranges_matches_oracle_pipeline(gpu):
    """scanCallback end to end: raw ranges -> ingest -> update on the device, vs oracle.ingest ->
    oracle process, 2 streams x 12 scans, 2 levels: poses, gate and maps bit-exact."""
    import torch
    S, T, LV, SIZE = 2, 12, 2, 512
    scans = synth.make_streams(S, T, with_points=False)
    L = _roll_pi_laser()
    fleet = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(0.4, 0.9)
    fleet.set_laser(L)
    oras = [O.HectorOracle(0.05, SIZE, (0.5, 0.5), LV, reduce_threads=0) for _ in range(S)]
    for o in oras:
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(0.4, 0.9)
    cs = O.unit_vectors(N, float(AMIN), float(AINC))
    scale = fleet.scale_to_map()
    for t in range(T):
        r = np.ascontiguousarray(scans.ranges[:, t, :])
        d_r = torch.from_numpy(r).cuda()
        fleet.step_ranges_device(d_r.data_ptr(), N)
        gp, _, gd, _ = fleet.poses()
        for s in range(S):
            pts, org = O.ingest(r[s], cs, L.as_oracle_dict(), scale)
            op, _, od = oras[s].process(pts, origo=tuple(org))
            assert gd[s] == od, (t, s)
            assert np.array_equal(_bits(gp[s]), _bits(op)), (t, s, gp[s], op)
    for s in range(S):
        for lvl in range(LV):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            assert np.array_equal(m["upd"], ou)
            assert np.array_equal(_bits(m["logodds"]), _bits(ol))


@pytest.mark.parametrize("NB,lo,hi", [(1440, 1280, 1440), (1200, 1152, 1280)])
def test_step_ranges_wide_scan_separate_ingest(gpu, NB, lo, hi):
    """Scans past the match kernel's register slots, in the reference order (the chain-wave match keeps
    <= 1152 points in registers):
    * 1440 beams (> 1280): the ingest runs as its own kernel and the match takes its strided HBM path;
    * 1200 beams, ranges clipped below 20 m so that 1153..1280 points survive the node's filters: the ingest
      stays fused into the match kernel (<= 1280 beams), whose non-register instance (max_points > 1152) then
      reads the points the same kernel's ingest wrote to HBM.
    Both equal oracle.ingest -> oracle process bit for bit."""
    import torch
    S, T, LV, SIZE = 2, 6, 2, 512
    scans = synth.make_streams(S, T, with_points=False, seed=3, n_beams=NB)
    if NB <= 1280:
        scans.ranges[:] = np.minimum(scans.ranges, np.float32(19.5))
    ang = synth.beam_angles(NB)
    L = HsLaser.defaults(NB, float(ang[0]), float(ang[1] - ang[0]))
    cs = np.ascontiguousarray(np.stack([np.cos(ang), np.sin(ang)], 1))
    fleet = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=NB)
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    fleet.set_laser(L, unit_vectors=cs)
    oras = [O.HectorOracle(0.05, SIZE, (0.5, 0.5), LV, reduce_threads=0) for _ in range(S)]
    for o in oras:
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(-1.0, -1.0)
    scale = fleet.scale_to_map()
    for t in range(T):
        r = np.ascontiguousarray(scans.ranges[:, t, :])
        d_r = torch.from_numpy(r).cuda()
        fleet.step_ranges_device(d_r.data_ptr(), NB)
        gp, _, gd, _ = fleet.poses()
        for s in range(S):
            pts, org = O.ingest(r[s], cs, L.as_oracle_dict(), scale)
            assert lo < pts.shape[0] <= hi, pts.shape[0]  # the path under test
            op, _, od = oras[s].process(pts, origo=tuple(org))
            assert gd[s] == od, (t, s)
            assert np.array_equal(_bits(gp[s]), _bits(op)), (t, s, gp[s], op)
    for s in range(S):
        for lvl in range(LV):
            m = fleet.get_map(s, lvl)
            ol, ou = oras[s].level(lvl)
            assert np.array_equal(m["upd"], ou)
            assert np.array_equal(_bits(m["logodds"]), _bits(ol))
    fleet.close()


def test_update_ranges_host_entry_equals_batch(gpu):
    import torch
    scans = synth.make_streams(1, 6, with_points=False)
    L = _roll_pi_laser()
    a = HectorFleet(1, 0.05, 256, (0.5, 0.5), 1, max_points=N)
    b = HectorFleet(1, 0.05, 256, (0.5, 0.5), 1, max_points=N)
    for f in (a, b):
        f.set_laser(L)
        f.set_thresholds(-1.0, -1.0)
    for t in range(6):
        r = np.ascontiguousarray(scans.ranges[0, t])
        pa, _, _ = a.update_ranges(0, r)
        d_r = torch.from_numpy(r[None]).cuda()
        b.step_ranges_device(d_r.data_ptr(), N)
        pb = b.poses()[0][0]
        assert np.array_equal(_bits(pa), _bits(pb)), t


def _maps_equal(fa, fb, S, LV):
    for s in range(S):
        for lvl in range(LV):
            ma, mb = fa.get_map(s, lvl), fb.get_map(s, lvl)
            assert np.array_equal(ma["upd"], mb["upd"]), (s, lvl)
            assert np.array_equal(_bits(ma["logodds"]), _bits(mb["logodds"])), (s, lvl)


@pytest.mark.parametrize("S,gate", [(5, (-1.0, -1.0)), (4, (0.4, 0.9))])
def test_fused_ingest_equals_separate_kernel(gpu, monkeypatch, S, gate):
    """Range-array steps run the scan ingest inside hs_match_kernel (default) or as hs_ingest_kernel
    (SLAM2D_FUSE_INGEST=0 at hs_create): every pose, gate and map cell equal bit for bit."""
    import torch
    T, LV, SIZE = 6, 2, 384
    scans = synth.make_streams(S, T, with_points=False, seed=91)
    L = _roll_pi_laser()
    monkeypatch.setenv("SLAM2D_FUSE_INGEST", "0")
    fa = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    monkeypatch.delenv("SLAM2D_FUSE_INGEST")
    fb = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    for f in (fa, fb):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(*gate)
        f.set_laser(L)
    r = np.ascontiguousarray(scans.ranges.transpose(1, 0, 2))      # [T][S][N]
    d_r = torch.from_numpy(r).cuda()
    hs = torch.cuda.current_stream().cuda_stream
    for t in range(T):
        fa.step_ranges_device(d_r[t].data_ptr(), N, hip_stream=hs)
        fb.step_ranges_device(d_r[t].data_ptr(), N, hip_stream=hs)
    torch.cuda.synchronize()
    pa, ca, da, _ = fa.poses()
    pb, cb, db, _ = fb.poses()
    assert np.array_equal(_bits(pa), _bits(pb)) and np.array_equal(_bits(ca), _bits(cb))
    assert np.array_equal(da, db)
    _maps_equal(fa, fb, S, LV)
    fa.close()
    fb.close()


def test_update_split_knob_same_maps(gpu, monkeypatch):
    """SLAM2D_UPD_SPLIT (more grid-update workgroups per level) changes only the work split: maps and
    poses equal the default split bit for bit."""
    import torch
    S, T, LV, SIZE = 3, 5, 3, 512
    scans = synth.make_streams(S, T, with_points=False, seed=17)
    L = _roll_pi_laser()
    monkeypatch.setenv("SLAM2D_UPD_SPLIT", "5,3,2")
    fa = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    monkeypatch.delenv("SLAM2D_UPD_SPLIT")
    fb = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    for f in (fa, fb):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(-1.0, -1.0)
        f.set_laser(L)
    r = np.ascontiguousarray(scans.ranges.transpose(1, 0, 2))
    d_r = torch.from_numpy(r).cuda()
    hs = torch.cuda.current_stream().cuda_stream
    for f in (fa, fb):
        f.run_ranges_device(T, d_r.data_ptr(), N, S * N, hip_stream=hs)
    torch.cuda.synchronize()
    pa, _, _, _ = fa.poses()
    pb, _, _, _ = fb.poses()
    assert np.array_equal(_bits(pa), _bits(pb))
    _maps_equal(fa, fb, S, LV)
    fa.close()
    fb.close()


@pytest.mark.parametrize("S,gate,pipeline,sweep", [(7, (-1.0, -1.0), "1", ""), (6, (0.4, 0.9), "1", ""),
                                                   (1, (-1.0, -1.0), "1", ""), (5, (0.4, 0.9), "0", ""),
                                                   (7, (-1.0, -1.0), "1", "3"), (5, (-1.0, -1.0), "0", "2")])
def test_run_ranges_equals_per_step(gpu, monkeypatch, S, gate, pipeline, sweep):
    """hs_run_ranges_device (K steps in one call; SLAM2D_PIPELINE=1: two fleet halves on two HIP streams,
    the grid update of one half beside the other half's match) == K calls of
    hs_step_ranges_batch_device, every pose, gate, map cell and pose-log entry bit for bit; odd fleets
    split unevenly, S = 1 runs unsplit.  Stream S-1 is also replayed on the oracle.  sweep: the run's ordinal
    sweep every few steps (SLAM2D_ORD_SWEEP; inside the two-half pipeline too) against the per-step fleet's
    default, so the decoded updateIndex of every cell is compared across the two representations."""
    import torch
    T, LV, SIZE = 8, 2, 384
    scans = synth.make_streams(S, T, with_points=False, seed=77)
    L = _roll_pi_laser()
    monkeypatch.setenv("SLAM2D_PIPELINE", pipeline)
    if sweep:
        monkeypatch.setenv("SLAM2D_ORD_SWEEP", sweep)
    fa = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    monkeypatch.delenv("SLAM2D_PIPELINE")
    monkeypatch.delenv("SLAM2D_ORD_SWEEP", raising=False)
    fb = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    logs = []
    for f in (fa, fb):
        f.set_update_factors(0.4, 0.9)
        f.set_thresholds(*gate)
        f.set_laser(L)
        d_log = torch.zeros((T, S, 3), dtype=torch.float32, device="cuda")
        f.set_pose_log(d_log.data_ptr(), S, T)
        logs.append(d_log)
    r = np.ascontiguousarray(scans.ranges.transpose(1, 0, 2))      # [T][S][N]
    d_r = torch.from_numpy(r).cuda()
    hs = torch.cuda.current_stream().cuda_stream   # the pose logs were zeroed on torch's stream
    fa.run_ranges_device(T, d_r.data_ptr(), N, S * N, hip_stream=hs)
    for t in range(T):
        fb.step_ranges_device(d_r[t].data_ptr(), N, hip_stream=hs)
    torch.cuda.synchronize()
    pa, ca, da, _ = fa.poses()
    pb, cb, db, _ = fb.poses()
    assert np.array_equal(_bits(pa), _bits(pb)) and np.array_equal(_bits(ca), _bits(cb))
    assert np.array_equal(da, db)
    assert np.array_equal(_bits(logs[0].cpu().numpy()), _bits(logs[1].cpu().numpy()))
    _maps_equal(fa, fb, S, LV)
    o = O.HectorOracle(0.05, SIZE, (0.5, 0.5), LV, reduce_threads=0)
    o.set_update_factors(0.4, 0.9)
    o.set_thresholds(*gate)
    cs = O.unit_vectors(N, float(AMIN), float(AINC))
    scale = fa.scale_to_map()
    lg = logs[0].cpu().numpy()
    for t in range(T):
        pts, org = O.ingest(r[t, S - 1], cs, L.as_oracle_dict(), scale)
        op, _, _ = o.process(pts, origo=tuple(org))
        assert np.array_equal(_bits(lg[t, S - 1]), _bits(op)), t


def test_device_calls_alternating_hip_streams(gpu):
    """Consecutive *_device calls on one context issued on two different HIP streams (the context's
    scratch -- update lists, ingest buffers -- is shared): each call waits for the previous one, so the
    result equals issuing all calls on one stream."""
    import torch
    S, T, LV, SIZE = 16, 6, 2, 256
    scans = synth.make_streams(S, T, with_points=False, seed=5)
    L = _roll_pi_laser()
    fa = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    fb = HectorFleet(S, 0.05, SIZE, (0.5, 0.5), LV, max_points=N)
    for f in (fa, fb):
        f.set_thresholds(-1.0, -1.0)
        f.set_laser(L)
    r = np.ascontiguousarray(scans.ranges.transpose(1, 0, 2))
    d_r = torch.from_numpy(r).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for t in range(T):
        half = S // 2
        # two disjoint stream ranges per step on two HIP streams, then the next step on the other pair
        fa.step_ranges_device(d_r[t].data_ptr(), N, stream_begin=0, count=half,
                              hip_stream=(s1 if t % 2 == 0 else s2).cuda_stream)
        fa.step_ranges_device(d_r[t, half:].data_ptr(), N, stream_begin=half, count=S - half,
                              hip_stream=(s2 if t % 2 == 0 else s1).cuda_stream)
        fb.step_ranges_device(d_r[t].data_ptr(), N)
    torch.cuda.synchronize()
    pa, _, da, _ = fa.poses()
    pb, _, db, _ = fb.poses()
    assert np.array_equal(_bits(pa), _bits(pb)) and np.array_equal(da, db)
    _maps_equal(fa, fb, S, LV)
