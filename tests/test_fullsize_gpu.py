"""GPU parity at the BASELINE.json configs' full sizes (c3 and GMapping at 1024 particles had
no GPU test, the Karto loop window was tested below its benched size).

  * north star -- the bench's fleet shape, 4608 streams x 2048^2 x 3 levels (242 GB), default issue path;
  * c3  -- lesson4 hector_slam 3-level 4096 x 4096 grid, a fleet of 1024 streams (225 GB of maps, so
           the last stream's cells sit above 2^32 words): streams 0, 511, 512 (the second fleet half of
           hs_run_ranges_device) and 1023 replayed on the oracle, poses every step and every cell of all
           three levels bit-exact;
  * GMapping -- make_gmapping_map with 1024 particles x 1081 beams (10 GB of particle maps, 64-bit
           offsets): particles 0, 511 and 1023 vs the oracle (itself pinned to the reference build), plus
           every particle's integer score;
  * Karto -- the benched loop-closure window 101 x 101 x 21 (search_size 10 m), 32 candidates in one
           batch, a sample vs the oracle.
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle as O
from slam2d import karto, synth
from slam2d.gmapping import GMappingFleet
from slam2d.hector import HectorFleet, HsLaser

pytestmark = pytest.mark.gpu

T_RED = 0  # reference summation order (the kernel default)


def _cround(x):
    """C round(): half away from zero."""
    f = math.floor(x)
    d = x - f
    return int(f + 1) if (d > 0.5 or (d == 0.5 and x > 0)) else int(f)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.mark.parametrize("pipeline,gate", [("0", "forced"), ("0", "reference"), ("1", "forced")])
def test_c3_4096x3_fleet_last_stream_bitexact(gpu, monkeypatch, request, pipeline, gate):
    """c3 at full size through hs_run_ranges_device: the default single-pass issue path (pipeline 0) and
    the two-half pipeline (1); the benchmark's forced map update and the node's 0.4 m / 0.9 rad gate.
    Every logged pose equals the oracle in the reference's sequential Hessian order bit for bit (the
    north star's pose bar by construction), and every cell of the 3 levels of the checked streams."""
    import torch

    B, LV, SIZE = 1024, 3, 4096
    T = 3 if gate == "forced" else 8
    thr = (-1.0, -1.0) if gate == "forced" else (0.4, 0.9)
    S = synth.make_streams(B, T, seed=31337)
    nb = S.ranges.shape[2]
    ang = synth.beam_angles(nb)
    monkeypatch.setenv("SLAM2D_PIPELINE", pipeline)
    fleet = HectorFleet(B, 0.05, SIZE, (0.5, 0.5), LV, max_points=1081)
    request.addfinalizer(fleet.close)  # 225 GB: free it even when an assertion fails
    assert fleet.reduction_order() == HectorFleet.ORDER_REFERENCE
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(*thr)
    fleet.set_laser(HsLaser.defaults(nb, float(ang[0]), float(ang[1] - ang[0])),
                    unit_vectors=np.stack([np.cos(ang), np.sin(ang)], 1))
    check = [0, B // 2 - 1, B // 2, B - 1]
    slot_of = np.full(B, -1, np.int32)
    slot_of[check] = np.arange(len(check), dtype=np.int32)
    d_slot = torch.from_numpy(slot_of).cuda()
    d_log = torch.zeros((T, len(check), 3), dtype=torch.float32, device="cuda")
    fleet.set_pose_log_slots(d_log.data_ptr(), d_slot.data_ptr(), len(check), T)
    d_r = torch.from_numpy(np.ascontiguousarray(S.ranges.transpose(1, 0, 2))).cuda()
    fleet.run_ranges_device(T, d_r.data_ptr(), nb, B * nb, hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del d_r
    log = d_log.cpu().numpy()
    _, _, did, cells = fleet.poses()
    if gate == "forced":
        assert did.all()
    for i, s in enumerate(check):
        o = O.HectorOracle(0.05, SIZE, (0.5, 0.5), LV, reduce_threads=T_RED)
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(*thr)
        od = False
        for k in range(T):
            op, _, od = o.process(S.points[s, k, : S.counts[s, k]])
            assert np.array_equal(_bits(log[k, i]), _bits(op)), (s, k, log[k, i], op)
        assert bool(did[s]) == od, s
        if od:
            assert cells[s] == o.sum_L(), s
        for lvl in range(LV):
            m = fleet.get_map(s, lvl)
            ol, ou = o.level(lvl)
            assert np.array_equal(m["upd"], ou), (s, lvl)
            assert np.array_equal(_bits(m["logodds"]), _bits(ol)), (s, lvl)
            assert m["update_index"] == o.update_index(lvl), (s, lvl)
        o.close()
    fleet.close()


def test_north_star_fleet_shape_bitexact(gpu, request):
    """The bench's own north-star shape (bench.py CONFIGS["northstar"]): 4608 streams x 2048^2 x 3 levels (242 GB
    of pyramids, three whole rounds of the match at 6 workgroups per CU), raw ranges through
    hs_run_ranges_device with the default issue path, stream pad and update split, forced map update -- 4 steps.
    Poses of every 64th stream and the last (the bench's pose log) equal the oracle in the reference order bit for
    bit at every step, and every cell of all three levels of the first, middle and last streams."""
    import torch

    B, LV, SIZE, T = 4608, 3, 2048, 4
    S = synth.make_streams(B, T, seed=5150)
    nb = S.ranges.shape[2]
    ang = synth.beam_angles(nb)
    fleet = HectorFleet(B, 0.05, SIZE, (0.5, 0.5), LV, max_points=1081)
    request.addfinalizer(fleet.close)  # 242 GB: free it even when an assertion fails
    fleet.set_update_factors(0.4, 0.9)
    fleet.set_thresholds(-1.0, -1.0)
    fleet.set_laser(HsLaser.defaults(nb, float(ang[0]), float(ang[1] - ang[0])),
                    unit_vectors=np.stack([np.cos(ang), np.sin(ang)], 1))
    logged = sorted(set(range(0, B, 64)) | {B - 1})
    slot_of = np.full(B, -1, np.int32)
    slot_of[logged] = np.arange(len(logged), dtype=np.int32)
    d_slot = torch.from_numpy(slot_of).cuda()
    d_log = torch.zeros((T, len(logged), 3), dtype=torch.float32, device="cuda")
    fleet.set_pose_log_slots(d_log.data_ptr(), d_slot.data_ptr(), len(logged), T)
    d_r = torch.from_numpy(np.ascontiguousarray(S.ranges.transpose(1, 0, 2))).cuda()
    fleet.run_ranges_device(T, d_r.data_ptr(), nb, B * nb, hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del d_r
    log = d_log.cpu().numpy()
    _, _, did, cells = fleet.poses()
    assert did.all()
    full = {0, B // 2, B - 1}
    for i, s in enumerate(logged + [B // 2]):
        o = O.HectorOracle(0.05, SIZE, (0.5, 0.5), LV, reduce_threads=T_RED)
        o.set_update_factors(0.4, 0.9)
        o.set_thresholds(-1.0, -1.0)
        for k in range(T):
            op, _, _ = o.process(S.points[s, k, : S.counts[s, k]])
            if slot_of[s] >= 0:
                got = log[k, slot_of[s]]
                assert np.array_equal(_bits(got), _bits(op)), (s, k, got, op)
        assert cells[s] == o.sum_L(), s
        if s in full:
            for lvl in range(LV):
                m = fleet.get_map(s, lvl)
                ol, ou = o.level(lvl)
                assert np.array_equal(m["upd"], ou), (s, lvl)
                assert np.array_equal(_bits(m["logodds"]), _bits(ol)), (s, lvl)
                assert m["update_index"] == o.update_index(lvl), (s, lvl)
        o.close()
    fleet.close()


def test_gmapping_1024_particles_bitexact(gpu):
    P, T = 1024, 2
    ang = synth.beam_angles().astype(np.float64)
    segs = synth.world_segments()
    gt = synth.trajectory(T, 0.0)
    rng = np.random.default_rng(2024)
    noise = rng.normal(0, [0.05, 0.05, 0.02], size=(P, 3))
    fleet = GMappingFleet(P)
    fleet.set_beams(ang)
    check = [0, 511, 1023]
    prev = {}
    for t in range(T):
        ranges = synth.cast_ranges(gt[t:t + 1], segs)[0].astype(np.float32)
        ranges += rng.normal(0, 0.01, ranges.shape).astype(np.float32)
        poses4 = GMappingFleet.poses4(gt[t] + noise)
        fleet.compute(poses4, ranges)
        s, h, f = fleet.scores()
        for p in check:
            on, ov, oacc, nfree, nh = O.gm_compute(ranges, np.cos(ang), np.sin(ang), tuple(poses4[p]))
            n, v, acc = fleet.particle_map(p)
            np.testing.assert_array_equal(v, ov, err_msg=f"t={t} particle {p} visits")
            np.testing.assert_array_equal(n, on, err_msg=f"t={t} particle {p} n")
            np.testing.assert_array_equal(acc.view(np.int32), oacc.view(np.int32), err_msg=f"t={t} particle {p} acc")
            assert h[p] == nh and f[p] == nfree, (t, p)
            if t:
                # hit beams on occupied cells (n / visits > 0.25) of the particle's previous map
                pn, pv = prev[p]
                sx, sy, sx2, sy2 = O.gm_geometry()
                gp = O.GM_DEFAULTS
                cx, cy = (gp["xmin"] + gp["xmax"]) / 2.0, (gp["ymin"] + gp["ymax"]) / 2.0
                px, py, ct, st = (float(v) for v in poses4[p])
                want = 0
                for i, r in enumerate(ranges.astype(np.float64)):
                    d = float(r)
                    if d > gp["max_range"] or d == 0.0 or not math.isfinite(d) or not d < gp["max_urange"]:
                        continue
                    ca, sa = math.cos(ang[i]), math.sin(ang[i])
                    wx, wy = px + d * (ct * ca - st * sa), py + d * (st * ca + ct * sa)
                    x = _cround((wx - cx) / gp["delta"]) + sx2   # Map::world2map, C round()
                    y = _cround((wy - cy) / gp["delta"]) + sy2
                    if 0 <= x < sx and 0 <= y < sy and pv[y, x] > 0 and pn[y, x] / pv[y, x] > 0.25:
                        want += 1
                assert int(s[p]) == want, (p, s[p], want)
            prev[p] = (on, ov)
        assert (h > 0).all() and (f > 0).all()
    fleet.close()


def test_karto_loop_window_101x101x21_batch(gpu):
    import torch

    lz = karto.laser(synth.N_BEAMS, float(synth.ANGLE_MIN), float(synth.ANGLE_INC), 0.1, 12.0)
    p = karto.default_params(loop=True)
    p.search_size = 10.0  # 101 x 101 x 21 coarse window at 0.05 m (bench.py --config karto_loop)
    M, K = 32, 10
    QR, qp, qt, CR, CP = synth.karto_loop(M, K, seed=4242)
    sm = karto.ScanMatcher(lz, p, max_matches=M, max_scans=M * (K + 1), max_base=K)
    pr = torch.tensor(np.concatenate([QR, CR.reshape(-1, synth.N_BEAMS)]), dtype=torch.float64, device="cuda")
    pp = torch.tensor(np.concatenate([qp, CP.reshape(-1, 3)]), dtype=torch.float64, device="cuda")
    sm.set_scans_device(0, M * (K + 1), pr.data_ptr(), pp.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
    q = torch.arange(M, dtype=torch.int32, device="cuda")
    beg = torch.arange(M + 1, dtype=torch.int32, device="cuda") * K
    idx = torch.arange(M, M + M * K, dtype=torch.int32, device="cuda")
    res = torch.zeros(M * C.sizeof(karto.KtResult), dtype=torch.uint8, device="cuda")
    sm.match_batch_device(M, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), res.data_ptr(), False, False, hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = karto.results_from_bytes(res.cpu().numpy())
    ol = O.KtLaser(lz.minimum_angle, lz.angular_resolution, lz.minimum_range, lz.range_threshold, lz.n_readings, 0)
    op = O.KtParams(*[getattr(p, f) for f, _ in karto.KtParams._fields_])
    for i in (0, 13, M - 1):
        om, oc, orr = O.karto_match(ol, op, QR[i], qp[i], CR[i], CP[i], False, False)
        assert out["status"][i] == 0
        np.testing.assert_array_equal(out["mean"][i], om)
        np.testing.assert_array_equal(out["covariance"][i].reshape(3, 3), oc)
        assert out["response"][i] == orr
