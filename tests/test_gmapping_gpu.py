"""GPU parity of the GMapping particle-map path (config 4): gm_compute_kernel through the C-ABI vs
the GMapping oracle (itself pinned bit-for-bit to the reference's own grid headers,
tests/test_gmapping_cpu.py).  Counts (n, visits) and the float hit accumulators are bit-exact."""
import math
import os

import numpy as np
import pytest

import oracle as O
from slam2d import synth
from slam2d.gmapping import GMappingFleet

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _oracle_maps(poses4, ranges, ang):
    out = []
    for p in poses4:
        n, v, acc, nfree, nh = O.gm_compute(ranges, np.cos(ang), np.sin(ang), tuple(p))
        out.append((n, v, acc, nfree, nh))
    return out


def _cround(x):
    """C round(): half away from zero."""
    f = math.floor(x)
    d = x - f
    if d > 0.5 or (d == 0.5 and x > 0):
        return f + 1
    return f


def _expected_score(prev, pose4, ranges, ang, p=O.GM_DEFAULTS, thresh=0.25):
    """Hit beams whose end cell is occupied (n/visits > thresh) in the previous map."""
    if prev is None:
        return 0
    n_prev, v_prev = prev
    sx, sy, sx2, sy2 = O.gm_geometry(p)
    cx, cy = (p["xmin"] + p["xmax"]) / 2.0, (p["ymin"] + p["ymax"]) / 2.0
    px, py, ct, st = (float(v) for v in pose4)
    score = 0
    for i, r in enumerate(ranges.astype(np.float64)):
        d = float(r)
        if d > p["max_range"] or d == 0.0 or not math.isfinite(d):
            continue
        if d > p["max_urange"]:
            d = p["max_urange"]
        if not d < p["max_urange"]:
            continue
        ca, sa = math.cos(ang[i]), math.sin(ang[i])
        dirx = ct * ca - st * sa
        diry = st * ca + ct * sa
        wx = px + d * dirx
        wy = py + d * diry
        x = _cround((wx - cx) / p["delta"]) + sx2
        y = _cround((wy - cy) / p["delta"]) + sy2
        if 0 <= x < sx and 0 <= y < sy and v_prev[y, x] > 0 and n_prev[y, x] / v_prev[y, x] > thresh:
            score += 1
    return score


def _check_maps(fleet, ref, P):
    for p in range(P):
        n, v, acc = fleet.particle_map(p)
        on, ov, oacc, _, _ = ref[p]
        np.testing.assert_array_equal(v, ov, err_msg=f"particle {p} visits")
        np.testing.assert_array_equal(n, on, err_msg=f"particle {p} n")
        np.testing.assert_array_equal(acc.view(np.int32), oacc.view(np.int32), err_msg=f"particle {p} acc")
        pub = np.empty_like(on, dtype=np.int8)
        O.gmapping_oracle_lib().gmo_publish(O._fp(np.ascontiguousarray(on)), O._fp(np.ascontiguousarray(ov)),
                                            on.shape[1], on.shape[0], 0.25, O._fp(pub))
        np.testing.assert_array_equal(fleet.publish(p), pub, err_msg=f"particle {p} publish")


def test_reference_fixture_scans(gpu):
    """The scans/poses of tests/golden/gmapping_ref.npz (reference build outputs) incl. d == 0,
    d > maxUrange (clamped, no hit), d > maxRange, inf."""
    d = np.load(os.path.join(GOLD, "gmapping_ref.npz"))
    ang = d["angles"]
    P = 4
    fleet = GMappingFleet(P, max_beams=len(ang))
    fleet.set_beams(ang)
    for i in range(4):
        poses4 = np.stack([d[f"p{k}_pose"] for k in range(4)])
        ranges = d[f"p{i}_ranges"]
        fleet.compute(poses4, ranges)
        _check_maps(fleet, _oracle_maps(poses4, ranges, ang), P)
        # the reference build's own sparse outputs for the matching pose
        n, v, acc = fleet.particle_map(i)
        idx = d[f"p{i}_idx"]
        np.testing.assert_array_equal(np.nonzero(v.ravel())[0], idx)
        np.testing.assert_array_equal(n.ravel()[idx], d[f"p{i}_n"])
        np.testing.assert_array_equal(v.ravel()[idx], d[f"p{i}_visits"])
        np.testing.assert_array_equal(acc.reshape(-1, 2)[idx].view(np.int32), d[f"p{i}_acc_bits"])


def test_particles_scores_and_fresh_maps(gpu):
    """Several steps of P particles around the synthetic trajectory: every map equals a fresh
    ComputeMap (cells of the previous footprint read 0), and each score equals the hit-on-occupied
    count against the particle's previous map."""
    rng = np.random.default_rng(777)
    P, T = 6, 4
    ang = synth.beam_angles().astype(np.float64)
    segs = synth.world_segments()
    gt = synth.trajectory(T, 0.0)
    fleet = GMappingFleet(P)
    fleet.set_beams(ang)
    noise = rng.normal(0, [0.05, 0.05, 0.02], size=(P, 3))
    prev = [None] * P
    for t in range(T):
        ranges = synth.cast_ranges(gt[t:t + 1], segs)[0].astype(np.float32)
        ranges += rng.normal(0, 0.01, ranges.shape).astype(np.float32)
        poses4 = GMappingFleet.poses4(gt[t] + noise)
        fleet.compute(poses4, ranges)
        ref = _oracle_maps(poses4, ranges, ang)
        _check_maps(fleet, ref, P)
        s, h, f = fleet.scores()
        for p in range(P):
            assert s[p] == _expected_score(prev[p], poses4[p], ranges, ang), (t, p)
            assert h[p] == ref[p][4] and f[p] == ref[p][3], (t, p)
            prev[p] = (ref[p][0], ref[p][1])
        if t:
            assert s.max() > 0


def test_beams_leaving_the_map_and_empty_scan(gpu):
    """A pose near the map edge: lines leave the +-40 m map (cells outside skipped, as the oracle
    does for the reference's assert); then an empty scan (n = 0) writes an empty map."""
    ang = synth.beam_angles().astype(np.float64)
    rng = np.random.default_rng(5)
    ranges = rng.uniform(0.0, 29.0, len(ang)).astype(np.float32)
    poses4 = GMappingFleet.poses4([[30.0, -35.0, 0.3], [-39.0, 39.0, 2.0]])
    fleet = GMappingFleet(2)
    fleet.set_beams(ang)
    fleet.compute(poses4, ranges)
    _check_maps(fleet, _oracle_maps(poses4, ranges, ang), 2)
    fleet.compute(poses4, np.zeros(0, np.float32))
    for p in range(2):
        n, v, acc = fleet.particle_map(p)
        assert v.sum() == 0 and n.sum() == 0


@pytest.mark.parametrize("n_beams", [2400, 6000])
def test_dense_scans(gpu, n_beams):
    """Scans of more beams than the default 1081: at 2400 the hit-cell slots and the ballot over 38 fan groups;
    at 6000, 94 fan groups, so gm_compute_kernel's groups past the ballot's first 64 take the scalar box-test
    path (raster and acc pass).  Counts, accumulators and publish bit-exact vs the oracle, two steps."""
    ang = synth.beam_angles(n_beams).astype(np.float64)
    segs = synth.world_segments()
    gt = synth.trajectory(2, 0.0)
    P = 3
    fleet = GMappingFleet(P, max_beams=n_beams)
    fleet.set_beams(ang)
    rng = np.random.default_rng(n_beams)
    for t in range(2):
        ranges = synth.cast_ranges(gt[t:t + 1], segs, n_beams)[0].astype(np.float32)
        ranges += rng.normal(0, 0.01, ranges.shape).astype(np.float32)
        poses4 = GMappingFleet.poses4(gt[t] + rng.normal(0, [0.05, 0.05, 0.02], size=(P, 3)))
        fleet.compute(poses4, ranges)
        _check_maps(fleet, _oracle_maps(poses4, ranges, ang), P)


def test_device_entry_and_scores_buffer(gpu):
    import torch

    ang = synth.beam_angles().astype(np.float64)
    segs = synth.world_segments()
    gt = synth.trajectory(2, 0.0)
    P = 5
    fleet = GMappingFleet(P)
    fleet.set_beams(ang)
    poses4 = GMappingFleet.poses4(np.repeat(gt[:1], P, axis=0) + np.linspace(-0.1, 0.1, P)[:, None])
    d_poses = torch.from_numpy(poses4).cuda()
    d_scores = torch.zeros(P, dtype=torch.int32, device="cuda")
    for t in range(2):
        ranges = synth.cast_ranges(gt[t:t + 1], segs)[0].astype(np.float32)
        d_r = torch.from_numpy(ranges).cuda()
        fleet.compute_device(d_poses.data_ptr(), d_r.data_ptr(), len(ranges), d_scores.data_ptr(),
                             hip_stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        s, _, _ = fleet.scores()
        np.testing.assert_array_equal(d_scores.cpu().numpy(), s)
        _check_maps(fleet, _oracle_maps(poses4, ranges, ang), P)


@pytest.mark.parametrize("use_comm", [True, False])
def test_normalize_weights_rccl_world1(gpu, use_comm):
    """gm_normalize_weights_device: the C-ABI form of the particle-weight exchange, with a real RCCL
    communicator made as a C++ host would (ncclGetUniqueId + ncclCommInitRank, world size 1 on the one
    GPU of the box) or none.  Sums are exact integers in double, weights equal the Python
    normalize_weights (torch) bit for bit.  On the CPU (gloo, world 2): RcclComm's unique-id broadcast
    with NUL bytes (test_rccl_unique_id_with_nul_bytes_gloo_world2) and the sums' algebra
    (test_particle_weight_allreduce_gloo_world2); sharding itself: test_sharded_fleet_equals_unsharded."""
    import torch

    from slam2d.gmapping import RcclComm, normalize_weights

    P = 1000
    fleet = GMappingFleet(4)
    scores = torch.from_numpy(np.random.default_rng(3).integers(0, 900, P).astype(np.int32)).cuda()
    w = torch.full((P,), -1.0, dtype=torch.float64, device="cuda")
    sums = torch.zeros(2, dtype=torch.float64, device="cuda")
    comm = RcclComm(1, 0) if use_comm else None
    try:
        fleet.normalize_weights_device(comm, scores.data_ptr(), P, w.data_ptr(), sums.data_ptr(),
                                       hip_stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        if comm:
            comm.close()
    s = scores.cpu().numpy().astype(np.float64) + 1.0
    assert sums.cpu().tolist() == [s.sum(), (s * s).sum()]
    wt, neff = normalize_weights(scores)
    np.testing.assert_array_equal(w.cpu().numpy(), wt.cpu().numpy())
    assert neff == pytest.approx(s.sum() ** 2 / (s * s).sum(), rel=1e-15)


@pytest.mark.parametrize("shards", [2, 8])
def test_sharded_fleet_equals_unsharded(gpu, shards):
    """P = 1024 particles split into `shards` GMappingFleet shards (what each of the
    ranks of `bench.py --config gmapping --gpus N` holds) give every particle the same map (n, visits,
    acc), score, hit and free counts as the unsharded fleet (GMapping::ComputeMap per particle,
    gmapping.cc:171-242), and combining the shards' exchange words [Σ(s+1), Σ(s+1)^2] -- what the RCCL
    all-reduce sums -- reproduces the unsharded gm_normalize_weights_device weights bit for bit."""
    import torch

    P, T = 1024, 2
    ang = synth.beam_angles().astype(np.float64)
    segs = synth.world_segments()
    gt = synth.trajectory(T, 0.0)
    rng = np.random.default_rng(4242)
    noise = rng.normal(0, [0.05, 0.05, 0.02], size=(P, 3))
    ranges = [synth.cast_ranges(gt[t:t + 1], segs)[0].astype(np.float32) for t in range(T)]
    hs = torch.cuda.current_stream().cuda_stream

    def run(lo, hi):
        f = GMappingFleet(hi - lo)
        f.set_beams(ang)
        d_sc = torch.zeros(hi - lo, dtype=torch.int32, device="cuda")
        for t in range(T):
            d_p = torch.from_numpy(GMappingFleet.poses4(gt[t] + noise[lo:hi])).cuda()
            d_r = torch.from_numpy(ranges[t]).cuda()
            f.compute_device(d_p.data_ptr(), d_r.data_ptr(), len(ranges[t]), d_sc.data_ptr(), hip_stream=hs)
        w = torch.zeros(hi - lo, dtype=torch.float64, device="cuda")
        sums = torch.zeros(2, dtype=torch.float64, device="cuda")
        f.normalize_weights_device(None, d_sc.data_ptr(), hi - lo, w.data_ptr(), sums.data_ptr(), hip_stream=hs)
        torch.cuda.synchronize()
        return f, f.scores(), w.cpu().numpy(), sums.cpu().numpy()

    full, (s0, h0, f0), w0, sums0 = run(0, P)
    assert s0.sum() > 0 and (h0 > 0).all()
    sample = {}
    bounds = np.linspace(0, P, shards + 1).astype(int)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        for p in (lo, hi - 1, (lo + hi) // 2):
            sample[p] = full.particle_map(p)
    full.close()
    tot = np.zeros(2)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        f, (s, h, fr), _, sums = run(lo, hi)
        np.testing.assert_array_equal(s, s0[lo:hi])
        np.testing.assert_array_equal(h, h0[lo:hi])
        np.testing.assert_array_equal(fr, f0[lo:hi])
        for p in (lo, hi - 1, (lo + hi) // 2):
            n, v, acc = f.particle_map(p - lo)
            np.testing.assert_array_equal(n, sample[p][0], err_msg=f"particle {p} n")
            np.testing.assert_array_equal(v, sample[p][1], err_msg=f"particle {p} visits")
            np.testing.assert_array_equal(acc.view(np.int32), sample[p][2].view(np.int32), err_msg=f"particle {p} acc")
        f.close()
        tot += sums  # the all-reduce: integer-valued doubles, exact in any order
    np.testing.assert_array_equal(tot, sums0)
    w_sharded = (s0.astype(np.float64) + 1.0) / tot[0]   # gm_weights_kernel with the all-reduced sums
    np.testing.assert_array_equal(w_sharded.view(np.int64), w0.view(np.int64))
