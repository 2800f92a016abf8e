"""GPU parity of the Karto correlative matcher (lesson6, config 5): the kt_* C-ABI vs the CPU
restatement oracle/karto_oracle.c of open_karto's ScanMatcher::MatchScan.  Bit-exact in every output
(mean, covariance, response).  open_karto itself needs boost and is not built: parity against the
library is unpinned (DESIGN.md "Karto")."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle as O
from slam2d import karto, synth

pytestmark = pytest.mark.gpu
D = math.pi / 180.0


def _laser(thr=12.0, n=synth.N_BEAMS):
    return karto.laser(n, float(synth.ANGLE_MIN), float(synth.ANGLE_INC), 0.1, thr)


def _olaser(l):
    return O.KtLaser(l.minimum_angle, l.angular_resolution, l.minimum_range, l.range_threshold, l.n_readings, 0)


def _oparams(p):
    return O.KtParams(*[getattr(p, f) for f, _ in karto.KtParams._fields_])


def _same(gpu_out, ora_out):
    gm, gc, gr = gpu_out
    om, oc, orr = ora_out
    np.testing.assert_array_equal(gm, om)
    np.testing.assert_array_equal(gc, oc)
    assert gr == orr


@pytest.mark.parametrize("penalize,refine", [(True, True), (False, True), (True, False)])
def test_sequential_match_bitexact(gpu, penalize, refine):
    """Mapper::Process's sequential match against 10 running scans (Mapper.cpp:2040)."""
    lz = _laser()
    p = karto.default_params()
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=16, max_base=12)
    R, T, Q = synth.karto_sequential(4, 10, seed=11)
    for i in range(10, 14):
        g = sm.MatchScan(R[i], Q[i], R[i - 10:i], T[i - 10:i], penalize, refine)
        o = O.karto_match(_olaser(lz), _oparams(p), R[i], Q[i], R[i - 10:i], T[i - 10:i], penalize, refine)
        _same(g, o)
    assert np.abs(g[0][:2] - T[13][:2]).max() < 0.08  # sanity: the match lands near the truth


def test_loop_window_bitexact(gpu):
    """MapperGraph::TryCloseLoop's coarse match (Mapper.cpp:991-992: doPenalize = doRefine = false) and
    the fine re-match (:1015-1016) on the loop matcher's 81x81x21 window."""
    lz = _laser()
    p = karto.default_params(loop=True)
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=16, max_base=10)
    QR, qp, qt, CR, CP = synth.karto_loop(2, seed=5)
    for i in range(2):
        for pen, ref in [(False, False), (False, True)]:
            g = sm.MatchScan(QR[i], qp[i], CR[i], CP[i], pen, ref)
            o = O.karto_match(_olaser(lz), _oparams(p), QR[i], qp[i], CR[i], CP[i], pen, ref)
            _same(g, o)


def test_response_expansion_and_empty_grid(gpu):
    """No base scans (empty grid: every pose ties at 0 -> average of the whole window) with response
    expansion on (3 widened passes, Mapper.cpp:244-271), and a query far from its base scans."""
    lz = _laser()
    p = karto.default_params()
    p.use_response_expansion = 1
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=16, max_base=4)
    R, T, Q = synth.karto_sequential(1, 4, seed=3)
    o = O.karto_match(_olaser(lz), _oparams(p), R[4], Q[4], R[:0], T[:0], True, True)
    _same(sm.MatchScan(R[4], Q[4], R[:0], T[:0], True, True), o)
    far = Q[4] + np.array([3.0, -2.0, 0.0])
    o = O.karto_match(_olaser(lz), _oparams(p), R[4], far, R[:4], T[:4], True, True)
    _same(sm.MatchScan(R[4], far, R[:4], T[:4], True, True), o)


def test_invalid_readings_and_clean_slots(gpu):
    """NaN / inf readings (INVALID_SCAN lookups indexed by point number, Karto.h:6476-6481), short
    range threshold, and back-to-back matches reusing the slot (the grid must be cleared exactly)."""
    lz = _laser(thr=6.0)
    p = karto.default_params()
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=16, max_base=6)
    R, T, Q = synth.karto_sequential(3, 6, seed=21)
    R = R.copy()
    R[7, 100:140] = np.nan
    R[7, 500] = np.inf
    R[8, ::7] = -np.inf
    for i in (6, 7, 8):
        g = sm.MatchScan(R[i], Q[i], R[i - 6:i], T[i - 6:i])
        o = O.karto_match(_olaser(lz), _oparams(p), R[i], Q[i], R[i - 6:i], T[i - 6:i])
        _same(g, o)


def test_batch_device_matches_single(gpu):
    """kt_match_batch_device over pooled scans: a batch of 136 sequential matches (ragged base counts)
    equals the oracle match by match."""
    import torch

    lz = _laser()
    p = karto.default_params()
    M, B = 136, 8  # >= 128: the binned AddScans path
    R, T, Q = synth.karto_sequential(M, B, seed=9)
    S = R.shape[0]
    # pool: slots [0, S) true-pose scans (bases), [S, S + M) the queries at their odometry poses
    sm = karto.ScanMatcher(lz, p, max_matches=M, max_scans=S + M, max_base=B)
    pr = torch.tensor(np.concatenate([R, R[B:]]), dtype=torch.float64, device="cuda")
    pp = torch.tensor(np.concatenate([T, Q[B:]]), dtype=torch.float64, device="cuda")
    sm.set_scans_device(0, S + M, pr.data_ptr(), pp.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
    counts = [B - (i % 3) for i in range(M)]
    beg = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    idx = np.concatenate([np.arange(B + i - c, B + i) for i, c in enumerate(counts)]).astype(np.int32)
    q = np.arange(S, S + M, dtype=np.int32)
    dq, db, di = (torch.tensor(a, device="cuda") for a in (q, beg, idx))
    res = torch.zeros(M * C.sizeof(karto.KtResult), dtype=torch.uint8, device="cuda")
    sm.match_batch_device(M, dq.data_ptr(), db.data_ptr(), di.data_ptr(), res.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = karto.results_from_bytes(res.cpu().numpy())
    for i in range(M):
        c = counts[i]
        o = O.karto_match(_olaser(lz), _oparams(p), R[B + i], Q[B + i], R[B + i - c:B + i], T[B + i - c:B + i])
        assert out["status"][i] == 0
        _same((out["mean"][i], out["covariance"][i].reshape(3, 3), out["response"][i]), o)


def test_grid_matches_oracle_addscans(gpu):
    """The device correlation grid after AddScans equals the oracle's byte for byte (grid of the last
    match is cleared afterwards: a second identical match must give the same result)."""
    lz = _laser()
    p = karto.default_params()
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=16, max_base=10)
    R, T, Q = synth.karto_sequential(1, 10, seed=4)
    a = sm.MatchScan(R[10], Q[10], R[:10], T[:10])
    b = sm.MatchScan(R[10], Q[10], R[:10], T[:10])
    _same(a, b)


def test_batch_device_loop_window(gpu):
    """A loop-closure candidate batch (>= 128 matches: binned AddScans) on a wide coarse window
    (21 x 21 positions: the 32 x 32-tile coarse kernel), doPenalize = doRefine = false as
    TryCloseLoop's first call (Mapper.cpp:991-992)."""
    import torch

    lz = _laser()
    p = karto.default_params(loop=True)
    p.search_size = 2.0  # 41 x 41 probability grid, 21 x 21 coarse positions
    M, K = 128, 6
    QR, qp, qt, CR, CP = synth.karto_loop(M, K, seed=17, perturb=(0.2, 0.2, 0.03))
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
    for i in range(0, M, 7):
        o = O.karto_match(_olaser(lz), _oparams(p), QR[i], qp[i], CR[i], CP[i], False, False)
        assert out["status"][i] == 0
        _same((out["mean"][i], out["covariance"][i].reshape(3, 3), out["response"][i]), o)


def _sharded_setup(lz, p, M, K, seed):
    QR, qp, qt, CR, CP = synth.karto_loop(M, K, seed=seed, perturb=(0.2, 0.2, 0.03))
    return QR, qp, CR, CP


@pytest.mark.parametrize("loop,nshards,penalize,refine,M", [(True, 2, False, False, 4), (True, 3, True, True, 4),
                                                             (False, 8, True, True, 6), (False, 2, True, True, 130)])
def test_sharded_window_equals_unsharded(gpu, loop, nshards, penalize, refine, M):
    """one batch with the coarse window split over `nshards` ranks (angles
    a = shard mod nshards), the exchange words combined by element-wise MAX exactly as the RCCL
    all-reduce does, then every shard's phase 2: identical results on every shard, bit-equal to the
    unsharded kt_match_batch_device (and so to the oracle).  Emulated on one GPU with one context per
    shard; the multi-process exchange itself is covered with gloo in tests/test_karto_cpu.py."""
    import torch

    lz = _laser()
    p = karto.default_params(loop=loop)
    if loop:
        p.search_size = 2.0
    K = 5
    QR, qp, CR, CP = _sharded_setup(lz, p, M, K, seed=23 + M)
    pr = torch.tensor(np.concatenate([QR, CR.reshape(-1, synth.N_BEAMS)]), dtype=torch.float64, device="cuda")
    pp = torch.tensor(np.concatenate([qp, CP.reshape(-1, 3)]), dtype=torch.float64, device="cuda")
    q = torch.arange(M, dtype=torch.int32, device="cuda")
    beg = torch.arange(M + 1, dtype=torch.int32, device="cuda") * K
    idx = torch.arange(M, M + M * K, dtype=torch.int32, device="cuda")
    nbytes = M * C.sizeof(karto.KtResult)

    def ctx():
        sm = karto.ScanMatcher(lz, p, max_matches=M, max_scans=M * (K + 1), max_base=K)
        sm.set_scans_device(0, M * (K + 1), pr.data_ptr(), pp.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
        return sm

    ref = ctx()
    r0 = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    ref.match_batch_device(M, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), r0.data_ptr(), penalize, refine, hip_stream=torch.cuda.current_stream().cuda_stream)
    shards = [ctx() for _ in range(nshards)]
    words = shards[0].exchange_words()
    xs = [torch.full((M, words), -1, dtype=torch.int64, device="cuda") for _ in range(nshards)]
    for k, sm in enumerate(shards):
        sm.match_sharded_begin_device(M, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), k, nshards, xs[k].data_ptr(),
                                      penalize, hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert all(bool((x >= 0).all()) for x in xs), "every exchange word is written and non-negative"
    x = xs[0].clone()
    for k in range(1, nshards):
        x = torch.maximum(x, xs[k])
    outs = []
    for sm in shards:
        r = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        sm.match_sharded_end_device(M, beg.data_ptr(), idx.data_ptr(), x.data_ptr(), r.data_ptr(), penalize, refine, hip_stream=torch.cuda.current_stream().cuda_stream)
        outs.append(r)
    torch.cuda.synchronize()
    want = r0.cpu().numpy()
    for r in outs:
        assert np.array_equal(r.cpu().numpy(), want)
    res = karto.results_from_bytes(want)
    o = O.karto_match(_olaser(lz), _oparams(p), QR[0], qp[0], CR[0], CP[0], penalize, refine)
    _same((res["mean"][0], res["covariance"][0].reshape(3, 3), res["response"][0]), o)
    # a context reused after the sharded path: the grids were cleared
    r2 = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    shards[0].match_batch_device(M, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), r2.data_ptr(), penalize, refine, hip_stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(r2.cpu().numpy(), want)


def test_sharded_rejects_expansion_and_bad_shard(gpu):
    import torch
    lz = _laser()
    p = karto.default_params()
    p.use_response_expansion = 1
    sm = karto.ScanMatcher(lz, p, max_matches=1, max_scans=2, max_base=1)
    x = torch.zeros((1, sm.exchange_words()), dtype=torch.int64, device="cuda")
    q = torch.zeros(1, dtype=torch.int32, device="cuda")
    beg = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    idx = torch.ones(1, dtype=torch.int32, device="cuda")
    with pytest.raises(karto.Slam2dError):
        sm.match_sharded_begin_device(1, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), 0, 2, x.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
    p.use_response_expansion = 0
    sm2 = karto.ScanMatcher(lz, p, max_matches=1, max_scans=2, max_base=1)
    with pytest.raises(karto.Slam2dError):
        sm2.match_sharded_begin_device(1, q.data_ptr(), beg.data_ptr(), idx.data_ptr(), 2, 2, x.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
