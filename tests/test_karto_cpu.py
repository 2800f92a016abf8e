"""Karto correlative matcher without a GPU: the CPU restatement (oracle/karto_oracle.c) behaves like
open_karto's ScanMatcher on the reference's own parameters, and kt_create validates parameters
before touching a device.  open_karto needs boost (absent): parity against it is unpinned."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle as O
from slam2d import synth

D = math.pi / 180.0


def laser(thr=12.0):
    return O.KtLaser(float(synth.ANGLE_MIN), float(synth.ANGLE_INC), 0.1, thr, synth.N_BEAMS, 0)


def params(loop=False, expansion=0):
    # Mapper::InitializeParameters (Mapper.cpp:1569-1660)
    if loop:
        return O.KtParams(8.0, 0.05, 0.03, 0.3 ** 2, (20 * D) ** 2, 0.2 * D, 20 * D, 2 * D, 0.9, 0.5, expansion, 0)
    return O.KtParams(0.3, 0.01, 0.03, 0.3 ** 2, (20 * D) ** 2, 0.2 * D, 20 * D, 2 * D, 0.9, 0.5, expansion, 0)


def test_grid_geometry_matches_create():
    """ScanMatcher::Create (Mapper.cpp:150-160) + CorrelationGrid border / WidthStep (Mapper.h:925,
    Karto.h:4442): 0.3 m / 0.01 m, range 12 m -> side 31, grid 31 + 2*1200, border Round(6)+1."""
    g = O.karto_grid_info(params(), laser())
    assert (g["side"], g["grid_size"], g["border"], g["width"], g["ws"]) == (31, 2431, 7, 2445, 2448)
    assert (g["half"], g["ksize"]) == (6, 13)
    lg = O.karto_grid_info(params(loop=True), laser())
    assert (lg["side"], lg["grid_size"], lg["border"], lg["ksize"]) == (161, 641, 2, 3)


def test_smear_kernel_values():
    """CalculateKernel (Mapper.h:1046-1086): Round(100 exp(-d^2 / (2 sigma^2))) on the 13x13 support."""
    k = np.zeros(169, np.uint8)
    assert O.karto_lib().ko_kernel(params(), laser(), O._fp(k), 169) == 169
    k = k.reshape(13, 13)
    i = np.arange(-6, 7)
    d2 = (i[:, None] * 0.01) ** 2 + (i[None, :] * 0.01) ** 2
    expect = np.floor(np.exp(-0.5 * d2 / 0.03 ** 2) * 100 + 0.5)
    assert np.array_equal(k, expect.astype(np.uint8))
    assert k[6, 6] == 100 and (k[np.arange(13) != 6].max() < 100)


def test_sequential_match_recovers_pose():
    R, T, Q = synth.karto_sequential(3, 10, seed=1)
    for i in range(10, 13):
        m, c, r = O.karto_match(laser(), params(), R[i], Q[i], R[i - 10:i], T[i - 10:i])
        assert np.abs(m[:2] - T[i][:2]).max() < 0.02
        assert abs(m[2] - T[i][2]) < 0.01
        assert 0.5 < r <= 1.0
        assert np.allclose(c, c.T) and np.all(np.diag(c) > 0)


def test_loop_match_recovers_drift():
    QR, qp, qt, CR, CP = synth.karto_loop(2, seed=2)
    for i in range(2):
        m, c, r = O.karto_match(laser(), params(loop=True), QR[i], qp[i], CR[i], CP[i], False, True)
        assert np.abs(m[:2] - qt[i][:2]).max() < 0.06, (m, qt[i])
        assert r > 0.3


def test_empty_grid_averages_whole_window():
    """No base scans: every response is 0, all 16x16x21 poses tie, the mean is the window centre and
    the covariance is MAX_VARIANCE (Mapper.cpp:545-551)."""
    R, T, Q = synth.karto_sequential(1, 1, seed=1)
    m, c, r = O.karto_match(laser(), params(), R[1], Q[1], R[:0], T[:0], True, False)
    assert r == 0.0
    assert abs(m[0] - Q[1][0]) < 1e-9 and abs(m[1] - Q[1][1]) < 1e-9
    assert c[0, 0] == 500.0 and c[1, 1] == 500.0


def test_kt_create_rejects_unsupported_params():
    """kt_create validates like ScanMatcher::Create / CalculateKernel before any device call."""
    from slam2d import karto

    L = karto._lib.lib()
    karto._declare(L)
    lz = karto.laser(synth.N_BEAMS, float(synth.ANGLE_MIN), float(synth.ANGLE_INC), 0.1, 12.0)
    h = C.c_void_p()
    bad = karto.default_params()
    bad.smear_deviation = 10 * bad.resolution  # off-centre kernel value 100 -> order-dependent AddScan
    assert L.kt_create(C.byref(h), C.byref(lz), C.byref(bad), 1, 4, 3) == -1
    assert b"off-centre" in L.kt_last_error()
    bad = karto.default_params()
    bad.smear_deviation = 0.1 * bad.resolution
    assert L.kt_create(C.byref(h), C.byref(lz), C.byref(bad), 1, 4, 3) == -1
    p = karto.default_params()
    assert p.search_size == 0.3 and p.resolution == 0.01 and abs(p.coarse_search_angle_offset - 20 * D) < 1e-15


# ----------------------------------------------------------------------------- sharded window (gloo)
def _window_case():
    lz = laser()
    p = params(loop=True)
    p.search_size = 2.0  # 21 x 21 coarse positions x 21 angles
    QR, qp, _, CR, CP = synth.karto_loop(1, 4, seed=31, perturb=(0.2, 0.2, 0.03))
    resp = O.karto_coarse_responses(lz, p, QR[0], qp[0], CR[0], CP[0], 21, 21, penalize=True)
    return resp


def _window_worker(rank, world, port, out):
    import os
    import torch
    import torch.distributed as dist

    from slam2d import karto

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    resp = _window_case()
    nA = resp.shape[2]
    mine = resp.copy()
    for a in range(nA):  # what this rank's kt_coarse_kernel leaves: other ranks' angles +0.0
        if not karto.shard_owns_angle(a, rank, world):
            mine[:, :, a] = 0.0
    posmax = mine.max(axis=2)
    best = mine.max()
    x = torch.from_numpy(np.concatenate([[best], posmax.ravel(), mine.ravel()]).view(np.int64).copy())
    karto.allreduce_window(x)
    out[rank] = x.numpy().tobytes()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_window_exchange_gloo(world):
    """the exchange step of a Karto window split over ranks by angle (the same
    slam2d.karto.allreduce_window the GPU path calls, here over gloo): after the int64 MAX all-reduce
    every rank holds, bit for bit, the unsharded window's responses, per-position maxima and best --
    the inputs of the tie average and covariance, which then run identically on every rank."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_window_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    resp = _window_case()
    assert np.all(resp >= 0.0) and resp.max() > 0.0
    want = np.concatenate([[resp.max()], resp.max(axis=2).ravel(), resp.ravel()])
    for r in range(world):
        got = np.frombuffer(res[r], np.float64)
        assert np.array_equal(got.view(np.int64), want.view(np.int64)), r
