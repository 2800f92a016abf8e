"""GPU parity of the PL-ICP path (lesson3 front-end): pl_icp_kernel through the C-ABI vs the CPU
restatement oracle/plicp_oracle.c in the kernel's summation order.  Bit-exact in every output
(x, valid, iterations, nvalid, error).  CSM itself is absent: parity against CSM is unpinned."""
import numpy as np
import pytest

import oracle as O
from slam2d import synth
from slam2d.plicp import PLICP, laser_scan_to_readings

pytestmark = pytest.mark.gpu


def _pairs(num, seed, noise=0.01, step=1, phase=0.3):
    rng = np.random.default_rng(seed)
    ang = synth.beam_angles().astype(np.float64)
    gt = synth.trajectory(num * step + 1, phase)
    R = synth.cast_ranges(gt, synth.world_segments())
    R = R + rng.normal(0, noise, R.shape)
    R = laser_scan_to_readings(R, 0.1, 29.9)
    pairs = [(R[k * step], R[k * step + 1]) for k in range(num)]
    return pairs, float(ang[0]), float(ang[1] - ang[0])


def _same(g, o):
    np.testing.assert_array_equal(g["x"], o["x"])
    assert g["valid"] == o["valid"] and g["iterations"] == o["iterations"] and g["nvalid"] == o["nvalid"]
    assert g["error"] == o["error"]


@pytest.mark.parametrize("noise", [0.0, 0.01, 0.03])
def test_consecutive_scans_bitexact(gpu, noise):
    pairs, amin, inc = _pairs(6, 3, noise)
    pl = PLICP(1, 1081)
    for ref, sens in pairs:
        _same(pl.icp(ref, sens, amin, inc), O.plicp(ref, sens, amin, inc, reduce_threads=256))


def test_first_guess_and_wide_motion(gpu):
    """Keyframe-style pairs (several scans apart) with a non-zero first guess (GetPrediction)."""
    pairs, amin, inc = _pairs(4, 9, 0.01, step=5)
    pl = PLICP(1, 1081)
    for k, (ref, sens) in enumerate(pairs):
        g = (0.3 * k - 0.2, 0.05, 0.02 * k)
        _same(pl.icp(ref, sens, amin, inc, g), O.plicp(ref, sens, amin, inc, g, reduce_threads=256))


def test_sparse_and_failing_scans(gpu):
    """Mostly invalid rays (fewer than 5 % correspondences -> valid = 0) and a short scan."""
    pairs, amin, inc = _pairs(2, 5)
    ref, sens = pairs[0]
    sparse = sens.copy()
    sparse[::1] = -1.0
    sparse[::40] = sens[::40]
    pl = PLICP(1, 1081)
    _same(pl.icp(ref, sparse, amin, inc), O.plicp(ref, sparse, amin, inc, reduce_threads=256))
    r_short, s_short = ref[300:700].copy(), sens[300:700].copy()
    _same(pl.icp(r_short, s_short, amin + 300 * inc, inc), O.plicp(r_short, s_short, amin + 300 * inc, inc, reduce_threads=256))


def test_batch_device(gpu):
    import ctypes as C

    import torch

    from slam2d.plicp import PlResult

    pairs, amin, inc = _pairs(12, 21, 0.01)
    B = len(pairs)
    ref = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    sens = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    guess = torch.zeros((B, 3), dtype=torch.float64, device="cuda")
    out = torch.zeros((B, C.sizeof(PlResult)), dtype=torch.uint8, device="cuda")
    pl = PLICP(B, 1081)
    pl.icp_batch_device(B, 1081, amin, inc, ref.data_ptr(), sens.data_ptr(), guess.data_ptr(), out.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    raw = out.cpu().numpy()
    for b in range(B):
        r = PlResult.from_buffer_copy(raw[b].tobytes())
        g = dict(x=np.array(r.x[:]), valid=bool(r.valid), iterations=r.iterations, nvalid=r.nvalid, error=r.error)
        _same(g, O.plicp(pairs[b][0], pairs[b][1], amin, inc, reduce_threads=256))


@pytest.mark.parametrize("n_beams,scale", [(1440, 1.0), (1081, 0.2), (1440, 0.12)])
def test_full_circle_and_near_scans(gpu, n_beams, scale):
    """The correspondence search prunes the polar interval by the angular distance bound (kept
    candidates visited in the same order): a 360-degree scan (1440 beams from -135 deg, wrapping past
    pi) and scaled-down worlds whose points sit around the pruning threshold (2.02 m) -- bit-exact vs
    the oracle's exhaustive interval scan."""
    rng = np.random.default_rng(77 + n_beams)
    ang0 = float(synth.ANGLE_MIN)
    inc = float(np.float64(synth.ANGLE_INC))
    gt = synth.trajectory(5, 1.1)
    R = synth.cast_ranges(gt, synth.world_segments(), n_beams) * scale
    R = R + rng.normal(0, 0.01 * scale, R.shape)
    R = laser_scan_to_readings(R, 0.05, 29.9)
    pl = PLICP(1, n_beams)
    for k in range(4):
        _same(pl.icp(R[k], R[k + 1], ang0, inc), O.plicp(R[k], R[k + 1], ang0, inc, reduce_threads=256))
