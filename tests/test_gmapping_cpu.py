"""GMapping single-scan grid (config 4) -- the oracle against the REFERENCE.

The reference's GMapping grid headers (lesson4/include/lesson4/gmapping/grid/*.h) compile
unmodified; oracle/Makefile builds them into oracle/_ref/libgmapping_ref.so (container only) and
oracle/make_golden.py stored their outputs in tests/golden/gmapping_ref.npz.  The C restatement
(oracle/gmapping_oracle.c) must reproduce them bit for bit: integer (n, visits) counts and the
float PointAccumulator sums.
"""
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                      "libgmapping_ref.so")


def _sparse(n, v, acc):
    idx = np.nonzero(v.ravel())[0].astype(np.int32)
    return idx, n.ravel()[idx], v.ravel()[idx], acc.reshape(-1, 2)[idx].view(np.int32)


def test_geometry():
    """ScanMatcherMap(Point(0,0), -40,-40,40,40, 0.05): 1600 x 1600, world2map(0,0) = (800,800)
    (SURVEY.md §8c probe)."""
    sx, sy, sx2, sy2 = O.gm_geometry()
    assert (sx, sy, sx2, sy2) == (1600, 1600, 800, 800)


@pytest.mark.parametrize("i", range(4))
def test_oracle_matches_reference_fixture(i):
    d = np.load(os.path.join(GOLD, "gmapping_ref.npz"))
    ang = d["angles"]
    x, y, c, s = (float(v) for v in d[f"p{i}_pose"])
    n, v, acc, nfree, nhits = O.gm_compute(d[f"p{i}_ranges"], np.cos(ang), np.sin(ang), (x, y, c, s))
    idx, nn, vv, ab = _sparse(n, v, acc)
    np.testing.assert_array_equal(idx, d[f"p{i}_idx"])
    np.testing.assert_array_equal(nn, d[f"p{i}_n"])
    np.testing.assert_array_equal(vv, d[f"p{i}_visits"])
    np.testing.assert_array_equal(ab, d[f"p{i}_acc_bits"])
    assert [nfree, nhits] == list(d[f"p{i}_counts"])


def test_fixture_edge_cases_present():
    """The fixture exercises d == 0, d > max_urange (clamped, no hit), d > max_range, inf."""
    d = np.load(os.path.join(GOLD, "gmapping_ref.npz"))
    r = d["p0_ranges"]
    assert (r == 0).any() and (r == 27.0).any() and (r == 35.0).any() and np.isinf(r).any()


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_matches_reference_live():
    """Random poses with theta != 0 and random ranges: oracle == reference build, every cell."""
    rng = np.random.default_rng(3)
    ang = np.linspace(-2.35619449, 2.35619449, 1081)
    for _ in range(6):
        x, y, th = rng.uniform(-10, 10), rng.uniform(-10, 10), rng.uniform(-np.pi, np.pi)
        r = rng.uniform(0.0, 32.0, 1081).astype(np.float32)
        pose = (x, y, np.cos(th), np.sin(th))
        a = O.gm_compute(r, np.cos(ang), np.sin(ang), pose, which="oracle")
        b = O.gm_compute(r, np.cos(ang), np.sin(ang), pose, which="ref")
        for u, w in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(u.view(np.int32) if u.dtype == np.float32 else u,
                                          w.view(np.int32) if w.dtype == np.float32 else w)
        assert a[3:] == b[3:]


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_grid_line_matches_reference():
    """GridLineTraversal::gridLine (gridlinetraversal.h:27-207) incl. the reversal to start at p0."""
    go, gr = O.gmapping_oracle_lib(), O.gmapping_ref_lib()
    rng = np.random.default_rng(11)
    buf_a = np.zeros(2 * 4000, np.int32)
    buf_b = np.zeros(2 * 4000, np.int32)
    for _ in range(2000):
        x0, y0 = (int(v) for v in rng.integers(0, 1600, 2))
        x1, y1 = x0 + int(rng.integers(-600, 600)), y0 + int(rng.integers(-600, 600))
        na = go.gmo_grid_line(x0, y0, x1, y1, O._fp(buf_a))
        nb = gr.gmr_grid_line(x0, y0, x1, y1, O._fp(buf_b), 4000)
        assert na == nb
        np.testing.assert_array_equal(buf_a[: 2 * na], buf_b[: 2 * nb])
