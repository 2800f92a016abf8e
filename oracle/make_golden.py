#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ -- TEST INFRASTRUCTURE.

  python oracle/make_golden.py            (needs oracle/build/*.so; gmapping_ref needs oracle/_ref)

The reference holds no tests, fixtures or known-answer vectors for this path, so:

* hector_*.npz -- inputs + outputs of the Hector C restatement (oracle/hector_oracle.c).  Hector is
  "parity unpinned" (Eigen3 absent, the reference's Hector core cannot be compiled here): these
  fixtures pin the oracle against regressions and carry the GPU's expected per-scan poses / map
  deltas; their arithmetic provenance is the restatement, cross-checked by the pure-Python
  Bresenham restatement (ray_cells) and the libm-vs-detmath tolerance tests.
* ray_cells.npz -- Bresenham cell lists of updateLineBresenhami (OccGridMapBase.h:220-299)
  computed by the pure-Python restatement in this file (independent of the C oracle).
* ref_hector_logodds.npz -- outputs of the REFERENCE Hector log-odds cell functions
  (lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h, std-only, compiled unmodified into
  oracle/_ref/libhector_logodds_ref.so by oracle/Makefile): probToLogOdds factors, cell update
  sequences (updateSetFree / updateUnsetFree / updateSetOccupied / resetGridCell) and
  getGridProbability on a strided sample of every float log-odds -- the Hector oracle's A9 rows and
  its probability evaluation are pinned against these.
* gmapping_ref.npz -- outputs of the REFERENCE GMapping grid headers (lesson4/include/lesson4/
  gmapping/grid/*.h, compiled unmodified into oracle/_ref/libgmapping_ref.so by oracle/Makefile)
  on synthetic scans: the GMapping oracle and the GPU path are pinned against these.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "creating-2d-laser-slam-from-scratch_amd", "python"))

import oracle as O  # noqa: E402
from slam2d import synth  # noqa: E402


# ------------------------------------------------------------------ pure-Python Bresenham (KAT)
def py_ray_cells(sx, sy, x0, y0, x1, y1):
    """OccGridMapBase::updateLineBresenhami + bresenham2D (OccGridMapBase.h:220-299), cells only:
    [start (free), abs_da-1 intermediate (free) ..., end (occupied)]; [] if cancelled (:226-238)."""
    if x0 < 0 or x0 >= sx or y0 < 0 or y0 >= sy:
        return []
    if x1 < 0 or x1 >= sx or y1 < 0 or y1 >= sy:
        return []
    dx, dy = x1 - x0, y1 - y0
    adx, ady = abs(dx), abs(dy)
    odx = 1 if dx > 0 else -1                      # util::sign: sign(0) = -1 (UtilFunctions.h:55-58)
    ody = (1 if dy > 0 else -1) * sx
    off = y0 * sx + x0
    if adx >= ady:
        da, db, oa, ob = adx, ady, odx, ody
    else:
        da, db, oa, ob = ady, adx, ody, odx
    err = da // 2
    out = [off]
    for _ in range(max(da - 1, 0)):                 # `end = abs_da - 1` steps (unsigned; da >= 1 here)
        off += oa
        err += db
        if err >= da:
            off += ob
            err -= da
        out.append(off)
    out.append(y1 * sx + x1)
    return out


def ray_cells_fixture(rng):
    sx, sy = 97, 61
    rays = [(10, 10, 10, 10), (0, 0, 96, 60), (96, 60, 0, 0), (5, 30, 90, 30), (50, 0, 50, 60),
            (20, 20, 40, 40), (40, 40, 20, 20), (20, 40, 40, 20), (3, 3, 4, 3), (3, 3, 3, 4),
            (0, 0, 1, 1), (10, 10, -1, 10), (10, 10, 97, 10), (10, 61, 10, 10)]
    for _ in range(200):
        rays.append(tuple(int(v) for v in (rng.integers(0, sx), rng.integers(0, sy),
                                           rng.integers(-3, sx + 3), rng.integers(-3, sy + 3))))
    rays = np.asarray(rays, np.int32)
    cells, offs = [], [0]
    for r in rays:
        c = py_ray_cells(sx, sy, *[int(v) for v in r])
        cells += c
        offs.append(len(cells))
    return dict(sx=np.int32(sx), sy=np.int32(sy), rays=rays, cells=np.asarray(cells, np.uint32),
                offsets=np.asarray(offs, np.int64))


# ------------------------------------------------------------------ Hector sequences
def level_delta(ora, lvl):
    lo, upd = ora.level(lvl)
    idx = np.nonzero(upd.ravel() >= 0)[0].astype(np.int32)
    return idx, lo.ravel()[idx].view(np.int32), upd.ravel()[idx]


def hector_fixture(size, levels, n_scans, beams_stride, thresholds, reduce_threads, stream_seed):
    S = synth.make_streams(1, n_scans, seed=stream_seed)
    pts = [S.points[0, k, : S.counts[0, k]][::beams_stride] for k in range(n_scans)]
    counts = np.asarray([len(p) for p in pts], np.int32)
    packed = np.zeros((n_scans, max(counts.max(), 1), 2), np.float32)
    for k, p in enumerate(pts):
        packed[k, : len(p)] = p
    ora = O.HectorOracle(0.05, size, (0.5, 0.5), levels, reduce_threads=reduce_threads)
    ora.set_update_factors(0.4, 0.9)
    ora.set_thresholds(*thresholds)
    poses, covs, did, sumL = [], [], [], []
    for k in range(n_scans):
        p, c, d = ora.process(packed[k, : counts[k]])
        poses.append(p)
        covs.append(c)
        did.append(d)
        sumL.append(ora.sum_L())
    out = dict(size=np.int32(size), levels=np.int32(levels), thresholds=np.asarray(thresholds, np.float32),
               reduce_threads=np.int32(reduce_threads), points=packed, counts=counts,
               poses=np.asarray(poses, np.float32), covs=np.asarray(covs, np.float32),
               did_update=np.asarray(did, np.int32), sum_L=np.asarray(sumL, np.uint64))
    for lvl in range(levels):
        idx, lbits, upd = level_delta(ora, lvl)
        out[f"l{lvl}_idx"], out[f"l{lvl}_logodds_bits"], out[f"l{lvl}_upd"] = idx, lbits, upd
        out[f"l{lvl}_publish"] = ora.publish(lvl).ravel()[idx]
        out[f"l{lvl}_update_index"] = np.int32(ora.update_index(lvl))
    ora.close()
    return out


# ------------------------------------------------------------------ GMapping (reference build)
def gmapping_fixture(rng):
    ang = synth.beam_angles().astype(np.float64)
    segs = synth.world_segments()
    poses = [(0.0, 0.0, 0.0), (1.3, -0.7, 0.0), (-2.25, 1.5, 0.6), (4.0, 3.0, -2.1)]
    out = {"angles": ang}
    for i, (x, y, th) in enumerate(poses):
        r = synth.cast_ranges(np.asarray([[x, y, th]]), segs)[0].astype(np.float32)
        r = r + rng.normal(0, 0.01, r.shape).astype(np.float32)
        r[::97] = 0.0                        # d == 0 is skipped (gmapping.cc:183)
        r[5::113] = 27.0                     # > max_urange: clamped, no hit (gmapping.cc:186-190)
        r[7::131] = 35.0                     # > max_range: skipped
        r[11::151] = np.inf                  # non-finite: skipped
        c, s = np.cos(th), np.sin(th)
        n, v, acc, nfree, nhits = O.gm_compute(r, np.cos(ang), np.sin(ang), (x, y, c, s), which="ref")
        idx = np.nonzero(v.ravel())[0].astype(np.int32)
        out[f"p{i}_pose"] = np.asarray([x, y, c, s], np.float64)
        out[f"p{i}_ranges"] = r
        out[f"p{i}_idx"] = idx
        out[f"p{i}_n"] = n.ravel()[idx]
        out[f"p{i}_visits"] = v.ravel()[idx]
        out[f"p{i}_acc_bits"] = acc.reshape(-1, 2)[idx].view(np.int32)
        out[f"p{i}_counts"] = np.asarray([nfree, nhits], np.int64)
    return out


# ------------------------------------------------------------------ Hector log-odds (reference build)
def hector_logodds_fixture():
    import ctypes as C
    R = C.CDLL(os.path.join(HERE, "_ref", "libhector_logodds_ref.so"))
    R.hlr_prob_to_logodds.restype = C.c_float
    R.hlr_prob_to_logodds.argtypes = [C.c_float]
    R.hlr_factors.argtypes = [C.c_float, C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    R.hlr_apply_ops.restype = C.c_float
    R.hlr_apply_ops.argtypes = [C.c_float, C.c_int, C.c_void_p, C.c_int, C.c_float, C.c_float, C.POINTER(C.c_int)]
    R.hlr_grid_probability_n.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong]
    rng = np.random.default_rng(4711)
    probs = np.concatenate([np.asarray([0.4, 0.6, 0.9, 0.5, 0.1, 0.99, 0.01, 0.45, 0.55], np.float32),
                            rng.uniform(0.001, 0.999, 200).astype(np.float32)])
    p2l = np.asarray([R.hlr_prob_to_logodds(float(p)) for p in probs], np.float32)
    pairs = np.asarray([(-1.0, -1.0), (0.4, 0.9), (0.4, 0.6), (0.3, 0.7)], np.float32)
    facs = []
    for a, b in pairs:
        lf, lo = C.c_float(), C.c_float()
        R.hlr_factors(float(a), float(b), C.byref(lf), C.byref(lo))
        facs.append((lf.value, lo.value))
    # update sequences: ops 0 setFree, 1 unsetFree, 2 setOccupied, 3 resetGridCell
    n_seq, max_len = 400, 64
    starts = np.concatenate([np.asarray([0.0, 49.9, 50.0, 49.99999, -50.0, 48.5], np.float32),
                             rng.uniform(-60, 60, n_seq - 6).astype(np.float32)])
    ops = rng.integers(0, 4, (n_seq, max_len)).astype(np.int32)
    ops[:6] = 2                      # saturating occupied runs from the clamp neighbourhood
    lens = rng.integers(1, max_len + 1, n_seq).astype(np.int32)
    lens[:6] = max_len
    which = rng.integers(0, len(pairs), n_seq).astype(np.int32)
    final, upd = np.zeros(n_seq, np.float32), np.zeros(n_seq, np.int32)
    for i in range(n_seq):
        u = C.c_int()
        a, b = pairs[which[i]]
        final[i] = R.hlr_apply_ops(float(starts[i]), 7, ops[i].ctypes.data, int(lens[i]), float(a), float(b),
                                   C.byref(u))
        upd[i] = u.value
    # getGridProbability on every 16384th float bit pattern (both signs) plus specials
    pos = np.arange(0, 0x7F800001, 16384, dtype=np.uint64)
    bits = np.concatenate([pos, pos | 0x80000000, np.asarray([0x7F800000, 0xFF800000, 0x7FC00000, 0x80000000,
                                                              0x00000001, 0x80000001], np.uint64)])
    xs = bits.astype(np.uint32).view(np.float32).copy()
    pr = np.zeros_like(xs)
    R.hlr_grid_probability_n(xs.ctypes.data, pr.ctypes.data, len(xs))
    return dict(probs=probs, p2l_bits=p2l.view(np.int32), factor_pairs=pairs,
                factors_bits=np.asarray(facs, np.float32).view(np.int32), seq_start=starts, seq_ops=ops,
                seq_len=lens, seq_pair=which, seq_final_bits=final.view(np.int32), seq_upd=upd,
                prob_x_bits=xs.view(np.int32), prob_bits=pr.view(np.int32))


def main():
    os.makedirs(GOLD, exist_ok=True)
    rng = np.random.default_rng(20250212)
    np.savez_compressed(os.path.join(GOLD, "ray_cells.npz"), **ray_cells_fixture(rng))
    cases = {
        "hector_512x2_seq": (512, 2, 20, 1, (0.4, 0.9), 0, 4242),
        "hector_512x2_tree256": (512, 2, 20, 1, (0.4, 0.9), 256, 4242),
        "hector_512x2_64beam_forced": (512, 2, 20, 17, (-1.0, -1.0), 256, 777),
        # 12.8 m map, 64 beams: the scan leaves the map, H turns singular and the pose diverges to
        # NaN (as the reference's would); afterwards every point is out of map and the pose stays NaN
        "hector_256x2_64beam_diverge": (256, 2, 20, 17, (-1.0, -1.0), 256, 777),
        "hector_1024x1_tree256": (1024, 1, 12, 1, (0.4, 0.9), 256, 99),
    }
    for name, args in cases.items():
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **hector_fixture(*args))
    if os.path.exists(os.path.join(HERE, "_ref", "libgmapping_ref.so")):
        np.savez_compressed(os.path.join(GOLD, "gmapping_ref.npz"), **gmapping_fixture(rng))
    else:
        print("oracle/_ref missing: gmapping_ref.npz not regenerated", file=sys.stderr)
    if os.path.exists(os.path.join(HERE, "_ref", "libhector_logodds_ref.so")):
        np.savez_compressed(os.path.join(GOLD, "ref_hector_logodds.npz"), **hector_logodds_fixture())
    else:
        print("oracle/_ref missing: ref_hector_logodds.npz not regenerated", file=sys.stderr)
    for f in sorted(os.listdir(GOLD)):
        print(f, os.path.getsize(os.path.join(GOLD, f)))


if __name__ == "__main__":
    main()
