#!/usr/bin/env python3
"""CPU model (no GPU) of a bitmap log for the update's ordinal plane.

Runs the oracle over one synthetic north-star stream (2048^2 x 3 levels, forced updates) and reports, per level:
cells marked per scan, 64 x 32 tiles with marks per scan, and for a fold every F scans the union of marked cells
and tiles -- the log's size (one bit word per marked tile and wave) and the fold's writes (each union cell once).
Box tiles (the kernel's tile loop) are printed last.
    python3 tools/ordlog_model.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "creating-2d-laser-slam-from-scratch_amd", "python"))
import oracle as O  # noqa: E402
from slam2d import synth  # noqa: E402

T = 40
S = synth.make_streams(1, T, seed=12345)
ora = O.HectorOracle(0.05, 2048, (0.5, 0.5), 3)
ora.set_update_factors(0.4, 0.9); ora.set_thresholds(-1.0, -1.0)
hist = {l: [] for l in range(3)}
for t in range(T):
    n = int(S.counts[0, t]) if hasattr(S, "counts") else S.points.shape[2]
    ora.process(S.points[0, t, :n])
    for l in range(3):
        _, u = ora.level(l)
        k = ora.cur_update_index(l) // 3 - 1
        m = (u == 3 * k + 1) | (u == 3 * k + 2)
        hist[l].append(m)
for l in range(3):
    H, W = hist[l][0].shape
    def tiles(m):
        th, tw = (H + 31) // 32, (W + 63) // 64
        mm = np.zeros((th * 32, tw * 64), bool); mm[:H, :W] = m
        return mm.reshape(th, 32, tw, 64).any(axis=(1, 3))
    cells = np.mean([m.sum() for m in hist[l][5:]])
    tv = np.mean([tiles(m).sum() for m in hist[l][5:]])
    for F in (1, 4, 8, 16, 32):
        uc = []; ut = []
        for s in range(5, T - F + 1, F):
            u = np.zeros_like(hist[l][0])
            for m in hist[l][s:s + F]: u |= m
            uc.append(u.sum()); ut.append(tiles(u).sum())
        print(f"L{l} {H}x{W}: cells/scan {cells:.0f} tiles/scan {tv:.0f} | F={F}: union cells {np.mean(uc):.0f} ({np.mean(uc)/F:.0f}/scan) union tiles {np.mean(ut):.0f}")
# box tiles per level: bbox of all marked cells (upper bound on the kernel's box is origin + end cells)
for l in range(3):
    bt = []
    for m in hist[l][5:]:
        ys, xs = np.nonzero(m)
        bt.append((xs.max() // 64 - xs.min() // 64 + 1) * (ys.max() // 32 - ys.min() // 32 + 1))
    print(f"L{l}: box tiles/scan {np.mean(bt):.0f} (max {max(bt)})")
