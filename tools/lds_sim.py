#!/usr/bin/env python3
"""Offline model of hs_update_kernel's raster LDS traffic: which mark words the lanes of one wave hit
with each free-mark atomic, and the LDS cycles that costs under the gfx950 banking rule for a 32-bit
LDS write / atomic (2 groups of 32 lanes, bank = word mod 32, one cycle per distinct lane on the
busiest bank: atomics do not broadcast).  Used to compare mark-array layouts and lane schedules
(stride, backward odd lanes, beam-to-lane order) before spending GPU time; not a test.

  python tools/lds_sim.py [--streams 2] [--scan 5]
"""
import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "creating-2d-laser-slam-from-scratch_amd", "python"))
from slam2d import synth  # noqa: E402

TILE, TH = int(os.environ.get("SIM_TW", 64)), int(os.environ.get("SIM_TH", 32))


def rays_for(points, pose_cell, theta, level):
    f = 1.0 / (1 << level)
    cs, sn = math.cos(theta), math.sin(theta)
    mx, my = pose_cell[0] * f, pose_cell[1] * f
    x0, y0 = int(mx + 0.5), int(my + 0.5)
    p = points * f
    ex = mx + (cs * p[:, 0] - sn * p[:, 1]) + 0.5
    ey = my + (sn * p[:, 0] + cs * p[:, 1]) + 0.5
    x1, y1 = ex.astype(np.int64), ey.astype(np.int64)
    return x0, y0, x1, y1


def walk(x0, y0, x1, y1):
    dx, dy = x1 - x0, y1 - y0
    adx, ady = abs(dx), abs(dy)
    sx, sy = (1 if dx > 0 else -1), (1 if dy > 0 else -1)
    if adx >= ady:
        return dict(xm=True, a0=x0, b0=y0, sa=sx, sb=sy, da=adx, db=ady, e0=adx // 2)
    return dict(xm=False, a0=y0, b0=x0, sa=sy, sb=sx, da=ady, db=adx, e0=ady // 2)


def cells_in_tile(w, X0, Y0):
    """free steps 0..da-1 of the walk inside the tile: list of (step, lx, ly)."""
    i = np.arange(w["da"])
    q = (w["e0"] + i * w["db"]) // max(w["da"], 1)
    a = w["a0"] + w["sa"] * i
    b = w["b0"] + w["sb"] * q
    x, y = (a, b) if w["xm"] else (b, a)
    m = (x >= X0) & (x < X0 + TILE) & (y >= Y0) & (y < Y0 + TH)
    return x[m] - X0, y[m] - Y0


ORDERS = {
    "id": lambda l: l,                                  # lane l: beam l of the fan
    "split": lambda l: 2 * (l & 31) + (l >> 5),         # lane group g (32 lanes): beams of parity g
}


def wave_cycles(fan_cells, stride, bwd_odd, order="id"):
    """fan_cells[b] = (lx, ly) arrays in walk order for beam b of the fan; lane l walks beam ORDERS[order](l)."""
    lanes_cells = [fan_cells[ORDERS[order](l)] for l in range(64)]
    n = [len(c[0]) for c in lanes_cells]
    addrs = []
    for l in range(64):
        lx, ly = lanes_cells[l]
        a = ly * stride + lx
        if (bwd_odd == 1 and (l & 1)) or (bwd_odd == 2 and l >= 32) or (bwd_odd == 3 and (l & 2)):
            a = a[::-1]
        addrs.append(a)
    # instruction schedule: 4-step trips, then one 2-step trip, then the last single step
    sched = []
    j = 0
    while any(4 * j + 3 < k for k in n):
        for u in range(4):
            sched.append([(l, 4 * j + u) for l in range(64) if 4 * j + 3 < n[l]])
        j += 1
    k4 = [4 * (k // 4) for k in n]
    if any(k - k4[l] >= 2 for l, k in enumerate(n)):
        for u in range(2):
            sched.append([(l, k4[l] + u) for l in range(64) if n[l] - k4[l] >= 2])
    k2 = [k4[l] + (2 if n[l] - k4[l] >= 2 else 0) for l in range(64)]
    if any(n[l] - k2[l] == 1 for l in range(64)):
        sched.append([(l, k2[l]) for l in range(64) if n[l] - k2[l] == 1])
    cyc = ideal = same = 0
    for ins in sched:
        for g in (0, 1):
            act = [addrs[l][s] for l, s in ins if (l >> 5) == g]
            if not act:
                continue
            act = np.asarray(act)
            banks = np.bincount(act % 32, minlength=32)
            cyc += int(banks.max())
            ideal += 1
            _, cnt = np.unique(act, return_counts=True)
            same += int(cnt.max() - 1)
    return cyc, ideal, len(sched), same



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--scan", type=int, default=5)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--map", type=int, default=2048)
    ap.add_argument("--detail", default="", help="variant: break its cycles down by level and origin tile")
    args = ap.parse_args()
    det = {}
    util = dict(pairs_bbox=0, pairs_line=0, tiles=0, tile_max4=0, tile_sum=0, tile_waves_busy=0, c_tests=0, c_chunks=0, c_cycles=0, c_instr=0, pairs=0, bbox_lanes=0, walk_lanes=0, lane_steps=0, walk_instr=0, waves_with_walk=0)
    S = synth.make_streams(args.streams, args.scan + 1, seed=4321)
    variants = {
        "s68": (68, 0, "id"), "s68_bidir_split": (68, 1, "split"), "s67_bidir_split": (67, 1, "split"),
        "s68_grpdir_id": (68, 2, "id"), "s67_grpdir_id": (67, 2, "id"), "s67_grpdir_split": (67, 2, "split"),
        "s68_pairdir_split": (68, 3, "split"), "s67_pairdir_split": (67, 3, "split"),
    }
    tot = {k: [0, 0, 0, 0] for k in variants}
    for s in range(args.streams):
        pts = S.points[s, args.scan, : S.counts[s, args.scan]].astype(np.float64)
        gt = S.gt[s, args.scan]
        pose_cell = (args.map / 2 + gt[0] * 20.0, args.map / 2 + gt[1] * 20.0)
        for lvl in range(args.levels):
            x0, y0, x1, y1 = rays_for(pts, pose_cell, gt[2], lvl)
            walks = [walk(x0, y0, int(a), int(b)) for a, b in zip(x1, y1)]
            nb = len(walks)
            xs = np.concatenate([[x0], x1]); ys = np.concatenate([[y0], y1])
            tx0, tx1 = xs.min() // TILE, xs.max() // TILE
            ty0, ty1 = ys.min() // TH, ys.max() // TH
            for ty in range(ty0, ty1 + 1):
                for tx in range(tx0, tx1 + 1):
                    X0, Y0 = tx * TILE, ty * TH
                    wave_instr = [0, 0, 0, 0]
                    for wv in range(4):
                        items = []
                        for g0 in range(64 * wv, nb, 256):
                            fb = [(min(x0, x1[b]), min(y0, y1[b]), max(x0, x1[b]), max(y0, y1[b])) for b in range(g0, min(g0 + 64, nb))]
                            if max(f[2] for f in fb) < X0 or min(f[0] for f in fb) >= X0 + TILE or max(f[3] for f in fb) < Y0 or min(f[1] for f in fb) >= Y0 + TH:
                                continue
                            util["c_tests"] += 1
                            for b in range(g0, min(g0 + 64, nb)):
                                c = cells_in_tile(walks[b], X0, Y0)
                                if len(c[0]):
                                    items.append(c)
                        for c0 in range(0, len(items), 64):
                            ch = items[c0:c0 + 64]
                            ch = ch + [(np.zeros(0, int), np.zeros(0, int))] * (64 - len(ch))
                            util["c_chunks"] += 1
                            r = wave_cycles(ch, 68, 1, "id")
                            util["c_cycles"] += r[0]; util["c_instr"] += r[2]
                            wave_instr[wv] += r[2]
                    if sum(wave_instr):
                        util["tiles"] += 1
                        util["tile_max4"] += 4 * max(wave_instr)
                        util["tile_sum"] += sum(wave_instr)
                        util["tile_waves_busy"] += sum(1 for x in wave_instr if x)
                    for g0 in range(0, nb, 64):
                        fb = [(x0, y0, x0, y0)] + [(min(x0, x1[b]), min(y0, y1[b]), max(x0, x1[b]), max(y0, y1[b]))
                                                   for b in range(g0, min(g0 + 64, nb))]
                        gx0 = min(f[0] for f in fb); gy0 = min(f[1] for f in fb)
                        gx1 = max(f[2] for f in fb); gy1 = max(f[3] for f in fb)
                        if gx1 < X0 or gx0 >= X0 + TILE or gy1 < Y0 or gy0 >= Y0 + TH:
                            continue
                        util["pairs"] += 1
                        bbl = sum(1 for f in fb[1:] if not (f[2] < X0 or f[0] >= X0 + TILE or f[3] < Y0 or f[1] >= Y0 + TH))
                        util["bbox_lanes"] += bbl
                        util["pairs_bbox"] += bbl > 0

                        def line_hits(b):  # segment vs the tile grown by one cell: corners not all on one side
                            if fb[1 + b - g0][2] < X0 or fb[1 + b - g0][0] >= X0 + TILE or fb[1 + b - g0][3] < Y0 or fb[1 + b - g0][1] >= Y0 + TH:
                                return False
                            nx, ny = y1[b] - y0, x0 - x1[b]
                            sv = [nx * (cx - x0) + ny * (cy - y0) for cx in (X0 - 1, X0 + TILE) for cy in (Y0 - 1, Y0 + TH)]
                            return not (min(sv) > 0 or max(sv) < 0)
                        util["pairs_line"] += any(line_hits(b) for b in range(g0, min(g0 + 64, nb)))
                        lanes = []
                        for l in range(64):
                            b = g0 + l
                            lanes.append(cells_in_tile(walks[b], X0, Y0) if b < nb else (np.zeros(0, int), np.zeros(0, int)))
                        nw = [len(c[0]) for c in lanes]
                        util["walk_lanes"] += sum(1 for k in nw if k)
                        util["lane_steps"] += sum(nw)
                        if not any(nw):
                            continue
                        util["waves_with_walk"] += 1
                        for k, (st, bw, od) in variants.items():
                            r = wave_cycles(lanes, st, bw, od)
                            for i in range(4):
                                tot[k][i] += r[i]
                            if k == args.detail:
                                key = (lvl, X0 <= x0 < X0 + TILE and Y0 <= y0 < Y0 + TH)
                                d = det.setdefault(key, [0, 0, 0, 0])
                                for i in range(4):
                                    d[i] += r[i]
    print("tiles with raster work %d, busy waves per tile %.2f, wave balance (sum / 4 max) %.3f" % (
        util["tiles"], util["tile_waves_busy"] / util["tiles"], util["tile_sum"] / util["tile_max4"]))
    print(util, "setup lanes busy %.3f (bbox) %.3f (walk) of 64 per pair" % (util["bbox_lanes"] / util["pairs"] / 64, util["walk_lanes"] / util["pairs"] / 64))
    base = tot["s68"][0]
    for k, (cyc, ideal, ins, same) in tot.items():
        if k == "s68":
            print(f"walk lane utilisation {util['lane_steps'] / (64 * ins):.3f} ({util['lane_steps']} lane-steps, {ins} walk instructions)")
        print(f"{k:12s} cycles {cyc:9d} ({cyc / base:5.3f})  conflict-free {ideal:9d}  instructions {ins:8d}  same-address extra {same:8d}")
    for (lvl, org), (cyc, ideal, ins, same) in sorted(det.items()):
        print(f"  {args.detail} level {lvl} {'origin tile' if org else 'other tiles'}: cycles {cyc:8d} conflict-free {ideal:8d} "
              f"instructions {ins:7d} same-address extra {same:7d}")


if __name__ == "__main__":
    main()
