#!/usr/bin/env python3
"""CPU model of hs_update_kernel's (tile, fan group) visits on the north-star scans (no GPU).

For a few synthetic scans (python/slam2d/synth.py, 2048^2 x 3 levels at 20 cells/m) counts, per level:
  tiles of the scan's box; (tile, group) pairs the box ballot passes; of those, pairs where some lane's own
  ray box meets the tile (the wave runs the clip setup); pairs where some lane's walk has a step in the tile
  (useful setups); the cone cull's (S2D_WEDGE) survivors; and the lane occupancy of the setups.
    python3 tools/visit_model.py [scans]

Round 6 adds the per-tile wave balance: each tile's raster is run by the four waves of the
workgroup, wave w taking the fan groups fi = w, w + 4, ...; a wave's raster cost on a tile is modelled as
SETUP instructions per (tile, group) clip setup plus STEP per step of the longest walk among the group's lanes
in that tile.  The barrier after the raster makes the busiest wave the tile's path, so the model prints, per
level, sum over tiles of the busiest wave's cost / sum of the mean wave's cost, the share of tiles (with steps)
crossed by <= 2 fan groups, and the same ratio for two alternatives: two-wave workgroups on 64 x 16 tiles
(groups fi = w, w + 2, ...), whose busiest wave summed over a 64 x 32 area is the last column; eight-wave
workgroups on 64 x 64 tiles; and the wave-slot time (waves x busiest wave) of those and of four waves sharing a
tile crossed by one or two groups (each group's walks split over 4 / G waves).  Both of the latter were built and
measured slower (profiles/r06/ab_r06y_update_8waves.md: +26 %, ab_r06z_update_split.md: +16.5 %), so neither the
busiest-wave nor the slot-time reading of this model predicts the kernel.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "creating-2d-laser-slam-from-scratch_amd", "python"))
from slam2d import synth  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_cone_cull_cpu import cone_meets, fan_cone, walk_cells  # noqa: E402

TILE, TILE_H = 64, 32
SETUP, STEP = 150, 5  # VALU-instruction model of one (tile, group) clip setup and one walk step


def level_rays(pts, pose, level, size=2048):
    f = 1.0 / (1 << level)
    cx = cy = size / (1 << level) / 2.0
    c, s = np.cos(pose[2]), np.sin(pose[2])
    mx, my = cx + pose[0] * 20.0 * f, cy + pose[1] * 20.0 * f
    x0, y0 = int(mx + 0.5), int(my + 0.5)
    px, py = pts[:, 0] * f, pts[:, 1] * f
    x1 = (mx + c * px - s * py + 0.5).astype(int)
    y1 = (my + s * px + c * py + 0.5).astype(int)
    return x0, y0, x1, y1


def main():
    nscans = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ss = synth.make_streams(nscans, 1, distinct_paths=nscans)
    tot = np.zeros((3, 7))
    segs = np.zeros(3)
    bal = {(lvl, nw): np.zeros(4) for lvl in range(3) for nw in (4, 2, 8)}
    split = np.zeros((3, 2))  # 4 waves, groups split over idle waves: sum of busiest, tiles
    for k in range(nscans):
        pts = ss.points[k, 0, :ss.counts[k, 0]]
        pose = ss.gt[k, 0] * 0  # first scan of each path: pose (0, 0, 0) in its own frame
        for lvl in range(3):
            x0, y0, x1, y1 = level_rays(pts, pose, lvl)
            n = len(x1)
            valid = ~((x1 == x0) & (y1 == y0))
            cells = [walk_cells(int(a - x0), int(b - y0)) if v else (np.zeros(0, int), np.zeros(0, int))
                     for a, b, v in zip(x1, y1, valid)]
            tiles_of = [set(zip(((cx + x0) // TILE).tolist(), ((cy + y0) // TILE_H).tolist())) for cx, cy in cells]
            bx0, bx1 = min(x0, x1.min()) // TILE, max(x0, x1.max()) // TILE
            by0, by1 = min(y0, y1.min()) // TILE_H, max(y0, y1.max()) // TILE_H
            ntiles = (bx1 - bx0 + 1) * (by1 - by0 + 1)
            ballot = setup = useful = cone_pass = cone_setup = seg_setup = 0
            lanes_setup = lanes_useful = 0
            for g in range(0, n, 64):
                idx = np.arange(g, min(g + 64, n))
                gv = idx[valid[idx]]
                if len(gv) == 0:
                    continue
                gx0, gx1 = min(x0, x1[gv].min()), max(x0, x1[gv].max())
                gy0, gy1 = min(y0, y1[gv].min()), max(y0, y1[gv].max())
                w = fan_cone([(int(x1[i] - x0), int(y1[i] - y0)) for i in gv])
                for tx in range(gx0 // TILE, gx1 // TILE + 1):
                    for ty in range(gy0 // TILE_H, gy1 // TILE_H + 1):
                        X0, Y0 = tx * TILE, ty * TILE_H
                        ballot += 1
                        own = [i for i in gv if max(x0, x1[i]) >= X0 and min(x0, x1[i]) < X0 + TILE and
                               max(y0, y1[i]) >= Y0 and min(y0, y1[i]) < Y0 + TILE_H]
                        use = [i for i in own if (tx, ty) in tiles_of[i]]
                        # segment test (round 6): the lane's ray line against the tile's integer box; a Bresenham cell
                        # lies within |cross| < (da + 1) / 2 of the line, so all four corners beyond +-da on one side
                        # means no cell of the ray in the tile (conservative)
                        seg = []
                        for i in own:
                            ddx, ddy = int(x1[i] - x0), int(y1[i] - y0)
                            da_ = max(abs(ddx), abs(ddy))
                            cr = [ddx * (cy - y0) - ddy * (cx - x0) for cx in (X0, X0 + TILE - 1) for cy in (Y0, Y0 + TILE_H - 1)]
                            if not (min(cr) > da_ or max(cr) < -da_):
                                seg.append(i)
                        assert set(use) <= set(seg), "segment test rejected a ray with steps in the tile"
                        seg_setup += bool(seg)
                        cm = bool(cone_meets(w, X0 - x0, X0 + TILE - 1 - x0, Y0 - y0, Y0 + TILE_H - 1 - y0))
                        cone_pass += cm
                        if own:
                            setup += 1
                            cone_setup += cm
                            lanes_setup += len(own)
                            lanes_useful += len(use)
                        if use:
                            useful += 1
            tot[lvl] += [ntiles, ballot, setup, useful, cone_setup, lanes_setup, lanes_useful]
            segs[lvl] += seg_setup
            # wave balance: per (tile, fan group) the clip setup and the longest walk of its lanes in the tile
            for th, nw in ((TILE_H, 4), (TILE_H // 2, 2), (TILE_H * 2, 8)):
                cost = {}  # tile -> per-wave cost
                ngroups = {}
                for i in range(n):
                    if not valid[i]:
                        continue
                    cx, cy = cells[i]
                    tx = (cx + x0) // TILE
                    ty = (cy + y0) // th
                    # free steps are cells 0..L-1 (the end cell is the hit); count per tile
                    keys, cnt = np.unique(np.stack([tx[:-1], ty[:-1]], 1), axis=0, return_counts=True) if len(tx) > 1 \
                        else (np.zeros((0, 2), int), np.zeros(0, int))
                    fi = i // 64
                    for (a, b), c in zip(keys.tolist(), cnt.tolist()):
                        d = cost.setdefault((a, b), {})
                        d[fi] = max(d.get(fi, 0), c)
                busy = mean = 0.0
                few = 0
                for t, d in cost.items():
                    w = np.zeros(nw)
                    for fi, steps in d.items():
                        w[fi % nw] += SETUP + STEP * steps
                    busy += w.max()
                    mean += w.mean()
                    few += len(d) <= 2
                    if nw == 4:
                        # split alternative: a tile crossed by G < 4 groups gives each group 4 // G waves, which split
                        # its lanes' walks (every wave runs the group's clip setup)
                        G = len(d)
                        kk = max(1, 4 // G)
                        ws = np.zeros(4)
                        for j, (fi, steps) in enumerate(sorted(d.items())):
                            for q in range(kk if G < 4 else 1):
                                ws[(j * kk + q) % 4 if G < 4 else fi % 4] += SETUP + STEP * -(-steps // kk)
                        split[lvl] += [ws.max(), 1]
                bal[(lvl, nw)] += np.array([busy, mean, few, len(cost)])
    print(f"{nscans} scans; per scan and level:")
    print("level  box-tiles  ballot-pairs  setups  useful-setups  setups-after-cone  lanes/setup  useful-lanes/setup")
    for lvl in range(3):
        t = tot[lvl] / nscans
        print(f"{lvl:5d} {t[0]:10.0f} {t[1]:13.0f} {t[2]:7.0f} {t[3]:14.0f} {t[4]:18.0f} {t[5] / max(t[2], 1):12.1f} "
              f"{t[6] / max(t[2], 1):19.1f}")
    print("setups surviving the segment test (some lane's ray line meets the tile's box; round 6):",
          ", ".join(f"level {lvl}: {segs[lvl] / nscans:.0f}" for lvl in range(3)))
    print(f"wave balance (model: {SETUP} per clip setup + {STEP} per walk step; busiest wave / mean wave, summed over tiles):")
    print("level  4 waves x 64x32: busiest/mean  tiles<=2 groups  raster per tile (busiest)  |  2 waves x 64x16: busiest/mean  "
          "raster per 64x32 area (busiest)")
    for lvl in range(3):
        b4, b2 = bal[(lvl, 4)], bal[(lvl, 2)]
        print(f"{lvl:5d} {b4[0] / b4[1]:31.2f} {b4[2] / b4[3]:16.2f} {b4[0] / b4[3]:26.0f}  |  {b2[0] / b2[1]:31.2f} "
              f"{b2[0] / b4[3]:31.0f}")
    print("8 waves x 64x64 tiles (512-thread workgroups): per level busiest/mean, busiest raster per 64x64 tile, per "
          "64x32 area, total raster work per 64x32 area vs the 4-wave design's")
    for lvl in range(3):
        b4, b8 = bal[(lvl, 4)], bal[(lvl, 8)]
        print(f"{lvl:5d} {b8[0] / b8[1]:8.2f} {b8[0] / b8[3]:10.0f} {b8[0] / b4[3]:10.0f}   total {8 * b8[1] / b4[3]:8.0f} vs "
              f"{4 * b4[1] / b4[3]:8.0f}   tiles with steps {b8[3] / nscans:6.0f} vs {b4[3] / nscans:6.0f}")
    # Wave-slot time: a wave waiting at the tile's barrier holds its slot (registers, LDS) -- with every slot of the
    # CU taken, the raster's throughput is set by waves x busiest, not by the busiest alone.  This is the reading
    # the 8-wave build measured (profiles/r06/ab_r06y_update_8waves.md: +33 % slot time here, +26 % update there).
    print("wave-slot time of the raster per 64x32 area (waves x busiest wave), relative to the 4-wave design:")
    print("level   4 waves   2 waves x 64x16   8 waves x 64x64   4 waves, groups split over idle waves")
    for lvl in range(3):
        b4, b2, b8 = bal[(lvl, 4)], bal[(lvl, 2)], bal[(lvl, 8)]
        s4 = 4 * b4[0]
        print(f"{lvl:5d} {s4 / b4[3]:9.0f} {2 * b2[0] / s4:17.2f} {8 * b8[0] / s4:17.2f} {4 * split[lvl][0] / s4:38.2f}")


if __name__ == "__main__":
    main()
