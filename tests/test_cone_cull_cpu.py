"""CPU emulation of the cone cull tried for the update kernel in round 4 (S2D_WEDGE: fan_cone / cone_meets in
profiles/r04/update_variants_octet_wedge_batch.patch; measured slower, not in the product sources -- this pins the
restatement tools/visit_model.py uses to count the clip setups it would remove).

The cull may only drop a (tile, fan group) pair when no ray of the group marks a cell of the tile: every
cell of the Bresenham walk of bresenham2D (lesson4/include/lesson4/hector_mapping/map/OccGridMapBase.h
:270-299 in the reference, closed form as in ray_walk) must pass cone_meets for its group's cone.
Integer arithmetic as in the kernel; the float ordering of fan_cone uses float32 like the GPU.
"""
import numpy as np


def walk_cells(dx, dy):
    adx, ady = abs(dx), abs(dy)
    sx = 1 if dx > 0 else -1
    sy = 1 if dy > 0 else -1
    xm = adx >= ady
    da, db = (adx, ady) if xm else (ady, adx)
    sa, sb = (sx, sy) if xm else (sy, sx)
    e0 = da // 2
    i = np.arange(da + 1, dtype=np.int64)
    q = (e0 + i * db) // da
    a, b = sa * i, sb * q
    return (a, b) if xm else (b, a)


def fan_cone(rays):
    if not rays:
        return (0, 0, 0, 0)
    rdx, rdy = rays[0]
    dots = [rdx * dx + rdy * dy for dx, dy in rays]
    if min(dots) <= 0:
        return (0, 0, 0, 0)
    t = [np.float32(rdx * dy - rdy * dx) * (np.float32(1) / np.float32(d)) for (dx, dy), d in zip(rays, dots)]
    la, lb = int(np.argmax(t)), int(np.argmin(t))
    return (*rays[la], *rays[lb])


def cone_meets(w, px0, px1, py0, py1):
    cw_max = w[2] * np.where(w[2] >= 0, py1, py0) - w[3] * np.where(w[3] >= 0, px0, px1)
    ccw_min = w[0] * np.where(w[0] >= 0, py0, py1) - w[1] * np.where(w[1] >= 0, px1, px0)
    return (cw_max >= -2 * max(abs(w[2]), abs(w[3]))) & (ccw_min <= 2 * max(abs(w[0]), abs(w[1])))


def _fans(seed, n):
    rng = np.random.default_rng(seed)
    for _ in range(n):
        length = rng.choice([3, 40, 700, 5000])
        th0 = rng.uniform(0, 2 * np.pi)
        span = np.radians(rng.choice([0.0, 1.0, 16.0, 60.0, 89.0, 120.0])) * rng.uniform(0.5, 1.0)
        rays = []
        for k in range(64):
            a = th0 + span * k / 63
            r = rng.uniform(0.1, 1.0) * length
            d = (int(round(r * np.cos(a))), int(round(r * np.sin(a))))
            if d != (0, 0) and rng.random() > 0.15:
                rays.append(d)
        yield rays


def test_every_marked_cell_inside_its_cone():
    for rays in _fans(7, 150):
        w = fan_cone(rays)
        for dx, dy in rays[:16]:
            x, y = walk_cells(dx, dy)
            assert cone_meets(w, x, x, y, y).all(), (w, dx, dy)


def test_cull_drops_tiles_and_keeps_marked_ones():
    culled = total = 0
    for rays in _fans(11, 60):
        w = fan_cone(rays)
        xs = [0] + [d[0] for d in rays]
        ys = [0] + [d[1] for d in rays]
        marked = set()
        for dx, dy in rays:
            x, y = walk_cells(dx, dy)
            marked.update(zip((x // 64).tolist(), (y // 32).tolist()))
        for tx in range(min(xs) // 64, max(xs) // 64 + 1):
            for ty in range(min(ys) // 32, max(ys) // 32 + 1):
                total += 1
                keep = bool(cone_meets(w, tx * 64, tx * 64 + 63, ty * 32, ty * 32 + 31))
                assert keep or (tx, ty) not in marked
                culled += not keep
    assert culled > total // 4  # the cone prunes a good share of the group boxes


def test_no_cone_when_rays_spread_over_90_degrees():
    assert fan_cone([(10, 0), (0, 10), (-10, 1)]) == (0, 0, 0, 0)
    assert fan_cone([]) == (0, 0, 0, 0)
    w = (0, 0, 0, 0)
    assert bool(cone_meets(w, -100, -50, 7, 9))  # no cone: every tile the box meets stays
