"""The tile order of hs_update_ring_kernel, restated in Python and checked on the CPU.

The kernel keeps one cursor per ray and visits the tiles of a level's box in rings around the tile of the
scan's begin cell (csrc/hector_kernels.hip: RingIter, ring_split, ray_cursor).  That is only correct if
every ray meets its tiles in the visit order -- (ring k = Chebyshev distance in tiles, secondary distance
s = min(|dx|, |dy|)) strictly increasing at every tile change along the Bresenham walk of
OccGridMapBase.h:220-299 -- and if the enumeration yields every tile of the box exactly once.  Both are
checked here on random rays and boxes (64 x 32-cell tiles, as the kernel's LDS tiles).
"""
import numpy as np
import pytest

TILE, TH = 64, 32


def walk(x0, y0, x1, y1):
    """Cells of steps 0..da of bresenham2D (OccGridMapBase.h:270-299; e0 = da / 2, sign(0) = -1)."""
    dx, dy = x1 - x0, y1 - y0
    adx, ady = abs(dx), abs(dy)
    sx, sy = (1 if dx > 0 else -1), (1 if dy > 0 else -1)
    xm = adx >= ady
    da, db = (adx, ady) if xm else (ady, adx)
    e, x, y = da // 2, x0, y0
    out = [(x, y)]
    for _ in range(da):
        e += db
        if xm:
            x += sx
        else:
            y += sy
        if e >= da:
            e -= da
            if xm:
                y += sy
            else:
                x += sx
        out.append((x, y))
    return out


def key(tx, ty, ox, oy):
    ax, ay = abs(tx - ox), abs(ty - oy)
    return (max(ax, ay), min(ax, ay))


def ring_iter(kb, ox, oy, box):
    """RingIter::next, statement by statement (j: (k,s) (k,-s) (-k,s) (-k,-s) (s,k) (-s,k) (s,-k) (-s,-k))."""
    tx0, tx1, ty0, ty1 = box
    k, s, j = kb, 0, -1
    kmax = max(ox - tx0, tx1 - ox, oy - ty0, ty1 - oy)
    while k <= kmax:
        j += 1
        if j == 8:
            j = 0
            s += 1
            if s > k:
                s = 0
                k += 1
                if k > kmax:
                    return
        if k == 0 and j != 0:
            continue
        if (s == 0 and (j & 1)) or (s == k and j >= 4):
            continue
        u, v = (k, s) if j < 4 else (s, k)
        dx = -u if ((j & 2) if j < 4 else (j & 1)) else u
        dy = -v if ((j & 1) if j < 4 else (j & 2)) else v
        tx, ty = ox + dx, oy + dy
        if tx0 <= tx <= tx1 and ty0 <= ty <= ty1:
            yield tx, ty


def tiles_within(k, ox, oy, box):
    tx0, tx1, ty0, ty1 = box
    if k < 0:
        return 0
    w = min(tx1, ox + k) - max(tx0, ox - k) + 1
    h = min(ty1, oy + k) - max(ty0, oy - k) + 1
    return w * h if (w > 0 and h > 0) else 0


def ring_split(p, parts, kmax, ox, oy, box):
    kb, ke = 0, kmax + 1
    if parts <= 1:
        return kb, ke
    total = tiles_within(kmax, ox, oy, box)
    lo, hi = total * p // parts, total * (p + 1) // parts
    kb = 0 if p == 0 else kmax + 1
    for k in range(0, kmax + 1):
        before = tiles_within(k - 1, ox, oy, box)
        if p > 0 and kb > kmax and before >= lo and k > 0:
            kb = k
        if p < parts - 1 and ke > kmax and before >= hi and k > 0:
            ke = k
    return kb, max(ke, kb)


@pytest.fixture(params=[32, 64], ids=["th32", "th64"])
def tile_h(request):
    """The ring kernel's LDS tile height (S2D_RING_TH: 32 with 256-thread workgroups, 64 with 512)."""
    global TH
    old, TH = TH, request.param
    yield request.param
    TH = old


def test_every_ray_meets_its_tiles_in_ring_order(tile_h):
    rng = np.random.default_rng(7)
    for _ in range(3000):
        x0, y0 = (int(v) for v in rng.integers(0, 2048, 2))
        x1, y1 = (int(v) for v in rng.integers(0, 2048, 2))
        if (x0, y0) == (x1, y1):
            continue
        ox, oy = x0 // TILE, y0 // TH
        keys = []
        for x, y in walk(x0, y0, x1, y1):
            t = (x // TILE, y // TH)
            if not keys or keys[-1][0] != t:
                keys.append((t, key(t[0], t[1], ox, oy)))
        ks = [k for _, k in keys]
        assert all(a < b for a, b in zip(ks, ks[1:])), (x0, y0, x1, y1, keys)


def test_ring_enumeration_covers_the_box_once_in_key_order():
    rng = np.random.default_rng(11)
    for _ in range(300):
        tx0, ty0 = (int(v) for v in rng.integers(0, 20, 2))
        box = (tx0, tx0 + int(rng.integers(0, 15)), ty0, ty0 + int(rng.integers(0, 25)))
        ox, oy = int(rng.integers(box[0], box[1] + 1)), int(rng.integers(box[2], box[3] + 1))
        seq = list(ring_iter(0, ox, oy, box))
        want = {(x, y) for x in range(box[0], box[1] + 1) for y in range(box[2], box[3] + 1)}
        assert len(seq) == len(want) and set(seq) == want
        ks = [key(x, y, ox, oy) for x, y in seq]
        assert ks == sorted(ks)
        # parts: contiguous ring ranges whose tile counts add up to the box, each enumerated from its first ring
        kmax = max(ox - box[0], box[1] - ox, oy - box[2], box[3] - oy)
        for parts in (2, 3, 8):
            got = []
            for p in range(parts):
                kb, ke = ring_split(p, parts, kmax, ox, oy, box)
                n = tiles_within(ke - 1, ox, oy, box) - tiles_within(kb - 1, ox, oy, box)
                it = ring_iter(kb, ox, oy, box)
                got += [next(it) for _ in range(n)]
            assert sorted(got) == sorted(want) and got == seq


def ray_cursor(x0, y0, x1, y1, K, ox, oy):
    """ray_cursor (csrc/hector_kernels.hip): the first step i of the walk inside ring >= K and its minor steps q."""
    dx, dy = x1 - x0, y1 - y0
    adx, ady = abs(dx), abs(dy)
    xm = adx >= ady
    da, db = (adx, ady) if xm else (ady, adx)
    sxn, syn = dx <= 0, dy <= 0
    if K == 0:
        return 0, 0
    e0 = da >> 1
    Dx = x0 - ((ox - K) * TILE + TILE - 1) if sxn else (ox + K) * TILE - x0
    Dy = y0 - ((oy - K) * TH + TH - 1) if syn else (oy + K) * TH - y0
    INF = 0x7FFF
    dma, dmi = (Dx, Dy) if xm else (Dy, Dx)
    im = dma if dma <= da else INF
    inn = (dmi * da - e0 + db - 1) // db if dmi <= db else INF
    i = min(im, inn)
    if i > da:
        return None
    return i, (e0 + i * db) // da


def test_ray_cursor_is_the_first_step_in_the_ring(tile_h):
    rng = np.random.default_rng(3)
    for _ in range(3000):
        x0, y0 = (int(v) for v in rng.integers(0, 2048, 2))
        x1, y1 = (int(v) for v in rng.integers(0, 2048, 2))
        if (x0, y0) == (x1, y1):
            continue
        ox, oy = x0 // TILE, y0 // TH
        cells = walk(x0, y0, x1, y1)
        xm = abs(x1 - x0) >= abs(y1 - y0)
        for K in (1, 2, 3, 5, 9, 20):
            want = next((i for i, (x, y) in enumerate(cells) if max(abs(x // TILE - ox), abs(y // TH - oy)) >= K), None)
            got = ray_cursor(x0, y0, x1, y1, K, ox, oy)
            if want is None:
                assert got is None, (x0, y0, x1, y1, K)
                continue
            # q = minor steps before step `want`: the minor coordinate's distance from the begin cell
            x, y = cells[want]
            assert got == (want, abs(y - y0) if xm else abs(x - x0)), (x0, y0, x1, y1, K, got, want)


STRIDE = 68  # LDS words per tile row (UPD_STRIDE)


def ring_visit(C, S, rx0, ry0, bwd):
    """ring_visit (csrc/hector_kernels.hip) statement by statement on integers: returns (new cursor, marked
    free cells in walk order as (lx, ly), the hit cell or None), or None if the cursor is not in the tile.
    The packed walk register V = f << 18 | LDS byte address is emulated exactly (32-bit wrap-around)."""
    da, db = C & 0x3FFF, (C >> 14) & 0x3FFF
    mx, my = -((C >> 28) & 1), -((C >> 29) & 1)
    xm = (C >> 30) & 1
    i, q = S & 0xFFFF, S >> 16
    ix, iy = (i, q) if xm else (q, i)
    lx, ly = rx0 + ((ix ^ mx) - mx), ry0 + ((iy ^ my) - my)
    if i > da or not (0 <= lx < TILE) or not (0 <= ly < TH):
        return None
    rx, ry = lx ^ ((TILE - 1) & ~mx), ly ^ ((TH - 1) & ~my)
    ra, rb = (rx, ry) if xm else (ry, rx)
    e = (da >> 1) + i * db - q * da
    n = min(ra + 1, da - i + 1)
    if db:
        n = min(n, ((rb + 1) * da - e + db - 1) // db)
    k, el = divmod(e + (n - 1) * db, da)
    last = i + n - 1
    hit = last == da
    Sn = (last + 1) | ((q + k + (1 if el + db >= da else 0)) << 16)
    hitcell = None
    if hit:
        ta, tb = (n - 1, k) if xm else (k, n - 1)
        hitcell = (lx + ((ta ^ mx) - mx), ly + ((tb ^ my) - my))
    nfree = n - int(hit)
    cells = []
    if nfree > 0:
        bm = -1 if bwd else 0
        um = hit and el < db
        ts = bm & (n - 1 - int(hit))
        ks = bm & (k - int(um))
        es = (el - (db if hit else 0) + (da if um else 0)) if bm else da - 1 - e
        sxs, sys_ = (ts, ks) if xm else (ks, ts)
        lxs, lys = lx + ((sxs ^ mx) - mx), ly + ((sys_ ^ my) - my)
        dx4, dy4 = (4 ^ mx) - mx, ((4 * STRIDE) ^ my) - my
        dab1, dab21 = (dx4 if xm else dy4), dx4 + dy4
        dab, dab2 = (dab1 ^ bm) - bm, (dab21 ^ bm) - bm
        M = 0xFFFFFFFF
        vdn = (db << 18) & M
        vk_major, vk_minor = dab & M, ((da << 18) + dab2) & M
        base = 4096  # any LDS byte address of the buffer
        v = ((es << 18) + base + (lys * STRIDE + lxs) * 4) & M
        for _ in range(nfree):
            a = ((v & 0x3FFFF) - base) // 4
            cells.append((a % STRIDE, a // STRIDE))
            borrow = v < vdn
            v = ((v - vdn) + (vk_minor if borrow else vk_major)) & M
    return Sn, cells, hitcell


def test_ring_visits_mark_exactly_the_walk(tile_h):
    """Every ray, visited tile by tile in ring order through ring_visit (forward and backward lanes), marks
    exactly the cells of its Bresenham walk: steps 0..da-1 free, step da the end cell."""
    rng = np.random.default_rng(5)
    for trial in range(1500):
        x0, y0 = (int(v) for v in rng.integers(0, 1024, 2))
        r = int(rng.choice([3, 40, 300, 900]))
        x1 = int(np.clip(x0 + rng.integers(-r, r + 1), 0, 1023))
        y1 = int(np.clip(y0 + rng.integers(-r, r + 1), 0, 1023))
        if (x0, y0) == (x1, y1):
            continue
        dx, dy = x1 - x0, y1 - y0
        xm = abs(dx) >= abs(dy)
        da, db = (abs(dx), abs(dy)) if xm else (abs(dy), abs(dx))
        C = da | (db << 14) | (int(dx <= 0) << 28) | (int(dy <= 0) << 29) | (int(xm) << 30)
        cells = walk(x0, y0, x1, y1)
        box = (min(x0, x1) // TILE, max(x0, x1) // TILE, min(y0, y1) // TH, max(y0, y1) // TH)
        ox, oy = x0 // TILE, y0 // TH
        for bwd in (False, True):
            S, free, hits = 0, [], []
            for tx, ty in ring_iter(0, ox, oy, box):
                out = ring_visit(C, S, x0 - tx * TILE, y0 - ty * TH, bwd)
                if out is None:
                    continue
                S, fc, hc = out
                fc = [(tx * TILE + a, ty * TH + b) for a, b in fc]
                free += fc[::-1] if bwd else fc
                if hc is not None:
                    hits.append((tx * TILE + hc[0], ty * TH + hc[1]))
            assert free == cells[:-1] and hits == [cells[-1]], (trial, bwd, x0, y0, x1, y1)
            assert (S & 0xFFFF) == da + 1


def ring_split_w(p, parts, kmax, ox, oy, box, hist, tile_w=64):
    """ring_split_w (csrc/hector_kernels.hip): ring k weighs tile_w per box tile + the rays reaching it."""
    w = []
    for k in range(kmax + 1):
        reach = sum(hist[min(k, len(hist) - 1):])
        w.append(tile_w * (tiles_within(k, ox, oy, box) - tiles_within(k - 1, ox, oy, box)) + reach)
    total = sum(w)
    lo, hi = total * p // parts, total * (p + 1) // parts
    before = np.concatenate([[0], np.cumsum(w)[:-1]])
    kb = 0 if p == 0 else next((k for k in range(1, kmax + 1) if before[k] >= lo), kmax + 1)
    ke = kmax + 1 if p == parts - 1 else next((k for k in range(1, kmax + 1) if before[k] >= hi), kmax + 1)
    return kb, max(ke, kb)


def test_weighted_ring_split_partitions_the_rings():
    rng = np.random.default_rng(13)
    for _ in range(400):
        tx0, ty0 = (int(v) for v in rng.integers(0, 20, 2))
        box = (tx0, tx0 + int(rng.integers(0, 15)), ty0, ty0 + int(rng.integers(0, 25)))
        ox, oy = int(rng.integers(box[0], box[1] + 1)), int(rng.integers(box[2], box[3] + 1))
        kmax = max(ox - box[0], box[1] - ox, oy - box[2], box[3] - oy)
        hist = rng.integers(0, 200, 128) * (np.arange(128) <= kmax)
        for parts in (2, 3, 8):
            cuts = [ring_split_w(p, parts, kmax, ox, oy, box, hist) for p in range(parts)]
            assert cuts[0][0] == 0 and cuts[-1][1] == kmax + 1
            assert all(cuts[p][1] == cuts[p + 1][0] for p in range(parts - 1)), cuts
