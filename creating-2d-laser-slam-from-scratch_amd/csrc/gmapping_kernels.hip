// gmapping_kernels.hip -- MI355X kernels of the GMapping particle-map path (config 4).
//
//   gm_score_kernel     one workgroup per particle: the particle's score of the new scan against its
//                       previous map (read before it is overwritten); opens the particle's new step.
//   gm_compute_kernel   `parts` 256-thread workgroups per particle: GMapping::ComputeMap
//                       (lesson4/src/gmapping/gmapping.cc:171-242) of the shared scan seen from the
//                       particle's pose, into the particle's tiled packed-count map (part q draws
//                       tiles q, q + parts, ...) and its hit-cell slots (one per beam: the slot of a
//                       cell's first hitting beam carries the cell and its accumulators).
//
// Per tile (round 6, the Hector update's idioms): one ballot picks the fan groups whose box meets the tile;
// the raster marks counts (and first-hit words) in LDS; an acc pass runs only when some beam ends in the tile;
// the counts are stored whole (a fresh map) by threads that zero the words they stored, so a tile needs
// no clear; first-hit words are restored by each hit cell's first beam.  Odd lanes walk backwards and each
// 32-lane half of a wave spans its 64-beam fan, spreading the LDS atomics near the scan origin.
//
// Raster: GridLineTraversal::gridLine (lesson4/include/lesson4/gmapping/grid/gridlinetraversal.h:
// 27-207) starts at the endpoint with the smaller major coordinate and, with decision variable
// d = 2 db - da, steps the minor axis when d >= 0.  In closed form, step i from that start is
//     (a_s + i, b_s + sb * q(i)),  q(i) = floor((2 db i + da) / (2 da)),  i in [0, da]
// (checked against the incremental walk on 200k random lines), so every lane clips its line to
// a tile directly.  points[0 .. num_points-2] (all but the end cell p1) get visits++ (:227-234);
// the end cell of a hit beam gets n++, visits++ and acc += (float)hit (:236-240, map.h:37-48).
// Counts are order-free integers (LDS atomicAdd on n << 16 | visits); acc is a float sum in beam
// order, so a cell hit by several beams is summed sequentially by its first beam's lane.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gmapping_internal.h"

namespace s2d {

// n / d for n < 2^31, 1 <= d < 2^16, exact when the quotient is < 2^16 (see hector_kernels.hip
// udiv_small; larger quotients only ever mean "beyond the line")
__device__ __forceinline__ unsigned gm_udiv(unsigned n, unsigned d)
{
    unsigned q = (unsigned)((float)n * __builtin_amdgcn_rcpf((float)d));
    int r = (int)(n - q * d);
    if (r < 0) {
        --q;
        r += (int)d;
    }
    if (r >= (int)d) ++q;
    return q;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations but not for its global
// stores (__syncthreads' release fence drains vmcnt, which parked every wave on the previous tile's
// 8 KB of count stores at each tile: 72 % of wave cycles waiting, r02o PMC).  The stores go to the
// particle's own map, which no wave of this kernel reads.
__device__ __forceinline__ void gm_lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#ifndef GM_BALLOT
#define GM_BALLOT 1  // fan groups culled per tile by one ballot (lane f tests group f); 0: a scalar box test per group
#endif
#ifndef GM_RESTORE
#define GM_RESTORE 1  // the count array is zeroed by the threads that store it (no clear + barrier per tile); 0: A/B
#endif
#ifndef GM_BWD
#define GM_BWD 1  // odd lanes walk their steps backwards (neighbouring beams at different radii: fewer lanes per LDS word)
#endif
#ifndef GM_FAN
#define GM_FAN 1  // lane l of a fan group rasters beam 2 (l % 32) + l / 32: each 32-lane half spans the fan (0: A/B)
#endif
#ifndef GM_PACKED
#define GM_PACKED 1  // the walk's error term and LDS address packed in one register, eight steps per trip (0: A/B)
#endif
#ifndef GM_PRICE
#define GM_PRICE 0  // timing-only pricing builds (wrong maps): 1 no acc pass, 2 no count stores (invalid with
                    // GM_RESTORE: the counts then pile up), 3 no walk steps
#endif
// 32-bit LDS byte address of an LDS pointer, and back (GM_PACKED carries addresses in packed registers)
typedef __attribute__((address_space(3))) unsigned gm_lds_u32;
__device__ __forceinline__ unsigned gm_lds_addr(unsigned *p) { return (unsigned)(size_t)(gm_lds_u32 *)p; }
__device__ __forceinline__ unsigned *gm_lds_ptr(unsigned a) { return (unsigned *)(gm_lds_u32 *)(size_t)a; }
constexpr int GM_STRIDE = 68;                          // LDS words per tile row (16-B rows)
constexpr int GM_LDS_WORDS = GM_TILE_H * GM_STRIDE;    // one LDS tile array

// Map::world2map (G/grid/map.h:171-174): round((p - center) / delta) + size/2, in double
__device__ __forceinline__ void gm_world2map(const GmGeom &g, double wx, double wy, int &mx, int &my)
{
    mx = (int)round((wx - g.cx) / g.delta) + g.sx2;
    my = (int)round((wy - g.cy) / g.delta) + g.sy2;
}

// packed ray: hit flag | (dy + 16384) << 16 | (dx + 16384), end cell relative to p0
constexpr int GM_REL = 16384;
__device__ __forceinline__ unsigned gm_pack(int dx, int dy, bool hit)
{
    return (hit ? GM_RAY_HIT : 0u) | ((unsigned)(dy + GM_REL) << 16) | (unsigned)(dx + GM_REL);
}

// One beam's grid line in (major a, minor b) coordinates, from its smaller-major end S.
struct GmLine {
    int as, bs, sb;   // start, minor direction
    int da, db;       // |major|, |minor| extent
    bool x_major;     // dy <= dx (gridlinetraversal.h:49)
    int ilo, ihi;     // free step range (the step of p1 excluded)
};

__device__ __forceinline__ GmLine gm_line(int x0, int y0, int x1, int y1)
{
    GmLine l;
    const int dx = abs(x1 - x0), dy = abs(y1 - y0);
    l.x_major = dy <= dx;
    int a0 = l.x_major ? x0 : y0, b0 = l.x_major ? y0 : x0;
    int a1 = l.x_major ? x1 : y1, b1 = l.x_major ? y1 : x1;
    const bool p1_is_start = a1 < a0;  // the walk starts at the smaller major coordinate
    l.as = p1_is_start ? a1 : a0;
    l.bs = p1_is_start ? b1 : b0;
    const int be = p1_is_start ? b0 : b1;
    l.sb = be > l.bs ? 1 : -1;
    l.da = l.x_major ? dx : dy;
    l.db = l.x_major ? dy : dx;
    l.ilo = p1_is_start ? 1 : 0;                // p1 = step 0 or step da is not freed
    l.ihi = p1_is_start ? l.da : l.da - 1;
    return l;
}

// Steps of the line inside [A0, A1) x [B0, B1) (major x minor), intersected with [lo, hi].
__device__ __forceinline__ bool gm_clip(const GmLine &l, int A0, int A1, int B0, int B1, int &lo, int &hi)
{
    lo = max(lo, A0 - l.as);
    hi = min(hi, A1 - 1 - l.as);
    if (lo > hi) return false;
    // minor range as q = (b - bs) * sb
    const int tlo = l.sb > 0 ? B0 - l.bs : l.bs - (B1 - 1);
    const int thi = l.sb > 0 ? B1 - 1 - l.bs : l.bs - B0;
    if (thi < 0) return false;
    if (l.db == 0) return tlo <= 0;  // q == 0 everywhere
    const unsigned two_da = 2u * (unsigned)l.da, two_db = 2u * (unsigned)l.db;
    if (tlo > 0) {  // smallest i with q(i) >= tlo
        const unsigned x = two_da * (unsigned)tlo - (unsigned)l.da;
        lo = max(lo, (int)gm_udiv(x + two_db - 1u, two_db));
    }
    {  // largest i with q(i) <= thi
        const unsigned y = two_da * (unsigned)(thi + 1) - (unsigned)l.da;
        hi = min(hi, (int)gm_udiv(y - 1u, two_db));
    }
    return lo <= hi;
}

// One beam of ComputeMap (:185-214): validity filter, clamp to maxUrange, end point in double.
struct GmBeam {
    bool valid, hit;
    int x1, y1;
    double wx, wy;
};

__device__ __forceinline__ GmBeam gm_beam(const GmGeom &g, double px, double py, double ct, double sn, float range,
                                          double ca, double sa)
{
    GmBeam e;
    double d = range;
    e.valid = !(d > g.max_range || d == 0.0 || !isfinite(d));
    e.hit = false;
    e.x1 = e.y1 = 0;
    e.wx = e.wy = 0.0;
    if (!e.valid) return e;
    if (d > g.max_urange) d = g.max_urange;
    const double dirx = ct * ca - sn * sa;  // build-defined particle pose (lp = (0,0,0) in :176)
    const double diry = sn * ca + ct * sa;
    double wx = px, wy = py;
    wx += d * dirx;
    wy += d * diry;
    gm_world2map(g, wx, wy, e.x1, e.y1);
    e.hit = d < g.max_urange;
    e.wx = wx;
    e.wy = wy;
    return e;
}

// Particle weight (build-defined, the reference has no particles): hit beams of this scan whose
// end cell is occupied (n/visits > occ_thresh, map.h:27 + gmapping.cc:150) in the particle's
// previous map.  Runs before gm_compute_kernel overwrites that map; opens the particle's new step.
// It also leaves the particle's rays for gm_compute_kernel: the packed end cell relative to p0 (or
// GM_RAY_INVALID) and the (float) hit point of every beam, so the compute workgroups of the particle
// neither redo the double-precision end points nor keep the hit points in LDS.
__global__ void __launch_bounds__(GM_THREADS)
gm_score_kernel(GmGeom g, const double *__restrict__ poses, const float *__restrict__ ranges, int n,
                const double *__restrict__ a_cos, const double *__restrict__ a_sin, const unsigned *__restrict__ maps,
                const int *__restrict__ stamps, GmState *__restrict__ state, int *__restrict__ scores_out,
                int particle_begin, unsigned *__restrict__ rays_out, float2 *__restrict__ hitxy_out,
                GmHitCell *__restrict__ hit_cells)
{
    __shared__ int s_red[GM_THREADS / 64][2];
    const int p = particle_begin + blockIdx.x;
    const int tid = threadIdx.x;
    const unsigned *pm = maps + (size_t)p * g.particle_words;
    const int *pstamp = stamps + (size_t)p * g.ntiles;
    GmState &st = state[p];
    const int prev_step = st.step;
    const int ptx0 = st.tx0, pty0 = st.ty0, ptx1 = st.tx1, pty1 = st.ty1;  // previous map's box
    const double px = poses[4 * blockIdx.x], py = poses[4 * blockIdx.x + 1];
    const double ct = poses[4 * blockIdx.x + 2], sn = poses[4 * blockIdx.x + 3];
    int x0, y0;
    gm_world2map(g, px, py, x0, y0);  // p0 = world2map(lp) (:176-179)
    unsigned *prays = rays_out + (size_t)p * g.max_beams;
    float2 *phxy = hitxy_out + (size_t)p * g.max_beams;
    GmHitCell *phits = hit_cells + (size_t)p * g.max_beams;
    int score = 0, hits = 0;
    for (int b = tid; b < n; b += GM_THREADS) {
        // the hit-cell list is indexed by beam: gm_compute_kernel fills the slot of a cell's first hitting beam
        phits[b].cell = -1;
        const GmBeam e = gm_beam(g, px, py, ct, sn, ranges[b], a_cos[b], a_sin[b]);
        unsigned r = GM_RAY_INVALID;
        // lines longer than 16383 cells are not representable (max_range / delta < 16384)
        if (e.valid && abs(e.x1 - x0) < GM_REL && abs(e.y1 - y0) < GM_REL) r = gm_pack(e.x1 - x0, e.y1 - y0, e.hit);
        prays[b] = r;
        phxy[b] = make_float2((float)e.wx, (float)e.wy);
        if (!e.valid || !e.hit) continue;
        hits += 1;
        const int x1 = e.x1, y1 = e.y1;
        if (prev_step > 0 && x1 >= 0 && x1 < g.sx && y1 >= 0 && y1 < g.sy) {
            const int tx = x1 / GM_TILE, ty = y1 / GM_TILE_H;
            if (tx >= ptx0 && tx <= ptx1 && ty >= pty0 && ty <= pty1 && pstamp[ty * g.tiles_x + tx] == prev_step) {
                const unsigned cv = pm[(size_t)(ty * g.tiles_x + tx) * GM_TILE_BLOCK_WORDS + (y1 % GM_TILE_H) * GM_TILE +
                                       (x1 % GM_TILE)];
                const int vis = (int)(cv & 0xFFFFu), nn = (int)(cv >> 16);
                const double occ = vis ? (double)nn * 1 / (double)vis : -1;
                score += occ > g.occ_thresh ? 1 : 0;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        score += __shfl_xor(score, off, 64);
        hits += __shfl_xor(hits, off, 64);
    }
    if ((tid & 63) == 0) {
        s_red[tid >> 6][0] = score;
        s_red[tid >> 6][1] = hits;
    }
    __syncthreads();
    if (tid == 0) {
        int sc = 0, hc = 0;
        for (int w = 0; w < GM_THREADS / 64; ++w) {
            sc += s_red[w][0];
            hc += s_red[w][1];
        }
        st.score = sc;
        st.hits = hc;
        st.step = prev_step + 1;   // tiles stamped with this step form the new map
        st.free_updates = 0;
        st.hit_cells = n;  // slots: one per beam, cell < 0 where no list entry
        if (scores_out) scores_out[blockIdx.x] = sc;
    }
}

// Grid: parts x count workgroups (part-major); part q draws tiles q, q + parts, ... of the particle's
// tile box.  Runs after gm_score_kernel of the same step.
__global__ void __launch_bounds__(GM_THREADS)
gm_compute_kernel(GmGeom g, const double *__restrict__ poses, int n, const unsigned *__restrict__ rays_in,
                  const float2 *__restrict__ hitxy, unsigned *__restrict__ maps, int *__restrict__ stamps,
                  GmHitCell *__restrict__ hit_cells, GmState *__restrict__ state, int particle_begin, int count,
                  int parts)
{
    extern __shared__ __attribute__((aligned(16))) unsigned smem[];
    unsigned *cnt = smem;                              // n << 16 | visits per cell of the tile
    unsigned *first_hit = smem + GM_LDS_WORDS;         // lowest hitting beam per cell
    unsigned *rays = smem + 2 * GM_LDS_WORDS;          // packed end cells
    int4 *gbox = reinterpret_cast<int4 *>(rays + ((n + 3) & ~3));        // per 64-beam fan group
    __shared__ int s_box[4];
    __shared__ int s_anyf[2];   // per tile parity: "some lane marked a cell"
    __shared__ int s_anyh[2];   // per tile parity: "some beam ends in the tile" (the acc pass runs)

    const int part = blockIdx.x / count;
    const int local = blockIdx.x - part * count;
    const int p = particle_begin + local;
    const int tid = threadIdx.x;
    unsigned *pm = maps + (size_t)p * g.particle_words;
    int *pstamp = stamps + (size_t)p * g.ntiles;
    GmHitCell *phits = hit_cells + (size_t)p * g.max_beams;
    GmState &st = state[p];
    const int cur_step = st.step;
    const double px = poses[4 * local], py = poses[4 * local + 1];
    int x0, y0;
    gm_world2map(g, px, py, x0, y0);  // p0 = world2map(lp) (:176-179)
    const unsigned *prays = rays_in + (size_t)p * g.max_beams;
    const float2 *phxy = hitxy + (size_t)p * g.max_beams;  // (float) hit points, read by the hit pass only

    if (tid == 0) {
        s_box[0] = g.sx; s_box[1] = g.sy; s_box[2] = -1; s_box[3] = -1;
    }
    __syncthreads();
    // ---- rays (:185-214), computed by gm_score_kernel
    int bx0 = x0, by0 = y0, bx1 = x0, by1 = y0;
    for (int b0 = __builtin_amdgcn_readfirstlane(tid & ~63); b0 < n; b0 += GM_THREADS) {
        const int b = b0 + (tid & 63);
        unsigned r = GM_RAY_INVALID;
        int gx0 = x0, gy0 = y0, gx1 = x0, gy1 = y0;
        if (b < n) {
            r = prays[b];
            if (r != GM_RAY_INVALID) {
                const int x1 = x0 + (int)(r & 0xFFFFu) - GM_REL, y1 = y0 + (int)((r >> 16) & 0x7FFFu) - GM_REL;
                gx0 = min(gx0, x1); gy0 = min(gy0, y1); gx1 = max(gx1, x1); gy1 = max(gy1, y1);
            }
            rays[b] = r;
        }
        bx0 = min(bx0, gx0); by0 = min(by0, gy0); bx1 = max(bx1, gx1); by1 = max(by1, gy1);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            gx0 = min(gx0, __shfl_xor(gx0, off, 64));
            gy0 = min(gy0, __shfl_xor(gy0, off, 64));
            gx1 = max(gx1, __shfl_xor(gx1, off, 64));
            gy1 = max(gy1, __shfl_xor(gy1, off, 64));
        }
        if ((tid & 63) == 0) gbox[b0 >> 6] = make_int4(gx0, gy0, gx1, gy1);
    }
    // first_hit starts empty once: afterwards each hit cell's first beam restores its word in the acc pass; with
    // GM_RESTORE the counts likewise (the store pass zeroes what it stored), and both tile flags start clear
    for (int k = tid; k < GM_LDS_WORDS / 4; k += GM_THREADS) {
        reinterpret_cast<uint4 *>(first_hit)[k] = make_uint4(~0u, ~0u, ~0u, ~0u);
        if (GM_RESTORE) reinterpret_cast<uint4 *>(cnt)[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < 2) s_anyf[tid] = s_anyh[tid] = 0;
    // the written tile box: the rays' box clamped to the map
    atomicMin(&s_box[0], max(bx0, 0)); atomicMin(&s_box[1], max(by0, 0));
    atomicMax(&s_box[2], min(bx1, g.sx - 1)); atomicMax(&s_box[3], min(by1, g.sy - 1));
    __syncthreads();

    const bool any_cell = s_box[0] <= s_box[2] && s_box[1] <= s_box[3];
    const int tx0 = any_cell ? s_box[0] / GM_TILE : 1, ty0 = any_cell ? s_box[1] / GM_TILE_H : 1;
    const int tx1 = any_cell ? s_box[2] / GM_TILE : 0, ty1 = any_cell ? s_box[3] / GM_TILE_H : 0;
    if (tid == 0 && part == 0) {
        st.tx0 = tx0; st.ty0 = ty0; st.tx1 = tx1; st.ty1 = ty1;
    }
    bool any_tile_marks = false, any_tile_hits = false;

    long long nfree = 0;
    const int ngr = (n + 63) >> 6;                                   // fan groups
    const int wbeam0 = __builtin_amdgcn_readfirstlane(tid & ~63);    // this wave's first beam
    const int ntx = tx1 - tx0 + 1, ntiles = (tx1 >= tx0) ? ntx * (ty1 - ty0 + 1) : 0;
    int it = 0;
    for (int t = part; t < ntiles; t += parts, ++it) {
        const int tx = tx0 + t % ntx, ty = ty0 + t / ntx;
        const int X0 = tx * GM_TILE, Y0 = ty * GM_TILE_H;
        const int X1 = min(X0 + GM_TILE, g.sx), Y1 = min(Y0 + GM_TILE_H, g.sy);
        if (!GM_RESTORE) {
            for (int k = tid; k < GM_LDS_WORDS / 4; k += GM_THREADS)
                reinterpret_cast<uint4 *>(cnt)[k] = make_uint4(0u, 0u, 0u, 0u);
            // the flag of this parity was last read two tiles ago, with barriers in between
            if (tid == 0) s_anyf[it & 1] = s_anyh[it & 1] = 0;
        } else if (tid == 0) {
            // the OTHER parity's flags, for the next tile: the previous tile read them after its raster barrier and
            // before its closing one (a tile without marks read s_anyf == 0, which this rewrites unchanged); this
            // tile's raster barrier orders the reset before the next tile's raster sets them
            s_anyf[(it & 1) ^ 1] = s_anyh[(it & 1) ^ 1] = 0;
        }
        // the fan groups (64 beams) whose box meets the tile: one ballot, lane f testing group f (groups past the
        // first 64, scans of > 4096 beams, test their box alone); this wave's groups are f = wave + 4 k
        unsigned long long fm = 0ull;
        if (GM_BALLOT) {
            int ol = tid & 63;  // opaque: the box address is not hoisted into a VGPR held across tiles
            asm volatile("" : "+v"(ol));
            const int4 gb = gbox[min(ol, ngr - 1)];
            fm = __ballot((int)(ol < ngr) & (int)(gb.z >= X0) & (int)(gb.x < X1) & (int)(gb.w >= Y0) & (int)(gb.y < Y1));
        }
        if (!GM_RESTORE) gm_lds_barrier();  // the cleared counts (GM_RESTORE: the previous tile's closing barrier)
        // one fan group's raster in the tile (a lambda: the ballot's groups and the scalar-tested groups past the
        // first 64 share it)
        auto raster_group = [&](int b0) {
            const int b = b0 + (GM_FAN ? 2 * (tid & 31) + ((tid >> 5) & 1) : (tid & 63));
            if (b >= n) return;
            const unsigned r = rays[b];
            if (r == GM_RAY_INVALID) return;
            const int x1 = x0 + (int)(r & 0xFFFFu) - GM_REL, y1 = y0 + (int)((r >> 16) & 0x7FFFu) - GM_REL;
            if (max(x0, x1) < X0 || min(x0, x1) >= X1 || max(y0, y1) < Y0 || min(y0, y1) >= Y1) return;
            if ((r & GM_RAY_HIT) && x1 >= X0 && x1 < X1 && y1 >= Y0 && y1 < Y1) {
                const int c = (y1 - Y0) * GM_STRIDE + (x1 - X0);
                atomicAdd(&cnt[c], 0x10001u);       // n++, visits++ (map.h:40-44)
                atomicMin(&first_hit[c], (unsigned)b);
                any_tile_marks = any_tile_hits = true;
            }
            const GmLine l = gm_line(x0, y0, x1, y1);
            int lo = l.ilo, hi = l.ihi;
            const bool in = l.x_major ? gm_clip(l, X0, X1, Y0, Y1, lo, hi) : gm_clip(l, Y0, Y1, X0, X1, lo, hi);
            if (!in) return;
            const unsigned two_da = 2u * (unsigned)l.da, two_db = 2u * (unsigned)l.db;
            // GM_BWD: odd lanes start at hi and walk down to lo (the same cells): near the scan origin the lanes of
            // a fan then sit at two radii per instruction, so half as many of them add to one LDS word (the
            // atomics to one address serialise)
            const bool bwd = GM_BWD && (tid & 1);
            const int s0 = bwd ? hi : lo;
            const unsigned num = two_db * (unsigned)s0 + (unsigned)l.da;
            const int q = l.da ? (int)gm_udiv(num, two_da) : 0;
            unsigned rem = num - (unsigned)q * two_da;
            const int la = l.x_major ? 1 : GM_STRIDE, lb = l.x_major ? GM_STRIDE : 1;
            const int A0 = l.x_major ? X0 : Y0, B0 = l.x_major ? Y0 : X0;
            const int li = (l.as + s0 - A0) * la + (l.bs + l.sb * q - B0) * lb;
            const int steps = hi - lo + 1;
            nfree += steps;
            any_tile_marks = true;
            // incremental walk with f = 2 da - 1 - rem in [0, 2 da): the minor axis steps when f < 2 db --
            // a subtract with borrow and two selects per step on byte offsets into the count array,
            // four steps per trip.  Backwards the same step with f = rem and the offsets negated: rem drops by
            // 2 db per step and the minor axis steps back exactly when it borrows (then + 2 da)
            if (GM_PRICE == 3) return;
            const int tda = (int)two_da, tdb = (int)two_db;
            const int dabf = la * 4, dab2f = dabf + l.sb * lb * 4;
            const int dab = bwd ? -dabf : dabf, dab2 = bwd ? -dab2f : dab2f;
            int f = bwd ? (int)rem : tda - 1 - (int)rem;
            int i = 0;
#if GM_PACKED
            // f and the step's LDS byte address in ONE register, V = f << 16 | address (LDS addresses < 2^16, f < 2 da
            // <= 2^15): subtracting 2 db << 16 borrows exactly when the minor axis steps, and one select + add then
            // moves both fields (the Hector update's walk); eight steps per trip
            const unsigned vdn = (unsigned)tdb << 16;
            const unsigned vk_major = (unsigned)dab, vk_minor = ((unsigned)tda << 16) + (unsigned)dab2;
            unsigned v = ((unsigned)f << 16) + gm_lds_addr(cnt) + (unsigned)li * 4u;
#define GM_WSTEP                                                                   \
    do {                                                                           \
        atomicAdd(gm_lds_ptr(v & 0xFFFFu), 1u); /* visits++ (:227-234) */          \
        unsigned vn_;                                                              \
        const bool c_ = __builtin_sub_overflow(v, vdn, &vn_);                      \
        v = vn_ + (c_ ? vk_minor : vk_major);                                      \
    } while (0)
            for (; i + 7 < steps; i += 8) {
                GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP;
            }
            if (i + 3 < steps) {
                GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP;
                i += 4;
            }
            if (i + 1 < steps) {
                GM_WSTEP; GM_WSTEP;
                i += 2;
            }
#undef GM_WSTEP
            if (i < steps) atomicAdd(gm_lds_ptr(v & 0xFFFFu), 1u);
#else
            char *pc = reinterpret_cast<char *>(cnt) + li * 4;
#define GM_WSTEP                                                                  \
    do {                                                                          \
        atomicAdd(reinterpret_cast<unsigned *>(pc), 1u); /* visits++ (:227-234) */ \
        unsigned fu_;                                                             \
        const bool c_ = __builtin_sub_overflow((unsigned)f, (unsigned)tdb, &fu_); \
        f = (int)fu_ + (c_ ? tda : 0);                                            \
        pc += c_ ? dab2 : dab;                                                    \
    } while (0)
            for (; i + 3 < steps; i += 4) {
                GM_WSTEP; GM_WSTEP; GM_WSTEP; GM_WSTEP;
            }
            for (; i + 1 < steps; i += 2) {
                GM_WSTEP; GM_WSTEP;
            }
#undef GM_WSTEP
            if (i < steps) atomicAdd(reinterpret_cast<unsigned *>(pc), 1u);
#endif
        };
        for (unsigned long long gmk = fm & (0x1111111111111111ull << (wbeam0 >> 6)); gmk; gmk &= gmk - 1ull)
            raster_group(__builtin_ctzll(gmk) << 6);
        for (int b0 = wbeam0 + (GM_BALLOT ? 64 * 64 : 0); b0 < n; b0 += GM_THREADS) {
            const int4 gb = gbox[b0 >> 6];
            const int gx0 = __builtin_amdgcn_readfirstlane(gb.x), gy0 = __builtin_amdgcn_readfirstlane(gb.y);
            const int gx1 = __builtin_amdgcn_readfirstlane(gb.z), gy1 = __builtin_amdgcn_readfirstlane(gb.w);
            if (gx1 < X0 || gx0 >= X1 || gy1 < Y0 || gy0 >= Y1) continue;
            raster_group(b0);
        }
        if (__ballot(any_tile_marks) && (tid & 63) == 0) s_anyf[it & 1] = 1;
        if (__ballot(any_tile_hits) && (tid & 63) == 0) s_anyh[it & 1] = 1;
        any_tile_hits = false;
        gm_lds_barrier();
        // tiles without any mark are not written: their stale stamp makes them read as fresh
        if (!s_anyf[it & 1]) continue;  // plain LDS accesses, ordered by gm_lds_barrier's memory clobber
        any_tile_marks = false;
        unsigned *tp = pm + (size_t)(ty * g.tiles_x + tx) * GM_TILE_BLOCK_WORDS;
        // acc: the first hitting beam of a cell sums every hit of that cell in beam order (:236-240)
        auto acc_group = [&](int b0) {
            const int b = b0 + (tid & 63);
            if (b >= n) return;
            const unsigned r = rays[b];
            if (r == GM_RAY_INVALID || !(r & GM_RAY_HIT)) return;
            const int x1 = x0 + (int)(r & 0xFFFFu) - GM_REL, y1 = y0 + (int)((r >> 16) & 0x7FFFu) - GM_REL;
            if (x1 < X0 || x1 >= X1 || y1 < Y0 || y1 >= Y1) return;
            const int c = (y1 - Y0) * GM_STRIDE + (x1 - X0);
            if (first_hit[c] != (unsigned)b) return;
            first_hit[c] = ~0u;  // restored for the next tile (a later beam of the cell then fails the test too)
            float ax = 0.0f, ay = 0.0f;
            const float2 h0 = phxy[b];
            ax += h0.x;
            ay += h0.y;
            // the other hits of the cell, in beam order; the raster counted them (n = cnt >> 16), so the
            // scan stops at the last one -- they are nearly always the next beams (a long serial scan
            // of every later beam per multiply-hit cell was most of this kernel's time)
            for (int need = (int)(cnt[c] >> 16) - 1, b2 = b + 1; need > 0 && b2 < n; ++b2)
                if (rays[b2] == r) {
                    const float2 h2 = phxy[b2];
                    ax += h2.x;
                    ay += h2.y;
                    --need;
                }
            GmHitCell hc;
            hc.cell = y1 * g.sx + x1;
            hc.ax = ax;
            hc.ay = ay;
            // the slot of the cell's first beam: no list counter (a returning global atomic per hit cell, on one
            // address per particle, was most of this pass's time)
            phits[b] = hc;
        };
        if (GM_PRICE != 1 && s_anyh[it & 1]) {  // (a tile where no beam ends has no acc pass)
            for (unsigned long long gmk = fm & (0x1111111111111111ull << (wbeam0 >> 6)); gmk; gmk &= gmk - 1ull)
                acc_group(__builtin_ctzll(gmk) << 6);
            for (int b0 = wbeam0 + (GM_BALLOT ? 64 * 64 : 0); b0 < n; b0 += GM_THREADS) {
                const int4 gb = gbox[b0 >> 6];
                const int gx0 = __builtin_amdgcn_readfirstlane(gb.x), gy0 = __builtin_amdgcn_readfirstlane(gb.y);
                const int gx1 = __builtin_amdgcn_readfirstlane(gb.z), gy1 = __builtin_amdgcn_readfirstlane(gb.w);
                if (gx1 < X0 || gx0 >= X1 || gy1 < Y0 || gy0 >= Y1) continue;
                acc_group(b0);
            }
        }
        // GM_RESTORE: the acc pass's count reads (n) precede the zeroing below
        if (GM_RESTORE && s_anyh[it & 1]) gm_lds_barrier();
        // counts: the whole tile (a fresh map: untouched cells written as zero), 16-B stores; GM_RESTORE: each
        // quad zeroed by the thread that stored it
        for (int qi = tid; qi < (GM_PRICE == 2 ? 0 : GM_TILE_CELLS / 4); qi += GM_THREADS) {
            const int row = qi >> 4, c4 = (qi & 15) << 2;
            uint4 *q = reinterpret_cast<uint4 *>(&cnt[row * GM_STRIDE + c4]);
            *reinterpret_cast<uint4 *>(&tp[row * GM_TILE + c4]) = *q;
            if (GM_RESTORE) *q = make_uint4(0u, 0u, 0u, 0u);
        }
        if (tid == 0) pstamp[ty * g.tiles_x + tx] = cur_step;
        gm_lds_barrier();  // the tile's LDS counts are read (GM_RESTORE: and zeroed) before the next tile's raster
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nfree += __shfl_xor(nfree, off, 64);
    if ((tid & 63) == 0 && nfree) atomicAdd(reinterpret_cast<unsigned long long *>(&st.free_updates), (unsigned long long)nfree);
}

// Particle weights, local half of the exchange: sums[0] = Σ (score + 1), sums[1] = Σ (score + 1)^2 over
// this rank's particles, as doubles.  Every term is an integer below 2^53, so the sums are exact and
// independent of the summation order (and of how the particles are sharded over ranks).
__global__ void __launch_bounds__(GM_THREADS) gm_weight_sums_kernel(const int *__restrict__ scores, int count,
                                                                    double *__restrict__ sums)
{
    __shared__ double s_red[GM_THREADS / 64][2];
    double a = 0.0, q = 0.0;
    for (int i = threadIdx.x; i < count; i += GM_THREADS) {
        const double v = (double)scores[i] + 1.0;
        a += v;
        q += v * v;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        q += __shfl_xor(q, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_red[threadIdx.x >> 6][0] = a;
        s_red[threadIdx.x >> 6][1] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tq = 0.0;
        for (int w = 0; w < GM_THREADS / 64; ++w) {
            ta += s_red[w][0];
            tq += s_red[w][1];
        }
        sums[0] = ta;
        sums[1] = tq;
    }
}

// w_p = (score_p + 1) / Σ_all (score + 1), from the all-reduced sums
__global__ void gm_weights_kernel(const int *__restrict__ scores, int count, const double *__restrict__ sums,
                                  double *__restrict__ w)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) w[i] = ((double)scores[i] + 1.0) / sums[0];
}

// GMapping::PublishMap conversion (gmapping.cc:141-159): -1 unvisited, 100 if n/visits > thresh, 0
__global__ void gm_publish_kernel(const unsigned *__restrict__ pm, const int *__restrict__ pstamp, GmGeom g, int step,
                                  int8_t *__restrict__ out)
{
    const size_t total = (size_t)g.sx * g.sy;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % g.sx), y = (int)(i / g.sx);
        const int t = (y / GM_TILE_H) * g.tiles_x + x / GM_TILE;
        int vis = 0, nn = 0;
        if (step > 0 && pstamp[t] == step) {
            const unsigned cv = pm[(size_t)t * GM_TILE_BLOCK_WORDS + (y % GM_TILE_H) * GM_TILE + (x % GM_TILE)];
            vis = (int)(cv & 0xFFFFu);
            nn = (int)(cv >> 16);
        }
        const double occ = vis ? (double)nn * 1 / (double)vis : -1;
        out[i] = occ < 0 ? (int8_t)-1 : (occ > g.occ_thresh ? (int8_t)100 : (int8_t)0);
    }
}

}  // namespace s2d
