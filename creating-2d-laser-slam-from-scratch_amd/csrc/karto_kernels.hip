// karto_kernels.hip -- MI355X kernels of the Karto correlative scan matcher (lesson6, config 5).
//
// One MatchScan (lesson6/lib/open_karto/src/Mapper.cpp:184-300) per "match slot"; a launch serves a
// whole batch of independent matches (a loop-closure candidate batch, or many robots' sequential
// matches).  Kernels, in stream order:
//   kt_prepare_kernel  one workgroup per pooled scan: LocalizedRangeScan::Update point readings
//                      (Karto.h:5362-5404, order-preserving compaction), the points in the scan's own
//                      frame (Transform::InverseTransformPose, Karto.h:2894-2901) and the
//                      viewpoint-independent half of FindValidPoints (Mapper.cpp:755-811): the
//                      "first point" reset events, found by one lane walking the points in LDS.
//   kt_begin_kernel    per match: centre the correlation grid on the query's pose (MatchScan 1-4).
//   kt_build_kernel    per (match, base scan): the viewpoint test of FindValidPoints, then AddScan +
//                      SmearPoint (Mapper.cpp:716-748, Mapper.h:971-1005) as a byte-wise max of the
//                      smear kernel: chunks of 16 consecutive points rendered in an LDS tile, merged
//                      into the grid by 64-bit compare-and-swap per non-zero qword.  Order-free because
//                      the kernel's only 100 is its centre (checked at kt_create).
//   kt_coarse_kernel   per (match, group of angles, 16x16 position tile): GridIndexLookup::ComputeOffsets per
//                      angle into LDS (Karto.h:6455-6501), then GetResponse (Mapper.cpp:819-856) for the
//                      tile's 256 positions -- each lane owns 4 positions two cells apart and reads
//                      them with ONE unaligned 8-byte gather per point (bytes 0, 2, 4, 6), summed as
//                      packed 16-bit lanes; the 4 waves split the points.  Penalty (Mapper.cpp:
//                      398-416), responses in the reference's pose order, per-position max over angles
//                      (the search-space probability grid) and the best response by 64-bit atomic max.
//   kt_select_kernel   per match: poses tying the best (DoubleEqual) compacted in pose order and
//                      averaged by one lane in that order (Mapper.cpp:456-487), the positional
//                      covariance (Mapper.cpp:535-626), response expansion (Mapper.cpp:244-271).
//   kt_fine_kernel     per match: the fine CorrelateScan (3x3 positions x fine angles) and
//                      ComputeAngularCovariance (Mapper.cpp:638-690) in one workgroup.
//   kt_build_kernel    again with clear = 1: zero the chunks' footprint boxes, so the slot's grid is
//                      clean for the next match without a 6 MB memset.
// All arithmetic is double, with -ffp-contract=off and the deterministic sin / cos / atan2 of
// detmath.h; the CPU restatement oracle/karto_oracle.c evaluates the same sequence (bit-exact parity).
#include <hip/hip_runtime.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>

#include "../../include/slam2d/karto.h"
#include "detmath.h"

namespace s2d {

constexpr int KT_THREADS = 256;
constexpr int KT_MAX_READINGS = 4096;
constexpr int KT_FINE_MAX_ANG = 64;
constexpr int KT_MAX_NXY = 1024;  // coarse positions per axis
constexpr int KT_SEL_ITEMS = 16;
constexpr int KT_INVALID = INT_MIN;  // INVALID_SCAN: any position index + this is negative -> skipped
constexpr double KT_PI = 3.14159265358979323846;
constexpr double KT_2PI = 6.28318530717958647692;
constexpr double KT_TOL = 1e-06;
constexpr double KT_MAX_VARIANCE = 500.0;
constexpr double KT_GAIN = 0.2;  // DISTANCE_PENALTY_GAIN == ANGLE_PENALTY_GAIN (Mapper.cpp:37-38)
constexpr int KT_OCC = 100;

// Host-computed geometry of one ScanMatcher (ScanMatcher::Create + CorrelateScan's search spaces).
struct KtGeom {
    double scale, res;                 // 1 / resolution, GetResolution() = 1 / scale
    int grid_size, border, width, height, ws, data_size;
    int side, probs_ws, half, ksize;
    int n;                             // readings per scan
    int nxy;                           // coarse positions per axis
    int ctx, cty, clw;                 // coarse position tiles along x / y; log2 of gather lanes per tile row
    int npass;                         // 1, or 4 with response expansion
    int nang[4];
    double aoff[4];                    // coarse angle offset per pass
    double coff, cres;                 // coarse search offset / resolution
    double foff;                       // fine search offset (resolution = res)
    int fn, fnang;                     // fine positions per axis, fine angles
    double faoff, fares;               // fine angle offset / resolution
    double min_angle, ang_res, min_range, range_thr;
    double dvp, avp, mdp, map_;        // penalties
    double cares;                      // coarse angle resolution
    int use_expansion;
    int max_poses;
    size_t grid_stride;                // bytes per match slot grid
    int tiles_x, tiles_y, ntiles;      // 64 x 64-cell tiles of the grid (kt_addscans_kernel)
};

struct KtPool {
    const double *ranges;  // [S][n]
    const double *poses;   // [S][3]
    int *npts;             // [S]
    double2 *pts;          // [S][n] world point readings
    double2 *loc;          // [S][n] points in the scan's frame
    unsigned char *bad;    // [S][n] raw reading k (k < npts) is NaN / inf (ComputeOffsets, Karto.h:6476-6481)
    int2 *evt;             // [S][n] (closing reset event, its first point) of point k, or (-1, -1)
};

struct KtState {
    double center[3];
    double gox, goy;
    double mean[3];
    double cov[9];
    double best;
    unsigned long long best_bits;
    int query, npts, pass, status;
};

// ---- Math.h (K/include/open_karto/Math.h:87-233) ----------------------------------------------
__device__ __forceinline__ double kt_round(double v) { return v >= 0.0 ? floor(v + 0.5) : ceil(v - 0.5); }
__device__ __forceinline__ bool kt_deq(double a, double b)
{
    const double d = a - b;
    return d < 0.0 ? d >= -KT_TOL : d <= KT_TOL;
}
__device__ __forceinline__ double kt_max(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double kt_sq(double v) { return v * v; }
__device__ inline double kt_norm_angle(double a)
{
    if (!isfinite(a)) return a;  // the reference would spin; a non-finite heading is passed through
    while (a < -KT_PI) {
        if (a < -KT_2PI) a += (double)(uint32_t)(a / -KT_2PI) * KT_2PI;
        else a += KT_2PI;
    }
    while (a > KT_PI) {
        if (a > KT_2PI) a -= (double)(uint32_t)(a / KT_2PI) * KT_2PI;
        else a -= KT_2PI;
    }
    return a;
}
__device__ inline double kt_norm_angle_diff(double minuend, double subtrahend)
{
    while (minuend - subtrahend < -KT_PI) minuend += KT_2PI;
    while (minuend - subtrahend > KT_PI) minuend -= KT_2PI;
    return minuend;
}
__device__ __forceinline__ int kt_w2g(double w, double o, double scale) { return (int)kt_round((w - o) * scale); }

__device__ __forceinline__ unsigned long long kt_bits(double v) { return (unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ double kt_dbl(unsigned long long b) { return __longlong_as_double((long long)b); }

// block-wide exclusive scan of v (256 threads); total returned through *total
__device__ __forceinline__ int kt_block_exscan(int v, int *sw, int *total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(inc, off, 64);
        if (lane >= off) inc += t;
    }
    if (lane == 63) sw[w] = inc;
    __syncthreads();
    int woff = 0;
    for (int i = 0; i < w; ++i) woff += sw[i];
    *total = sw[0] + sw[1] + sw[2] + sw[3];
    __syncthreads();
    return woff + inc - v;
}

__device__ __forceinline__ int kt_block_max_int(int v, int *sw)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = v;
    __syncthreads();
    const int r = max(max(sw[0], sw[1]), max(sw[2], sw[3]));
    __syncthreads();
    return r;
}

// rotation part of Transform(sensorPose).InverseTransformPose: Matrix3::FromAxisAngle(0, 0, 1, 0 - h)
// (Karto.h:2392-2420, :2909-2935) and Matrix3 * Pose2 (Karto.h:2574-2583)
__device__ __forceinline__ void kt_inv_rot(double h, double r[6])
{
    const double rad = 0.0 - h;
    const double c = sdm_cos(rad), s = sdm_sin(rad);
    const double omc = 1.0 - c;
    const double zomc = (0.0 * 0.0) * omc;
    r[0] = 0.0 * omc + c;
    r[1] = zomc - 1.0 * s;
    r[2] = zomc + 0.0 * s;
    r[3] = zomc + 1.0 * s;
    r[4] = 0.0 * omc + c;
    r[5] = zomc - 0.0 * s;
}

// =================================================================================================
// kt_prepare_kernel: pooled scans -> point readings, local points, reset events
// =================================================================================================
__global__ void __launch_bounds__(KT_THREADS)
kt_prepare_kernel(KtGeom g, KtPool P, int first)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char kt_smem[];
    double2 *spts = reinterpret_cast<double2 *>(kt_smem);       // [n]
    int *sev = reinterpret_cast<int *>(spts + g.n);              // [n] reset events
    int *snext = sev + g.n;                                      // [n] next point beyond 0.1 m
    __shared__ int sw[4];
    __shared__ int s_nev;

    const int s = first + blockIdx.x;
    const int tid = threadIdx.x;
    const int n = g.n;
    const double *raw = P.ranges + (size_t)s * n;
    const double px = P.poses[3 * s], py = P.poses[3 * s + 1], ph = P.poses[3 * s + 2];

    // order-preserving compaction of the readings InRange(r, minimumRange, rangeThreshold)
    const int chunk = (n + KT_THREADS - 1) / KT_THREADS;
    const int i0 = min(tid * chunk, n), i1 = min(i0 + chunk, n);
    int cnt = 0;
    for (int i = i0; i < i1; ++i) {
        const double r = raw[i];
        cnt += (r >= g.min_range && r <= g.range_thr) ? 1 : 0;
    }
    int npts;
    int k = kt_block_exscan(cnt, sw, &npts);
    double R[6];
    kt_inv_rot(ph, R);
    const double dth = kt_norm_angle(0.0 - ph);
    double2 *pts = P.pts + (size_t)s * n;
    double2 *loc = P.loc + (size_t)s * n;
    for (int i = i0; i < i1; ++i) {
        const double r = raw[i];
        if (!(r >= g.min_range && r <= g.range_thr)) continue;
        const double angle = ph + g.min_angle + (double)(uint32_t)i * g.ang_res;
        const double x = px + (r * sdm_cos(angle));
        const double y = py + (r * sdm_sin(angle));
        pts[k] = make_double2(x, y);
        spts[k] = make_double2(x, y);
        const double dx = x - px, dy = y - py;
        const double lx = R[0] * dx + R[1] * dy + R[2] * dth;
        const double ly = R[3] * dx + R[4] * dy + R[5] * dth;
        loc[k] = make_double2(lx, ly);
        ++k;
    }
    unsigned char *bad = P.bad + (size_t)s * n;
    for (int j = tid; j < npts; j += KT_THREADS) {
        const double r = raw[j];  // the reference indexes the raw readings with the point index
        bad[j] = (isnan(r) || isinf(r)) ? 1 : 0;
    }
    if (tid == 0) P.npts[s] = npts;
    __syncthreads();
    // FindValidPoints' reset events (the viewpoint-independent walk): the walk keeps an anchor point and
    // resets it at the first later point farther than 0.1 m from it.  next(j) = that point for anchor j
    // (the same squared-distance test), found for every j in parallel; one lane then follows the chain
    // 0 -> next(0) -> ..., one LDS read per event instead of one per point.
    const double min_sq = 0.1 * 0.1;
    for (int j = tid; j < npts; j += KT_THREADS) {
        const double fx = spts[j].x, fy = spts[j].y;
        int nx = j + 1;
        for (; nx < npts; ++nx) {
            const double2 c = spts[nx];
            const double dx = fx - c.x, dy = fy - c.y;
            if (dx * dx + dy * dy > min_sq) break;
        }
        snext[j] = nx;
    }
    __syncthreads();
    if (tid == 0) {
        int nev = 0;
        if (npts > 0)
            for (int a = snext[0]; a < npts; a = snext[a]) sev[nev++] = a;
        s_nev = nev;
    }
    __syncthreads();
    const int nev = s_nev;
    int2 *evt = P.evt + (size_t)s * n;
    for (int j = tid; j < npts; j += KT_THREADS) {
        int lo = 0, hi = nev;  // first event > j
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sev[mid] > j) hi = mid;
            else lo = mid + 1;
        }
        evt[j] = lo < nev ? make_int2(sev[lo], lo > 0 ? sev[lo - 1] : 0) : make_int2(-1, -1);
    }
}

// =================================================================================================
// kt_begin_kernel: centre the correlation grid on the scan pose (MatchScan steps 1-4)
// =================================================================================================
__global__ void __launch_bounds__(KT_THREADS)
kt_begin_kernel(KtGeom g, KtPool P, const int *__restrict__ query, KtState *st, unsigned long long *posmax)
{
    const int m = blockIdx.x;
    const int q = query[m];
    if (threadIdx.x == 0) {
        KtState &S = st[m];
        S.center[0] = P.poses[3 * q];
        S.center[1] = P.poses[3 * q + 1];
        S.center[2] = P.poses[3 * q + 2];
        S.gox = S.center[0] - (0.5 * (g.grid_size - 1) * g.res);
        S.goy = S.center[1] - (0.5 * (g.grid_size - 1) * g.res);
        S.best_bits = 0ull;
        S.best = 0.0;
        S.query = q;
        S.npts = P.npts[q];
        S.pass = 0;
        S.status = KT_OK;
    }
    unsigned long long *pm = posmax + (size_t)m * g.nxy * g.nxy;
    for (int i = threadIdx.x; i < g.nxy * g.nxy; i += KT_THREADS) pm[i] = 0ull;
}

// =================================================================================================
// kt_build_kernel: AddScans (clear = 0) / zero the same footprints (clear = 1)
//
// Every wave takes chunks of KT_CHUNK consecutive points of one base scan (consecutive readings land
// next to each other, so their smear footprints overlap heavily).  A chunk whose footprint bounding
// box fits the wave's LDS tile is rendered there first (byte max, points in turn, lanes over the
// kernel cells), then every non-zero word of the tile is merged into the grid with one 32-bit
// compare-and-swap (first tried against 0: most words are fresh).  Chunks that do not fit (a jump
// between walls) smear their points straight into the grid.  clear = 1 zeroes the chunk's whole
// bounding box (every non-zero cell of the grid lies in some footprint, so the grid ends all-zero).
// =================================================================================================
constexpr int KT_CHUNK = 16;
constexpr int KT_BT_W = 12;   // LDS tile: 12 qwords (96 cells) wide
constexpr int KT_BT_H = 96;   // ... 96 rows tall
constexpr int KT_FAST_KS = 15;  // kernels up to 15x15 (<= 4 cells per lane) use per-lane cell tables

__device__ __forceinline__ unsigned long long kt_bytemax8(unsigned long long a, unsigned long long b)
{
    unsigned long long r = 0;
#pragma unroll
    for (int t = 0; t < 64; t += 8) r |= (unsigned long long)max((unsigned)(a >> t) & 0xFFu, (unsigned)(b >> t) & 0xFFu) << t;
    return r;
}

// Render the footprints of the points in `gmask` into the wave's LDS tile and merge the tile into the
// grid (clear: zero the footprints' box).  False when their box does not fit the tile.
__device__ __forceinline__ bool kt_group(unsigned long long gmask, bool ok, int cx, int cy, int lane, int h, int ks,
                                         int wsw, unsigned long long *gw, unsigned long long *tile, const unsigned char *sk,
                                         const int *cell_off, const int *cell_off2, const unsigned char *cell_kv,
                                         int clear)
{
    const bool in = ok && ((gmask >> lane) & 1ull);
    int x0 = in ? cx : INT_MAX, x1 = in ? cx : INT_MIN, y0 = in ? cy : INT_MAX, y1 = in ? cy : INT_MIN;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        x0 = min(x0, __shfl_xor(x0, off, 64));
        x1 = max(x1, __shfl_xor(x1, off, 64));
        y0 = min(y0, __shfl_xor(y0, off, 64));
        y1 = max(y1, __shfl_xor(y1, off, 64));
    }
    const int bx0 = (x0 - h) & ~7, by0 = y0 - h;
    const int ww = ((x1 + h) - bx0) / 8 + 1, hh = (y1 + h) - by0 + 1;
    if (ww > KT_BT_W || hh > KT_BT_H) return false;
    const int wbase = by0 * wsw + (bx0 >> 3);
    const int nw = ww * hh;
    if (clear) {
        for (int t = lane; t < nw; t += 64) {
            const int r = t / ww, q = t - r * ww;
            gw[wbase + r * wsw + q] = 0ull;
        }
        return true;
    }
    unsigned char *tileb = reinterpret_cast<unsigned char *>(tile);
    for (int t = lane; t < nw; t += 64) tile[t] = 0ull;
    unsigned long long mm = gmask & __ballot(ok);
    if (ks <= KT_FAST_KS) {
        while (mm) {  // points in turn; every lane owns the same <= 4 kernel cells for each point
            const int src = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int pbase = (__shfl(cy, src, 64) - h - by0) * (ww * 8) + (__shfl(cx, src, 64) - h - bx0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (cell_kv[u] == 0) continue;
                unsigned char *cell = tileb + pbase + cell_off[u] * (ww * 8) + cell_off2[u];
                if (cell_kv[u] > *cell) *cell = cell_kv[u];
            }
        }
    } else {
        while (mm) {
            const int src = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int px = __shfl(cx, src, 64) - h - bx0, py = __shfl(cy, src, 64) - h - by0;
            for (int t = lane; t < ks * ks; t += 64) {
                const int jj = t / ks, ii = t - jj * ks;
                const unsigned char kv = sk[ii + ks * jj];
                unsigned char *cell = tileb + (py + jj) * (ww * 8) + (px + ii);
                if (kv > *cell) *cell = kv;
            }
        }
    }
    // merge: 8 64-bit compare-and-swaps in flight per lane (a fresh word finishes in one), then the words that
    // already held data
    for (int t0 = lane; t0 < nw; t0 += 64 * 8) {
        unsigned long long want[8], old[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = t0 + 64 * u;
            want[u] = t < nw ? tile[t] : 0ull;
            old[u] = 0ull;
            if (want[u] != 0ull) {
                const int r = t / ww, q = t - r * ww;
                old[u] = atomicCAS(gw + wbase + r * wsw + q, 0ull, want[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (old[u] == 0ull) continue;
            const int t = t0 + 64 * u;
            const int r = t / ww, q = t - r * ww;
            unsigned long long *w = gw + wbase + r * wsw + q;
            unsigned long long o = old[u];
            while (true) {
                const unsigned long long nv = kt_bytemax8(o, want[u]);
                if (nv == o) break;
                const unsigned long long prev = atomicCAS(w, o, nv);
                if (prev == o) break;
                o = prev;
            }
        }
    }
    return true;
}

template <int clear, int WAVES>
__global__ void __launch_bounds__(WAVES * 64)
kt_build_kernel(KtGeom g, KtPool P, const KtState *__restrict__ st, const int *__restrict__ bbeg,
                const int *__restrict__ bidx, const unsigned char *__restrict__ kernel, unsigned char *grids, int count,
                int max_base)
{
    __shared__ unsigned char sk[41 * 41];
    __shared__ unsigned long long stile[WAVES][KT_BT_H * KT_BT_W];
    // WAVES == 4: one workgroup per (match, base scan), XCD-aware (every block of match m on XCD m % 8);
    // otherwise one workgroup per match whose waves share out all (base scan, chunk) pairs, so the
    // overlapping chunks of different base scans rarely race for the same grid words.
    int m, jlo, jhi;
    if (WAVES == 4) {
        const int b = blockIdx.x;
        const int xcd = b & 7, q8 = b >> 3;
        const int grp = q8 / max_base, j = q8 - grp * max_base;
        m = grp * 8 + xcd;
        if (m >= count) return;
        jlo = bbeg[m] + j;
        jhi = jlo + 1;
        if (jlo >= bbeg[m + 1]) return;
    } else {
        m = blockIdx.x;
        jlo = bbeg[m];
        jhi = bbeg[m + 1];
    }
    for (int i = threadIdx.x; i < g.ksize * g.ksize; i += WAVES * 64) sk[i] = kernel[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const KtState &S = st[m];
    const double vx = S.center[0], vy = S.center[1];
    const double gox = S.gox, goy = S.goy;
    unsigned char *grid = grids + (size_t)m * g.grid_stride;
    unsigned long long *gw = reinterpret_cast<unsigned long long *>(grid);
    const int wsw = g.ws >> 3;  // qwords per grid row (ws is a multiple of 8)
    const int h = g.half, ks = g.ksize;
    unsigned long long *tile = stile[wave];
    int cell_off[4], cell_off2[4];
    unsigned char cell_kv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = lane + 64 * u;
        const int jj = t / ks, ii = t - jj * ks;
        const bool in = ks <= KT_FAST_KS && t < ks * ks;
        cell_off[u] = in ? jj : 0;
        cell_off2[u] = in ? ii : 0;
        cell_kv[u] = in ? sk[ii + ks * jj] : 0;
    }
    const int cmax = (g.n + KT_CHUNK - 1) / KT_CHUNK;  // chunk slots per base scan
    for (int id = wave; id < (jhi - jlo) * cmax; id += WAVES) {
        const int jb = id / cmax, c = id - jb * cmax;
        const int s = bidx[jlo + jb];
        const int npts = P.npts[s];
        if (c * KT_CHUNK >= npts) continue;
        const double2 *pts = P.pts + (size_t)s * g.n;
        const int2 *evt = P.evt + (size_t)s * g.n;
        // ---- this chunk's points: FindValidPoints' viewpoint test, AddScan's ROI test ----
        const int k = c * KT_CHUNK + lane;
        bool ok = false;
        int cx = 0, cy = 0;
        if (lane < KT_CHUNK && k < npts) {
            const int2 e = evt[k];
            if (e.x >= 0) {
                const double2 f = pts[e.y], cu = pts[e.x];
                const double a = vy - f.y;
                const double b = f.x - vx;
                const double cc = f.y * vx - f.x * vy;
                const double ss = cu.x * a + cu.y * b + cc;
                if (!(ss < 0.0)) {  // wrong side of the viewpoint otherwise (Mapper.cpp:795-799)
                    const double2 p = pts[k];
                    const int gx = kt_w2g(p.x, gox, g.scale), gy = kt_w2g(p.y, goy, g.scale);
                    if (gx >= 0 && gx < g.grid_size && gy >= 0 && gy < g.grid_size) {
                        ok = true;
                        cx = gx + g.border;
                        cy = gy + g.border;
                    }
                }
            }
        }
        const unsigned long long mask = __ballot(ok);
        if (mask == 0ull) continue;
        if (kt_group(mask, ok, cx, cy, lane, h, ks, wsw, gw, tile, sk, cell_off, cell_off2, cell_kv, clear)) continue;
        // the chunk's box is too large (a jump between walls): quarters, then single points
        for (int q = 0; q < KT_CHUNK; q += 4) {
            const unsigned long long m4 = mask & (0xFull << q);
            if (m4 == 0ull || kt_group(m4, ok, cx, cy, lane, h, ks, wsw, gw, tile, sk, cell_off, cell_off2, cell_kv, clear))
                continue;
            unsigned long long mm = m4;
            while (mm) {  // one footprint always fits the tile (ks <= 41)
                const int src = __builtin_ctzll(mm);
                mm &= mm - 1;
                kt_group(1ull << src, ok, cx, cy, lane, h, ks, wsw, gw, tile, sk, cell_off, cell_off2, cell_kv, clear);
            }
        }
    }
}

// =================================================================================================
// kt_addscans_kernel: AddScans of one match per workgroup, binned by 64 x 64-cell grid tiles
//
// 1. every valid (FindValidPoints) in-ROI point of the match's base scans -> its cell, into a
//    per-slot scratch list (all 512 threads: the dependent loads overlap across the breadth);
// 2. passes over as many base scans as the LDS item store holds: count the points per tile their
//    smear footprint overlaps, prefix, scatter the cells tile-sorted into LDS;
// 3. every wave takes whole tiles: renders the tile's footprints into a 4 KB LDS tile (byte max,
//    points in turn, lanes over kernel cells) and writes the tile with plain 8-byte stores -- the
//    workgroup owns its match's grid, so no atomics touch global memory.  A tile written by an
//    earlier pass is re-read first.  Written tiles are listed per slot for kt_clear_tiles_kernel.
// =================================================================================================
#if defined(KT_DIAG_STAMPS)
__device__ unsigned long long kt_diag[65536 * 8];
#define KT_STAMP(i) do { if (threadIdx.x == 0) kt_diag[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define KT_STAMP(i) do { } while (0)
#endif
constexpr int KT_AS_WAVES = 8;
constexpr int KT_AS_ITEMS = 15360;     // tile-sorted footprint items per pass (60 KB of LDS)
constexpr int KT_AS_MARGIN = 16;       // LDS tile margin (footprints of kernel half <= 8 stay inside)
constexpr int KT_AS_TW = 64 + 2 * KT_AS_MARGIN;
constexpr int KT_AS_MAX_TILES = 2048;  // tiles per grid (e.g. 2896 x 2896 cells)
constexpr int KT_AS_MAX_BASE = 1024;
constexpr int KT_AS_CLASSES = 12;  // tile size classes of the render order

__device__ __forceinline__ int kt_size_class(int c)  // 0 for c >= 2^11, 11 for c == 1
{
    const int lg = 31 - __builtin_clz((unsigned)c);
    return lg >= KT_AS_CLASSES - 1 ? 0 : KT_AS_CLASSES - 1 - lg;
}

template <int NW>
__device__ __forceinline__ int kt_block_exscan_n(int v, int *sw, int *total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(inc, off, 64);
        if (lane >= off) inc += t;
    }
    if (lane == 63) sw[w] = inc;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        woff += i < w ? sw[i] : 0;
        tot += sw[i];
    }
    *total = tot;
    __syncthreads();
    return woff + inc - v;
}

__device__ __forceinline__ int kt_tiles_of(int cx, int cy, int h, int tiles_x, int *t)
{
    const int tx0 = (cx - h) >> 6, tx1 = (cx + h) >> 6, ty0 = (cy - h) >> 6, ty1 = (cy + h) >> 6;
    int c = 0;
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) t[c++] = ty * tiles_x + tx;
    return c;
}

// One wave renders the items [c0, c1) of a tile into its LDS tile (fast path, ks <= KT_FAST_KS): lane
// slot u < NS holds kernel cell (lane + 64 u) mod ks^2 at byte offset koff[u] from the footprint's
// origin.  Lanes past the last cell duplicate a cell another slot (or lane) also holds, with the same
// kernel value: both write max(old, kv) or max(max(old, kv), kv), the same byte, so every slot runs on
// all lanes, unmasked and with no trash bytes.  The items are read 64 at a time (one LDS read, then
// v_readlane per item).  Item j is paired with item j + half of the chunk:
// when their footprints are disjoint, both are read before either is written (one LDS round trip for
// the two); otherwise they run one after the other.  Byte max is order-free, so any order is exact.
template <int NS>
__device__ __forceinline__ void kt_render_items(unsigned char *tileb, const unsigned *sitem, int c0, int c1, int base,
                                                int ks, const int (&koff)[4], const unsigned (&kv)[4])
{
    const int lane = threadIdx.x & 63;
    auto one = [&](int o) {
        unsigned cur[NS];
#pragma unroll
        for (int u = 0; u < NS; ++u) cur[u] = tileb[koff[u] + o];
#pragma unroll
        for (int u = 0; u < NS; ++u) tileb[koff[u] + o] = (unsigned char)max(cur[u], kv[u]);
    };
    auto two = [&](int oa, int ob) {
        unsigned ca[NS], cb[NS];
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            ca[u] = tileb[koff[u] + oa];
            cb[u] = tileb[koff[u] + ob];
        }
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            tileb[koff[u] + oa] = (unsigned char)max(ca[u], kv[u]);
            tileb[koff[u] + ob] = (unsigned char)max(cb[u], kv[u]);
        }
    };
    for (int cb = c0; cb < c1; cb += 64) {
        const int ne = min(64, c1 - cb);
        const int mine = lane < ne ? (int)sitem[cb + lane] : 0;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), as in kt_render_items_dw
        const int half = ne >> 1;
        for (int j = 0; j < half; ++j) {
            const int a = __builtin_amdgcn_readlane(mine, j), b = __builtin_amdgcn_readlane(mine, j + half);
            const int ax = a & 0xFFFF, ay = a >> 16, bx = b & 0xFFFF, by = b >> 16;
            const int oa = base + ay * KT_AS_TW + ax, ob = base + by * KT_AS_TW + bx;  // scalar
            if (abs(ax - bx) >= ks || abs(ay - by) >= ks) {
                two(oa, ob);
            } else {
                one(oa);
                one(ob);
            }
        }
        if (ne & 1) {
            const int a = __builtin_amdgcn_readlane(mine, ne - 1);
            one(base + (a >> 16) * KT_AS_TW + (a & 0xFFFF));
        }
    }
}

// Dword form of the render for kernels up to KT_DW_KS wide: a footprint row of ks bytes starting at
// any byte lies in 4 aligned dwords, so lane (r, k) of the first ks * nd lanes owns aligned dword k of
// footprint row r (nd = dwords per row), one ds_read_b32 + one ds_write_b32 per item.  Its 4 kernel
// bytes depend on the origin's alignment s: they are bytes 3 - s .. 6 - s of the lane's 8 bytes of the
// row's kernel padded with 3 leading zeros (klo, khi), one v_alignbyte.  Bytes outside the footprint
// get kernel 0 (max(x, 0) = x) and lanes past ks * nd duplicate a lane's dword (same value written).
// Items run one after the other (pairs with disjoint dword spans read before either write measured
// slower here).  Byte max is per-byte SWAR, exact because every grid byte and kernel value is <= 100.
constexpr int KT_DW_KS = 13;

__device__ __forceinline__ unsigned kt_bytemax7(unsigned a, unsigned b)
{
    const unsigned t = ((a | 0x80808080u) - b) & 0x80808080u;  // 0x80 in every byte where a >= b
    return b ^ ((a ^ b) & (t - (t >> 7)));
}

__device__ __forceinline__ void kt_render_items_dw(unsigned char *tileb, const unsigned *sitem, int c0, int c1, int bx,
                                                   int by, int ks, int nd, int koffd, unsigned klo, unsigned khi)
{
    const int lane = threadIdx.x & 63;
    auto one = [&](int row, int col) {
        unsigned *w = reinterpret_cast<unsigned *>(tileb + row * KT_AS_TW + (col & ~3) + koffd);
        const unsigned kv = __builtin_amdgcn_alignbyte(khi, klo, 3 - (col & 3));
        const unsigned x = *w;
        *w = kt_bytemax7(x, kv);
    };
    for (int cb = c0; cb < c1; cb += 64) {
        const int ne = min(64, c1 - cb);
        const int mine = lane < ne ? (int)sitem[cb + lane] : 0;
        // wait for the item read here: left to the compiler, the wait lands inside the loop, where it
        // also waits for every item's store before the next item's load is issued
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        for (int j = 0; j < ne; ++j) {
            const int a = __builtin_amdgcn_readlane(mine, j);
            one(by + (a >> 16), bx + (a & 0xFFFF));
        }
    }
}

__global__ void __launch_bounds__(KT_AS_WAVES * 64)
kt_addscans_kernel(KtGeom g, KtPool P, const KtState *__restrict__ st, const int *__restrict__ bbeg,
                   const int *__restrict__ bidx, const unsigned char *__restrict__ kernel, unsigned char *grids,
                   int *scratch, size_t scratch_stride, int *dirty_list, int *dirty_count)
{
    __shared__ unsigned sitem[KT_AS_ITEMS];
    __shared__ int soff[KT_AS_MAX_TILES + 1];
    __shared__ int scur[KT_AS_MAX_TILES];
    __shared__ unsigned char sdirty[KT_AS_MAX_TILES];
    __shared__ int sscan[KT_AS_MAX_BASE];
    __shared__ unsigned long long stile[KT_AS_WAVES][KT_AS_TW * KT_AS_TW / 8 + 8];  // + 64 trash bytes
    __shared__ unsigned char sk[41 * 41];
    __shared__ int sw[KT_AS_WAVES];
    __shared__ int s_ndirty, s_pass_end, s_next;
    __shared__ int sbk[2 * KT_AS_CLASSES + 1];  // per size class: list offset, cursor; then the list length
    constexpr int NT = KT_AS_WAVES * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = blockIdx.x;
    const int jlo = bbeg[m], nb = bbeg[m + 1] - jlo;
    const KtState &S = st[m];
    const double vx = S.center[0], vy = S.center[1];
    const double gox = S.gox, goy = S.goy;
    const int n = g.n, h = g.half, ks = g.ksize, NTL = g.ntiles;
    const int wsw = g.ws >> 3;
    unsigned long long *gw = reinterpret_cast<unsigned long long *>(grids + (size_t)m * g.grid_stride);
    int *cellv = scratch + (size_t)m * scratch_stride;
    KT_STAMP(0);
    for (int i = tid; i < ks * ks; i += NT) sk[i] = kernel[i];
    for (int t = tid; t < NTL; t += NT) sdirty[t] = 0;
    for (int j = tid; j < nb; j += NT) sscan[j] = 0;
    if (tid == 0) {
        s_ndirty = 0;
        s_next = 0;
    }
    __syncthreads();
    // ---- 1. cells of the valid in-ROI points ----
    // four points per thread and trip, every load of the four issued before any is used (the chain
    // bidx -> npts / evt -> pts is three dependent loads; out-of-range lanes read in-bounds index 0)
    constexpr int KT_P1_U = 4;
    for (int i0 = tid; i0 < nb * n; i0 += KT_P1_U * NT) {
        int jv[KT_P1_U], kv[KT_P1_U], sv[KT_P1_U];
#pragma unroll
        for (int u = 0; u < KT_P1_U; ++u) {
            const int i = i0 + u * NT;
            const int ic = i < nb * n ? i : 0;
            jv[u] = ic / n;
            kv[u] = ic - jv[u] * n;
            sv[u] = bidx[jlo + jv[u]];
        }
        int np[KT_P1_U];
        int2 ev[KT_P1_U];
#pragma unroll
        for (int u = 0; u < KT_P1_U; ++u) {
            np[u] = P.npts[sv[u]];
            ev[u] = P.evt[(size_t)sv[u] * n + kv[u]];
        }
        double2 fv[KT_P1_U], cv[KT_P1_U], pv[KT_P1_U];
        bool ok[KT_P1_U];
#pragma unroll
        for (int u = 0; u < KT_P1_U; ++u) {
            const double2 *pts = P.pts + (size_t)sv[u] * n;
            ok[u] = i0 + u * NT < nb * n && kv[u] < np[u] && ev[u].x >= 0;
            fv[u] = pts[ok[u] ? ev[u].y : 0];
            cv[u] = pts[ok[u] ? ev[u].x : 0];
            pv[u] = pts[kv[u]];
        }
#pragma unroll
        for (int u = 0; u < KT_P1_U; ++u) {
            const int i = i0 + u * NT;
            if (i >= nb * n) break;
            int cell = -1;
            if (ok[u]) {
                const double2 f = fv[u], cu = cv[u];
                const double a = vy - f.y;
                const double b = f.x - vx;
                const double cc = f.y * vx - f.x * vy;
                const double ss = cu.x * a + cu.y * b + cc;
                if (!(ss < 0.0)) {  // wrong side of the viewpoint otherwise (Mapper.cpp:795-799)
                    const int gx = kt_w2g(pv[u].x, gox, g.scale), gy = kt_w2g(pv[u].y, goy, g.scale);
                    if (gx >= 0 && gx < g.grid_size && gy >= 0 && gy < g.grid_size)
                        cell = (gx + g.border) | ((gy + g.border) << 16);
                }
            }
            cellv[i] = cell;
            if (cell >= 0) {
                int tl[4];
                atomicAdd(&sscan[jv[u]], kt_tiles_of(cell & 0xFFFF, cell >> 16, h, g.tiles_x, tl));
            }
        }
    }
    __syncthreads();
    KT_STAMP(1);
    // per-lane kernel cells (ks <= 15: at most 4 of the <= 225 cells per lane), as byte offsets in the
    // LDS tile from the footprint's origin
    int koff[4];
    unsigned kvv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = (lane + 64 * u) % (ks * ks);  // past the last cell: a duplicate (kt_render_items)
        const int jj = t / ks, ii = t - jj * ks;
        const bool in = ks <= KT_FAST_KS;
        koff[u] = in ? jj * KT_AS_TW + ii : 0;
        kvv[u] = in ? sk[ii + ks * jj] : 0u;
    }
    const int nslot = (ks * ks + 63) >> 6;
    // dword form (ks <= KT_DW_KS): lane -> (row r, dword k), klo / khi = padded kernel bytes 4k .. 4k + 7
    const int nd = (ks + 6) >> 2;
    int koffd = 0;
    unsigned klo = 0u, khi = 0u;
    if (ks <= KT_DW_KS) {
        const int t = lane % (ks * nd);
        const int r = t / nd, k = t - r * nd;
        koffd = r * KT_AS_TW + 4 * k;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = 4 * k + j - 3;
            const unsigned v = (c >= 0 && c < ks) ? (unsigned)sk[c + ks * r] : 0u;
            if (j < 4) klo |= v << (8 * j);
            else khi |= v << (8 * (j - 4));
        }
    }
    unsigned long long *tile = stile[wave];
    unsigned char *tileb = reinterpret_cast<unsigned char *>(tile);
    int pa = 0;
    while (pa < nb) {
        if (tid == 0) {  // as many base scans as the item store holds (one always fits: <= 4 * 4096)
            int tot = 0, pb = pa;
            while (pb < nb && tot + sscan[pb] <= KT_AS_ITEMS) tot += sscan[pb++];
            s_pass_end = pb;
        }
        for (int t = tid; t < NTL; t += NT) scur[t] = 0;
        if (tid < 2 * KT_AS_CLASSES + 1) sbk[tid] = 0;
        __syncthreads();
        const int pb = s_pass_end;
        // ---- 2. count per tile, prefix, scatter tile-sorted ----
        for (int i = pa * n + tid; i < pb * n; i += NT) {
            const int cell = cellv[i];
            if (cell < 0) continue;
            int tl[4];
            const int c = kt_tiles_of(cell & 0xFFFF, cell >> 16, h, g.tiles_x, tl);
            for (int q = 0; q < c; ++q) atomicAdd(&scur[tl[q]], 1);
        }
        __syncthreads();
        {
            const int per = (NTL + NT - 1) / NT;
            const int t0 = min(tid * per, NTL), t1 = min(t0 + per, NTL);
            int loc = 0;
            for (int t = t0; t < t1; ++t) loc += scur[t];
            int tot;
            int pre = kt_block_exscan_n<KT_AS_WAVES>(loc, sw, &tot);
            for (int t = t0; t < t1; ++t) {
                const int c = scur[t];
                soff[t] = pre;
                scur[t] = pre;
                pre += c;
            }
            if (tid == 0) soff[NTL] = tot;
        }
        __syncthreads();
        if (pa == 0) KT_STAMP(2);
        for (int i = pa * n + tid; i < pb * n; i += NT) {
            const int cell = cellv[i];
            if (cell < 0) continue;
            int tl[4];
            const int c = kt_tiles_of(cell & 0xFFFF, cell >> 16, h, g.tiles_x, tl);
            for (int q = 0; q < c; ++q) sitem[atomicAdd(&scur[tl[q]], 1)] = (unsigned)cell;
        }
        // the tiles with items by size class (class 0: >= 2^(KT_AS_CLASSES - 1) items, then halving)
        for (int t = tid; t < NTL; t += NT) {
            const int c = soff[t + 1] - soff[t];
            if (c) atomicAdd(&sbk[kt_size_class(c)], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int k = 0; k < KT_AS_CLASSES; ++k) {
                const int v = sbk[k];
                sbk[k] = acc;
                acc += v;
            }
            sbk[2 * KT_AS_CLASSES] = acc;
        }
        __syncthreads();
        // the scatter is done, so scur becomes the tile list, heaviest class first: the waves take tiles
        // from it in turn (greedy largest-first; round-robin by tile index left one wave a third above
        // the mean)
        int *slist = scur;
        for (int t = tid; t < NTL; t += NT) {
            const int c = soff[t + 1] - soff[t];
            if (c) {
                const int k = kt_size_class(c);
                slist[sbk[k] + atomicAdd(&sbk[KT_AS_CLASSES + k], 1)] = t;
            }
        }
        __syncthreads();
        if (pa == 0) KT_STAMP(3);
        // ---- 3. render whole tiles, plain stores ----
        // The LDS tile is the 64 x 64 tile plus a 16-cell margin on every side, so a footprint of any
        // point listed for the tile (kernel half <= 8 in this path) lies inside it: no bounds tests,
        // no divergence; cells a lane does not own get max(x, 0) = x written back.
        const int nlist = sbk[2 * KT_AS_CLASSES];
        for (;;) {
            int k = 0;
            if (lane == 0) k = atomicAdd(&s_next, 1);
            k = __builtin_amdgcn_readfirstlane(k);
            if (k >= nlist) break;
            const int t = __builtin_amdgcn_readfirstlane(slist[k]);
            const int c0 = soff[t], c1 = soff[t + 1];
            const int ty = t / g.tiles_x, tx = t - ty * g.tiles_x;
            const int x0 = tx * 64, y0 = ty * 64;
            const bool was = sdirty[t] != 0;
            for (int q = lane; q < KT_AS_TW * KT_AS_TW / 8; q += 64) tile[q] = 0ull;
            if (was)
                for (int q = lane; q < 512; q += 64) {
                    const int r = q >> 3, xq = (x0 >> 3) + (q & 7), y = y0 + r;
                    if (y < g.height && xq < wsw)
                        tile[((r + KT_AS_MARGIN) * KT_AS_TW + KT_AS_MARGIN) / 8 + (q & 7)] = gw[(size_t)y * wsw + xq];
                }
            if (ks <= KT_DW_KS) {
                kt_render_items_dw(tileb, sitem, c0, c1, KT_AS_MARGIN - h - x0, KT_AS_MARGIN - h - y0, ks, nd, koffd, klo,
                                   khi);
            } else if (ks <= KT_FAST_KS) {
                // The LDS tile is the 64 x 64 tile plus a 16-cell margin on every side, so a footprint of
                // any point listed for the tile (kernel half <= 8 in this path) lies inside it: no bounds
                // tests.  base + (cell row) * TW + (cell col) is the footprint origin's byte (scalar).
                const int base = __builtin_amdgcn_readfirstlane((KT_AS_MARGIN - h - y0) * KT_AS_TW + (KT_AS_MARGIN - h - x0));
                switch (nslot) {
                case 1: kt_render_items<1>(tileb, sitem, c0, c1, base, ks, koff, kvv); break;
                case 2: kt_render_items<2>(tileb, sitem, c0, c1, base, ks, koff, kvv); break;
                case 3: kt_render_items<3>(tileb, sitem, c0, c1, base, ks, koff, kvv); break;
                default: kt_render_items<4>(tileb, sitem, c0, c1, base, ks, koff, kvv); break;
                }
            } else {
                for (int c = c0; c < c1; ++c) {
                    const unsigned cell = sitem[c];
                    const int bx = (int)(cell & 0xFFFFu) - h - x0, by = (int)(cell >> 16) - h - y0;
                    for (int q = lane; q < ks * ks; q += 64) {
                        const int jj = q / ks, ii = q - jj * ks;
                        const int x = bx + ii, y = by + jj;
                        if ((unsigned)x >= 64u || (unsigned)y >= 64u) continue;
                        const unsigned char kv = sk[ii + ks * jj];
                        unsigned char *b = tileb + (y + KT_AS_MARGIN) * KT_AS_TW + x + KT_AS_MARGIN;
                        if (kv > *b) *b = kv;
                    }
                }
            }
            for (int q = lane; q < 512; q += 64) {
                const int r = q >> 3, xq = (x0 >> 3) + (q & 7), y = y0 + r;
                if (y < g.height && xq < wsw)
                    gw[(size_t)y * wsw + xq] = tile[((r + KT_AS_MARGIN) * KT_AS_TW + KT_AS_MARGIN) / 8 + (q & 7)];
            }
            if (lane == 0 && !was) {
                sdirty[t] = 1;
                dirty_list[(size_t)m * NTL + atomicAdd(&s_ndirty, 1)] = t;
            }
        }
        __syncthreads();
        if (tid == 0) s_next = 0;
        if (pa == 0) KT_STAMP(4);
        pa = pb;
    }
    if (tid == 0) dirty_count[m] = s_ndirty;
    KT_STAMP(5);
}

// zero every tile kt_addscans_kernel wrote for the slot
__global__ void __launch_bounds__(KT_THREADS)
kt_clear_tiles_kernel(KtGeom g, unsigned char *grids, const int *__restrict__ dirty_list,
                      const int *__restrict__ dirty_count)
{
    const int m = blockIdx.x;
    const int cnt = dirty_count[m];
    const int wsw = g.ws >> 3;
    unsigned long long *gw = reinterpret_cast<unsigned long long *>(grids + (size_t)m * g.grid_stride);
    // gridDim.y workgroups per match share its tiles (more stores in flight than one workgroup's)
    for (int i = threadIdx.x + blockIdx.y * KT_THREADS; i < cnt * 512; i += KT_THREADS * gridDim.y) {
        const int t = dirty_list[(size_t)m * g.ntiles + (i >> 9)];
        const int q = i & 511;
        const int ty = t / g.tiles_x, tx = t - ty * g.tiles_x;
        const int y = ty * 64 + (q >> 3), xq = tx * 8 + (q & 7);
        if (y < g.height && xq < wsw) gw[(size_t)y * wsw + xq] = 0ull;
    }
}

// =================================================================================================
// kt_coarse_kernel: GetResponse over a tile of 256 positions for a group of `ag` consecutive angles
//
// The workgroup keeps its positions and walks its angles: per angle the query's offsets
// (GridIndexLookup::ComputeOffsets) into LDS, the gathers, the responses.  A position's `ag` responses
// are stored angle-major (resp[a * npos + pos], the select kernel reads them back in the reference's
// pose order pos * nA + a), so each angle's 256 responses leave as one contiguous 2 KB run: stored
// position-major, each workgroup wrote 8-byte pieces 8 * nA bytes apart and the launch wrote 157 MB for
// 55 MB of responses (r01el, r02ae).  The per-position maximum over the group's angles is kept in a
// register for the match's best response only: the per-position maximum over all angles is derived
// from the stored responses by kt_select_kernel (no 64-bit atomic per position and angle).  ag = 1 by
// default (grouping measured slower: fewer workgroups in flight for the gathers); SLAM2D_KT_AG sets it.
// =================================================================================================
__global__ void __launch_bounds__(KT_THREADS)
kt_coarse_kernel(KtGeom g, KtPool P, KtState *st, const unsigned char *__restrict__ grids, double *resp,
                 unsigned long long *posmax, int count, int pass, int penalize, int shard, int nshards, int ag)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char kt_smem[];
    int *soff = reinterpret_cast<int *>(kt_smem);  // [npts]
    __shared__ unsigned scnt[4][KT_THREADS];
    __shared__ double sbest[4];

    const int nA = g.nang[pass];
    const int ngrp = (nA + ag - 1) / ag;
    const int T2 = g.ctx * g.cty;
    const int W = ngrp * T2;
    // XCD-aware: all work of one match runs on one XCD (blocks are dealt round-robin to the 8 XCDs)
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = b >> 3;
    const int grp = q8 / W, w = q8 - grp * W;
    const int m = grp * 8 + xcd;
    if (m >= count) return;
    KtState &S = st[m];
    if (S.pass != pass) return;
    const int agrp = w / T2, t = w - agrp * T2;
    const int a0 = agrp * ag, a1 = min(a0 + ag, nA);
    const int ty = t / g.ctx, tx = t - ty * g.ctx;
    // tile of 256 positions, TW = 4 << clw wide and TH = 64 >> clw high: a lane gathers 4 positions of a
    // row (8 bytes), 1 << clw lanes per row
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    const double cxs = S.center[0], cys = S.center[1], chs = S.center[2];
    const double gox = S.gox, goy = S.goy;
    const double aoff = g.aoff[pass];
    const double start = chs - aoff;
    const int q = S.query, npts = S.npts;
    const double2 *loc = P.loc + (size_t)q * g.n;
    const unsigned char *bad = P.bad + (size_t)q * g.n;
    // this lane's 4 gather positions: row iy, columns ix0 .. ix0 + 3
    const int clw = g.clw, lmask = (1 << clw) - 1;
    const int iy = ty * (64 >> clw) + (lane >> clw);
    const int ix0 = tx * (4 << clw) + (lane & lmask) * 4;
    const double startX = -g.coff;
    int gpos[4];
    bool fast = true;
    {
        const double y = startX + (double)(uint32_t)iy * g.cres;
        const int gy = kt_w2g(cys + y, goy, g.scale) + g.border;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ix = ix0 + j;
            gpos[j] = 0;
            if (ix < g.nxy && iy < g.nxy) {
                const double x = startX + (double)(uint32_t)ix * g.cres;
                const int gx = kt_w2g(cxs + x, gox, g.scale) + g.border;
                if (gx < 0 || gx >= g.width || gy < 0 || gy >= g.height) {
                    S.status = KT_ERANGE;  // GridIndex would throw (Karto.h:4488-4499)
                    continue;
                }
                gpos[j] = gx + gy * g.ws;
                if (gpos[j] != gpos[0] + 2 * j) fast = false;
            }
        }
    }
    // the position this thread finalises (one per thread of the tile)
    const int pl = tid >> 2, pj = tid & 3;
    const int piy = ty * (64 >> clw) + (pl >> clw);
    const int pix = tx * (4 << clw) + (pl & lmask) * 4 + pj;
    const bool pin = piy < g.nxy && pix < g.nxy;
    const size_t pos = (size_t)piy * g.nxy + pix;
    // responses angle-major (resp[a * npos + pos]): a workgroup's 256 positions are one contiguous 2 KB run
    const size_t npos = (size_t)g.nxy * g.nxy;
    double *rpos = resp + (size_t)m * g.max_poses + pos;
    double pmax = 0.0;   // max over this group's angles at this position (responses are >= 0)

    const unsigned ds = (unsigned)g.data_size;
    const unsigned lim = ds - 6u;
    const unsigned char *grid = grids + (size_t)m * g.grid_stride;
    for (int a = a0; a < a1; ++a) {
        // window sharded over GPUs (kt_match_sharded_begin_device): this rank owns the angles
        // a = shard (mod nshards); the others' responses are left +0.0 for the MAX all-reduce
        if ((a % nshards) != shard) {  // block-uniform
            if (pin) rpos[(size_t)a * npos] = 0.0;
            continue;
        }
        const double angle = start + (double)(uint32_t)a * g.cares;
        const double cs = sdm_cos(angle), sn = sdm_sin(angle);
        __syncthreads();  // the previous angle's offsets are no longer read
        for (int k = tid; k < npts; k += KT_THREADS) {
            int o = KT_INVALID;
            if (!bad[k]) {
                const double2 l = loc[k];
                const double ox = cs * l.x - sn * l.y;
                const double oy = sn * l.x + cs * l.y;
                const int gx = kt_w2g(ox + gox, gox, g.scale), gy = kt_w2g(oy + goy, goy, g.scale);
                o = gx + gy * g.ws;
            }
            soff[k] = o;
        }
        __syncthreads();
        unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        unsigned acc01 = 0, acc23 = 0;
        int since = 0;
        if (fast) {
            // 8 points per iteration: 8 independent 8-byte gathers in flight per lane
            const int base = gpos[0];
            int k = wave;
            for (; k + 28 < npts; k += 32) {
                int bi[8];
                bool allin = true;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    bi[j] = base + soff[k + 4 * j];
                    allin = allin && (unsigned)bi[j] < lim;
                }
                if (allin) {
                    uint2 v[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) __builtin_memcpy(&v[j], grid + bi[j], 8);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        acc01 += v[j].x & 0x00FF00FFu;
                        acc23 += v[j].y & 0x00FF00FFu;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int b = bi[j];
                        if ((unsigned)b < ds) c0 += grid[b];
                        if ((unsigned)(b + 2) < ds) c1 += grid[b + 2];
                        if ((unsigned)(b + 4) < ds) c2 += grid[b + 4];
                        if ((unsigned)(b + 6) < ds) c3 += grid[b + 6];
                    }
                }
                since += 8;
                if (since >= 504) {  // 512 * 100 < 65536: flush the packed 16-bit sums
                    c0 += acc01 & 0xFFFFu; c1 += acc01 >> 16; c2 += acc23 & 0xFFFFu; c3 += acc23 >> 16;
                    acc01 = acc23 = 0;
                    since = 0;
                }
            }
            for (; k < npts; k += 4) {
                const int bi = base + soff[k];
                if ((unsigned)bi < lim) {
                    uint2 v;
                    __builtin_memcpy(&v, grid + bi, 8);
                    acc01 += v.x & 0x00FF00FFu;
                    acc23 += v.y & 0x00FF00FFu;
                } else {
                    if ((unsigned)bi < ds) c0 += grid[bi];
                    if ((unsigned)(bi + 2) < ds) c1 += grid[bi + 2];
                    if ((unsigned)(bi + 4) < ds) c2 += grid[bi + 4];
                    if ((unsigned)(bi + 6) < ds) c3 += grid[bi + 6];
                }
            }
            c0 += acc01 & 0xFFFFu; c1 += acc01 >> 16; c2 += acc23 & 0xFFFFu; c3 += acc23 >> 16;
        } else {
            for (int k = wave; k < npts; k += 4) {
                const int o = soff[k];
                const int i0 = gpos[0] + o, i1 = gpos[1] + o, i2 = gpos[2] + o, i3 = gpos[3] + o;
                if ((unsigned)i0 < ds) c0 += grid[i0];
                if ((unsigned)i1 < ds) c1 += grid[i1];
                if ((unsigned)i2 < ds) c2 += grid[i2];
                if ((unsigned)i3 < ds) c3 += grid[i3];
            }
        }
        scnt[wave][lane * 4 + 0] = c0;
        scnt[wave][lane * 4 + 1] = c1;
        scnt[wave][lane * 4 + 2] = c2;
        scnt[wave][lane * 4 + 3] = c3;
        __syncthreads();
        // one thread per position of the tile
        const unsigned total = scnt[0][tid] + scnt[1][tid] + scnt[2][tid] + scnt[3][tid];
        if (pin) {
            double response = 0.0;
            if (npts > 0) response = (double)total / (double)(uint32_t)(npts * KT_OCC);
            if (penalize && !kt_deq(response, 0.0)) {
                const double x = startX + (double)(uint32_t)pix * g.cres;
                const double y = startX + (double)(uint32_t)piy * g.cres;
                const double sqd = kt_sq(x) + kt_sq(y);
                double dp = 1.0 - (KT_GAIN * sqd / g.dvp);
                dp = kt_max(dp, g.mdp);
                const double sqa = kt_sq(angle - chs);
                double ap = 1.0 - (KT_GAIN * sqa / g.avp);
                ap = kt_max(ap, g.map_);
                response *= (dp * ap);
            }
            rpos[(size_t)a * npos] = response;
            pmax = kt_max(pmax, response);
        }
    }
    double best = pmax;  // posmax itself is taken from the stored responses by kt_select_kernel
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) best = kt_max(best, __shfl_xor(best, off, 64));
    if (lane == 0) sbest[wave] = best;
    __syncthreads();
    if (tid == 0) {
        const double bb = kt_max(kt_max(sbest[0], sbest[1]), kt_max(sbest[2], sbest[3]));
        atomicMax(&S.best_bits, kt_bits(bb));
    }
}

// =================================================================================================
// kt_exchange_kernel: the per-match state a sharded window exchanges (dir 0: export, 1: import)
//   x[m] = [best bits, ERANGE flag, posmax (nxy^2 bits), responses (nxy^2 * nA bits)]
// every value is a non-negative double, so the int64 MAX all-reduce of the ranks' exports is exactly
// the union of their angles (non-owned responses are +0.0, posmax / best are maxima already).
// =================================================================================================
__global__ void __launch_bounds__(KT_THREADS)
kt_exchange_kernel(KtGeom g, KtState *st, double *resp, unsigned long long *posmax, long long *xbuf, int dir)
{
    const int m = blockIdx.x, tid = threadIdx.x;
    KtState &S = st[m];
    const int nxy2 = g.nxy * g.nxy;
    const int np = nxy2 * g.nang[0];
    long long *x = xbuf + (size_t)m * (2 + nxy2 + np);
    unsigned long long *pm = posmax + (size_t)m * nxy2;
    long long *r = reinterpret_cast<long long *>(resp + (size_t)m * g.max_poses);
    if (dir == 0) {
        if (tid == 0) {
            x[0] = (long long)S.best_bits;
            x[1] = S.status == KT_ERANGE ? 1 : 0;
        }
        for (int i = tid; i < nxy2; i += KT_THREADS) x[2 + i] = (long long)pm[i];
        for (int i = tid; i < np; i += KT_THREADS) x[2 + nxy2 + i] = r[i];
    } else {
        if (tid == 0) {
            S.best_bits = (unsigned long long)x[0];
            if (x[1]) S.status = KT_ERANGE;
        }
        for (int i = tid; i < nxy2; i += KT_THREADS) pm[i] = (unsigned long long)x[2 + i];
        for (int i = tid; i < np; i += KT_THREADS) r[i] = x[2 + nxy2 + i];
    }
}

// =================================================================================================
// kt_select_kernel: best, tie average, positional covariance, response expansion
// (KT_SEL_THREADS = 1024 for large windows: the loop window's 101 x 101 positions take 10 block rounds
// instead of 40; 256 for the sequential matcher's 16 x 16, where the wider block measured slower)
// =================================================================================================
template <int KT_SEL_THREADS>
__global__ void __launch_bounds__(KT_SEL_THREADS)
kt_select_kernel(KtGeom g, KtState *st, const double *__restrict__ resp, unsigned long long *posmax, int *tie_idx,
                 double4 *tie_val, int pass, int refine, kt_result *out)
{
    __shared__ int sw[KT_SEL_THREADS / 64];
    __shared__ int s_n;
    __shared__ double s_mean[3];
    __shared__ int s_err;
    __shared__ int s_pcx[KT_MAX_NXY], s_pcy[KT_MAX_NXY];
    const int m = blockIdx.x;
    KtState &S = st[m];
    if (S.pass != pass) return;
    const int tid = threadIdx.x;
    const int nA = g.nang[pass];
    const int nxy = g.nxy;
    const double best = kt_dbl(S.best_bits);
    const double *r = resp + (size_t)m * g.max_poses;
    int *ti = tie_idx + (size_t)m * g.max_poses;
    double4 *tv = tie_val + (size_t)m * g.max_poses;
    const double cx = S.center[0], cy = S.center[1], ch = S.center[2];
    const double startX = -g.coff;
    const double astart = ch - g.aoff[pass];
    if (tid == 0) {
        s_n = 0;
        s_err = 0;
    }
    __syncthreads();
    // Poses with DoubleEqual(response, best), in the reference's pose order i = pos * nA + a, and the
    // per-position maximum over the angles (the search-space probability grid, posmax).  kt_coarse_kernel
    // stores the responses angle-major, so thread tid takes position base + tid and walks its angles
    // (coalesced across the threads); ordering the ties by thread within a round keeps pose order.
    const int npos = nxy * nxy;
    unsigned long long *pmw = posmax + (size_t)m * npos;
    for (int base = 0; base < npos; base += KT_SEL_THREADS) {
        const int pos = base + tid;
        int c = 0;
        double mx = 0.0;
        if (pos < npos)
            for (int a0 = 0; a0 < nA; a0 += 8) {  // 8 independent loads in flight per thread
                double v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = a0 + j < nA ? r[(size_t)(a0 + j) * npos + pos] : 0.0;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (a0 + j < nA) {
                        mx = kt_max(mx, v[j]);
                        c += kt_deq(v[j], best) ? 1 : 0;
                    }
            }
        if (pos < npos) pmw[pos] = kt_bits(mx);
        int tot;
        int pre = kt_block_exscan_n<KT_SEL_THREADS / 64>(c, sw, &tot);
        const int n0 = s_n;
        if (c)
            for (int a = 0; a < nA; ++a)
                if (kt_deq(r[(size_t)a * npos + pos], best)) ti[n0 + pre++] = pos * nA + a;
        __syncthreads();
        if (tid == 0) s_n = n0 + tot;
        __syncthreads();
    }
    const int nt = s_n;
    for (int t = tid; t < nt; t += KT_SEL_THREADS) {
        const int i = ti[t];
        const int a = i % nA, pos = i / nA;
        const int ix = pos % nxy, iy = pos / nxy;
        const double x = cx + (startX + (double)(uint32_t)ix * g.cres);
        const double y = cy + (startX + (double)(uint32_t)iy * g.cres);
        const double h = kt_norm_angle(astart + (double)(uint32_t)a * g.cares);
        tv[t] = make_double4(x, y, sdm_cos(h), sdm_sin(h));
    }
    __syncthreads();
    if (tid == 0) {
        double ax = 0.0, ay = 0.0, tx = 0.0, ty = 0.0;
        for (int t = 0; t < nt; ++t) {
            const double4 v = tv[t];
            ax += v.x;
            ay += v.y;
            tx += v.z;
            ty += v.w;
        }
        if (nt > 0) {
            ax /= nt;
            ay /= nt;
            tx /= nt;
            ty /= nt;
            s_mean[0] = ax;
            s_mean[1] = ay;
            s_mean[2] = sdm_atan2(ty, tx);
        } else {
            s_mean[0] = s_mean[1] = s_mean[2] = 0.0;
            s_err = 1;
        }
    }
    __syncthreads();
    // ComputePositionalCovariance over the search-space probability grid
    double cov[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double pgox = cx - g.coff, pgoy = cy - g.coff;
    if (best < KT_TOL) {
        cov[0] = KT_MAX_VARIANCE;
        cov[4] = KT_MAX_VARIANCE;
        cov[8] = 4 * kt_sq(g.cares);
    } else {
        const unsigned long long *pm = posmax + (size_t)m * nxy * nxy;
        const double lo = best - 0.1;
        __syncthreads();
        if (tid == 0) s_n = 0;
        __syncthreads();
        const int npos = nxy * nxy;
        // probability-grid cell of every coarse column / row (WorldToGrid of the pose positions)
        for (int i = tid; i < nxy; i += KT_SEL_THREADS) {
            const double v = startX + (double)(uint32_t)i * g.cres;
            const int pgx = kt_w2g(cx + v, pgox, g.scale), pgy = kt_w2g(cy + v, pgoy, g.scale);
            s_pcx[i] = pgx;
            s_pcy[i] = pgy;
            if (pgx < 0 || pgx >= g.side || pgy < 0 || pgy >= g.side)
                s_err = 2;  // "Index out of range in probability search" (Mapper.cpp:446)
        }
        __syncthreads();
        for (int base = 0; base < npos; base += KT_SEL_THREADS) {
            const int i = base + tid;
            int f = 0;
            double val = 0.0;
            if (i < npos) {
                const int ix = i % nxy, iy = i / nxy;
                // the probability cell holds the max over every pose that lands in it: this position
                // and any neighbour whose coordinates round to the same cell
                const int px = s_pcx[ix], py = s_pcy[iy];
                const bool xl = ix > 0 && s_pcx[ix - 1] == px, xr = ix + 1 < nxy && s_pcx[ix + 1] == px;
                const bool yl = iy > 0 && s_pcy[iy - 1] == py, yr = iy + 1 < nxy && s_pcy[iy + 1] == py;
                unsigned long long v = pm[i];
                if (xl | xr | yl | yr) {
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            if ((dx < 0 && !xl) || (dx > 0 && !xr) || (dy < 0 && !yl) || (dy > 0 && !yr)) continue;
                            v = max(v, pm[(iy + dy) * nxy + ix + dx]);
                        }
                }
                val = kt_dbl(v);
                f = val >= lo ? 1 : 0;
            }
            int tot;
            const int pre = kt_block_exscan_n<KT_SEL_THREADS / 64>(f, sw, &tot);
            const int n0 = s_n;
            if (f) {
                const int ix = i % nxy, iy = i / nxy;
                tv[n0 + pre] = make_double4(startX + (double)(uint32_t)ix * g.cres,
                                            startX + (double)(uint32_t)iy * g.cres, val, 0.0);
            }
            __syncthreads();
            if (tid == 0) s_n = n0 + tot;
            __syncthreads();
        }
        if (tid == 0) {
            const int nc = s_n;
            double axx = 0, axy = 0, ayy = 0, norm = 0;
            const double dx = s_mean[0] - cx, dy = s_mean[1] - cy;
            for (int t = 0; t < nc; ++t) {
                const double4 v = tv[t];
                const double x = v.x, y = v.y, response = v.z;
                norm += response;
                axx += (kt_sq(x - dx) * response);
                axy += ((x - dx) * (y - dy) * response);
                ayy += (kt_sq(y - dy) * response);
            }
            if (norm > KT_TOL) {
                double vxx = axx / norm, vxy = axy / norm, vyy = ayy / norm;
                const double vtt = 4 * kt_sq(g.cares);
                const double minxx = 0.1 * kt_sq(g.cres), minyy = 0.1 * kt_sq(g.cres);
                vxx = kt_max(vxx, minxx);
                vyy = kt_max(vyy, minyy);
                const double mult = 1.0 / best;
                cov[0] = vxx * mult;
                cov[1] = vxy * mult;
                cov[3] = vxy * mult;
                cov[4] = vyy * mult;
                cov[8] = vtt;
            }
            if (kt_deq(cov[0], 0.0)) cov[0] = KT_MAX_VARIANCE;
            if (kt_deq(cov[4], 0.0)) cov[4] = KT_MAX_VARIANCE;
        }
    }
    if (tid == 0) {
        const double clamped = best > 1.0 ? 1.0 : best;
        for (int i = 0; i < 3; ++i) S.mean[i] = s_mean[i];
        for (int i = 0; i < 9; ++i) S.cov[i] = cov[i];
        S.best = clamped;
        if (s_err) S.status = KT_ERANGE;
        if (g.use_expansion && pass + 1 < g.npass && kt_deq(clamped, 0.0)) {
            S.pass = pass + 1;  // MatchScan: widen the angular window by 20 degrees and retry
            S.best_bits = 0ull;
        } else {
            S.pass = -1;
            if (!refine) {
                kt_result &o = out[m];
                for (int i = 0; i < 3; ++i) o.mean[i] = s_mean[i];
                for (int i = 0; i < 9; ++i) o.covariance[i] = cov[i];
                o.response = clamped;
                o.status = S.status;
                o.pad_ = 0;
            }
        }
    }
    __syncthreads();
    if (S.pass == pass + 1) {
        unsigned long long *pm = posmax + (size_t)m * nxy * nxy;
        for (int i = tid; i < nxy * nxy; i += KT_SEL_THREADS) pm[i] = 0ull;
    }
}

// =================================================================================================
// kt_fine_kernel: fine CorrelateScan + ComputeAngularCovariance, one workgroup per match
//
// Each thread holds its points (k = tid + u * KT_THREADS, up to KT_FINE_PPT) in registers for every
// angle, the angles' sin / cos are computed once into LDS, and every angle's counts go to LDS by one
// atomic add per wave (integer sums, order-free): no barrier between angles, and four points' offsets
// and gathers (36 bytes) in flight per lane instead of one point's.
// =================================================================================================
constexpr int KT_FINE_THREADS = KT_THREADS;  // 1024 threads (4 waves per SIMD) measured slower
constexpr int KT_FINE_PPT = 16;              // points per thread held in registers: n <= 4096 = 16 * 256
__device__ __forceinline__ int kt_offset(const KtGeom &g, double cs, double sn, double2 l, double gox, double goy)
{
    const double ox = cs * l.x - sn * l.y;
    const double oy = sn * l.x + cs * l.y;
    return kt_w2g(ox + gox, gox, g.scale) + kt_w2g(oy + goy, goy, g.scale) * g.ws;
}

__global__ void __launch_bounds__(KT_FINE_THREADS)
kt_fine_kernel(KtGeom g, KtPool P, KtState *st, const unsigned char *__restrict__ grids, int penalize,
               kt_result *out)
{
    __shared__ unsigned scnt[KT_FINE_MAX_ANG][9];
    __shared__ unsigned scov[KT_FINE_MAX_ANG];
    __shared__ double s_cs[KT_FINE_MAX_ANG][2];
    __shared__ double sresp[KT_FINE_MAX_ANG * 9];
    __shared__ double s_mean[3];
    __shared__ double s_best;
    __shared__ int s_gi;
    const int m = blockIdx.x;
    KtState &S = st[m];
    const int tid = threadIdx.x, lane = tid & 63;
    const double cx = S.mean[0], cy = S.mean[1], ch = S.mean[2];  // rSearchCenter = coarse rMean
    const double gox = S.gox, goy = S.goy;
    const int q = S.query, npts = S.npts;
    const double2 *loc = P.loc + (size_t)q * g.n;
    const unsigned char *bad = P.bad + (size_t)q * g.n;
    const unsigned char *grid = grids + (size_t)m * g.grid_stride;
    const unsigned ds = (unsigned)g.data_size;
    const int nA = g.fnang;
    const double startX = -g.foff;
    const double astart = ch - g.faoff;
    int err = 0;
    int gpos[9];
#pragma unroll
    for (int p = 0; p < 9; ++p) {
        const int ix = p % 3, iy = p / 3;
        const double x = startX + (double)(uint32_t)ix * g.res;
        const double y = startX + (double)(uint32_t)iy * g.res;
        const int gx = kt_w2g(cx + x, gox, g.scale) + g.border, gy = kt_w2g(cy + y, goy, g.scale) + g.border;
        if (gx < 0 || gx >= g.width || gy < 0 || gy >= g.height) err = 1;
        gpos[p] = gx + gy * g.ws;
    }
    for (int i = tid; i < nA * 9; i += KT_FINE_THREADS) scnt[i / 9][i % 9] = 0u;
    for (int a = tid; a < nA; a += KT_FINE_THREADS) {
        const double angle = astart + (double)(uint32_t)a * g.fares;
        s_cs[a][0] = sdm_cos(angle);
        s_cs[a][1] = sdm_sin(angle);
        scov[a] = 0u;
    }
    double2 lp[KT_FINE_PPT];
    bool ok[KT_FINE_PPT];
#pragma unroll
    for (int u = 0; u < KT_FINE_PPT; ++u) {
        const int k = tid + u * KT_FINE_THREADS;
        ok[u] = k < npts && !bad[k];
        lp[u] = ok[u] ? loc[k] : make_double2(0.0, 0.0);
    }
    __syncthreads();
    for (int a = 0; a < nA; ++a) {
        const double cs = s_cs[a][0], sn = s_cs[a][1];
        unsigned c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int u0 = 0; u0 < KT_FINE_PPT; u0 += 4) {
            if (u0 * KT_FINE_THREADS >= npts) break;  // block-uniform
            int o[4];
            unsigned char v[4][9];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                o[u] = kt_offset(g, cs, sn, lp[u0 + u], gox, goy);
                // branch-free: out-of-range cells read cell 0 and count 0, so all gathers are in flight
#pragma unroll
                for (int p = 0; p < 9; ++p) {
                    const int idx = gpos[p] + o[u];
                    v[u][p] = grid[(unsigned)idx < ds ? idx : 0];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int p = 0; p < 9; ++p) {
                    const int idx = gpos[p] + o[u];
                    c[p] += (ok[u0 + u] && (unsigned)idx < ds) ? v[u][p] : 0u;
                }
        }
#pragma unroll
        for (int p = 0; p < 9; ++p) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) c[p] += __shfl_xor(c[p], off, 64);
            if (lane == 0) atomicAdd(&scnt[a][p], c[p]);
        }
    }
    __syncthreads();
    // responses in pose order (y, x, angle)
    const int np = 9 * nA;
    for (int i = tid; i < np; i += KT_FINE_THREADS) {
        const int a = i % nA, p = i / nA;
        double response = 0.0;
        if (npts > 0) response = (double)scnt[a][p] / (double)(uint32_t)(npts * KT_OCC);
        if (penalize && !kt_deq(response, 0.0)) {
            const double x = startX + (double)(uint32_t)(p % 3) * g.res;
            const double y = startX + (double)(uint32_t)(p / 3) * g.res;
            const double sqd = kt_sq(x) + kt_sq(y);
            double dp = 1.0 - (KT_GAIN * sqd / g.dvp);
            dp = kt_max(dp, g.mdp);
            const double angle = astart + (double)(uint32_t)a * g.fares;
            const double sqa = kt_sq(angle - ch);
            double ap = 1.0 - (KT_GAIN * sqa / g.avp);
            ap = kt_max(ap, g.map_);
            response *= (dp * ap);
        }
        sresp[i] = response;
    }
    __syncthreads();
    if (tid == 0) {
        double best = -1;
        for (int i = 0; i < np; ++i) best = kt_max(best, sresp[i]);
        double ax = 0.0, ay = 0.0, tx = 0.0, ty = 0.0;
        int nt = 0;
        for (int i = 0; i < np; ++i) {
            if (!kt_deq(sresp[i], best)) continue;
            const int a = i % nA, p = i / nA;
            ax += cx + (startX + (double)(uint32_t)(p % 3) * g.res);
            ay += cy + (startX + (double)(uint32_t)(p / 3) * g.res);
            const double h = kt_norm_angle(astart + (double)(uint32_t)a * g.fares);
            tx += sdm_cos(h);
            ty += sdm_sin(h);
            ++nt;
        }
        ax /= nt;
        ay /= nt;
        tx /= nt;
        ty /= nt;
        s_mean[0] = ax;
        s_mean[1] = ay;
        s_mean[2] = sdm_atan2(ty, tx);
        s_best = best;
        const int gx = kt_w2g(ax, gox, g.scale) + g.border, gy = kt_w2g(ay, goy, g.scale) + g.border;
        if (gx < 0 || gx >= g.width || gy < 0 || gy >= g.height) {
            err = 1;
            s_gi = 0;
        } else {
            s_gi = gx + gy * g.ws;
        }
    }
    __syncthreads();
    // ComputeAngularCovariance: GetResponse at the best pose for every fine angle
    const int gi = s_gi;
    for (int a = 0; a < nA; ++a) {
        const double cs = s_cs[a][0], sn = s_cs[a][1];
        unsigned c = 0;
#pragma unroll
        for (int u0 = 0; u0 < KT_FINE_PPT; u0 += 4) {
            if (u0 * KT_FINE_THREADS >= npts) break;  // block-uniform
            int idx[4];
            unsigned char v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                idx[u] = gi + kt_offset(g, cs, sn, lp[u0 + u], gox, goy);
                v[u] = grid[(unsigned)idx[u] < ds ? idx[u] : 0];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) c += (ok[u0 + u] && (unsigned)idx[u] < ds) ? v[u] : 0u;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
        if (lane == 0) atomicAdd(&scov[a], c);
    }
    if (err) S.status = KT_ERANGE;
    __syncthreads();
    if (tid == 0) {
        const double best = s_best;
        const double best_angle = kt_norm_angle_diff(s_mean[2], ch);
        double norm = 0.0, acc = 0.0;
        for (int a = 0; a < nA; ++a) {
            const double angle = astart + (double)(uint32_t)a * g.fares;
            const double response = npts > 0 ? (double)scov[a] / (double)(uint32_t)(npts * KT_OCC) : 0.0;
            if (response >= (best - 0.1)) {
                norm += response;
                acc += (kt_sq(angle - best_angle) * response);
            }
        }
        if (norm > KT_TOL) {
            if (acc < KT_TOL) acc = kt_sq(g.fares);
            acc /= norm;
        } else {
            acc = 1000 * kt_sq(g.fares);
        }
        kt_result &o = out[m];
        for (int i = 0; i < 3; ++i) o.mean[i] = s_mean[i];
        for (int i = 0; i < 9; ++i) o.covariance[i] = S.cov[i];
        o.covariance[8] = acc;
        o.response = best > 1.0 ? 1.0 : best;
        o.status = S.status;
        o.pad_ = 0;
    }
}

}  // namespace s2d
