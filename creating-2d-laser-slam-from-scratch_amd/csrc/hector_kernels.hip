// hector_kernels.hip -- MI355X (gfx950) kernels for the Hector scan-to-map matcher and the
// once-per-scan Bresenham log-odds grid update (reference: lesson4/include/lesson4/hector_mapping/,
// abbreviated H/ below).  Host orchestration + C-ABI live in hector_capi.hip.
//
// Data layout in HBM (per context):
//   cells  : LogOddsCell {float l; int upd} (H/map/GridMapLogOdds.h:37-87) stored tiled: per stream,
//            per level, 64 x 32-cell tiles of 20 KB each = [2048 log-odds floats][2048 16-bit update
//            ordinals][2048 updateIndex ints] (hector_internal.h cell_word, ORD_OFF, COLD_OFF: the grid update
//            writes the ordinals, a periodic sweep the ints); the tile is the grid update's unit of work.
//   state  : StreamState per stream (pose, last map-update pose, covariance, update indices).
//   points : float2 per beam in level-0 map scale, padded to xy_stride per stream.
//
// One step = one HectorSlamProcessor::update per stream (H/slam_main/HectorSlamProcessor.h:81-108):
//   k1 hs_match_kernel      one 256-thread workgroup per stream: all levels coarse->fine, all
//                           Gauss-Newton iterations, block reduction of H/b, 3x3 solve, gating.
//   k2 hs_update_kernel     256-thread workgroups per (stream, level, part): the tiles of the scan's
//                           bounding box (64 x 32 cells, the storage tile) are dealt round-robin to
//                           the level's parts (split by the number of updating streams, upd_split);
//                           each ray's cells inside a tile come from the closed-form Bresenham step
//                           range, the once-per-scan semantics of bresenhamCellFree/Occ
//                           (H/map/OccGridMapBase.h:302-330) are resolved in LDS event words, then
//                           every marked cell's log-odds is read once and written once with its
//                           16-bit update ordinal (neither index plane is read).  No global atomics;
//                           see DESIGN.md.
// Wrong-result pricing builds (no atomics, no walk, no apply, hardware exp) are not in this file:
// tools/build_diag.py derives them from a copy of the sources.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "detmath.h"
#include "hector_internal.h"

namespace s2d {

// ---------------------------------------------------------------------------------------- helpers
__device__ __forceinline__ void map_from_world(const LevelGeom &g, const float *w, float *m)
{
    // GridMapBase::getMapCoordsPose  H/map/GridMapBase.h:238-242  (Affine2f * Vector2f)
    m[0] = g.map_t[0] + (g.scale * w[0] + 0.0f * w[1]);
    m[1] = g.map_t[1] + (0.0f * w[0] + g.scale * w[1]);
    m[2] = w[2];
}

__device__ __forceinline__ void world_from_map(const LevelGeom &g, const float *m, float *w)
{
    // GridMapBase::getWorldCoordsPose  H/map/GridMapBase.h:229-233
    w[0] = g.inv_t[0] + (g.inv_l[0] * m[0] + g.inv_l[1] * m[1]);
    w[1] = g.inv_t[1] + (g.inv_l[2] * m[0] + g.inv_l[3] * m[1]);
    w[2] = m[2];
}

__device__ __forceinline__ float normalize_angle(float angle)
{
    // util::normalize_angle  H/util/UtilFunctions.h:36-48 (evaluated in double)
    const double two_pi = 2.0f * S2D_PI;
    float a = (float)fmod(fmod((double)angle, two_pi) + two_pi, two_pi);
    if ((double)a > S2D_PI) a = (float)((double)a - two_pi);
    return a;
}

__device__ __forceinline__ bool pose_diff_larger(const float *p1, const float *p2, float dist, float ang)
{
    // util::poseDifferenceLargerThan  H/util/UtilFunctions.h:72-91
    float dx = p1[0] - p2[0];
    float dy = p1[1] - p2[1];
    float n = __fsqrt_rn(dx * dx + dy * dy);
    if (n > dist) return true;
    float ad = p1[2] - p2[2];
    if ((double)ad > S2D_PI) ad = (float)((double)ad - S2D_PI * 2.0f);
    else if ((double)ad < -S2D_PI) ad = (float)((double)ad + S2D_PI * 2.0f);
    return fabsf(ad) > ang;
}

// Clock probe (hs_set_clock_probe): every CLK_SAMPLE-th workgroup subtracts its entry stamps and adds
// its exit stamps -- s_memtime (shader cycles) and s_memrealtime (100-MHz constant ticks) -- so clk[4k]
// / clk[4k + 1] x 100 MHz is the effective shader clock over the sampled lifetimes of kernel k
// (MI355X_MICROARCH.md, in-kernel clock).  The stamps go straight to memory (vector atomics), so no
// register is held across the kernel; with the probe off it is one uniform branch at entry and exit.
__device__ __forceinline__ void clk_stamp(unsigned long long *clk, int kernel, bool entry)
{
    if (clk == nullptr || (blockIdx.x % CLK_SAMPLE) != 0 || threadIdx.x != 0) return;
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the stamps are back before any LDS wait is counted
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long *k = clk + 4 * kernel;
    if (entry) {
        atomicAdd(k, 0ull - c);
        atomicAdd(k + 1, 0ull - r);
    } else {
        atomicAdd(k, c);
        atomicAdd(k + 1, r);
        atomicAdd(k + 2, 1ull);
    }
}

// exp's 2^(j/128) table (detmath.h): read once per workgroup into LDS by the kernels that call
// cell_prob (hs_match_kernel, load_exptab), so the per-lane table reads are LDS reads
__constant__ double c_exptab[SDM_EXPTAB_N] = {SDM_EXPTAB_VALUES};
__shared__ double s_exptab[SDM_EXPTAB_N];
__device__ __forceinline__ void load_exptab()  // all threads; a barrier must follow before cell_prob
{
    for (int k = threadIdx.x; k < SDM_EXPTAB_N; k += blockDim.x) s_exptab[k] = c_exptab[k];
}

// GridMapLogOddsFunctions::getGridProbability  H/map/GridMapLogOdds.h:136-140
__device__ __forceinline__ float cell_prob(float l)
{
    float odds = sdm_expf_tab(l, s_exptab);
    return __fdiv_rn(odds, odds + 1.0f);
}

// Matrix3f::inverse() * dTr  (ScanMatcher.h:120; Eigen 3.3 cofactor inverse, halving redux)
__device__ __forceinline__ void solve3(const float *m, const float *b, float *d)
{
#define M(i, j) m[(i)*3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    float c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    float det = c00 * M(0, 0) + (c10 * M(1, 0) + c20 * M(2, 0));
    float invdet = __fdiv_rn(1.0f, det);
    float inv[9];
    inv[0] = c00 * invdet;
    inv[1] = c10 * invdet;
    inv[2] = c20 * invdet;
    inv[3] = COF(0, 1) * invdet;
    inv[4] = COF(1, 1) * invdet;
    inv[5] = COF(2, 1) * invdet;
    inv[6] = COF(0, 2) * invdet;
    inv[7] = COF(1, 2) * invdet;
    inv[8] = COF(2, 2) * invdet;
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = inv[i * 3] * b[0] + (inv[i * 3 + 1] * b[1] + inv[i * 3 + 2] * b[2]);
#undef COF
#undef M
}

// ---- scan ingest ---------------------------------------------------------------------------------
// HectorMappingRos::scanCallback (hector_slam.cc:186-198) for a batch of range arrays, one 256-thread
// workgroup per stream: laser_geometry's projectLaser(scan, cloud, 30.0) (double products of the
// cached unit vectors, rounded to the float Point32) and rosPointCloudToDataContainer (:320-362)
// statement by statement, then an order-preserving compaction (wave ballots + a per-chunk prefix over
// the 4 waves), so point k of the DataContainer is the k-th surviving beam as in the node's loop.
// hs_ingest_kernel runs it alone; hs_match_kernel runs it as its prologue when handed a MatchIngest
// (hs_run_ranges_device: one launch less per step, the points go straight into the match registers).
struct IngestGeom {
    double cutoff, use_max_sq;
    double tf[12];  // basis rows, origin
    float range_min, sqr_min, sqr_max, z_min, z_max, scale;
    float2 origo;
    int n;
};

struct MatchIngest {       // the fused ingest's buffers (ranges == nullptr: points come from xy / counts)
    const float *ranges;   // [stream][rstride] range arrays
    int rstride;
    const double2 *cs;     // unit vectors
    float2 *xy_out;        // DataContainer points, written for the grid update ([stream][xy_stride])
    int *n_out;            // point count per stream
    float2 *origo_out;     // DataContainer origo per stream
};

// one beam of projectLaser + rosPointCloudToDataContainer: true if it becomes a DataContainer point
__device__ __forceinline__ bool ingest_beam(const IngestGeom &ig, double2 u, float range, float2 &p)  // u = cs[beam]
{
    bool keep = false;
    if (((double)range < ig.cutoff) && (range >= ig.range_min)) {  // projectLaser_
        const float x = (float)((double)range * u.x);
        const float y = (float)((double)range * u.y);
        const float z = 0.0f;
        const float d2 = __fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y));          // :334
        keep = (d2 > ig.sqr_min) && (d2 < ig.sqr_max);                          // :336
        if ((x < 0.0f) && (d2 < 0.50f)) keep = false;                           // :338-341
        if ((double)d2 > ig.use_max_sq) keep = false;                           // :344-345
        if (keep) {
            const double vx = (double)x, vy = (double)y, vz = (double)z;        // :348 tf dot products
            const double px = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(ig.tf[0], vx), __dmul_rn(ig.tf[1], vy)),
                                                  __dmul_rn(ig.tf[2], vz)), ig.tf[9]);
            const double py = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(ig.tf[3], vx), __dmul_rn(ig.tf[4], vy)),
                                                  __dmul_rn(ig.tf[5], vz)), ig.tf[10]);
            const double pz = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(ig.tf[6], vx), __dmul_rn(ig.tf[7], vy)),
                                                  __dmul_rn(ig.tf[8], vz)), ig.tf[11]);
            const float zl = (float)(pz - ig.tf[11]);                            // :351
            keep = zl > ig.z_min && zl < ig.z_max;                               // :353
            p = make_float2(__fmul_rn((float)px, ig.scale), __fmul_rn((float)py, ig.scale));  // :356
        }
    }
    return keep;
}

// the whole scan of one stream by a 256-thread workgroup: surviving points in beam order to out (and to
// stage, an LDS copy, when given); returns the count (uniform).  s_w: ING_SW ints of LDS.
// Scans of up to ING_CHUNKS x 256 beams: every range and unit vector is loaded up front (one memory latency
// instead of one per 256-beam chunk) and the compaction takes ONE barrier (each wave's count per chunk, then
// every thread's offset = the counts of the earlier chunks and of the lower waves of its own); longer scans
// take the chunk loop (two barriers per chunk).
constexpr int ING_CHUNKS = 5;  // 1280 beams
#ifndef S2D_ING_PRELOAD
#define S2D_ING_PRELOAD 1  // 0: the chunk loop for every scan (A/B)
#endif
constexpr int ING_SW = 4 * ING_CHUNKS;
__device__ __forceinline__ int ingest_scan(const IngestGeom &ig, const double2 *__restrict__ cs,
                                           const float *__restrict__ r, float2 *__restrict__ out, float2 *stage,
                                           int *s_w)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (S2D_ING_PRELOAD && ig.n <= 256 * ING_CHUNKS) {
        float rr[ING_CHUNKS];
        double2 uu[ING_CHUNKS];
#pragma unroll
        for (int c = 0; c < ING_CHUNKS; ++c) {
            const int i = c * 256 + tid;
            rr[c] = 0.0f;
            uu[c] = make_double2(0.0, 0.0);
            if (i < ig.n) {
                rr[c] = r[i];
                uu[c] = cs[i];
            }
        }
        float2 pp[ING_CHUNKS];
        unsigned keepm = 0u;  // bit c: this thread's beam of chunk c survives
#pragma unroll
        for (int c = 0; c < ING_CHUNKS; ++c) {
            pp[c] = make_float2(0.0f, 0.0f);
            const bool keep = c * 256 + tid < ig.n && ingest_beam(ig, uu[c], rr[c], pp[c]);
            const unsigned long long m = __ballot(keep);
            if (lane == 0) s_w[c * 4 + wv] = __popcll(m);
            keepm |= keep ? 1u << c : 0u;
        }
        __syncthreads();
        int base = 0;
#pragma unroll
        for (int c = 0; c < ING_CHUNKS; ++c) {
            const int c0 = s_w[c * 4], c1 = s_w[c * 4 + 1], c2 = s_w[c * 4 + 2], c3 = s_w[c * 4 + 3];
            const unsigned long long m = __ballot((keepm >> c) & 1u);
            if ((keepm >> c) & 1u) {
                const int off = base + (wv > 0 ? c0 : 0) + (wv > 1 ? c1 : 0) + (wv > 2 ? c2 : 0);
                const int k = off + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                out[k] = pp[c];
                if (stage) stage[k] = pp[c];
            }
            base += c0 + c1 + c2 + c3;
        }
        __syncthreads();  // s_w read by every thread before a caller reuses it
        return base;
    }
    int base = 0;
    for (int b0 = 0; b0 < ig.n; b0 += 256) {
        const int i = b0 + tid;
        float2 p = make_float2(0.0f, 0.0f);
        const bool keep = i < ig.n && ingest_beam(ig, cs[i], r[i], p);
        const unsigned long long m = __ballot(keep);
        if (lane == 0) s_w[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int k = 0; k < wv; ++k) off += s_w[k];
        if (keep) {
            const int k = off + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            out[k] = p;
            if (stage) stage[k] = p;
        }
        base += s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
    }
    return base;
}

__global__ void __launch_bounds__(256)
hs_ingest_kernel(IngestGeom ig, const double2 *__restrict__ cs, const float *__restrict__ ranges, int rstride,
                 float2 *__restrict__ xy, int xy_stride, int *__restrict__ n_out, float2 *__restrict__ origo_out)
{
    __shared__ int s_w[ING_SW];
    const int s = blockIdx.x;
    const int n = ingest_scan(ig, cs, ranges + (size_t)s * rstride, xy + (size_t)s * xy_stride, nullptr, s_w);
    if (threadIdx.x == 0) {
        n_out[s] = n;
        if (origo_out) origo_out[s] = ig.origo;
    }
}

// --------------------------------------------------------------------------------- k1: match
// Per point: OccGridMapUtil::getCompleteHessianDerivs body (H/map/OccGridMapUtil.h:94-126) with
// interpMapValueWithDerivatives (:139-228), split in two phases so that a thread's gathers for a
// batch of points are all in flight before the first one is consumed:
//   point_fetch: transform, bounds test, the 4 neighbour log-odds (raw);
//   point_accum: probabilities, bilinear value + corrected gradients, accumulate into acc[9] =
//                {dTr0, dTr1, dTr2, H00, H11, H22, H01, H02, H12}.
struct PointFetch {
    float px, py, fx, fy;
    float l[4];
    bool in;
};

__device__ __forceinline__ void point_fetch(const float *__restrict__ lvl_words, const LevelGeom &g, float tx,
                                            float ty, float cs, float sn, float px, float py, PointFetch &pf)
{
    float nsn = -sn;
    float x = tx + (cs * px + nsn * py);
    float y = ty + (sn * px + cs * py);
    pf.px = px;
    pf.py = py;
    pf.in = (x >= 0.0f) && (x <= g.lim[0]) && (y >= 0.0f) && (y <= g.lim[1]);  // NaN -> out of map
    if (pf.in) {
        int ix = (int)x, iy = (int)y;
        pf.fx = x - (float)ix;
        pf.fy = y - (float)iy;
        // 4 neighbours (:160-192); ix <= sx-2, iy <= sy-2 by the bounds check
        const unsigned ux = (unsigned)ix, uy = (unsigned)iy;  // >= 0 by the bounds check
        const float *r0 = lvl_words + cell_word(g, (int)ux, (int)uy);
        const float *r1 = lvl_words + cell_word(g, (int)ux, (int)(uy + 1));
        if ((ux & (CELL_BLK - 1)) != CELL_BLK - 1) {
            // (ix, ix + 1) are adjacent words of one block row: one 8-byte (4-byte aligned) gather per row
            float2 a, b;
            __builtin_memcpy(&a, r0, 8);
            __builtin_memcpy(&b, r1, 8);
            pf.l[0] = a.x; pf.l[1] = a.y; pf.l[2] = b.x; pf.l[3] = b.y;
        } else {
            pf.l[0] = r0[0];
            pf.l[1] = lvl_words[cell_word(g, (int)(ux + 1), (int)uy)];
            pf.l[2] = r1[0];
            pf.l[3] = lvl_words[cell_word(g, (int)(ux + 1), (int)(uy + 1))];
        }
    }
}

// The 9 per-point terms t = {dTr0, dTr1, dTr2, H00, H11, H22, H01, H02, H12} of one point
// (OccGridMapUtil.h:106-125: the products the reference adds into dTr / H).
// probs: pf.l already holds the 4 probabilities (neighbourhood cache) instead of log-odds
template <bool probs = false>
__device__ __forceinline__ void point_terms(const PointFetch &pf, float cs, float sn, float *t)
{
    float v, gx, gy;
    if (!pf.in) {
        v = 0.0f;
        gx = 0.0f;
        gy = 0.0f;
    } else {
        const float fx = pf.fx, fy = pf.fy;
        float i0 = probs ? pf.l[0] : cell_prob(pf.l[0]);
        float i1 = probs ? pf.l[1] : cell_prob(pf.l[1]);
        float i2 = probs ? pf.l[2] : cell_prob(pf.l[2]);
        float i3 = probs ? pf.l[3] : cell_prob(pf.l[3]);
        float dx1 = i0 - i1;
        float dx2 = i2 - i3;
        float dy1 = i0 - i2;
        float dy2 = i1 - i3;
        float xfi = 1.0f - fx;
        float yfi = 1.0f - fy;
        v = ((i0 * xfi + i1 * fx) * yfi) + ((i2 * xfi + i3 * fx) * fy);
        gx = -((dx1 * yfi) + (dx2 * fy));
        gy = -((dy1 * xfi) + (dy2 * fx));
    }
    const float px = pf.px, py = pf.py;
    float fun = 1.0f - v;
    // sinRot/cosRot (:87-88) are the same values as the transform's sn/cs
    float rot = ((-sn * px - cs * py) * gx + (cs * px - sn * py) * gy);
    t[0] = gx * fun;
    t[1] = gy * fun;
    t[2] = rot * fun;
    t[3] = gx * gx;
    t[4] = gy * gy;
    t[5] = rot * rot;
    t[6] = gx * gy;
    t[7] = gx * rot;
    t[8] = gy * rot;
}

// acc[k] += t[k]: one thread's strided partial sums (the tree order, below)
template <bool probs = false>
__device__ __forceinline__ void point_accum(const PointFetch &pf, float cs, float sn, float *acc)
{
    float t[9];
    point_terms<probs>(pf, cs, sn, t);
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k] = acc[k] + t[k];
}

// ---- the reference's summation order (default) -------------------------------------------------
// getCompleteHessianDerivs adds the points' terms one after the other in point order
// (OccGridMapUtil.h:94-126: dTr[k] += ..., H(i, j) += ... for i = 0 .. size-1, in float).  Float
// addition is not associative, so the only way to get the reference's H / b bit for bit is that same
// chain of adds.  The points are processed in chunks of 256 (point i = chunk * 256 + thread); a chunk's
// 9 x 256 terms go to LDS term-major, and 9 lanes of one wave (lane k = term k) extend the 9 running
// sums over the chunk in point order while the other waves compute the next chunk's terms.
// Rows are SEQ_STRIDE words: 16-B aligned, and row k starts on bank 4k, so the 9 lanes' 16-B reads
// hit distinct banks.
constexpr int SEQ_STRIDE = MATCH_THREADS + 4;
constexpr int SEQ_WORDS = 9 * SEQ_STRIDE;

// run + T[lane][0] + T[lane][1] + ... + T[lane][cnt - 1], left to right.  The adds are one dependent
// chain; the LDS reads of the next 16 terms are issued before the current 16 are added.
#define S2D_ADD4(v) do { run = run + (v).x; run = run + (v).y; run = run + (v).z; run = run + (v).w; } while (0)
template <int STRIDE>
__device__ __forceinline__ float seq_chain_t(const float *T, int lane, int cnt, float run)
{
    const float4 *row = reinterpret_cast<const float4 *>(T + lane * STRIDE);
    const int c4 = cnt >> 2;
    int i = 0;
    if (c4 >= 8) {
        // two register sets of 16 terms, alternating: one set's reads are in flight while the other's
        // adds run
        float4 a0 = row[0], a1 = row[1], a2 = row[2], a3 = row[3];
        float4 b0, b1, b2, b3;
        for (i = 4; i + 7 < c4; i += 8) {
            b0 = row[i]; b1 = row[i + 1]; b2 = row[i + 2]; b3 = row[i + 3];
            __builtin_amdgcn_sched_barrier(0);  // keep the reads above the adds (the scheduler sinks them)
            S2D_ADD4(a0); S2D_ADD4(a1); S2D_ADD4(a2); S2D_ADD4(a3);
            a0 = row[i + 4]; a1 = row[i + 5]; a2 = row[i + 6]; a3 = row[i + 7];
            __builtin_amdgcn_sched_barrier(0);
            S2D_ADD4(b0); S2D_ADD4(b1); S2D_ADD4(b2); S2D_ADD4(b3);
        }
        S2D_ADD4(a0); S2D_ADD4(a1); S2D_ADD4(a2); S2D_ADD4(a3);
    }
    for (; i < c4; ++i) {
        const float4 a = row[i];
        S2D_ADD4(a);
    }
    const float *tail = T + lane * STRIDE + (c4 << 2);
    for (int r = 0; r < (cnt & 3); ++r) run = run + tail[r];
    return run;
}
#undef S2D_ADD4
__device__ __forceinline__ float seq_chain(const float *T, int lane, int cnt, float run)
{
    return seq_chain_t<SEQ_STRIDE>(T, lane, cnt, run);
}

// The wave that runs a workgroup's sequential sums and step tail.  Workgroups co-resident on one CU
// tend to have block ids 256 apart (round-robin dispatch over the CUs), so the block id's bits 8-9 are
// mixed in: their chain waves then sit on different SIMDs instead of sharing one.
__device__ __forceinline__ int chain_wave()
{
    return (int)((blockIdx.x + (blockIdx.x >> 8)) & (MATCH_WAVES - 1));
}

// Workgroup barrier for LDS hand-offs only (waits for this wave's LDS operations, not for its global
// memory operations; see hs_update_kernel)
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One chunk of the sequential sum: store this thread's terms t (if has), hand the chunk to the chain
// wave cw, which extends run (lane k < 9: term k).  first: no earlier chunk of this step is still
// being read (the previous step ended with a workgroup barrier after the chain).
__device__ __forceinline__ void seq_chunk(float *T, const float *t, bool has, bool first, int cnt, int cw, float &run)
{
    const int tid = threadIdx.x, lane = tid & 63;
    if (!first) lds_barrier();  // the chain wave has finished reading the previous chunk
    if (has) {
#pragma unroll
        for (int k = 0; k < 9; ++k) T[k * SEQ_STRIDE + tid] = t[k];
    }
    lds_barrier();
    if ((tid >> 6) == cw) {
        // the chain is the workgroup's critical path (the other waves wait for it at the next barrier):
        // it issues ahead of the co-resident workgroups' waves (s_setprio; back to 0 after the step tail)
        __builtin_amdgcn_s_setprio(3);
        if (lane < 9) run = seq_chain(T, lane, cnt, run);
    }
}

// the 9 sums held by lanes 0..8 of the calling (chain) wave, in every lane of it
__device__ __forceinline__ void seq_gather(float run, float *s)
{
#pragma unroll
    for (int k = 0; k < 9; ++k) s[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(run), k));
}

// The 64-lane xor butterfly of the Hessian terms, offsets 32, 16, 8, 4, 2, 1 (the oracle's
// reduce_threads = 256 order).  Offsets 32 and 16 go through ds_bpermute; after them a lane's value
// equals that of lanes i ^ 16, i ^ 32, so the xor-8 partner is also the lane 8 further round its
// 16-lane row (DPP row_ror:8), after that the xor-4 partner the lane 4 further (row_ror:4), and the
// xor-2 / xor-1 partners are quad permutations.  Every lane adds exactly the value its xor partner
// holds, in the same operand order, so the sums are bit-identical to the __shfl_xor butterfly.
template <int NV>
__device__ __forceinline__ void wave_butterfly(float (&acc)[NV])
{
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = acc[k] + __shfl_xor(acc[k], 32, 64);
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = acc[k] + __shfl_xor(acc[k], 16, 64);
#pragma unroll
    for (int k = 0; k < NV; ++k)
        acc[k] = acc[k] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[k]), 0x128, 0xF, 0xF, false));
#pragma unroll
    for (int k = 0; k < NV; ++k)
        acc[k] = acc[k] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[k]), 0x124, 0xF, 0xF, false));
#pragma unroll
    for (int k = 0; k < NV; ++k)
        acc[k] = acc[k] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[k]), 0x4E, 0xF, 0xF, false));
#pragma unroll
    for (int k = 0; k < NV; ++k)
        acc[k] = acc[k] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[k]), 0xB1, 0xF, 0xF, false));
}

#ifndef S2D_MATCH_BATCH
#define S2D_MATCH_BATCH 2
#endif
constexpr int MATCH_BATCH = S2D_MATCH_BATCH;  // points per thread with gathers in flight together

// One Gauss-Newton step, ScanMatcher::estimateTransformationLogLh (H/matcher/ScanMatcher.h:107-139),
// points read from HBM (scans of more than MATCH_THREADS * MATCH_REG_PTS points).
// Every thread ends with the same H, b and estimate.  SEQ: the reference's sequential sum (seq_chunk);
// else the tree order (xor butterflies, symmetric).
template <bool SEQ>
__device__ __forceinline__ void gn_step(const float *__restrict__ cells, const LevelGeom &g,
                                        const float2 *__restrict__ pts, int n, float f, float *est, float *H,
                                        float (*red)[MATCH_WAVES][9], int parity, int *clamps, float *seqT)
{
    const int tid = threadIdx.x;
    const float cs = sdm_cosf(est[2]);
    const float sn = sdm_sinf(est[2]);
    float s[9];
    if constexpr (SEQ) {
        const int cw = chain_wave();
        float run = 0.0f;
        for (int c0 = 0; c0 < n; c0 += MATCH_THREADS) {
            const int i = c0 + tid;
            float t[9];
            if (i < n) {
                PointFetch pf;
                const float2 p = pts[i];
                point_fetch(cells, g, est[0], est[1], cs, sn, p.x * f, p.y * f, pf);
                point_terms(pf, cs, sn, t);
            }
            seq_chunk(seqT, t, i < n, c0 == 0, min(MATCH_THREADS, n - c0), cw, run);
        }
        if ((tid >> 6) == cw && (tid & 63) < 9) red[parity][0][tid & 63] = run;
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 9; ++k) s[k] = red[parity][0][k];
    } else {
        float acc[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] = 0.0f;
        // per-thread order of the points is i = tid, tid + 256, ... (the oracle's reduce_threads order)
        for (int i0 = tid; i0 < n; i0 += MATCH_THREADS * MATCH_BATCH) {
            PointFetch pf[MATCH_BATCH];
#pragma unroll
            for (int j = 0; j < MATCH_BATCH; ++j) {
                const int i = i0 + j * MATCH_THREADS;
                if (i < n) {
                    const float2 p = pts[i];
                    point_fetch(cells, g, est[0], est[1], cs, sn, p.x * f, p.y * f, pf[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < MATCH_BATCH; ++j)
                if (i0 + j * MATCH_THREADS < n) point_accum(pf[j], cs, sn, acc);
        }
        wave_butterfly(acc);  // 64-lane xor butterfly, offsets 32..1
        const int wave = tid >> 6;
        if ((tid & 63) == 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) red[parity][wave][k] = acc[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            // xor butterfly over the 4 wave sums: off 2 then off 1
            float a0 = red[parity][0][k] + red[parity][2][k];
            float a1 = red[parity][1][k] + red[parity][3][k];
            s[k] = a0 + a1;
        }
    }
    float b[3] = {s[0], s[1], s[2]};
    H[0] = s[3]; H[4] = s[4]; H[8] = s[5];
    H[1] = s[6]; H[2] = s[7]; H[5] = s[8];
    H[3] = H[1]; H[6] = H[2]; H[7] = H[5];
    if ((H[0] != 0.0f) && (H[4] != 0.0f)) {
        float d[3];
        solve3(H, b, d);
        if (d[2] > 0.2f) {
            d[2] = 0.2f;
            (*clamps)++;
        } else if (d[2] < -0.2f) {
            d[2] = -0.2f;
            (*clamps)++;
        }
        est[0] = est[0] + d[0];
        est[1] = est[1] + d[1];
        est[2] = est[2] + d[2];
    }
}

// gn_step with the thread's points resident in registers (n <= MATCH_THREADS * NP): every gather of
// the step is issued before the first is consumed -- one memory round trip per Gauss-Newton step.
// Accumulation order per thread is i = tid, tid + 256, ... as in gn_step.
// Neighbourhood cache: the 4 cell probabilities a point computed last time (GridMapCacheArray's role,
// GridMapCacheArray.h:48-171), keyed by its cell (iy << 16 | ix), in thread-private LDS slots.  The map
// is constant during the match, so a point whose cell did not change since the previous Gauss-Newton
// step (most of them once the pose converges) reuses the values bit for bit and skips the gathers, the
// 4 exp and the 4 divisions; only waves with a moved point pay a gather round.  Keys reset per level.
constexpr unsigned NB_NONE = 0xFFFFFFFFu;

// Misses are compacted per wave: a lane that gathered a moved point's 4 log-odds parks them in the
// point's cache slot and appends the slot to its wave's list; the wave then converts the listed slots
// 64 at a time (4 exp + 4 divisions each) -- with per-slot branches the whole wave would pay the
// conversion of slot j whenever ANY of its 64 lanes missed there, i.e. on nearly every step.
// The step's uniform tail -- H / b from the wave sums, the 3x3 solve, the clamp, the new estimate and
// the sin / cos (in double) of its angle for the next step -- runs on ONE wave of the workgroup (wave
// blockIdx.x % 4, so the four SIMDs share the duty across workgroups) and is broadcast through LDS
// (s_pose[parity]: est[3], cos, sin, H[9], clamp flag); the other waves would only repeat it.
constexpr int POSE_WORDS = 16;

template <int NP, bool SEQ>
__device__ __forceinline__ void gn_step_reg(const float *__restrict__ cells, const LevelGeom &g, const float2 (&p)[NP],
                                            int n, float f, float *est, float &cs, float &sn, float *H,
                                            float (*red)[MATCH_WAVES][9], int parity, unsigned *nb_key,
                                            float4 *nb_val, unsigned short *mlist, float (*s_pose)[POSE_WORDS],
                                            float *seqT)
{
    const int tid = threadIdx.x;
    PointFetch pf[NP];
    unsigned key[NP];
    bool miss[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int slot = tid + j * MATCH_THREADS;
        miss[j] = false;
        key[j] = NB_NONE;
        if (slot < n) {
            // transform + bounds (point_fetch without the gathers)
            const float px = p[j].x * f, py = p[j].y * f;
            const float nsn = -sn;
            const float x = est[0] + (cs * px + nsn * py);
            const float y = est[1] + (sn * px + cs * py);
            pf[j].px = px;
            pf[j].py = py;
            pf[j].in = (x >= 0.0f) && (x <= g.lim[0]) && (y >= 0.0f) && (y <= g.lim[1]);  // NaN -> out of map
            if (pf[j].in) {
                const int ix = (int)x, iy = (int)y;
                pf[j].fx = x - (float)ix;
                pf[j].fy = y - (float)iy;
                key[j] = ((unsigned)iy << 16) | (unsigned)ix;
                miss[j] = nb_key[slot] != key[j];
                if (miss[j]) {
                    const unsigned ux = (unsigned)ix, uy = (unsigned)iy;
                    const float *r0 = cells + cell_word(g, (int)ux, (int)uy);
                    const float *r1 = cells + cell_word(g, (int)ux, (int)(uy + 1));
                    if ((ux & (CELL_BLK - 1)) != CELL_BLK - 1) {  // (ix, ix + 1) adjacent in a block row
                        float2 a, b;
                        __builtin_memcpy(&a, r0, 8);
                        __builtin_memcpy(&b, r1, 8);
                        pf[j].l[0] = a.x; pf[j].l[1] = a.y; pf[j].l[2] = b.x; pf[j].l[3] = b.y;
                    } else {
                        pf[j].l[0] = r0[0];
                        pf[j].l[1] = cells[cell_word(g, (int)(ux + 1), (int)uy)];
                        pf[j].l[2] = r1[0];
                        pf[j].l[3] = cells[cell_word(g, (int)(ux + 1), (int)(uy + 1))];
                    }
                }
            }
        }
    }
    // park the gathered log-odds of every miss in its slot, list the slot for its wave
    const int lane = tid & 63;
    unsigned short *wl = mlist + (tid >> 6) * (NP * 64);
    int nmiss = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int slot = tid + j * MATCH_THREADS;
        const unsigned long long bm = __ballot(miss[j]);
        if (miss[j]) {
            nb_val[slot] = make_float4(pf[j].l[0], pf[j].l[1], pf[j].l[2], pf[j].l[3]);
            nb_key[slot] = key[j];
            wl[nmiss + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))] =
                (unsigned short)slot;
        }
        nmiss += __popcll(bm);
    }
    // the wave's own LDS writes are seen by its later LDS reads (in-order per wave); keep the compiler
    // from moving the reads above them
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int e = lane; e < nmiss; e += 64) {
        const int slot = wl[e];
        const float4 v = nb_val[slot];
        nb_val[slot] = make_float4(cell_prob(v.x), cell_prob(v.y), cell_prob(v.z), cell_prob(v.w));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int wave = tid >> 6;
    const int cw = chain_wave();  // the chain / step-tail wave
    float run = 0.0f;                                       // SEQ: lane k < 9 of wave cw: sum of term k
    if constexpr (SEQ) {
        // chunk j = points j * 256 .. j * 256 + 255 = slot j of every thread, in point order
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (j * MATCH_THREADS >= n) break;  // uniform
            const int slot = tid + j * MATCH_THREADS;
            float t[9];
            if (slot < n) {
                if (pf[j].in) {
                    const float4 v = nb_val[slot];
                    pf[j].l[0] = v.x; pf[j].l[1] = v.y; pf[j].l[2] = v.z; pf[j].l[3] = v.w;
                }
                point_terms<true>(pf[j], cs, sn, t);
            }
            seq_chunk(seqT, t, slot < n, j == 0, min(MATCH_THREADS, n - j * MATCH_THREADS), cw, run);
        }
    } else {
        float acc[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] = 0.0f;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int slot = tid + j * MATCH_THREADS;
            if (slot >= n) continue;
            if (pf[j].in) {
                const float4 v = nb_val[slot];
                pf[j].l[0] = v.x; pf[j].l[1] = v.y; pf[j].l[2] = v.z; pf[j].l[3] = v.w;
            }
            point_accum<true>(pf[j], cs, sn, acc);
        }
        wave_butterfly(acc);  // 64-lane xor butterfly, offsets 32..1
        if ((tid & 63) == 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) red[parity][wave][k] = acc[k];
        }
        __syncthreads();
    }
    float *sp = s_pose[parity];
    if (wave == cw) {
        float s[9];
        if constexpr (SEQ) {
            seq_gather(run, s);
        } else {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                float a0 = red[parity][0][k] + red[parity][2][k];
                float a1 = red[parity][1][k] + red[parity][3][k];
                s[k] = a0 + a1;
            }
        }
        float b[3] = {s[0], s[1], s[2]};
        H[0] = s[3]; H[4] = s[4]; H[8] = s[5];
        H[1] = s[6]; H[2] = s[7]; H[5] = s[8];
        H[3] = H[1]; H[6] = H[2]; H[7] = H[5];
        float clamp = 0.0f;
        if ((H[0] != 0.0f) && (H[4] != 0.0f)) {
            float d[3];
            solve3(H, b, d);
            if (d[2] > 0.2f) {
                d[2] = 0.2f;
                clamp = 1.0f;
            } else if (d[2] < -0.2f) {
                d[2] = -0.2f;
                clamp = 1.0f;
            }
            est[0] = est[0] + d[0];
            est[1] = est[1] + d[1];
            est[2] = est[2] + d[2];
        }
        if ((tid & 63) == 0) {
            sp[0] = est[0];
            sp[1] = est[1];
            sp[2] = est[2];
            sp[3] = sdm_cosf(est[2]);
            sp[4] = sdm_sinf(est[2]);
#pragma unroll
            for (int k = 0; k < 9; ++k) sp[5 + k] = H[k];
            sp[14] = clamp;
        }
        __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    est[0] = sp[0];
    est[1] = sp[1];
    est[2] = sp[2];
    cs = sp[3];
    sn = sp[4];
#pragma unroll
    for (int k = 0; k < 9; ++k) H[k] = sp[5 + k];
}

// ---- the reference's summation order with a dedicated chain wave (default, round 4) ---------------
// Round 3 ran the sequential sums on one wave that ALSO computed a quarter of every chunk's terms, so each
// chunk cost the chain (256 dependent adds) plus that wave's share of the next chunk's terms, and the
// other waves waited for it at every hand-off (chunk loop 15.4 k of a GN step's 24 k cycles).  Here the
// chain wave cw holds no points: the other three waves own the scan (point i = chunk * CW_PTS + pt, pt the
// thread's rank among the 192 point threads, CW_NP slots each: scans of <= 1152 points) and fill two
// alternating term buffers, one barrier per chunk -- at barrier j the point waves have stored chunk j and
// the chain wave has finished chunk j - 1, whose buffer the point waves fill next.  The chain wave goes from
// chunk to chunk without waiting for terms.  The adds are the same chain in the same order as
// getCompleteHessianDerivs (OccGridMapUtil.h:94-126), so H / b are bit-identical to round 3's.
constexpr int CW_PTS = MATCH_THREADS - 64;        // point threads
constexpr int CW_NP = 6;                           // slots per point thread
constexpr int CW_MAXN = CW_PTS * CW_NP;            // 1152 points in registers
constexpr int CW_STRIDE = CW_PTS + 4;              // term-buffer row (words): 16-B aligned, row k on bank 4k
constexpr int CW_BUF = 9 * CW_STRIDE;              // one chunk's terms
// term buffers: 1 (default: two barriers per chunk; 31.3 KB of LDS with REGS, 5 workgroups per CU) or 2 (one
// barrier per chunk; 38.3 KB, 4 workgroups per CU).  Measured (profiles/r04/ab_r04d*): match 0.340 / 0.345 ms at
// 2048 streams; at 2560 streams (two whole rounds at 5 per CU) the one-buffer match is 0.395 ms, 1.56 M scans/s
#ifndef S2D_CW_BUFS
#define S2D_CW_BUFS 1
#endif
constexpr int CW_BUFS = S2D_CW_BUFS;
#ifndef S2D_MATCH_CW
#define S2D_MATCH_CW 1  // 0: round 3's chain wave that also computes terms (A/B builds)
#endif
// 1 (default; one term buffer only): the moved points' probability conversions are shared by all four waves --
// the idle chain wave too -- over the three point waves' miss lists, between two barriers, instead of each point
// wave converting its own list (the longest list set the start of chunk 0).  0: per-wave lists (A/B).
#ifndef S2D_CW_SHARECONV
#define S2D_CW_SHARECONV 1
#endif
constexpr bool CW_SHARE = S2D_CW_SHARECONV && CW_BUFS == 1;
// wave priority of every wave from a Gauss-Newton step's start to chunk 0's store (the phase the chain waits
// for: transform, gathers, conversions, chunk 0's terms), so it issues ahead of co-resident workgroups' point
// waves working ahead on later chunks; 0 = default priority (A/B)
#ifndef S2D_PRECHAIN_PRIO
#define S2D_PRECHAIN_PRIO 2
#endif
#ifndef S2D_PROLOGUE_PRIO
#define S2D_PROLOGUE_PRIO 1  // the kernel's prologue and every level's start at that priority too (0: A/B)
#endif

// cell_word for a cell inside the level (x, y < 2^15) in unsigned 32-bit arithmetic: shifts, masks and one
// 24-bit multiply (the tile index < 2^13 times the block words), no 64-bit address math.  The match's gathers
// index the level's uniform base with 4 x this: as 64-bit VGPR addresses (cell_word) they needed 64-bit
// temporaries, and the compiler's reuse of a slot's load registers for those put a vmcnt(0) between slots
// 3 and 4 of the gather loop -- two memory round trips per Gauss-Newton step instead of one.
__device__ __forceinline__ unsigned cell_off(const LevelGeom &g, unsigned x, unsigned y)
{
    return __umul24((y / TILE_H) * (unsigned)g.tiles_x + x / TILE, (unsigned)TILE_BLOCK_WORDS) +
           (unsigned)tile_cell((int)(x % TILE), (int)(y % TILE_H));
}

template <int NP, bool BIG>
__device__ __forceinline__ void gn_step_cw(const float *__restrict__ cells, const LevelGeom &g, const float2 (&p)[NP],
                                           int n, float f, float *est, float &cs, float &sn, int parity,
                                           unsigned (&kreg)[NP], float4 *nb_val, float (*s_pose)[POSE_WORDS], float *seqT,
                                           int cw, int pt, bool first)
{
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = tid >> 6;
    const int nch = (n + CW_PTS - 1) / CW_PTS;  // chunks (uniform)
    float run = 0.0f;                           // chain wave, lane k < 9: the running sum of term k
    __shared__ int s_mcnt[4];                   // CW_SHARE: each point wave's miss count
    unsigned short *wl0 = reinterpret_cast<unsigned short *>(seqT + (CW_BUFS - 1) * CW_BUF);  // the miss lists
    if (S2D_PRECHAIN_PRIO) __builtin_amdgcn_s_setprio(S2D_PRECHAIN_PRIO);
    if (wave != cw) {
        // the moved points' neighbourhoods go straight from HBM into the cache planes by LDS-DMA (no VGPRs hold
        // them; the transform is recomputed for the terms below)
        unsigned key[NP];
        bool miss[NP];
        // every slot's key first, then the gathers of the moved points (the cached keys are registers: a slot
        // is only ever looked up by the thread that owns it)
        const unsigned (&kv)[NP] = kreg;
        const float lim0 = g.lim[0], lim1 = g.lim[1];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int slot = pt + j * CW_PTS;
            const float px = p[j].x * f, py = p[j].y * f;
            const float nsn = -sn;
            const float x = est[0] + (cs * px + nsn * py);
            const float y = est[1] + (sn * px + cs * py);
            const bool in = (slot < n) & (x >= 0.0f) & (x <= lim0) & (y >= 0.0f) & (y <= lim1);  // NaN -> out of map
            key[j] = in ? ((unsigned)(int)y << 16) | (unsigned)(int)x : NB_NONE;  // a slot >= n: no miss
        }
        const int pw = pt >> 6;
        float *nbf = reinterpret_cast<float *>(nb_val);  // four planes of CW_MAXN floats (cell 00, 10, 01, 11)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            miss[j] = key[j] != NB_NONE && kv[j] != key[j];
            if (miss[j]) {
                // LDS-DMA: lane l of this wave lands at plane + (pw * 64 + j * CW_PTS) + l = its slot
                const int sb = pw * 64 + j * CW_PTS;
                const unsigned ux = key[j] & 0xFFFFu, uy = key[j] >> 16;
                const float *a0, *a1, *a2, *a3;
                if (BIG) {  // (levels of 2^30 words or more: 64-bit addresses)
                    a0 = cells + cell_word(g, (int)ux, (int)uy);
                    a1 = cells + cell_word(g, (int)ux + 1, (int)uy);
                    a2 = cells + cell_word(g, (int)ux, (int)uy + 1);
                    a3 = cells + cell_word(g, (int)ux + 1, (int)uy + 1);
                } else {
                    const char *cb = reinterpret_cast<const char *>(cells);
                    a0 = reinterpret_cast<const float *>(cb + 4u * cell_off(g, ux, uy));
                    a1 = reinterpret_cast<const float *>(cb + 4u * cell_off(g, ux + 1u, uy));
                    a2 = reinterpret_cast<const float *>(cb + 4u * cell_off(g, ux, uy + 1u));
                    a3 = reinterpret_cast<const float *>(cb + 4u * cell_off(g, ux + 1u, uy + 1u));
                }
                typedef __attribute__((address_space(1))) void gv;
                typedef __attribute__((address_space(3))) void lv;
                __builtin_amdgcn_global_load_lds((gv *)a0, (lv *)(nbf + 0 * CW_MAXN + sb), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((gv *)a1, (lv *)(nbf + 1 * CW_MAXN + sb), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((gv *)a2, (lv *)(nbf + 2 * CW_MAXN + sb), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((gv *)a3, (lv *)(nbf + 3 * CW_MAXN + sb), 4, 0, 0);
            }
        }
        // park the gathered log-odds of every miss in its slot and list the slot for this wave (the list lives
        // in the last term buffer: with two, first written after chunk 0's barrier; with one, chunk 0 is stored
        // after a barrier that follows every wave's conversions), then convert 64 at a time
        unsigned short *wl = reinterpret_cast<unsigned short *>(seqT + (CW_BUFS - 1) * CW_BUF) + pw * (NP * 64);
        int nmiss = 0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int slot = pt + j * CW_PTS;
            const unsigned long long bm = __ballot(miss[j]);
            if (miss[j]) {
                kreg[j] = key[j];
                // (a first step keeps no list: its terms may already fill the buffer the lists live in)
                if (!first)
                    wl[nmiss + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))] =
                        (unsigned short)slot;
            }
            nmiss += __popcll(bm);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's LDS-DMA landed (the barrier below publishes it)
        if (first) {
            // a level's first step: every in-map point missed (the keys were reset); each point thread converts its
            // own slots chunk by chunk below, so chunk 0's terms -- and the chain -- start after one sixth of the
            // conversions, and chunk j + 1's overlap the chain's chunk j
        } else if constexpr (CW_SHARE) {
            if (lane == 0) s_mcnt[pw] = nmiss;
        } else {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            float *nbf = reinterpret_cast<float *>(nb_val);
            for (int e = lane; e < nmiss; e += 64) {
                const int slot = wl[e];
#pragma unroll
                for (int c = 0; c < 4; ++c) nbf[c * CW_MAXN + slot] = cell_prob(nbf[c * CW_MAXN + slot]);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
    }
    if (CW_SHARE && !first) {
        // every wave converts entries wave * 64 + lane + 256 k of the three lists laid end to end; the second
        // barrier also retires the lists before chunk 0's terms overwrite them
        lds_barrier();
        const int c0 = s_mcnt[0], c1 = s_mcnt[1], tot = c0 + c1 + s_mcnt[2];
        for (int e = tid; e < tot; e += MATCH_THREADS) {
            const int l = e < c0 ? 0 : (e < c0 + c1 ? 1 : 2);
            const int slot = wl0[l * (NP * 64) + e - (l == 0 ? 0 : (l == 1 ? c0 : c0 + c1))];
            float *nbf = reinterpret_cast<float *>(nb_val);
#pragma unroll
            for (int c = 0; c < 4; ++c) nbf[c * CW_MAXN + slot] = cell_prob(nbf[c * CW_MAXN + slot]);
        }
        lds_barrier();
    }
    if (wave != cw) {
        // chunk j = slot j of every point thread, in point order; buffer j & 1
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (j >= nch) break;  // uniform
            const int slot = pt + j * CW_PTS;
            float t[9];
            if (slot < n) {
                PointFetch pf;  // the gather phase's transform, recomputed (the same operations, the same bits)
                pf.px = p[j].x * f;
                pf.py = p[j].y * f;
                const float nsn = -sn;
                const float x = est[0] + (cs * pf.px + nsn * pf.py);
                const float y = est[1] + (sn * pf.px + cs * pf.py);
                pf.in = (x >= 0.0f) && (x <= g.lim[0]) && (y >= 0.0f) && (y <= g.lim[1]);
                if (pf.in) {
                    pf.fx = x - (float)(int)x;
                    pf.fy = y - (float)(int)y;
                    float *nbf = reinterpret_cast<float *>(nb_val);
#pragma unroll
                    for (int c = 0; c < 4; ++c) pf.l[c] = nbf[c * CW_MAXN + slot];
                    if (first) {  // this thread's own gathered log-odds (its LDS-DMA landed: vmcnt(0) above)
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            pf.l[c] = cell_prob(pf.l[c]);
                            nbf[c * CW_MAXN + slot] = pf.l[c];
                        }
                    }
                }
                point_terms<true>(pf, cs, sn, t);
            }
            // (barriers only in wave-uniform control flow: a wave whose lanes straddle n runs both sides of
            // the slot test)
            if (CW_BUFS == 1 && (!CW_SHARE || j > 0)) lds_barrier();  // the chain wave is done with chunk j - 1 (j = 0: the miss lists)
            if (slot < n) {
                float *T = seqT + (CW_BUFS == 2 ? (j & 1) * CW_BUF : 0);
#pragma unroll
                for (int k = 0; k < 9; ++k) T[k * CW_STRIDE + pt] = t[k];
            }
            lds_barrier();  // chunk j stored (two buffers: and the chain wave is done with chunk j - 1)
            if (S2D_PRECHAIN_PRIO && j == 0) __builtin_amdgcn_s_setprio(0);
        }
    } else {
        // the chain: lane k < 9 extends the sum of term k over each chunk, at s_setprio 3 through the step tail
        // (the workgroup's critical path issues ahead of co-resident workgroups' waves)
        __builtin_amdgcn_s_setprio(3);
        for (int j = 0; j < nch; ++j) {
            if (CW_BUFS == 1 && (!CW_SHARE || j > 0)) lds_barrier();
            lds_barrier();
            if (lane < 9)
                run = seq_chain_t<CW_STRIDE>(seqT + (CW_BUFS == 2 ? (j & 1) * CW_BUF : 0), lane, min(CW_PTS, n - j * CW_PTS),
                                             run);
        }
    }
    float *sp = s_pose[parity];
    if (wave == cw) {
        float s[9], H[9];
        seq_gather(run, s);
        float b[3] = {s[0], s[1], s[2]};
        H[0] = s[3]; H[4] = s[4]; H[8] = s[5];
        H[1] = s[6]; H[2] = s[7]; H[5] = s[8];
        H[3] = H[1]; H[6] = H[2]; H[7] = H[5];
        float clamp = 0.0f;
        if ((H[0] != 0.0f) && (H[4] != 0.0f)) {
            float d[3];
            solve3(H, b, d);
            if (d[2] > 0.2f) {
                d[2] = 0.2f;
                clamp = 1.0f;
            } else if (d[2] < -0.2f) {
                d[2] = -0.2f;
                clamp = 1.0f;
            }
            est[0] = est[0] + d[0];
            est[1] = est[1] + d[1];
            est[2] = est[2] + d[2];
        }
        if (lane == 0) {
            sp[0] = est[0];
            sp[1] = est[1];
            sp[2] = est[2];
            sp[3] = sdm_cosf(est[2]);
            sp[4] = sdm_sinf(est[2]);
#pragma unroll
            for (int k = 0; k < 9; ++k) sp[5 + k] = H[k];
            sp[14] = clamp;
        }
        __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    // (H stays in s_pose, read once at the level's end)
    est[0] = sp[0];
    est[1] = sp[1];
    est[2] = sp[2];
    cs = sp[3];
    sn = sp[4];
}

constexpr int MATCH_REG_PTS = 5;  // points per thread kept in registers: scans of up to 1280 points

// register budget of the reference-order register instances (gn_step_cw): waves per SIMD the compiler must fit
// them into.  6 (default, round 6): 80 VGPRs; with the cache keys in registers and the gathers by LDS-DMA the
// instance needs 26.1 KB of LDS, so six workgroups share a CU (5 before: 31.3 KB, 89 VGPRs).  Measured
// (profiles/r06/ab_r06h*, ab_r06i*): match -1.9 % at the north star, -2.9 % under the node's gate; the
// other instances (tree order, HBM path) stay unconstrained (1)
#ifndef S2D_MATCH_WAVES
#define S2D_MATCH_WAVES 6
#endif
// SEQ (default): H / b summed in the reference's sequential point order; else the tree order
// (SLAM2D_MATCH_ORDER=tree / hs_set_reduction_order: faster, poses within float reassociation of the
// reference's).
// REGS: every scan of the launch fits the registers (max_points <= CW_MAXN for SEQ, 1280 for the tree
// order): the HBM-strided Gauss-Newton path is compiled out -- it alone lifted the kernel from 83 to 140
// VGPRs (SEQ), so the common case no longer pays its register allocation
// BIG: some level holds 2^30 words or more (maps above ~20000^2 cells): the reference-order gathers use 64-bit
// addresses (cell_word) instead of 32-bit byte offsets from the level base (cell_off)
template <bool SEQ, bool REGS, bool BIG>
__global__ void __launch_bounds__(MATCH_THREADS) __attribute__((amdgpu_waves_per_eu((SEQ && REGS) ? S2D_MATCH_WAVES : 1)))
hs_match_kernel(FleetGeom geom, const float *__restrict__ cells, StreamState *__restrict__ state,
                const float2 *__restrict__ xy, int xy_stride, const int *__restrict__ counts,
                const float2 *__restrict__ origo, const float *__restrict__ hints, int stream_begin, int mode,
                float *__restrict__ out_pose, float *__restrict__ out_cov, PoseLog plog, WorkQueue *__restrict__ wq,
                UpdList *__restrict__ wl, IngestGeom ig, MatchIngest mi, float2 *__restrict__ mc, int mc_stride)
{
    static_assert(MATCH_THREADS == 64 * MATCH_WAVES && MATCH_WAVES == 4, "reduction tree assumes 4 waves");
    __shared__ float red[2][MATCH_WAVES][9];
    // SEQ: two chunks' terms for the chain wave (gn_step_cw; its miss lists live in the second), or one
    // 256-point chunk of the HBM path (gn_step); tree order: the miss lists
    constexpr bool CW = SEQ && S2D_MATCH_CW;                          // gn_step_cw (else round 3's gn_step_reg)
    constexpr int NPR = CW ? CW_NP : MATCH_REG_PTS;                   // point slots per thread in registers
    constexpr int NSLOT = CW ? CW_MAXN : MATCH_REG_PTS * MATCH_THREADS;
    constexpr int SEQ_LDS = !CW ? SEQ_WORDS : ((CW_BUFS * CW_BUF > SEQ_WORDS || REGS) ? CW_BUFS * CW_BUF : SEQ_WORDS);
    __shared__ __attribute__((aligned(16))) float seqT[SEQ ? SEQ_LDS : 4];
    __shared__ unsigned nb_key[CW ? 4 : NSLOT];  // (the chain-wave path keeps its cached keys in registers: kreg)
    __shared__ float4 nb_val[NSLOT];
    __shared__ unsigned short mlist[CW ? 4 : MATCH_REG_PTS * MATCH_THREADS];  // tree order: per wave, the slots whose cell moved
    __shared__ float s_pose[2][POSE_WORDS];                             // a step's result, by parity
    const int local = blockIdx.x;
    const int s = stream_begin + local;
    StreamState &st = state[s];
    clk_stamp(geom.clk, 0, true);
    // fused ingest (mi.ranges): the scan's points in beam order to mi.xy_out (for the grid update) and to
    // an LDS copy in nb_val's space, read into registers below before nb_val's first use
    const bool fused = mi.ranges != nullptr;
    // the prologue (ingest, pose) and every level's start are on the stream's path like a step's pre-chain phase
    if (S2D_PRECHAIN_PRIO && S2D_PROLOGUE_PRIO) __builtin_amdgcn_s_setprio(S2D_PRECHAIN_PRIO);
    load_exptab();
    if (!fused) __syncthreads();  // (fused: the ingest's barriers order the table before its first use)
    const float *scells = cells + (size_t)s * geom.stream_words;
    __shared__ int s_w[ING_SW];
    float2 *stage = reinterpret_cast<float2 *>(nb_val);
    const float2 *pts = fused ? mi.xy_out + (size_t)local * xy_stride : xy + (size_t)local * xy_stride;
    // a caller's count is clamped to [0, max_points] (= mc_stride, the per-stream container's capacity;
    // hs_step_batch_device documents the range): the register-only instance has no path for more points, and
    // the update kernel sizes its ray groups by max_points
    const int n = fused ? ingest_scan(ig, mi.cs, mi.ranges + (size_t)local * mi.rstride,
                                      mi.xy_out + (size_t)local * xy_stride, stage, s_w)
                        : min(max(counts[local], 0), mc_stride);

    float hint[3];
    if (hints) {
        hint[0] = hints[3 * local];
        hint[1] = hints[3 * local + 1];
        hint[2] = hints[3 * local + 2];
    } else {
        hint[0] = st.pose[0];
        hint[1] = st.pose[1];
        hint[2] = st.pose[2];
    }

    float np_[3] = {hint[0], hint[1], hint[2]};
    // the covariance: the last level's H after a match, else the stream's stored one (read only then, in the
    // epilogue -- held from here it kept nine registers live through the whole match)
    float cov[9];
    bool cov_h = false;

    int clamps = 0;
    int parity = 0;
    if (mode == MODE_PROCESS || mode == MODE_MATCH_ONLY) {
        // MapRepMultiMap::matchData  H/slam_main/MapRepMultiMap.h:144-167
        float tmp[3] = {hint[0], hint[1], hint[2]};
        // SEQ: the chain wave cw holds no points; point thread pt owns points pt + j * CW_PTS (gn_step_cw)
        const int cw = chain_wave();
        const int wv = (int)threadIdx.x >> 6;
        const bool owner = !CW || wv != cw;
        const int pt = CW ? ((wv < cw ? wv : wv - 1) * 64 + ((int)threadIdx.x & 63)) : (int)threadIdx.x;
        const int pstride = CW ? CW_PTS : MATCH_THREADS;
        const bool in_regs = n <= pstride * NPR;
        float2 preg[NPR];
        unsigned kreg[NPR];  // CW: each owned slot's neighbourhood-cache key (NB_NONE: nothing cached)
#pragma unroll
        for (int j = 0; j < NPR; ++j) {
            const int i = pt + j * pstride;
            preg[j] = make_float2(0.0f, 0.0f);
            if (owner && in_regs && i < n) {
                if (fused) preg[j] = stage[i];  // LDS (kept apart from the global read: no flat access)
                else preg[j] = pts[i];
            }
        }
        if (fused) __syncthreads();  // stage read before nb_val is written
        // MapRepMultiMap keeps the scan it matched: dataContainers[l - 1].setFrom(container, 1 / 2^l)
        // (MapRepMultiMap.h:161) is what updateByScan later draws into levels >= 1 (:187).  The stream's
        // stored container (level-0 scale, scaled at use exactly as setFrom does) is mc[s]; the fused
        // ingest already wrote the points there.
        float2 *mcs = mc ? mc + (size_t)s * mc_stride : nullptr;
        if (mcs && mcs != pts && geom.levels > 1) {
            if (in_regs) {
#pragma unroll
                for (int j = 0; j < NPR; ++j) {
                    const int i = pt + j * pstride;
                    if (owner && i < n) mcs[i] = preg[j];
                }
            } else {
                for (int i = threadIdx.x; i < n; i += MATCH_THREADS) mcs[i] = pts[i];
            }
        }
        for (int lvl = geom.levels - 1; lvl >= 0; --lvl) {
            const LevelGeom &g = geom.lv[lvl];
            const int iters = lvl == 0 ? 5 : 3;
            if (n == 0) continue;  // ScanMatcher::matchData returns the hint (ScanMatcher.h:65, :96)
            if (S2D_PRECHAIN_PRIO && S2D_PROLOGUE_PRIO) __builtin_amdgcn_s_setprio(S2D_PRECHAIN_PRIO);
            const float *lc = scells + g.word_offset;
            float est[3], H[9];
            map_from_world(g, tmp, est);
#pragma unroll
            for (int j = 0; j < NPR; ++j) {
                if constexpr (CW) kreg[j] = NB_NONE;
                else if (owner) nb_key[pt + j * pstride] = NB_NONE;  // own slots
            }
            float cs = sdm_cosf(est[2]), sn = sdm_sinf(est[2]);
            for (int it = 0; it <= iters; ++it) {
                if (in_regs) {
                    if constexpr (CW)
                        gn_step_cw<NPR, BIG>(lc, g, preg, n, g.pts_scale, est, cs, sn, parity, kreg, nb_val, s_pose, seqT,
                                             cw, pt, it == 0);
                    else
                        gn_step_reg<NPR, SEQ>(lc, g, preg, n, g.pts_scale, est, cs, sn, H, red, parity, nb_key,
                                              nb_val, mlist, s_pose, seqT);
                    clamps += s_pose[parity][14] != 0.0f ? 1 : 0;
                } else if constexpr (!REGS) {
                    gn_step<SEQ>(lc, g, pts, n, g.pts_scale, est, H, red, parity, &clamps, seqT);
                }
                parity ^= 1;
            }
            est[2] = normalize_angle(est[2]);
            // the last step's H: the chain-wave path left it in s_pose only (parity has moved past it)
#pragma unroll
            for (int k = 0; k < 9; ++k) cov[k] = (CW && in_regs) ? s_pose[parity ^ 1][5 + k] : H[k];
            cov_h = true;
            world_from_map(g, est, tmp);
        }
        np_[0] = tmp[0];
        np_[1] = tmp[1];
        np_[2] = tmp[2];
    }
    clk_stamp(geom.clk, 0, false);
    if (threadIdx.x != 0) return;
    if (local == 0) {  // reset the grid-update work queue for this step (consumed by k2/k3)
        wq->seg_used = 0;
        wq->item_used = 0;
        wq->whole_used = 0;
    }

    if (!cov_h) {
#pragma unroll
        for (int k = 0; k < 9; ++k) cov[k] = st.cov[k];
    }
    if (out_pose) {
        out_pose[3 * local] = np_[0];
        out_pose[3 * local + 1] = np_[1];
        out_pose[3 * local + 2] = np_[2];
    }
    if (out_cov) {
        for (int k = 0; k < 9; ++k) out_cov[9 * local + k] = cov[k];
    }
    st.clamp_count += clamps;
    st.tot_steps += 1;
    const int slot = plog.slot_of ? plog.slot_of[s] : s;
    if (plog.buf && slot >= 0 && slot < plog.streams && st.step_index < plog.capacity) {
        float *row = plog.buf + ((size_t)st.step_index * plog.streams + slot) * 3;
        row[0] = np_[0];
        row[1] = np_[1];
        row[2] = np_[2];
    }
    st.step_index += 1;
    if (mode == MODE_PROCESS || mode == MODE_MATCH_ONLY) {
        unsigned long long it = 0;
        for (int lvl = 0; lvl < geom.levels; ++lvl) it += (lvl == 0 ? 6 : 4);
        st.tot_gn_points += it * (unsigned long long)n;
    }
    st.n = n;
    const float2 org = fused ? ig.origo : (origo ? origo[local] : make_float2(0.0f, 0.0f));
    st.origo[0] = org.x;
    st.origo[1] = org.y;
    if (mode == MODE_PROCESS || mode == MODE_MATCH_ONLY) {  // the stored container (see above)
        st.mc_n = n;
        st.mc_origo[0] = org.x;
        st.mc_origo[1] = org.y;
    }
    if (fused) {
        mi.n_out[local] = n;
        mi.origo_out[local] = org;
    }
    int do_update = 0;
    if (mode == MODE_PROCESS || mode == MODE_NO_MATCH_FORCE) {
        // HectorSlamProcessor::update  H/slam_main/HectorSlamProcessor.h:91-107
        st.pose[0] = np_[0];
        st.pose[1] = np_[1];
        st.pose[2] = np_[2];
        for (int k = 0; k < 9; ++k) st.cov[k] = cov[k];
        if (mode == MODE_NO_MATCH_FORCE || pose_diff_larger(np_, st.last_upd_pose, geom.min_dist, geom.min_ang)) {
            do_update = 1;
            st.last_upd_pose[0] = np_[0];
            st.last_upd_pose[1] = np_[1];
            st.last_upd_pose[2] = np_[2];
        }
    } else if (mode == MODE_UPDATE_ONLY) {
        do_update = 1;  // MapRepMultiMap::updateByScan with the given pose
    }
    st.do_update = do_update;
    if (do_update) {
        st.upd_pose[0] = np_[0];
        st.upd_pose[1] = np_[1];
        st.upd_pose[2] = np_[2];
        st.mark_base = st.cur_update_index;  // currMarkFreeIndex = +1, currMarkOccIndex = +2 (OccGridMapBase.h:120-121)
        // the hot ordinal of this update k = currUpdateIndex / 3 (hector_internal.h ORD_OFF): freed cells get
        // 2 (k - E) + 1, occupied ones + 1
        st.ord_base = 2 * (st.cur_update_index / 3 - st.ord_epoch) + 1;
        if (st.ord_base >= 0xFFFF) st.ord_overflow = 1;  // its occupied ordinal would not fit 16 bits (no sweep)
        st.cur_update_index += 3;            // OccGridMapBase.h:167
        st.map_updates += 1;                 // GridMapBase::setUpdated (GridMapBase.h:333)
        st.step_cells = 0;
        st.tot_updates += 1;
        if (wl) wl->stream[atomicAdd(&wl->count, 1)] = local;
    }
}

// ------------------------------------------------------------------------------- ray geometry
// OccGridMapBase::updateByScan (H/map/OccGridMapBase.h:118-161) + updateLineBresenhami (:220-267).
// Every ray starts at the common begin cell; a ray is stored as its end cell (packed y<<16 | x) or
// RAY_INVALID when updateByScan would skip it (begin == end :157, or begin/end outside :226-238).
constexpr unsigned RAY_INVALID = 0xFFFFFFFFu;
// waves per hs_update_kernel workgroup: 4 (default: 256 threads, 64 x 32-cell LDS tiles, 8 workgroups per CU) or 8
// (512 threads, 64 x 64-cell tiles, 4 per CU: the same 32 waves per CU, half the tile visits and clip setups)
#ifndef S2D_UPD_WAVES
#define S2D_UPD_WAVES 4
#endif
constexpr int UPD_WAVES = S2D_UPD_WAVES;
static_assert(UPD_WAVES == 4 || UPD_WAVES == 8, "hs_update_kernel: 4 or 8 waves per workgroup");
constexpr int UPD_THREADS = 64 * UPD_WAVES;
// two LDS words per tile cell, both updated with blind atomicMin (no read-modify-write chain):
//   first_hit[c]  = smallest beam whose end cell is c      (NONE if none)
//   first_free[c] = smallest beam that frees c            (NONE if none)
// the reference's per-cell outcome depends only on these: free only -> l + lf; hit -> if freed
// first (first_free < first_hit) ((l + lf) - lf), then + lo if l < 50.
constexpr unsigned W_NONE = 0xFFFFFFFFu;

// (int)v of :135/:154 for v in int range; NaN / out of range -> -1 (cancelled by the bounds check,
// as x86's INT_MIN is in the reference; the GPU's saturating convert would turn NaN into cell 0)
__device__ __forceinline__ int cell_of(float v)
{
    return (v > -2147483648.0f && v < 2147483648.0f) ? (int)v : -1;
}

struct RayFrame {
    float mx, my, cs, sn;
    int bxi, byi;
};

__device__ __forceinline__ RayFrame ray_frame(const LevelGeom &g, const StreamState &st, const float *org)
{
    RayFrame fr;
    float mp[3];
    map_from_world(g, st.upd_pose, mp);  // getMapCoordsPose (:124)
    fr.mx = mp[0];
    fr.my = mp[1];
    fr.cs = sdm_cosf(mp[2]);
    fr.sn = sdm_sinf(mp[2]);
    const float f = g.pts_scale;
    float ox = org[0] * f, oy = org[1] * f;  // setFrom: origo * factor (DataPointContainer.h:48)
    float nsn = -fr.sn;
    float bx = fr.mx + (fr.cs * ox + nsn * oy);   // poseTransform * origo (:132)
    float by = fr.my + (fr.sn * ox + fr.cs * oy);
    fr.bxi = cell_of(bx + 0.5f);                   // (:135)
    fr.byi = cell_of(by + 0.5f);
    return fr;
}

__device__ __forceinline__ unsigned make_ray(const LevelGeom &g, const RayFrame &fr, float2 p)
{
    const float f = g.pts_scale;
    float px = p.x * f, py = p.y * f;
    float nsn = -fr.sn;
    float ex = fr.mx + (fr.cs * px + nsn * py);  // poseTransform * point (:147)
    float ey = fr.my + (fr.sn * px + fr.cs * py);
    ex += 0.5f;                                   // (:151)
    ey += 0.5f;
    int x1 = cell_of(ex), y1 = cell_of(ey);       // (:154)
    int x0 = fr.bxi, y0 = fr.byi;
    if (x0 == x1 && y0 == y1) return RAY_INVALID;
    if ((x0 < 0) || (x0 >= g.sx) || (y0 < 0) || (y0 >= g.sy)) return RAY_INVALID;
    if ((x1 < 0) || (x1 >= g.sx) || (y1 < 0) || (y1 >= g.sy)) return RAY_INVALID;
    return ((unsigned)y1 << 16) | (unsigned)x1;
}

// Bresenham walk of bresenham2D (:270-299) in closed form: major axis a, minor axis b,
//   step i in [0, da]:  a(i) = a0 + sa*i,  b(i) = b0 + sb*q(i),  q(i) = floor((e0 + i*db) / da),
// e0 = da/2 (error_b start, :254/:260).  The incremental error walk keeps error in [0, da), so this
// is exactly the cell sequence of the reference; steps 0..da-1 are freed, step da is the end cell.
#ifndef S2D_FAST_UDIV
#define S2D_FAST_UDIV 1
#endif
// n / d for n < 2^31, 1 <= d < 2^16: a float reciprocal estimate (relative error < 2^-22) and one
// correction step each way -- ~8 instructions instead of the ~25 of the integer division sequence.
// Exact whenever the quotient is < 2^16, which covers every step index (<= 32767) it is compared
// with; a larger quotient stays > 2^15 and only ever means "beyond the walk".
// The products here use the full-rate 24-bit multiply (v_mul_u32_u24; v_mul_lo_u32 is quarter rate): q * d
// is exact while q < 2^24 (d < 2^16, so the product < 2^32); a larger q -- a true quotient of at least
// ~2^24 -- stays within +-1 of it, still "beyond the walk".
__device__ __forceinline__ unsigned udiv_rcp(unsigned n, unsigned d, float rcp_d)  // rcp_d = rcp((float)d)
{
    unsigned q = (unsigned)((float)n * rcp_d);
    int r = (int)(n - __umul24(q, d));
    if (r < 0) {
        --q;
        r += (int)d;
    }
    if (r >= (int)d) ++q;
    return q;
}
__device__ __forceinline__ unsigned udiv_small(unsigned n, unsigned d, unsigned &rem)  // quotient and remainder
{
#if S2D_FAST_UDIV
    unsigned q = (unsigned)((float)n * __builtin_amdgcn_rcpf((float)d));
    int r = (int)(n - __umul24(q, d));  // callers: quotient < 2^16 (see udiv_rcp)
    if (r < 0) {
        --q;
        r += (int)d;
    }
    if (r >= (int)d) {
        ++q;
        r -= (int)d;
    }
    rem = (unsigned)r;  // (the caller's own n - q * d compiled to a quarter-rate 32-bit multiply)
    return q;
#else
    rem = n % d;
    return n / d;
#endif
}

struct RayWalk {
    int a0, b0, sa, sb, da, db, e0;
    bool x_major;
};

__device__ __forceinline__ RayWalk ray_walk(int x0, int y0, int x1, int y1)
{
    RayWalk w;
    int dx = x1 - x0, dy = y1 - y0;
    int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    int sx = dx > 0 ? 1 : -1, sy = dy > 0 ? 1 : -1;  // util::sign (UtilFunctions.h:55-58)
    w.x_major = adx >= ady;                         // (:252)
    if (w.x_major) {
        w.a0 = x0; w.b0 = y0; w.sa = sx; w.sb = sy; w.da = adx; w.db = ady;
    } else {
        w.a0 = y0; w.b0 = x0; w.sa = sy; w.sb = sx; w.da = ady; w.db = adx;
    }
    w.e0 = w.da / 2;
    return w;
}

// Steps [lo, hi] of the walk whose cell lies in the rectangle [A0,A1) x [B0,B1) (major x minor);
// returns false if none.  q(i) >= Q  <=>  i >= ceil((Q*da - e0)/db);  q(i) <= Q  <=>  i <= floor(((Q+1)*da - e0 - 1)/db).
__device__ __forceinline__ bool walk_range(const RayWalk &w, int A0, int A1, int B0, int B1, int &lo, int &hi)
{
    // branch-free (lanes of one fan differ in the step signs): the steps whose major coordinate lies in
    // [A0, A1), then the minor constraint q(i) in [qlo, qhi] through the two divisions by db (one
    // reciprocal), each taken only where its numerator is meaningful (qlo > 0 / qhi >= 0, db > 0)
    const int d0 = A0 - w.a0, d1 = A1 - 1 - w.a0;
    lo = w.sa > 0 ? d0 : -d1;
    hi = w.sa > 0 ? d1 : -d0;
    lo = lo > 0 ? lo : 0;
    hi = hi < w.da ? hi : w.da;
    const int e0 = B0 - w.b0, e1 = B1 - 1 - w.b0;
    const int qlo = w.sb > 0 ? e0 : -e1, qhi = w.sb > 0 ? e1 : -e0;
    const unsigned dbs = w.db ? (unsigned)w.db : 1u;
    const float rdb = __builtin_amdgcn_rcpf((float)dbs);
    // numerator > 0 when qlo > 0: qlo * da - e0 >= da - da / 2   (|qlo|, |qhi|, da < 2^15: 24-bit products)
    const int n1 = qlo > 0 ? __mul24(qlo, w.da) - w.e0 + w.db - 1 : 0;
    // numerator >= 0 when qhi >= 0: (qhi + 1) * da - e0 - 1 >= da - da / 2 - 1
    const int n2 = qhi >= 0 ? __mul24(qhi + 1, w.da) - w.e0 - 1 : 0;
    const int t = (int)udiv_rcp((unsigned)n1, dbs, rdb), t2 = (int)udiv_rcp((unsigned)n2, dbs, rdb);
    if (w.db != 0) {
        if (qlo > 0 && t > lo) lo = t;
        if (t2 < hi) hi = t2;
    }
    // db == 0: q(i) == 0 for every step, so the walk is in the band iff qlo <= 0 <= qhi
    return lo <= hi && qhi >= 0 && !(w.db == 0 && qlo > 0);
}

// ------------------------------------------------------------ k2/k3: binned, tiled grid update
// The grid update of one scan level is split into 64 x TILE_H tiles of the map:
//   k2 hs_bin_kernel   (one workgroup per stream): builds every level's rays, walks each ray's tile
//                      crossings in closed form (two divisions per crossing), counting-sorts the
//                      ray segments by tile in LDS, and appends one work item per NON-EMPTY tile
//                      (plus its segment list) to global queues.  Oversized scans fall back to one
//                      WHOLE item per level (every ray tested against every tile of the bbox).
//   k3 hs_tile_kernel  (grid-stride over work items): per tile, two LDS words per cell updated with
//                      blind atomicMin --
//                        first_hit[c]  = smallest beam whose end cell is c
//                        first_free[c] = smallest beam that frees c
//                      -- then ONE coalesced 8-byte read-modify-write per touched cell applying the
//                      reference's float sequence: free only: l + lf; hit: ((l + lf) - lf) if freed
//                      first (first_free < first_hit), then + lo if l < 50.
// This equals running bresenhamCellFree / bresenhamCellOcc (:302-330) beam by beam.
constexpr unsigned W_NONE_ = 0xFFFFFFFFu;
constexpr int BIN_THREADS = 256;
constexpr int MAX_BIN_TILES = 1024;  // per level; larger bounding boxes use a WHOLE item
constexpr int ITEM_TILE = 0, ITEM_WHOLE = 1;

// Enumerate the tiles crossed by steps 0..da of a walk: f(tile_x, tile_y, lo, hi).
template <class F>
__device__ __forceinline__ void for_each_segment(const RayWalk &w, F f)
{
    const int A = w.x_major ? TILE : TILE_H;   // tile extent along the major axis
    const int Bt = w.x_major ? TILE_H : TILE;  // along the minor axis
    int i = 0;
    int q = 0;  // q(0) = floor(e0 / da) = 0
    while (i <= w.da) {
        const int a = w.a0 + w.sa * i;
        const int b = w.b0 + w.sb * q;
        const int ta = a / A, tb = b / Bt;
        const int ra = w.sa > 0 ? (ta * A + A - 1 - a) : (a - ta * A);    // steps left along a
        int iend = i + ra;
        if (w.db > 0) {
            const int rb = w.sb > 0 ? (tb * Bt + Bt - 1 - b) : (b - tb * Bt);  // b-steps left
            const int qmax = q + rb;
            const int ib = (int)(((unsigned)(qmax + 1) * (unsigned)w.da - (unsigned)w.e0 - 1u) / (unsigned)w.db);
            if (ib < iend) iend = ib;
        }
        if (iend > w.da) iend = w.da;
        if (w.x_major) f(ta, tb, i, iend);
        else f(tb, ta, i, iend);
        i = iend + 1;
        q = (int)(((unsigned)w.e0 + (unsigned)i * (unsigned)w.db) / (unsigned)w.da);
    }
}

// block-wide exclusive scan of v (256 threads); returns the exclusive prefix, *total = sum
__device__ __forceinline__ int block_exscan(int v, int *s_wave, int *total)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int t = __shfl_up(x, off, 64);
        if (lane >= off) x += t;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BIN_THREADS / 64; ++k) {
        const int ws = s_wave[k];
        if (k < wave) base += ws;
        tot += ws;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__global__ void __launch_bounds__(BIN_THREADS)
hs_bin_kernel(FleetGeom geom, StreamState *__restrict__ state, const float2 *__restrict__ xy, int xy_stride,
              const float2 *__restrict__ mc, int mc_stride, int stream_begin, int max_points, unsigned *__restrict__ rays_g, uint4 *__restrict__ segs,
              WorkItem *__restrict__ items, WorkItem *__restrict__ wholes, WorkQueue *__restrict__ wq,
              unsigned seg_cap, unsigned item_cap)
{
    __shared__ int s_bbox[4];
    __shared__ int s_cnt[MAX_BIN_TILES];
    __shared__ int s_off[MAX_BIN_TILES];
    __shared__ unsigned s_rows[MAX_BIN_TILES];  // per tile: mask of tile rows touched
    __shared__ int s_wave[BIN_THREADS / 64];
    __shared__ unsigned s_base[2];
    const int local = blockIdx.x;
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    const int tid = threadIdx.x;
    unsigned long long Ltot = 0, Rtot = 0;

    for (int lvl = 0; lvl < geom.levels; ++lvl) {
        const LevelGeom &g = geom.lv[lvl];
        // level 0: this step's DataContainer; levels >= 1: the stored one (MapRepMultiMap.h:181-188)
        const int n = lvl == 0 ? st.n : st.mc_n;
        const float2 *pts = lvl == 0 ? xy + (size_t)local * xy_stride : mc + (size_t)s * mc_stride;
        unsigned *rays = rays_g + ((size_t)s * geom.levels + lvl) * max_points;
        const RayFrame fr = ray_frame(g, st, lvl == 0 ? st.origo : st.mc_origo);
        const int x0 = fr.bxi, y0 = fr.byi;
        if (tid == 0) {
            s_bbox[0] = x0; s_bbox[1] = y0; s_bbox[2] = x0; s_bbox[3] = y0;
        }
        __syncthreads();
        int bx0 = x0, by0 = y0, bx1 = x0, by1 = y0, R = 0;
        for (int b = tid; b < n; b += BIN_THREADS) {
            unsigned r = make_ray(g, fr, pts[b]);
            rays[b] = r;
            if (r != RAY_INVALID) {
                int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
                bx0 = min(bx0, x1); by0 = min(by0, y1); bx1 = max(bx1, x1); by1 = max(by1, y1);
                Ltot += (unsigned long long)(max(abs(x1 - x0), abs(y1 - y0)) + 1);
                R += 1;
            }
        }
        Rtot += R;
        if (R) {
            atomicMin(&s_bbox[0], bx0); atomicMin(&s_bbox[1], by0);
            atomicMax(&s_bbox[2], bx1); atomicMax(&s_bbox[3], by1);
        }
        if (!__syncthreads_or(R != 0)) continue;  // nothing drawn on this level
        const int tx0 = s_bbox[0] / TILE, ty0 = s_bbox[1] / TILE_H;
        const int ntx = s_bbox[2] / TILE - tx0 + 1, nty = s_bbox[3] / TILE_H - ty0 + 1;
        const int nt = ntx * nty;
        const unsigned begin_xy = (unsigned)x0 | ((unsigned)y0 << 16);
        bool whole = nt > MAX_BIN_TILES;
        if (!whole) {
            for (int t = tid; t < nt; t += BIN_THREADS) {
                s_cnt[t] = 0;
                s_rows[t] = 0;
            }
            __syncthreads();
            // pass 1: count segments per tile
            for (int b = tid; b < n; b += BIN_THREADS) {
                unsigned r = rays[b];
                if (r == RAY_INVALID) continue;
                RayWalk w = ray_walk(x0, y0, (int)(r & 0xFFFFu), (int)(r >> 16));
                for_each_segment(w, [&](int tx, int ty, int lo, int hi) {
                    const int t = (ty - ty0) * ntx + (tx - tx0);
                    atomicAdd(&s_cnt[t], 1);
                    // rows spanned by steps lo..hi (monotone along the walk)
                    int ylo, yhi;
                    if (w.x_major) {
                        ylo = w.b0 + w.sb * (int)(((unsigned)w.e0 + (unsigned)lo * (unsigned)w.db) / (unsigned)w.da);
                        yhi = w.b0 + w.sb * (int)(((unsigned)w.e0 + (unsigned)hi * (unsigned)w.db) / (unsigned)w.da);
                    } else {
                        ylo = w.a0 + w.sa * lo;
                        yhi = w.a0 + w.sa * hi;
                    }
                    const int r0 = min(ylo, yhi) - ty * TILE_H, r1 = max(ylo, yhi) - ty * TILE_H;
                    const unsigned m1 = r1 >= 31 ? 0xFFFFFFFFu : ((2u << r1) - 1u);
                    const unsigned m0 = (1u << r0) - 1u;
                    atomicOr(&s_rows[t], m1 & ~m0);
                });
            }
            __syncthreads();
            // exclusive scans: segment offsets and non-empty tile ranks (each thread owns a chunk)
            const int per = (nt + BIN_THREADS - 1) / BIN_THREADS;
            const int t0 = tid * per, t1 = min(nt, t0 + per);
            int csum = 0, cne = 0;
            for (int t = t0; t < t1; ++t) {
                csum += s_cnt[t];
                cne += s_cnt[t] > 0;
            }
            int seg_total, ne_total;
            int seg_pre = block_exscan(csum, s_wave, &seg_total);
            int ne_pre = block_exscan(cne, s_wave, &ne_total);
            if (tid == 0) {
                unsigned sb = atomicAdd(&wq->seg_used, (unsigned)seg_total);
                unsigned ib = atomicAdd(&wq->item_used, (unsigned)ne_total);
                if (sb + (unsigned)seg_total > seg_cap || ib + (unsigned)ne_total > item_cap) {
                    atomicAdd(&wq->overflow, 1u);
                    sb = 0xFFFFFFFFu;  // -> WHOLE item (the reserved ranges stay unused)
                }
                s_base[0] = sb;
                s_base[1] = ib;
            }
            __syncthreads();
            const unsigned seg_base = s_base[0], item_base = s_base[1];
            whole = seg_base == 0xFFFFFFFFu;
            if (whole) {
                // the item slots reserved above are read by hs_tile_kernel (it walks every slot below
                // item_used): fill the in-capacity ones with empty items (no segment, no row)
                for (int k = tid; k < ne_total; k += BIN_THREADS) {
                    const unsigned idx = item_base + (unsigned)k;
                    if (idx >= item_cap) break;
                    WorkItem it;
                    it.s = s;
                    it.lvl_kind = lvl | (ITEM_TILE << 8);
                    it.tile_xy = (unsigned)tx0 | ((unsigned)ty0 << 16);
                    it.begin_xy = begin_xy;
                    it.seg_begin = 0;
                    it.seg_count = 0;
                    it.mark_base = (unsigned)st.ord_base;
                    it.n = 0;
                    items[idx] = it;
                }
            }
            if (!whole) {
                // offsets + work items for this thread's chunk of tiles; s_off becomes the fill cursor
                for (int t = t0; t < t1; ++t) {
                    const int c = s_cnt[t];
                    s_off[t] = seg_pre;
                    if (c > 0) {
                        WorkItem it;
                        it.s = s;
                        it.lvl_kind = lvl | (ITEM_TILE << 8);
                        it.tile_xy = (unsigned)(tx0 + t % ntx) | ((unsigned)(ty0 + t / ntx) << 16);
                        it.begin_xy = begin_xy;
                        it.seg_begin = seg_base + (unsigned)seg_pre;
                        it.seg_count = (unsigned)c;
                        it.mark_base = (unsigned)st.ord_base;
                        it.n = s_rows[t];  // tile items: touched-row mask
                        items[item_base + (unsigned)ne_pre] = it;
                        ++ne_pre;
                    }
                    seg_pre += c;
                }
                __syncthreads();
                // pass 2: scatter segments {beam | lo<<16, hi}
                for (int b = tid; b < n; b += BIN_THREADS) {
                    unsigned r = rays[b];
                    if (r == RAY_INVALID) continue;
                    RayWalk w = ray_walk(x0, y0, (int)(r & 0xFFFFu), (int)(r >> 16));
                    for_each_segment(w, [&](int tx, int ty, int lo, int hi) {
                        const int slot = atomicAdd(&s_off[(ty - ty0) * ntx + (tx - tx0)], 1);
                        segs[seg_base + (unsigned)slot] = make_uint4((unsigned)b | ((unsigned)lo << 16), (unsigned)hi, r, 0u);
                    });
                }
            }
        }
        if (whole && tid == 0) {
            const unsigned k = atomicAdd(&wq->whole_used, 1u);
            WorkItem it;
            it.s = s;
            it.lvl_kind = lvl | (ITEM_WHOLE << 8);
            it.tile_xy = (unsigned)tx0 | ((unsigned)ty0 << 16);
            it.begin_xy = begin_xy;
            it.seg_begin = (unsigned)ntx | ((unsigned)nty << 16);
            it.seg_count = 0;
            it.mark_base = (unsigned)st.ord_base;
            it.n = (unsigned)n;
            wholes[k] = it;
        }
        __syncthreads();
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        Ltot += __shfl_xor(Ltot, off, 64);
        Rtot += __shfl_xor(Rtot, off, 64);
    }
    if ((tid & 63) == 0 && Rtot) {
        atomicAdd(&state[s].step_cells, Ltot);
        atomicAdd(&state[s].tot_cells, Ltot);
        atomicAdd(&state[s].tot_rays, Rtot);
    }
}

#ifndef S2D_TILE_MINW
#define S2D_TILE_MINW 1
#endif
// Diagnostic build only (-DS2D_STAMPS): per-phase s_memtime sums of hs_tile_kernel, wave 0 of each
// workgroup: [0] wait+clear, [1] raster, [2] apply, [3] tiles, [4] workgroup lifetime.
__device__ unsigned long long g_stamps[8];
#ifdef S2D_STAMPS
#define S2D_STAMP(v) do { __builtin_amdgcn_sched_barrier(0); v = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define S2D_STAMP(v) do { } while (0)
#endif

// lds_barrier (defined with the match kernel): waits for this wave's LDS operations (lgkmcnt) but not
// for its global loads/stores (__syncthreads' release fence would also drain vmcnt, serialising the
// prefetched cell loads and the previous tile's stores into every barrier).

// Tile kernel: ONE WAVE per workgroup and per tile, so there is no workgroup barrier and many tiles
// are in flight per CU (latency, not issue, bounds this phase).  Workgroup w takes items w, w+G, ...
// (G = grid); the next item and its first 64 segments are loaded one tile ahead.
//   LDS: two key arrays per tile, rows padded to 65 words (vertical neighbours on different banks);
//        key = (0xFFFF - gen) << 16 | beam, gen = 1 + tiles processed by this wave, so atomicMin
//        overwrites stale keys of earlier tiles and no per-tile clear is needed.
//   raster: one segment per lane (closed-form start, Bresenham increments), blind LDS atomicMin.
//        (Flattening the (segment, step) pairs over the lanes was measured 1.9x slower: its serial
//        LDS reads are not hidden at this occupancy.)
//   apply: only the tile rows flagged in the item's row mask are loaded (issued at tile start,
//        overlapping the raster); touched cells are stored; nothing waits for the stores.
constexpr int TILE_THREADS = 64;
constexpr int LDS_STRIDE = TILE + 1;
constexpr int TILE_WORDS = TILE_H * LDS_STRIDE;
static_assert(TILE_H <= 32, "row masks are 32-bit");

__global__ void __launch_bounds__(TILE_THREADS, S2D_TILE_MINW)
hs_tile_kernel(FleetGeom geom, float *__restrict__ cells, const StreamState *__restrict__ state,
               const unsigned *__restrict__ rays_g, const uint4 *__restrict__ segs, const WorkItem *__restrict__ items,
               const WorkItem *__restrict__ wholes, const WorkQueue *__restrict__ wq, int max_points)
{
    __shared__ __attribute__((aligned(16))) unsigned s_hit[TILE_WORDS];
    __shared__ __attribute__((aligned(16))) unsigned s_free[TILE_WORDS];
    const unsigned n_items = wq->item_used < wq->item_cap ? wq->item_used : wq->item_cap;
    const unsigned n_total = n_items + wq->whole_used;
    const int lane = threadIdx.x;
    const float lf = geom.lf, lo = geom.lo;
    unsigned long long ts0 = 0, ta = 0, tb = 0, tc = 0, td = 0, acc0 = 0, acc1 = 0, acc2 = 0, ntiles = 0;
    S2D_STAMP(ts0);
    for (int k = lane; k < TILE_WORDS; k += TILE_THREADS) {
        s_hit[k] = 0xFFFFFFFFu;
        s_free[k] = 0xFFFFFFFFu;
    }
    unsigned gen = 1;  // gen 0's key prefix 0xFFFF would alias the 0xFFFFFFFF fill
    unsigned it = blockIdx.x;
    WorkItem nxt;
    uint4 sg_nxt = make_uint4(0, 0, RAY_INVALID, 0);
    if (it < n_total) {
        nxt = it < n_items ? items[it] : wholes[it - n_items];
        if ((nxt.lvl_kind >> 8) == ITEM_TILE && (unsigned)lane < nxt.seg_count) sg_nxt = segs[nxt.seg_begin + lane];
    }
    for (; it < n_total; it += gridDim.x) {
        S2D_STAMP(ta);
        const WorkItem item = nxt;
        const uint4 sg_cur = sg_nxt;
        const unsigned itn = it + gridDim.x;
        if (itn < n_total) nxt = itn < n_items ? items[itn] : wholes[itn - n_items];  // prefetch item
        const int s = item.s;
        const int lvl = item.lvl_kind & 0xFF;
        const int kind = item.lvl_kind >> 8;
        const LevelGeom &g = geom.lv[lvl];
        // hot ordinals of currMarkFreeIndex / currMarkOccIndex (:120-121; hector_internal.h ORD_OFF)
        const unsigned short mark_free = (unsigned short)item.mark_base;
        const unsigned short mark_occ = (unsigned short)(item.mark_base + 1u);
        float *lvw = cells + (size_t)s * geom.stream_words + g.word_offset;
        const int x0 = (int)(item.begin_xy & 0xFFFFu), y0 = (int)(item.begin_xy >> 16);
        const int ttx0 = (int)(item.tile_xy & 0xFFFFu), tty0 = (int)(item.tile_xy >> 16);
        const int ntx = kind == ITEM_TILE ? 1 : (int)(item.seg_begin & 0xFFFFu);
        const int nty = kind == ITEM_TILE ? 1 : (int)(item.seg_begin >> 16);
        const unsigned rowmask = kind == ITEM_TILE ? item.n : 0xFFFFFFFFu;
        for (int tt = 0; tt < ntx * nty; ++tt) {
            if (gen == 0xFFFFu) {  // key space exhausted: reset (never reached at realistic sizes)
                for (int k = lane; k < TILE_WORDS; k += TILE_THREADS) {
                    s_hit[k] = 0xFFFFFFFFu;
                    s_free[k] = 0xFFFFFFFFu;
                }
                gen = 1;
            }
            const unsigned gkey = (0xFFFFu - gen) << 16;
            const int X0 = (ttx0 + tt % ntx) * TILE, Y0 = (tty0 + tt / ntx) * TILE_H;
            const int gx = X0 + lane;
            const bool colok = gx < g.sx;
            // this tile's contiguous block: log-odds plane, then the 16-bit ordinal plane
            float *tl = lvw + (size_t)((ttx0 + tt % ntx) + (tty0 + tt / ntx) * g.tiles_x) * TILE_BLOCK_WORDS;
            unsigned short *tu = reinterpret_cast<unsigned short *>(tl + ORD_OFF);
            float cl[TILE_H];
#pragma unroll
            for (int row = 0; row < TILE_H; ++row) {
                const int gy = Y0 + row;
                if (((rowmask >> row) & 1u) && colok && gy < g.sy) cl[row] = tl[tile_cell(lane, row)];
            }
            S2D_STAMP(tb);
            bool any = false;
            if (kind == ITEM_TILE) {
                any = item.seg_count > 0;
                uint4 sg = sg_cur;
                for (unsigned k = lane; k < item.seg_count; k += TILE_THREADS) {
                    if (k != (unsigned)lane) sg = segs[item.seg_begin + k];
                    const unsigned key = gkey | (sg.x & 0xFFFFu);
                    RayWalk w = ray_walk(x0, y0, (int)(sg.z & 0xFFFFu), (int)(sg.z >> 16));
                    const int slo = (int)(sg.x >> 16), shi = (int)sg.y;
                    const unsigned num = (unsigned)w.e0 + (unsigned)slo * (unsigned)w.db;
                    const int qq = (int)(num / (unsigned)w.da);
                    int err = (int)(num - (unsigned)qq * (unsigned)w.da);
                    const int la = w.x_major ? 1 : LDS_STRIDE;
                    const int lb = w.x_major ? LDS_STRIDE : 1;
                    int li = (w.a0 + w.sa * slo - (w.x_major ? X0 : Y0)) * la + (w.b0 + w.sb * qq - (w.x_major ? Y0 : X0)) * lb;
                    const int da_step = w.sa * la, db_step = w.sb * lb;
                    const int ifree = min(shi, w.da - 1);
                    for (int i = slo; i <= ifree; ++i) {
                        atomicMin(&s_free[li], key);  // bresenhamCellFree (:302-312)
                        li += da_step;
                        err += w.db;
                        if (err >= w.da) {
                            err -= w.da;
                            li += db_step;
                        }
                    }
                    if (shi == w.da) atomicMin(&s_hit[li], key);  // end cell (:265-266)
                }
            } else {
                // fallback for oversized scans: every ray against this tile (closed-form step range)
                const unsigned *rays = rays_g + ((size_t)s * geom.levels + lvl) * max_points;
                const int n = (int)item.n;
                const int X1 = X0 + TILE, Y1 = Y0 + TILE_H;
                for (int b = lane; b < n; b += TILE_THREADS) {
                    const unsigned r = rays[b];
                    if (r == RAY_INVALID) continue;
                    const int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
                    if (max(x0, x1) < X0 || min(x0, x1) >= X1 || max(y0, y1) < Y0 || min(y0, y1) >= Y1) continue;
                    RayWalk w = ray_walk(x0, y0, x1, y1);
                    int lo_i, hi_i;
                    bool in = w.x_major ? walk_range(w, X0, X1, Y0, Y1, lo_i, hi_i)
                                        : walk_range(w, Y0, Y1, X0, X1, lo_i, hi_i);
                    if (!in) continue;
                    any = true;
                    const unsigned key = gkey | (unsigned)b;
                    const unsigned num = (unsigned)w.e0 + (unsigned)lo_i * (unsigned)w.db;
                    const int qq = (int)(num / (unsigned)w.da);
                    int err = (int)(num - (unsigned)qq * (unsigned)w.da);
                    const int la = w.x_major ? 1 : LDS_STRIDE;
                    const int lb = w.x_major ? LDS_STRIDE : 1;
                    int li = (w.a0 + w.sa * lo_i - (w.x_major ? X0 : Y0)) * la + (w.b0 + w.sb * qq - (w.x_major ? Y0 : X0)) * lb;
                    const int ifree = min(hi_i, w.da - 1);
                    for (int i = lo_i; i <= ifree; ++i) {
                        atomicMin(&s_free[li], key);
                        li += w.sa * la;
                        err += w.db;
                        if (err >= w.da) {
                            err -= w.da;
                            li += w.sb * lb;
                        }
                    }
                    if (hi_i == w.da) atomicMin(&s_hit[li], key);
                }
            }
            // prefetch the next item's first segments (the item load was issued at the top)
            if (tt == ntx * nty - 1 && itn < n_total && (nxt.lvl_kind >> 8) == ITEM_TILE &&
                (unsigned)lane < nxt.seg_count)
                sg_nxt = segs[nxt.seg_begin + lane];
            S2D_STAMP(tc);
            if (__any(any)) {
                unsigned touched = 0;
                // apply: lane = column -> 256 B / 512 B coalesced row accesses
#pragma unroll
                for (int row = 0; row < TILE_H; ++row) {
                    const int gy = Y0 + row;
                    if (!((rowmask >> row) & 1u) || !colok || gy >= g.sy) continue;
                    const unsigned hk = s_hit[row * LDS_STRIDE + lane];
                    const unsigned fk = s_free[row * LDS_STRIDE + lane];
                    const bool hit = (hk & 0xFFFF0000u) == gkey;
                    const bool fre = (fk & 0xFFFF0000u) == gkey;
                    if (!hit && !fre) continue;
                    float l = cl[row];
                    unsigned short upd;
                    if (!hit) {
                        l = l + lf;        // updateSetFree (GridMapLogOdds.h:120-124)
                        upd = mark_free;
                    } else {
                        if (fre && (fk & 0xFFFFu) < (hk & 0xFFFFu)) {
                            l = l + lf;    // bresenhamCellFree by an earlier beam
                            l = l - lf;    // updateUnsetFree (GridMapLogOdds.h:126-129)
                        }
                        if (l < 50.0f) l = l + lo;  // updateSetOccupied (:108-114)
                        upd = mark_occ;
                    }
                    tl[tile_cell(lane, row)] = l;
                    tu[tile_cell(lane, row)] = upd;
                    ++touched;
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) touched += __shfl_xor(touched, off, 64);
                if (lane == 0 && touched)
                    atomicAdd(&const_cast<StreamState *>(state)[s].tot_touched, (unsigned long long)touched);
            }
            ++gen;
            S2D_STAMP(td);
            acc0 += tb - ta;
            acc1 += tc - tb;
            acc2 += td - tc;
            ntiles += 1;
            ta = td;
        }
    }
#ifdef S2D_STAMPS
    unsigned long long te;
    S2D_STAMP(te);
    if (lane == 0) {
        atomicAdd(&g_stamps[0], acc0);
        atomicAdd(&g_stamps[1], acc1);
        atomicAdd(&g_stamps[2], acc2);
        atomicAdd(&g_stamps[3], ntiles);
        atomicAdd(&g_stamps[4], te - ts0);
    }
#else
    (void)ts0; (void)acc0; (void)acc1; (void)acc2; (void)ntiles; (void)tb; (void)tc; (void)td;
#endif
}

// ------------------------------------------------- k2 (default): per-(stream, level) grid update
// Default update path (SLAM2D_UPDATE=binned selects the bin + tile kernels above).  One 256-thread
// workgroup per (stream, level); the level's rays (packed end cells) stay in LDS.  For each
// 64 x TILE_H tile of the scan's bounding box:
//   (1) raster: every ray whose fan group can reach the tile clips itself to the tile (closed-form
//       Bresenham step range) and marks LDS: atomicMin(first_free, beam) per free step,
//       atomicMin(first_hit, beam) at its end cell -- blind atomics, no read-modify-write chain;
//   (2) apply: one coalesced read-modify-write per 4-cell quad holding a mark, applying the
//       reference's float sequence per cell: free only: l + lf; hit: ((l + lf) - lf) if an earlier
//       beam freed it, then + lo if l < 50.
// This equals running bresenhamCellFree / bresenhamCellOcc (:302-330) beam by beam.
//
// Fan groups: beams b with the same b / 64 (one wave's lanes in one pass) share a bounding box
// (origin + their end cells, computed once); a tile outside a group's box is skipped by the whole
// wave with one scalar test.  Laser scans are angle-ordered, so a group is a narrow fan.
#ifndef S2D_UPD_STRIDE
#define S2D_UPD_STRIDE 68
#endif
// LDS words per tile row: 16-B rows (the apply reads and restores a quad's marks as one uint4) whose
// stride is not a multiple of 32 banks.  (67, odd, spreads a column of cells over all 32 banks of an
// atomic's lane group instead of 8, but the raster's conflicts are mostly lanes on the SAME word, which
// no stride changes -- tools/lds_sim.py: 2 % fewer raster LDS cycles -- and the unaligned quads cost the
// apply more: measured 0.005 ms slower.)
constexpr int UPD_STRIDE = S2D_UPD_STRIDE;
#ifndef S2D_UPD_PRIO
#define S2D_UPD_PRIO 0  // 1: hs_update_kernel raises a wave's priority by its share of the tile's fan groups (A/B)
#endif
#ifndef S2D_APPLY_FAST
#define S2D_APPLY_FAST 1  // 0: every marked quad takes the full apply_cell sequence (A/B)
#endif
#ifndef S2D_UPD_TH
#define S2D_UPD_TH (8 * S2D_UPD_WAVES)  // 32 rows with 4 waves, 64 with 8: every thread owns two quads of a tile
#endif
#ifndef S2D_UPD_MINB
#define S2D_UPD_MINB 8  // __launch_bounds__ minimum: 8 waves per SIMD, which caps the VGPRs at 64 (full occupancy; with 8-wave
                        // workgroups the value 4 let the compiler settle for 7 waves per SIMD, i.e. 3 workgroups per CU)
#endif
constexpr int UPD_TH = S2D_UPD_TH;                    // LDS tile height (a multiple of the storage TILE_H)
static_assert(UPD_TH % TILE_H == 0, "an LDS tile covers whole storage tiles");
constexpr int UPD_TILE_WORDS = UPD_TH * UPD_STRIDE;   // one LDS mark array
// r * UPD_STRIDE for a tile row r in [0, UPD_TH): the mask shows the compiler a 16-bit operand, so it
// selects the full-rate v_mul_u32_u24 (r * 68 of an int of unknown range, and even __mul24 or a
// shift-and-add it recombined, became a quarter-rate v_mul_lo_u32)
__device__ __forceinline__ int lds_row(int r) { return (int)(((unsigned)r & 0xFFFFu) * (unsigned)UPD_STRIDE); }
static_assert(UPD_STRIDE % 4 == 0 && UPD_STRIDE >= TILE, "quad-aligned LDS rows");
constexpr int UPD_QUADS = TILE * UPD_TH / 4 / UPD_THREADS;  // apply quads per thread per tile

// Tile marks: ONE LDS word per tile cell, lowered with blind atomicMin of a beam EVENT code
//   free step of beam b -> 2b + 1,    end (hit) cell of beam b -> 2b,
// plus one hit bit per cell.  The word ends as the earliest event at the cell in beam order (the
// order updateByScan walks the beams).  A beam never frees its own end cell, so with the hit bit
// set an odd word means a lower-index beam freed the cell before the first beam that hits it, an
// even word that the hit came first -- all that bresenhamCellFree / bresenhamCellOcc (:302-330)
// depend on within one scan.  A quad's marks are carried in registers as 12 bits: bit c "marked",
// bit 4 + c "odd event word", bit 8 + c "hit" for its cells c = 0..3.
// GridMapLogOddsFunctions (GridMapLogOdds.h:108-129) applied to one marked cell:
// bit k of m set ? a : b, as a bitwise select on the float bits (no compare, no exec-mask branch)
// The apply's stores: plain, or non-temporal (S2D_NT_STORE=1: a written cell is next touched one scan later,
// after ~3.5 GB of other traffic, so keeping its line in L2 / the Infinity Cache buys nothing)
#ifndef S2D_NT_STORE
#define S2D_NT_STORE 0
#endif
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef int nt_i4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void upd_store(float4 *p, float4 v)
{
#if S2D_NT_STORE
    const nt_f4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<nt_f4 *>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ void upd_store(int4 *p, int4 v)
{
#if S2D_NT_STORE
    const nt_i4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<nt_i4 *>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ void upd_store(int *p, int v)
{
#if S2D_NT_STORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__device__ __forceinline__ float bit_select(unsigned m, int k, float a, float b)
{
    const int sel = ((int)(m << (31 - k))) >> 31;  // 0 or -1
    return __int_as_float((__float_as_int(a) & sel) | (__float_as_int(b) & ~sel));
}

// A quad's mark bits as hs_update_kernel carries them from the mark read to the apply.
//   S2D_PACK_PERM 1 (default): the quad's four event words gathered by two byte permutes and one bit-field
//   insert -- bit 7 + 8 c set when cell c is unmarked (the top bit of W_NONE; an event 2 b + {0, 1} is below
//   2^31), bit QB_OD(c) the low bit of its event (odd: freed before its first hit), bit 1 + c its hit bit
//   (rotated out of the row's hit word), all other bits don't-care: 6 VALU per quad instead of ~24 for
//   the twelve compares / selects / shifts that built the compact nibbles.  A hit cell is always marked
//   (its atomicMin of 2 b), so the hit and odd bits need no masking with the marks.
//   0: the compact nibbles, bits c / 4 + c / 8 + c = marked / odd / hit (A/B).
#ifndef S2D_PACK_PERM
#define S2D_PACK_PERM 1
#endif
#if S2D_PACK_PERM
__device__ __forceinline__ constexpr int qb_un(int c) { return 7 + 8 * c; }
__device__ __forceinline__ constexpr int qb_od(int c) { return c < 2 ? 16 + 8 * c : 8 * (c - 2); }
__device__ __forceinline__ constexpr int qb_hit(int c) { return 1 + c; }
constexpr unsigned QB_UNMASK = 0x80808080u, QB_HITMASK = 0x1Eu;
__device__ __forceinline__ unsigned qb_pack(uint4 m, unsigned hitw, int s)  // s: the quad's bit in hitw
{
    // P: bytes x.b3 y.b3 x.b0 y.b0 (unmarked x 7, y 15; odd x 16, y 24); Q: z.b0 w.b0 z.b3 w.b3 (odd z 0, w 8;
    // unmarked z 23, w 31)
    const unsigned P = __builtin_amdgcn_perm(m.y, m.x, 0x04000703u);
    const unsigned Q = __builtin_amdgcn_perm(m.w, m.z, 0x07030400u);
    const unsigned R = (P & 0x01018080u) | (Q & ~0x01018080u);
    const unsigned h = __builtin_amdgcn_alignbit(hitw, hitw, (unsigned)(s - 1) & 31u);  // bits s..s+3 -> 1..4
    return (h & QB_HITMASK) | (R & ~QB_HITMASK);
}
__device__ __forceinline__ bool qb_any(unsigned mb) { return (mb & QB_UNMASK) != QB_UNMASK; }
__device__ __forceinline__ bool qb_all(unsigned mb) { return (mb & QB_UNMASK) == 0u; }
__device__ __forceinline__ unsigned qb_count(unsigned mb) { return __popc(~mb & QB_UNMASK); }
__device__ __forceinline__ bool qb_cell(unsigned mb, int c) { return !((mb >> qb_un(c)) & 1u); }
__device__ __forceinline__ unsigned qb_hits(unsigned mb) { return mb & QB_HITMASK; }
__device__ __forceinline__ float qb_sel_marked(unsigned mb, int c, float a, float b) { return bit_select(mb, qb_un(c), b, a); }
#else
__device__ __forceinline__ constexpr int qb_od(int c) { return 4 + c; }
__device__ __forceinline__ constexpr int qb_hit(int c) { return 8 + c; }
__device__ __forceinline__ unsigned qb_pack(uint4 m, unsigned hitw, int s)
{
    const unsigned h = (hitw >> s) & 15u;
    const unsigned mk = (unsigned)(m.x != W_NONE) | ((unsigned)(m.y != W_NONE) << 1) | ((unsigned)(m.z != W_NONE) << 2) |
                        ((unsigned)(m.w != W_NONE) << 3);
    const unsigned od = (m.x & 1u) | ((m.y & 1u) << 1) | ((m.z & 1u) << 2) | ((m.w & 1u) << 3);
    return mk | ((od & mk) << 4) | ((h & mk) << 8);
}
__device__ __forceinline__ bool qb_any(unsigned mb) { return (mb & 15u) != 0u; }
__device__ __forceinline__ bool qb_all(unsigned mb) { return (mb & 15u) == 15u; }
__device__ __forceinline__ unsigned qb_count(unsigned mb) { return __popc(mb & 15u); }
__device__ __forceinline__ bool qb_cell(unsigned mb, int c) { return (mb >> c) & 1u; }
__device__ __forceinline__ unsigned qb_hits(unsigned mb) { return (mb >> 8) & 15u; }
__device__ __forceinline__ float qb_sel_marked(unsigned mb, int c, float a, float b) { return bit_select(mb, c, a, b); }
#endif

__device__ __forceinline__ float apply_cell(float l, unsigned odd, unsigned hit, float lf, float lo)
{
    if (!hit) return l + lf;   // updateSetFree (:120-124)
    if (odd) {
        l = l + lf;            // bresenhamCellFree by an earlier beam
        l = l - lf;            // updateUnsetFree (:126-129)
    }
    if (l < 50.0f) l = l + lo; // updateSetOccupied (:108-114)
    return l;
}

// word offset of the quad at (c4, row) of the LDS tile (c4 % 4 == 0: 4 contiguous cells of a block row)
// inside the level's tiled storage, relative to the LDS tile's first storage tile (rows past TILE_H
// continue in the storage tile below)
__device__ __forceinline__ int upd_off(int row, int c4, int tiles_x)
{
    if constexpr (UPD_TH == TILE_H) return tile_cell(c4, row);
    return (row / TILE_H) * tiles_x * TILE_BLOCK_WORDS + tile_cell(c4, row % TILE_H);
}

constexpr int UPD_HIT_WORDS = UPD_TH * (TILE / 32);                  // one hit bit per tile cell
constexpr int UPD_MARK_WORDS = (UPD_TILE_WORDS + UPD_HIT_WORDS + 3) & ~3;

constexpr int UPD_FIXED_WORDS = 2 * UPD_MARK_WORDS + 4;  // two mark buffers + 4 spare words; then rays, fan-group boxes

// the free mark of one raster step: blind LDS atomicMin of the event code
__device__ __forceinline__ void upd_mark(unsigned *p, unsigned ev) { atomicMin(p, ev); }
// 32-bit LDS byte address of an LDS pointer, and back (the walk carries addresses in packed registers)
typedef __attribute__((address_space(3))) unsigned lds_u32;
__device__ __forceinline__ unsigned lds_addr(unsigned *p) { return (unsigned)(size_t)(lds_u32 *)p; }
__device__ __forceinline__ unsigned *lds_ptr(unsigned a) { return (unsigned *)(lds_u32 *)(size_t)a; }

__device__ __forceinline__ int lane_rank(unsigned long long m)  // set lanes below this one
{
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Fan groups: the 64 beams a wave rasters together.  S2D_FAN_STRIDE 1 (default): 64 consecutive beams
// (a 16 deg fan at 0.25 deg), lane l walking beam 2 (l % 32) + l / 32: each 32-lane half of an LDS
// atomic (its banking group) spans the whole fan, and with the odd lanes walking backwards (see the
// raster) the forward lanes of a half are 1 deg apart instead of 0.25 -- near the scan origin fewer
// lanes land on one word (tools/lds_sim.py: 0.66 vs 0.75 of the consecutive order's raster LDS cycles).
// 4: beams 256 G + 4 k + w for wave w of super-group G (a 64 deg fan, 1 deg apart), so that near the
// scan origin the lanes of one LDS atomic address distinct cells -- measured slower (round 2, 0.82 vs
// 0.78 ms): the wider fans lose more to culling than the conflicts cost.
#ifndef S2D_FAN_STRIDE
#define S2D_FAN_STRIDE 1
#endif
__device__ __forceinline__ int fan_beam(int b0, int lane)  // b0 = 256 G + 64 w
{
#if S2D_FAN_STRIDE == 4
    return (b0 & ~255) + 4 * lane + ((b0 >> 6) & 3);
#else
    return b0 + 2 * (lane & 31) + (lane >> 5);
#endif
}
__host__ __device__ constexpr int fan_groups(int max_points)
{
    return ((max_points + UPD_THREADS - 1) / UPD_THREADS) * UPD_WAVES;
}
constexpr int UPD_GROUP_WORDS = 4;  // LDS words per fan group: its bounding box

// Grid: for level l, upd_parts[l] x count blocks (level-major, then part, then stream); part p of a
// level draws the tiles t = p, p + parts, ... of the scan's tile box (t row-major over the box).
// RREG > 0: scans of at most RREG * 256 points keep each lane's packed rays (one per fan group it
// rasters) in registers instead of an LDS array of max_points words -- 4.3 KB less LDS per workgroup
// at 1081 beams, 8 instead of 7 workgroups per CU (the kernel's VGPRs allow 8).  RREG = 0: rays in LDS.
// The rays are five named registers picked by selects on the wave-uniform fan-group index (an array
// or a struct indexed by it ends up in scratch).
constexpr int UPD_RREG = (1280 + UPD_THREADS - 1) / UPD_THREADS;  // scans of <= 1280 (4 waves) / 1536 (8) points
static_assert(UPD_RREG <= 5, "five ray registers at most");
template <int RREG>
__global__ void __launch_bounds__(UPD_THREADS, S2D_UPD_MINB)
hs_update_kernel(FleetGeom geom, float *__restrict__ cells, StreamState *__restrict__ state,
                 const float2 *__restrict__ xy, int xy_stride, const float2 *__restrict__ mc, int mc_stride,
                 int stream_begin, int count, int max_points, const UpdList *__restrict__ wl,
                 UpdList *__restrict__ wl_next, int ncu)
{
    extern __shared__ __attribute__((aligned(16))) unsigned smem[];
    // two mark buffers (tile i rasters into buffer i & 1 while tile i - 1's cells are applied),
    // each UPD_TILE_WORDS event words + UPD_HIT_WORDS hit bits; then 4 spare words, rays, fan boxes
    // "tile has a mark" per buffer: a plain LDS array (a volatile pointer into smem loses the LDS address
    // space -- flat accesses with a vmcnt(0) wait that drains the loads the pipeline keeps in flight);
    // lds_barrier's memory clobber orders the accesses
    __shared__ unsigned s_any[2];
    unsigned *rays = smem + UPD_FIXED_WORDS;               // max_points packed end cells (RREG == 0)
    int4 *gbox = reinterpret_cast<int4 *>(rays + (RREG > 0 ? 0 : ((max_points + 3) & ~3)));  // per fan group: x0 y0 x1 y1
    static_assert(RREG == 0 || RREG == UPD_RREG, "RayRegs holds UPD_RREG rays");
    // RREG > 0: this lane's ray of fan group k = b0 / 256
    unsigned rr0 = RAY_INVALID, rr1 = RAY_INVALID, rr2 = RAY_INVALID, rr3 = RAY_INVALID, rr4 = RAY_INVALID;
    const int lane = threadIdx.x & 63;
    __shared__ int s_bbox[4];

    // level-major block order: every stream's level 0 (the largest) is dispatched first
    int lvl = 0, idx = (int)blockIdx.x, parts, part, local;
    if (wl) {
        // the U streams the match kernel listed, split by U (not by the batch size): with the node's
        // map-update gate only a fraction of the streams update, and they get the whole grid
        const int U = wl->count;
        if (blockIdx.x == 0 && threadIdx.x == 0) wl_next->count = 0;
        int pl[MAX_LEVELS];
        upd_split(U, ncu, geom.levels, pl, geom.upd_minp);
        while (lvl + 1 < geom.levels && idx >= pl[lvl] * U) idx -= pl[lvl++] * U;
        if (idx >= pl[lvl] * U) return;  // the grid is sized for the largest split (host)
        parts = pl[lvl];
        part = idx / U;
        local = wl->stream[idx - part * U];
    } else {
        while (lvl + 1 < geom.levels && idx >= geom.upd_parts[lvl] * count) idx -= geom.upd_parts[lvl++] * count;
        parts = geom.upd_parts[lvl];
        part = idx / count;
        local = idx - part * count;
    }
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    clk_stamp(geom.clk, 1, true);
    const LevelGeom &g = geom.lv[lvl];
    // level 0: this step's DataContainer; levels >= 1: the stored one of the last match
    // (MapRepMultiMap::updateByScan, MapRepMultiMap.h:181-188; equal to this step's after a match)
    const int n = lvl == 0 ? st.n : st.mc_n;
    const int tid = threadIdx.x;
    float *lvw = cells + (size_t)s * geom.stream_words + g.word_offset;

    const RayFrame fr = ray_frame(g, st, lvl == 0 ? st.origo : st.mc_origo);
    const int x0 = fr.bxi, y0 = fr.byi;
    if (tid == 0) {
        s_bbox[0] = x0; s_bbox[1] = y0; s_bbox[2] = x0; s_bbox[3] = y0;
    }
    __syncthreads();
    int bx0 = x0, by0 = y0, bx1 = x0, by1 = y0;
    unsigned long long L = 0, R = 0;
    const float2 *pts = lvl == 0 ? xy + (size_t)local * xy_stride : mc + (size_t)s * mc_stride;
    // the wave's first beam in a scalar register: the fan-group loops and the ray-register selects below
    // then compile to scalar control (tid & ~63 in a VGPR made them divergent loops with exec-mask code)
    const int wave_beam0 = __builtin_amdgcn_readfirstlane(tid & ~63);
    for (int b0 = wave_beam0; (b0 & ~(UPD_THREADS - 1)) < n; b0 += UPD_THREADS) {   // wave-uniform trip count
        const int b = fan_beam(b0, lane);
        unsigned r = RAY_INVALID;
        if (b < n) {
            r = make_ray(g, fr, pts[b]);
            if constexpr (RREG == 0) rays[b] = r;
        }
        if constexpr (RREG > 0) {
            const int k = (int)((unsigned)b0 / UPD_THREADS);
            rr0 = k == 0 ? r : rr0;
            rr1 = k == 1 ? r : rr1;
            rr2 = k == 2 ? r : rr2;
            rr3 = (RREG > 3 && k == 3) ? r : rr3;  // (8 waves: three registers)
            rr4 = (RREG > 4 && k == 4) ? r : rr4;
        }
        int gx0 = x0, gy0 = y0, gx1 = x0, gy1 = y0;  // fan group box: origin + valid ends
        if (r != RAY_INVALID) {
            const int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
            gx0 = min(gx0, x1); gy0 = min(gy0, y1); gx1 = max(gx1, x1); gy1 = max(gy1, y1);
            const int adx = abs(x1 - x0), ady = abs(y1 - y0);
            L += (unsigned long long)(max(adx, ady) + 1);
            R += 1;
        }
        bx0 = min(bx0, gx0); by0 = min(by0, gy0); bx1 = max(bx1, gx1); by1 = max(by1, gy1);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            gx0 = min(gx0, __shfl_xor(gx0, off, 64));
            gy0 = min(gy0, __shfl_xor(gy0, off, 64));
            gx1 = max(gx1, __shfl_xor(gx1, off, 64));
            gy1 = max(gy1, __shfl_xor(gy1, off, 64));
        }
        if (lane == 0) gbox[b0 >> 6] = make_int4(gx0, gy0, gx1, gy1);
    }
    if (R) {
        atomicMin(&s_bbox[0], bx0); atomicMin(&s_bbox[1], by0);
        atomicMax(&s_bbox[2], bx1); atomicMax(&s_bbox[3], by1);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        L += __shfl_xor(L, off, 64);
        R += __shfl_xor(R, off, 64);
    }
    if (lane == 0 && R && part == 0) {
        atomicAdd(&state[s].step_cells, L);
        atomicAdd(&state[s].tot_cells, L);
        atomicAdd(&state[s].tot_rays, R);
    }
    // both mark buffers start clean (afterwards each tile's readers restore what its raster marked)
    for (int k = tid; k < 2 * UPD_MARK_WORDS / 4; k += UPD_THREADS)
        reinterpret_cast<uint4 *>(smem)[k] = (k % (UPD_MARK_WORDS / 4)) < UPD_TILE_WORDS / 4
                                                 ? make_uint4(W_NONE, W_NONE, W_NONE, W_NONE)
                                                 : make_uint4(0u, 0u, 0u, 0u);
    if (tid < 2) s_any[tid] = 0u;
    if (!__syncthreads_or(R != 0)) {  // no ray drawn on this level
        clk_stamp(geom.clk, 1, false);
        return;
    }
    const int tx0 = s_bbox[0] / TILE, ty0 = s_bbox[1] / UPD_TH;
    const int tx1 = s_bbox[2] / TILE, ty1 = s_bbox[3] / UPD_TH;
    // hot ordinals of currMarkFreeIndex (:120) / currMarkOccIndex (:121): hector_internal.h ORD_OFF
    const unsigned mark_free = (unsigned)st.ord_base;  // (+1: currMarkOccIndex, the hit bit added per cell)
    const float lf = geom.lf, lo = geom.lo;
    unsigned touched = 0;

    const int ntx = tx1 - tx0 + 1, ntiles = ntx * (ty1 - ty0 + 1);
    const int nfans = ((n + UPD_THREADS - 1) / UPD_THREADS) * (UPD_THREADS / 64);  // groups with a box in gbox
    const int my_tiles = ntiles > part ? (ntiles - part + parts - 1) / parts : 0;
    // Two-stage pipeline over this workgroup's tiles t_i = part + i * parts, ONE barrier per tile:
    //   iteration i: raster tile i into buffer i & 1 -> apply tile i - 1 from registers (its cell
    //   loads were issued one raster earlier) -> barrier -> read tile i's marks into registers, issue the
    //   loads of its marked quads and restore the words just read to "no mark".
    // Every mark word is read and restored by the thread that owns its quad (a hit-bit word by one
    // lane of the 8 that read it, all in one wave, after the read), so a buffer is clean again before
    // the barrier of iteration i + 1 that precedes its next raster; a tile without marks wrote nothing.
    // s_any[buf] holds the number (i + 1) of the last tile of that buffer that had a mark, so it needs no
    // reset.  The barrier only waits for LDS traffic (lds_barrier), so the loads and the previous tile's
    // stores stay in flight across it.  (Skipping the tiles no fan group reaches outright -- no barrier,
    // buffers alternating over the rastered tiles only -- measured no faster: the skeleton of an empty
    // tile is now a ballot, and the extra state cost the kernel two spilled VGPRs.)
    float4 ql[UPD_QUADS];      // pending tile: log-odds of the marked quads (loads in flight)
    unsigned qb[UPD_QUADS];    // pending tile: 12 mark bits per quad (see apply_cell)

    float *pend_tl = nullptr;  // pending tile's storage block (null: nothing pending)
    // tile t = part + i * parts of the box (row-major): its column and row are carried from tile to tile
    // (a division of t by the box width per tile was ~20 scalar instructions of signed-division code)
    int tcol = part % ntx, trow = part / ntx;
    for (int ii = 0; ii <= my_tiles; ++ii) {
        const int i = __builtin_amdgcn_readfirstlane(ii);  // uniform (the compiler had put it in a VGPR)
        const int qtid = tid;  // (the quads' offsets derive from it)
        const int ty = ty0 + trow, tx = tx0 + tcol;
        tcol += parts;
        while (tcol >= ntx) {
            tcol -= ntx;
            ++trow;
        }
        const int X0 = tx * TILE, Y0 = ty * UPD_TH;
        const int X1 = X0 + TILE, Y1 = Y0 + UPD_TH;
        const int buf = i & 1;
        unsigned *marks = smem + buf * UPD_MARK_WORDS;
        unsigned *hitb = marks + UPD_TILE_WORDS;
        if (i < my_tiles) {
            unsigned anyv = 0u;  // a VGPR flag: no exec-mask merging of a divergent bool
            // the fan groups whose box meets the tile, one bit each: lane f tests group f, one ballot (the
            // scalar box test of every group of the wave on every tile cost ~20 SALU a time, most of them
            // on tiles no fan reaches); groups past the first 64 (scans of > 4096 points) test their box alone
            unsigned long long fm;
            {
                int ol = lane;  // opaque: the lane's box address is not hoisted into a VGPR held across tiles
                asm volatile("" : "+v"(ol));
                const int4 gb = gbox[min(ol, nfans - 1)];
                fm = __ballot((int)(ol < nfans) & (int)(gb.z >= X0) & (int)(gb.x < X1) & (int)(gb.w >= Y0) &
                              (int)(gb.y < Y1));
            }
            {
                // this wave's groups (fi = wave + 4 k) among the first 64 that meet the tile, one set bit each:
                // the loop visits only those (scalar find-first-set), then the groups past 64 test their box
                unsigned long long gm = fm & ((UPD_WAVES == 8 ? 0x0101010101010101ull : 0x1111111111111111ull)
                                              << (wave_beam0 >> 6));
                int b0x = wave_beam0 + 64 * 64;  // groups >= 64 (scans of > 4096 points)
                if constexpr (S2D_UPD_PRIO) {
                    // the waves with more of this tile's groups issue first: the four meet at the tile's barrier,
                    // so the busiest one is the workgroup's path (back to 0 after the raster)
                    const int c = __popcll(gm);
                    if (c >= 3) __builtin_amdgcn_s_setprio(3);
                    else if (c == 2) __builtin_amdgcn_s_setprio(2);
                    else if (c == 1) __builtin_amdgcn_s_setprio(1);
                }
                for (;;) {
                    int b0;
                    if (gm) {
                        b0 = __builtin_ctzll(gm) << 6;
                        gm &= gm - 1ull;
                    } else {
                        if ((b0x & ~(UPD_THREADS - 1)) >= n) break;
                        b0 = b0x;
                        b0x += UPD_THREADS;
                        const int4 gb = gbox[b0 >> 6];
                        const int gx0 = __builtin_amdgcn_readfirstlane(gb.x), gy0 = __builtin_amdgcn_readfirstlane(gb.y);
                        const int gx1 = __builtin_amdgcn_readfirstlane(gb.z), gy1 = __builtin_amdgcn_readfirstlane(gb.w);
                        if (gx1 < X0 || gx0 >= X1 || gy1 < Y0 || gy0 >= Y1) continue;
                    }
                    const int b = fan_beam(b0, lane);
                    unsigned r;
                    if constexpr (RREG > 0) {
                        const int k = (int)((unsigned)b0 / UPD_THREADS);
                        r = k == 0 ? rr0 : (k == 1 ? rr1 : (k == 2 ? rr2 : (k == 3 ? rr3 : rr4)));
                    }
                    else r = b < n ? rays[b] : RAY_INVALID;
                    // the tests below are combined with bitwise ors: one divergent branch (exec-mask save,
                    // test, restore: SALU work) per early exit instead of one per condition
                    const int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
                    if ((int)(r == RAY_INVALID) | (int)(max(x0, x1) < X0) | (int)(min(x0, x1) >= X1) |
                        (int)(max(y0, y1) < Y0) | (int)(min(y0, y1) >= Y1))
                        continue;
                    if (x1 >= X0 && x1 < X1 && y1 >= Y0 && y1 < Y1) {  // bresenhamCellOcc (:266)
                        const int c = (y1 - Y0) * TILE + (x1 - X0);
                        atomicMin(&marks[lds_row(y1 - Y0) + (x1 - X0)], 2u * (unsigned)b);
                        atomicOr(&hitb[c >> 5], 1u << (c & 31));
                        anyv = 1u;
                    }
                    const RayWalk w = ray_walk(x0, y0, x1, y1);
                    // the tile in (major, minor) order, selected before ONE clip (lanes of a fan that straddles
                    // a diagonal differ in x_major)
                    const int A0 = w.x_major ? X0 : Y0, A1 = w.x_major ? X1 : Y1;
                    const int B0 = w.x_major ? Y0 : X0, B1 = w.x_major ? Y1 : X1;
                    int lo_i, hi_i;
                    const bool met = walk_range(w, A0, A1, B0, B1, lo_i, hi_i);
                    if (hi_i > w.da - 1) hi_i = w.da - 1;  // steps 0..da-1 are freed (:277-298)
                    if ((int)!met | (int)(lo_i > hi_i)) continue;
                    anyv = 1u;
                    const int scnt = hi_i - lo_i + 1;     // free steps of this beam inside the tile
                    // Odd lanes walk their segment backwards, from hi_i down to lo_i (the same cells; the step
                    // below is its own inverse in g = da - 1 - f): at one instruction neighbouring beams then sit
                    // at different radii, so near the scan origin half as many lanes hit one LDS word (the
                    // atomics to one address serialise).
                    const bool bwd = (lane & 1) != 0;
                    const int s0 = bwd ? hi_i : lo_i;
                    // (s0, db, q, da < 2^15 and the tile offsets < 2^7: 24-bit multiplies throughout)
                    const unsigned num = (unsigned)w.e0 + __umul24((unsigned)s0, (unsigned)w.db);
                    unsigned rem;
                    const int q = (int)udiv_small(num, (unsigned)w.da, rem);
                    const int err = (int)rem;
                    const unsigned ev = 2u * (unsigned)b + 1u;
                    // LDS index of step s0 and its increments along the major / minor axis
                    const int la = w.x_major ? 1 : UPD_STRIDE;
                    const int lb = w.x_major ? UPD_STRIDE : 1;
                    const int ia = w.a0 + (w.sa > 0 ? s0 : -s0) - A0, ib = w.b0 + (w.sb > 0 ? q : -q) - B0;
                    const int li = __mul24(ia, la) + __mul24(ib, lb);
                    // incremental walk, f = da - 1 - error_b in [0, da) (backwards: g = error_b), packed with
                    // the LDS byte address of the step's mark word into ONE register, V = f << 18 | address
                    // (LDS addresses < 2^18, f < da <= 2^14: the host sends larger maps to the binned kernels,
                    // upd_single_ok): the subtraction of db << 18 borrows exactly when
                    // f < db -- the minor axis steps -- and one select + add then moves both fields.  Three
                    // VALU per step plus the address mask, instead of five.
                    const int dab1 = w.sa > 0 ? 4 * la : -4 * la;              // (no quarter-rate 32-bit multiply)
                    const int dab21 = dab1 + (w.sb > 0 ? 4 * lb : -4 * lb);
                    const int dab = bwd ? -dab1 : dab1, dab2 = bwd ? -dab21 : dab21;
                    const int fw0 = bwd ? err : w.da - 1 - err;
                    const unsigned vdn = (unsigned)w.db << 18;
                    const unsigned vk_major = (unsigned)dab;                            // f -= db, no minor step
                    const unsigned vk_minor = ((unsigned)w.da << 18) + (unsigned)dab2;  // f += da - db, minor step
                    unsigned v = ((unsigned)fw0 << 18) + lds_addr(marks) + (unsigned)li * 4u;
                    int k = 0;
#define S2D_WSTEP                                                          \
    do {                                                                   \
        upd_mark(lds_ptr(v & 0x3FFFFu), ev); /* bresenhamCellFree */       \
        unsigned vn_;                                                      \
        const bool c_ = __builtin_sub_overflow(v, vdn, &vn_);              \
        v = vn_ + (c_ ? vk_minor : vk_major);                              \
    } while (0)
                    // eight steps per trip (the loop control -- a scalar counter, the exec mask update and
                    // the branch -- is per trip), then at most one trip of four and of two
                    for (; k + 7 < scnt; k += 8) {
                        S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP;
                    }
                    if (k + 3 < scnt) {
                        S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP;
                        k += 4;
                    }
                    if (k + 1 < scnt) {
                        S2D_WSTEP; S2D_WSTEP;
                        k += 2;
                    }
#undef S2D_WSTEP
                    if (k < scnt) upd_mark(lds_ptr(v & 0x3FFFFu), ev);
                }
            }
            if (S2D_UPD_PRIO) __builtin_amdgcn_s_setprio(0);
            if (__ballot(anyv != 0u) && lane == 0) s_any[buf] = (unsigned)(i + 1);
        }
        // every pending load first (only LDS work came after them): with the loads conditional the compiler
        // cannot count them and would otherwise wait on each quad's stores before the next.  Waited for on
        // every iteration, with or without a pending tile (then only old stores remain, long drained): the
        // compiler then knows no load into ql is outstanding past this point, and the next tile's address
        // arithmetic in those registers needs no wait -- conditional, it cost a vmcnt(0) at the next loads,
        // i.e. a wait for all of this apply's stores.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        if (pend_tl) {
            // apply the previous tile: log-odds of every marked cell, and its hot ordinal (see below); the
            // ordinal plane is never read -- a cell's stored index always predates this scan's marks
            // (currUpdateIndex += 3 per scan)
            unsigned short *tu = reinterpret_cast<unsigned short *>(pend_tl + ORD_OFF);
#pragma unroll
            for (int j = 0; j < UPD_QUADS; ++j) {
                const unsigned mb = qb[j];
                if (!qb_any(mb)) continue;
                const int qi = qtid + j * UPD_THREADS;
                const unsigned o = (unsigned)upd_off(qi >> 4, (qi & 15) << 2, g.tiles_x);
                // the quad's ordinals, in 16-bit units from this tile block's plane: an LDS tile taller than a storage
                // tile continues in the block below, whose plane is one block (2 x TILE_BLOCK_WORDS halves) further
                const unsigned ou = UPD_TH == TILE_H ? o
                                                     : o + (unsigned)((qi >> 4) / TILE_H * g.tiles_x * TILE_BLOCK_WORDS);
                float4 v = ql[j];
                const float lv[4] = {v.x, v.y, v.z, v.w};
                float nv[4];
                unsigned uv[4];
                if (S2D_APPLY_FAST && !__any(qb_hits(mb))) {
                    // no end cell in this quad slot of the whole wave (about three quarters of level 0's on the
                    // synthetic scans): every marked cell is free only -- updateSetFree alone, two VALU per cell
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        nv[c] = qb_sel_marked(mb, c, lv[c] + lf, lv[c]);
                        uv[c] = mark_free;
                    }
                } else {
                    // apply_cell on the 4 cells without branches: every candidate value computed, then picked by
                    // bit selects on the sign-extended mark bits (v_bfe_i32 + v_bfi_b32: two VALU per choice; the
                    // branchy form compiled to exec-mask code around each cell)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float l = lv[c];
                        const float t = l + lf;                       // updateSetFree
                        const float u = t - lf;                       // ... then updateUnsetFree
                        const float h = bit_select(mb, qb_od(c), u, l);  // an earlier beam freed the hit cell
                        const float oc = h < 50.0f ? h + lo : h;         // updateSetOccupied
                        nv[c] = qb_sel_marked(mb, c, bit_select(mb, qb_hit(c), oc, t), l);
                        uv[c] = mark_free + ((mb >> qb_hit(c)) & 1u);
                    }
                }
                // log-odds: the whole quad was loaded, so it is stored whole (one instruction; unmarked
                // cells rewrite their own value); ordinals: the quad's 8 bytes when every cell is marked, else
                // per marked cell (its unmarked cells were never read)
                upd_store(reinterpret_cast<float4 *>(&pend_tl[o]), make_float4(nv[0], nv[1], nv[2], nv[3]));
                if (qb_all(mb)) {
                    *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        if (qb_cell(mb, c)) tu[ou + (unsigned)c] = (unsigned short)uv[c];
                }
                touched += qb_count(mb);
            }
            pend_tl = nullptr;
        }
        if (i < my_tiles) {
            lds_barrier();  // tile i's marks complete
            if (s_any[buf] == (unsigned)(i + 1)) {
                // thread owns quads q = tid + j * 256 (16 quads per 64-cell row); cells outside the map
                // (padding of edge tiles) never carry marks
                pend_tl = lvw + (size_t)(tx + ty * (UPD_TH / TILE_H) * g.tiles_x) * TILE_BLOCK_WORDS;
#pragma unroll
                for (int j = 0; j < UPD_QUADS; ++j) {
                    const unsigned qi = (unsigned)qtid + j * UPD_THREADS;
                    const int row = (int)(qi >> 4), c4 = (int)((qi & 15u) << 2);
                    const int mw = lds_row(row) + c4;
                    const uint4 m = *reinterpret_cast<const uint4 *>(&marks[mw]);
                    qb[j] = qb_pack(m, hitb[row * (TILE / 32) + (c4 >> 5)], c4 & 31);
                    const bool mk = qb_any(qb[j]);
                    // unsigned 32-bit offset: the load takes the scalar-base + VGPR-offset form, so nothing but
                    // the load itself writes its destination registers
                    if (mk) ql[j] = *reinterpret_cast<const float4 *>(pend_tl + (unsigned)upd_off(row, c4, g.tiles_x));
                    // restore: the quad's event words (read by this thread only) and, by the first of
                    // the 8 lanes sharing it, the hit-bit word (its readers are this wave's lanes, whose
                    // read above precedes this write)
                    if (mk) *reinterpret_cast<uint4 *>(&marks[mw]) = make_uint4(W_NONE, W_NONE, W_NONE, W_NONE);
                    if ((tid & 7) == 0) hitb[row * (TILE / 32) + (c4 >> 5)] = 0u;
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) touched += __shfl_xor(touched, off, 64);
    if (lane == 0 && touched) atomicAdd(&state[s].tot_touched, (unsigned long long)touched);
    clk_stamp(geom.clk, 1, false);
}

// ------------------------------- k2 (opt-in, SLAM2D_UPD_KERNEL=ring): ring-ordered grid update with ray cursors
// (the default update is the clip kernel hs_update_kernel above; hector_capi.hip upd_ring_ok)
// The same once-per-scan update as hs_update_kernel (tiles of 64 x UPD_TH cells, LDS event words + hit
// bits, the two-stage raster / apply pipeline, fan groups culled per tile with one ballot), with the
// per-(tile, ray) clip replaced by a cursor per ray.
//
// Tile order.  The tiles of the level's box are visited in RINGS around the tile of the scan's begin
// cell: ring k = the tiles at Chebyshev distance k (in tile units), and inside a ring by the secondary
// distance s = min(|dx|, |dy|).  Along a ray both tile coordinates move monotonically away from the
// begin tile (the ray starts inside it), so each tile change strictly increases (k, s) in lexicographic
// order: every ray meets its tiles in the visit order, one after the other.  So each lane keeps, per ray,
// the walk's position -- the next step i and the minor steps q before it -- and a tile visit starts where
// the previous one stopped: no clipping of the ray against the tile (round 3: ray_walk + walk_range + the
// start division, ~150 VALU per (tile, fan group) visit), only the exit of the tile (one division by db
// for the minor boundary, one by da for the minor steps taken).
// Parts: part p of a level takes a contiguous range of rings (split by tile count, ring_split); its
// cursors start at the first step of each ray inside its first ring (ray_cursor).
// Per ray two registers (scans of <= RING_GROUPS * 256 points; larger scans use hs_update_kernel<0>):
//   consts  = da | db << 14 | (x step < 0) << 28 | (y step < 0) << 29 | x major << 30   (0: no ray)
//   cursor  = i | q << 16: step i is next, q = its minor steps (i > da: the ray is done)
// (da, db < 2^14: maps of at most 16384 cells per side, upd_ring_ok).
// LDS tile height of the ring kernel: 32 rows with 256-thread workgroups (default), or 64 rows with 512-thread
// workgroups (S2D_RING_TH=64: a ray crosses fewer tiles; the same LDS and registers per wave, 2 quads per
// thread in the apply, 8 waves at every tile barrier)
#ifndef S2D_RING_TH
#define S2D_RING_TH 32
#endif
constexpr int RTH = S2D_RING_TH;
constexpr int RTHREADS = RTH == 64 ? 512 : 256;
constexpr int RWAVES = RTHREADS / 64;
static_assert(RTH % TILE_H == 0 && (RTH == 32 || RTH == 64), "ring tiles: 32 or 64 rows");
constexpr int RTILE_WORDS = RTH * UPD_STRIDE;                       // one LDS mark array
constexpr int RHIT_WORDS = RTH * (TILE / 32);                       // one hit bit per tile cell
constexpr int RMARK_WORDS = (RTILE_WORDS + RHIT_WORDS + 3) & ~3;
constexpr int RFIXED_WORDS = 2 * RMARK_WORDS + 4;                  // two mark buffers + 4 spare words; then fan boxes
constexpr int RQUADS = TILE * RTH / 4 / RTHREADS;                   // apply quads per thread per tile
constexpr unsigned long long RGROUP_MASK = RWAVES == 4 ? 0x1111111111111111ull : 0x0101010101010101ull;
constexpr int RING_GROUPS = (5 * 256 + RTHREADS - 1) / RTHREADS;    // fan groups per lane: scans of <= 1280 points
__host__ __device__ constexpr int ring_fan_groups(int max_points) { return ((max_points + RTHREADS - 1) / RTHREADS) * RWAVES; }
__host__ __device__ constexpr int ring_shmem_words(int max_points) { return RFIXED_WORDS + UPD_GROUP_WORDS * ring_fan_groups(max_points); }
// word offset of the quad at (c4, row) of the LDS tile in the level's tiled storage (see upd_off)
__device__ __forceinline__ int ring_off(int row, int c4, int tiles_x)
{
    if constexpr (RTH == TILE_H) return tile_cell(c4, row);
    return (row / TILE_H) * tiles_x * TILE_BLOCK_WORDS + tile_cell(c4, row % TILE_H);
}
constexpr unsigned CUR_DONE = 0xFFFFu;

__device__ __forceinline__ unsigned ray_consts(int x0, int y0, unsigned r)
{
    if (r == RAY_INVALID) return 0u;
    const int dx = (int)(r & 0xFFFFu) - x0, dy = (int)(r >> 16) - y0;
    const int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    const bool xm = adx >= ady;                                   // (:252)
    const unsigned da = (unsigned)(xm ? adx : ady), db = (unsigned)(xm ? ady : adx);
    // util::sign (UtilFunctions.h:55-58): sign(0) = -1
    return da | (db << 14) | ((unsigned)(dx <= 0) << 28) | ((unsigned)(dy <= 0) << 29) | ((unsigned)xm << 30);
}

// tiles of the box [tx0, tx1] x [ty0, ty1] within Chebyshev distance k of (ox, oy) (k < 0: none)
__device__ __forceinline__ int tiles_within(int k, int ox, int oy, int tx0, int tx1, int ty0, int ty1)
{
    if (k < 0) return 0;
    const int w = min(tx1, ox + k) - max(tx0, ox - k) + 1, h = min(ty1, oy + k) - max(ty0, oy - k) + 1;
    return (w > 0 && h > 0) ? w * h : 0;
}

// The cursor of a ray at its first step inside ring >= K (K = 0: step 0).  Along x the ring starts
// Dx cells from the begin cell (the ray's x moves away from the begin tile), along y Dy; a major-axis
// distance D is reached at step D, a minor-axis one at the first i with q(i) = floor((e0 + i db) / da) >= D.
__device__ __forceinline__ unsigned ray_cursor(unsigned C, int K, int x0, int y0, int ox, int oy)
{
    const int da = (int)(C & 0x3FFFu), db = (int)((C >> 14) & 0x3FFFu);
    if (da == 0) return CUR_DONE;
    if (K == 0) return 0u;
    const bool sxn = (C >> 28) & 1u, syn = (C >> 29) & 1u, xm = (C >> 30) & 1u;
    const int e0 = da >> 1;
    const int Dx = sxn ? x0 - ((ox - K) * TILE + TILE - 1) : (ox + K) * TILE - x0;
    const int Dy = syn ? y0 - ((oy - K) * RTH + RTH - 1) : (oy + K) * RTH - y0;
    const int INF = 0x7FFF;
    const int Dma = xm ? Dx : Dy, Dmi = xm ? Dy : Dx;
    const int im = Dma <= da ? Dma : INF;
    const int in = (Dmi <= db) ? (Dmi * da - e0 + db - 1) / db : INF;  // db >= Dmi >= 1 here
    const int i = min(im, in);
    if (i > da) return CUR_DONE;
    const int q = (e0 + i * db) / da;
    return (unsigned)i | ((unsigned)q << 16);
}

// One fan group's visit of the tile at (X0, Y0) for this lane's ray (consts C, cursor S): if the cursor
// is inside the tile, the ray's steps from there to where it leaves the tile (or ends) are marked --
// free steps with event 2b + 1 (bresenhamCellFree, OccGridMapBase.h:302-312), the end cell with 2b and
// its hit bit (bresenhamCellOcc, :314-330) -- and the cursor moves past them.  Direction handling is
// select-free where it can be: with the sign masks mx, my (0 or -1), a signed step is (t ^ m) - m and
// the steps left to a tile edge are l ^ 63 or l ^ 31 (63 - l, 31 - l for l in range) or l itself.
__device__ __forceinline__ void ring_visit(unsigned C, unsigned &S, unsigned b, int rx0, int ry0, unsigned *marks,
                                           unsigned *hitb, unsigned &anyv, int bm)
{
    const int i = (int)(S & 0xFFFFu);
    const int q = (int)(S >> 16);
    const int da = (int)(C & 0x3FFFu);
    const int db = (int)((C >> 14) & 0x3FFFu);
    const int mx = ((int)(C << 3)) >> 31, my = ((int)(C << 2)) >> 31;  // bits 28 / 29: x / y step < 0
    const bool xm = (C >> 30) & 1u;
    // the cursor's cell relative to the tile (rx0 = begin x - X0, ry0 = begin y - Y0)
    const int ix = xm ? i : q, iy = xm ? q : i;
    const int lx = rx0 + ((ix ^ mx) - mx), ly = ry0 + ((iy ^ my) - my);
    // done rays (i > da) and cursors outside the tile: nothing here (one branch)
    if ((int)(i > da) | (int)((unsigned)lx >= (unsigned)TILE) | (int)((unsigned)ly >= (unsigned)RTH)) return;
    // steps after this one that stay inside the tile along x / y
    const int rx = lx ^ ((TILE - 1) & ~mx), ry = ly ^ ((RTH - 1) & ~my);
    const int ra = xm ? rx : ry, rb = xm ? ry : rx;
    const int e = (da >> 1) + (int)__umul24((unsigned)i, (unsigned)db) - (int)__umul24((unsigned)q, (unsigned)da);
    // steps inside the tile, this one included: the major axis leaves after ra + 1, the walk ends at step
    // da, the minor axis leaves at the first step with rb + 1 minor steps: ceil(((rb + 1) da - e) / db)
    int n = min(ra + 1, da - i + 1);
    const unsigned dbs = db ? (unsigned)db : 1u;
    const unsigned nb = udiv_rcp(__umul24((unsigned)(rb + 1), (unsigned)da) - (unsigned)e + dbs - 1u, dbs,
                                 __builtin_amdgcn_rcpf((float)dbs));
    n = db ? min(n, (int)nb) : n;
    // the last step in the tile: its minor steps k after this one and its error el
    unsigned el;
    const int k = (int)udiv_small((unsigned)e + __umul24((unsigned)(n - 1), (unsigned)db), (unsigned)da, el);
    const int last = i + n - 1;
    const bool hit = last == da;
    anyv = 1u;
    // the cursor's next step: error el + db, a minor step iff it reaches da (a done ray keeps i = da + 1)
    S = (unsigned)(last + 1) | ((unsigned)(q + k + (int)(el + (unsigned)db >= (unsigned)da)) << 16);
    if (hit) {  // bresenhamCellOcc (:266): the end cell, n - 1 major and k minor steps from the cursor
        const int ta = xm ? n - 1 : k, tb = xm ? k : n - 1;
        const int lxl = lx + ((ta ^ mx) - mx), lyl = ly + ((tb ^ my) - my);
        const int c = lyl * TILE + lxl;
        atomicMin(&marks[lds_row(lyl) + lxl], 2u * b);
        atomicOr(&hitb[c >> 5], 1u << (c & 31));
    }
    const int nfree = n - (int)hit;
    if (nfree <= 0) return;
    // start of the walk: forward lanes (bm = 0) at the cursor; backward lanes (bm = -1) at the last free
    // step -- the last step, or the one before it when the last is the end cell (un-stepped: the end cell was
    // reached by a minor step iff el < db)
    const bool um = hit && el < (unsigned)db;
    const int ts = bm & (n - 1 - (int)hit);                       // major steps from the cursor
    const int ks = bm & (k - (int)um);                            // minor steps from the cursor
    const int es = bm ? (int)el - (hit ? db : 0) + (um ? da : 0) : da - 1 - e;  // g = error (bwd) / f (fwd)
    const int sxs = xm ? ts : ks, sys = xm ? ks : ts;
    const int lxs = lx + ((sxs ^ mx) - mx), lys = ly + ((sys ^ my) - my);
    // LDS byte steps along the major / minor axis, negated for backward lanes
    const int dx4 = (4 ^ mx) - mx, dy4 = ((4 * UPD_STRIDE) ^ my) - my;
    const int dab1 = xm ? dx4 : dy4, dab21 = dx4 + dy4;
    const int dab = (dab1 ^ bm) - bm, dab2 = (dab21 ^ bm) - bm;
    const unsigned vdn = (unsigned)db << 18;
    const unsigned vk_major = (unsigned)dab;
    const unsigned vk_minor = ((unsigned)da << 18) + (unsigned)dab2;
    unsigned v = ((unsigned)es << 18) + lds_addr(marks) + (unsigned)(lds_row(lys) + lxs) * 4u;
    const unsigned ev = 2u * b + 1u;
    int kk = 0;
#define S2D_WSTEP                                                          \
    do {                                                                   \
        upd_mark(lds_ptr(v & 0x3FFFFu), ev); /* bresenhamCellFree */       \
        unsigned vn_;                                                      \
        const bool c_ = __builtin_sub_overflow(v, vdn, &vn_);              \
        v = vn_ + (c_ ? vk_minor : vk_major);                              \
    } while (0)
    for (; kk + 7 < nfree; kk += 8) {
        S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP;
    }
    if (kk + 3 < nfree) {
        S2D_WSTEP; S2D_WSTEP; S2D_WSTEP; S2D_WSTEP;
        kk += 4;
    }
    if (kk + 1 < nfree) {
        S2D_WSTEP; S2D_WSTEP;
        kk += 2;
    }
#undef S2D_WSTEP
    if (kk < nfree) upd_mark(lds_ptr(v & 0x3FFFFu), ev);
}

// The ring range [kb, ke) of part p of `parts` for a box of `total` tiles: parts split the tiles of the
// box in ring order by count (every part's range is whole rings).
__device__ __forceinline__ void ring_split(int p, int parts, int kmax, int ox, int oy, int tx0, int tx1, int ty0,
                                           int ty1, int &kb, int &ke)
{
    kb = 0;
    ke = kmax + 1;
    if (parts <= 1) return;
    const int total = tiles_within(kmax, ox, oy, tx0, tx1, ty0, ty1);
    const int lo = (int)(((long long)total * p) / parts), hi = (int)(((long long)total * (p + 1)) / parts);
    // kb: the first ring whose preceding rings hold >= lo tiles (p = 0: ring 0); ke likewise for hi
    kb = p == 0 ? 0 : kmax + 1;
    ke = p == parts - 1 ? kmax + 1 : kmax + 1;
    for (int k = 0; k <= kmax; ++k) {
        const int before = tiles_within(k - 1, ox, oy, tx0, tx1, ty0, ty1);
        if (p > 0 && kb > kmax && before >= lo && k > 0) kb = k;
        if (p < parts - 1 && ke > kmax && before >= hi && k > 0) ke = k;
    }
    if (ke < kb) ke = kb;
}

// block-wide exclusive scan over the ring kernel's RTHREADS threads (s_wave: RWAVES ints)
__device__ __forceinline__ int ring_exscan(int v, int *s_wave, int *total)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(x, off, 64);
        if (lane >= off) x += t;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < RWAVES; ++k) {
        const int ws = s_wave[k];
        if (k < wave) base += ws;
        tot += ws;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// Weighted variant (default): ring k weighs RING_TILE_W per box tile plus one per ray that reaches it (the
// rays' end rings are histogrammed in LDS, s_rh[RING_HIST]; rings past the last bin count in it).  Inner
// rings hold few tiles but every ray's first steps, so a split by tiles alone left the inner part the
// heaviest.  All threads call it (two block barriers); s_cut[2] receives [kb, ke).
constexpr int RING_HIST = 128;
#ifndef S2D_RING_SPLIT_TILES
#define S2D_RING_SPLIT_TILES 0  // 1: split by tile count alone (A/B)
#endif
#ifndef S2D_RING_TILE_W
#define S2D_RING_TILE_W 64
#endif
__device__ __forceinline__ void ring_split_w(int p, int parts, int kmax, int ox, int oy, int tx0, int tx1, int ty0,
                                             int ty1, const unsigned *s_rh, int *s_wave, int *s_cut, int &kb, int &ke)
{
    const int tid = threadIdx.x;
    // thread k: ring k's weight; rays reaching ring k = rays whose end ring is >= k
    int w = 0;
    if (tid <= kmax) {
        const int kk = min(tid, RING_HIST - 1);
        unsigned reach = 0;
        for (int j = kk; j < RING_HIST; ++j) reach += s_rh[j];
        const int tk = tiles_within(tid, ox, oy, tx0, tx1, ty0, ty1) - tiles_within(tid - 1, ox, oy, tx0, tx1, ty0, ty1);
        w = S2D_RING_TILE_W * tk + (int)reach;
    }
    if (tid == 0) {
        s_cut[0] = p == 0 ? 0 : kmax + 1;
        s_cut[1] = kmax + 1;
    }
    int total;
    const int before = ring_exscan(w, s_wave, &total);  // weight of the rings < tid
    const int lo = (int)(((long long)total * p) / parts), hi = (int)(((long long)total * (p + 1)) / parts);
    if (tid >= 1 && tid <= kmax) {
        if (p > 0 && before >= lo) atomicMin(&s_cut[0], tid);
        if (p < parts - 1 && before >= hi) atomicMin(&s_cut[1], tid);
    }
    __syncthreads();
    kb = s_cut[0];
    ke = max(s_cut[1], kb);
}

// Next tile of the box in ring order: candidates (k, s, j), j = 0..7 the 8 tiles (+-k, +-s), (+-s, +-k),
// duplicates skipped (s == 0: odd j; s == k: j >= 4; k == 0: j = 0 only).  The caller knows how many
// tiles remain, so a candidate is always found.
struct RingIter {
    int k, s, j;
    int ox, oy, tx0, tx1, ty0, ty1;
    __device__ __forceinline__ void next(int &tx, int &ty)
    {
        for (;;) {
            if (++j == 8) {
                j = 0;
                if (++s > k) {
                    s = 0;
                    ++k;
                }
            }
            if (k == 0 && j != 0) continue;
            if ((s == 0 && (j & 1)) || (s == k && j >= 4)) continue;
            const int u = j < 4 ? k : s, v = j < 4 ? s : k;
            const int dx = ((j < 4 ? (j & 2) : (j & 1)) != 0) ? -u : u;
            const int dy = ((j < 4 ? (j & 1) : (j & 2)) != 0) ? -v : v;
            tx = ox + dx;
            ty = oy + dy;
            if (tx >= tx0 && tx <= tx1 && ty >= ty0 && ty <= ty1) return;
        }
    }
};

__global__ void __launch_bounds__(RTHREADS, S2D_UPD_MINB * 256 / RTHREADS)
hs_update_ring_kernel(FleetGeom geom, float *__restrict__ cells, StreamState *__restrict__ state,
                      const float2 *__restrict__ xy, int xy_stride, const float2 *__restrict__ mc, int mc_stride,
                      int stream_begin, int count, int max_points, const UpdList *__restrict__ wl,
                      UpdList *__restrict__ wl_next, int ncu)
{
    extern __shared__ __attribute__((aligned(16))) unsigned smem[];
    __shared__ unsigned s_any[2];
    __shared__ unsigned s_touched;
    __shared__ unsigned s_rh[RING_HIST];  // rays per end ring (ring_split_w)
    __shared__ int s_wave[RWAVES], s_cut[2];
    int4 *gbox = reinterpret_cast<int4 *>(smem + RFIXED_WORDS);  // per fan group: x0 y0 x1 y1
    const int lane = threadIdx.x & 63;
    __shared__ int s_bbox[4];

    int lvl = 0, idx = (int)blockIdx.x, parts, part, local;
    if (wl) {
        const int U = wl->count;
        if (blockIdx.x == 0 && threadIdx.x == 0) wl_next->count = 0;
        int pl[MAX_LEVELS];
        upd_split(U, ncu, geom.levels, pl, geom.upd_minp);
        while (lvl + 1 < geom.levels && idx >= pl[lvl] * U) idx -= pl[lvl++] * U;
        if (idx >= pl[lvl] * U) return;
        parts = pl[lvl];
        part = idx / U;
        local = wl->stream[idx - part * U];
    } else {
        while (lvl + 1 < geom.levels && idx >= geom.upd_parts[lvl] * count) idx -= geom.upd_parts[lvl++] * count;
        parts = geom.upd_parts[lvl];
        part = idx / count;
        local = idx - part * count;
    }
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    clk_stamp(geom.clk, 1, true);
    const LevelGeom &g = geom.lv[lvl];
    const int n = lvl == 0 ? st.n : st.mc_n;  // MapRepMultiMap::updateByScan (MapRepMultiMap.h:181-188)
    const int tid = threadIdx.x;
    float *lvw = cells + (size_t)s * geom.stream_words + g.word_offset;

    const RayFrame fr = ray_frame(g, st, lvl == 0 ? st.origo : st.mc_origo);
    const int x0 = fr.bxi, y0 = fr.byi;
    if (tid == 0) {
        s_bbox[0] = x0; s_bbox[1] = y0; s_bbox[2] = x0; s_bbox[3] = y0;
    }
    if (tid < RING_HIST) s_rh[tid] = 0u;
    __syncthreads();
    int bx0 = x0, by0 = y0, bx1 = x0, by1 = y0;
    unsigned long long L = 0, R = 0;
    const float2 *pts = lvl == 0 ? xy + (size_t)local * xy_stride : mc + (size_t)s * mc_stride;
    const int wave_beam0 = __builtin_amdgcn_readfirstlane(tid & ~63);
    const int wave = wave_beam0 >> 6;
    const int ox = x0 / TILE, oy = y0 / RTH;  // the begin tile (x0, y0 >= 0 whenever a ray is valid)
    unsigned Ck[RING_GROUPS], Sk[RING_GROUPS];
#pragma unroll
    for (int k = 0; k < RING_GROUPS; ++k) {
        Ck[k] = 0u;
        const int b0 = wave_beam0 + k * RTHREADS;
        if ((b0 & ~(RTHREADS - 1)) >= n) continue;  // uniform: every group of a started block gets its box
        const int b = fan_beam(b0, lane);
        const unsigned r = b < n ? make_ray(g, fr, pts[b]) : RAY_INVALID;
        Ck[k] = ray_consts(x0, y0, r);
        int gx0 = x0, gy0 = y0, gx1 = x0, gy1 = y0;  // fan group box: origin + valid ends
        if (r != RAY_INVALID) {
            const int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
            gx0 = min(gx0, x1); gy0 = min(gy0, y1); gx1 = max(gx1, x1); gy1 = max(gy1, y1);
            L += (unsigned long long)((Ck[k] & 0x3FFFu) + 1u);
            R += 1;
            if (parts > 1) {
                const int er = max(abs(x1 / TILE - ox), abs(y1 / RTH - oy));
                atomicAdd(&s_rh[min(er, RING_HIST - 1)], 1u);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            gx0 = min(gx0, __shfl_xor(gx0, off, 64));
            gy0 = min(gy0, __shfl_xor(gy0, off, 64));
            gx1 = max(gx1, __shfl_xor(gx1, off, 64));
            gy1 = max(gy1, __shfl_xor(gy1, off, 64));
        }
        // the wave's box from its (wave-uniform) group boxes
        bx0 = min(bx0, gx0); by0 = min(by0, gy0); bx1 = max(bx1, gx1); by1 = max(by1, gy1);
        if (lane == 0) gbox[b0 >> 6] = make_int4(gx0, gy0, gx1, gy1);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        L += __shfl_xor(L, off, 64);
        R += __shfl_xor(R, off, 64);
    }
    // one lane per wave: per-lane atomics here compiled to a scalar loop over the active lanes per word
    if (lane == 0 && R) {
        atomicMin(&s_bbox[0], bx0); atomicMin(&s_bbox[1], by0);
        atomicMax(&s_bbox[2], bx1); atomicMax(&s_bbox[3], by1);
    }
    if (lane == 0 && R && part == 0) {
        atomicAdd(&state[s].step_cells, L);
        atomicAdd(&state[s].tot_cells, L);
        atomicAdd(&state[s].tot_rays, R);
    }
    for (int k = tid; k < 2 * RMARK_WORDS / 4; k += RTHREADS)
        reinterpret_cast<uint4 *>(smem)[k] = (k % (RMARK_WORDS / 4)) < RTILE_WORDS / 4
                                                 ? make_uint4(W_NONE, W_NONE, W_NONE, W_NONE)
                                                 : make_uint4(0u, 0u, 0u, 0u);
    if (tid < 2) s_any[tid] = 0u;
    if (tid == 0) s_touched = 0u;
    if (!__syncthreads_or(R != 0)) {  // no ray drawn on this level
        clk_stamp(geom.clk, 1, false);
        return;
    }
    const int tx0 = s_bbox[0] / TILE, ty0 = s_bbox[1] / RTH;
    const int tx1 = s_bbox[2] / TILE, ty1 = s_bbox[3] / RTH;
    const int kmax = max(max(ox - tx0, tx1 - ox), max(oy - ty0, ty1 - oy));
    int kb = 0, ke = kmax + 1;
    if (parts > 1) {
#if S2D_RING_SPLIT_TILES
        ring_split(part, parts, kmax, ox, oy, tx0, tx1, ty0, ty1, kb, ke);
#else
        ring_split_w(part, parts, kmax, ox, oy, tx0, tx1, ty0, ty1, s_rh, s_wave, s_cut, kb, ke);
#endif
    }
    const int my_tiles = tiles_within(ke - 1, ox, oy, tx0, tx1, ty0, ty1) - tiles_within(kb - 1, ox, oy, tx0, tx1, ty0, ty1);
#pragma unroll
    for (int k = 0; k < RING_GROUPS; ++k) Sk[k] = ray_cursor(Ck[k], kb, x0, y0, ox, oy);
    // hot ordinals of currMarkFreeIndex (:120) / currMarkOccIndex (:121): hector_internal.h ORD_OFF
    const unsigned mark_free = (unsigned)st.ord_base;  // (+1: currMarkOccIndex, the hit bit added per cell)
    const float lf = geom.lf, lo = geom.lo;
    unsigned touched = 0;
    const int nfans = ((n + RTHREADS - 1) / RTHREADS) * (RTHREADS / 64);
    const int bm = -(lane & 1);  // odd lanes (bm = -1) walk their segments backwards (see hs_update_kernel)
    RingIter it;
    it.k = kb;
    it.s = 0;
    it.j = -1;
    it.ox = ox; it.oy = oy; it.tx0 = tx0; it.tx1 = tx1; it.ty0 = ty0; it.ty1 = ty1;

    float4 ql[RQUADS];
    unsigned qb[RQUADS];
    float *pend_tl = nullptr;
    for (int ii = 0; ii <= my_tiles; ++ii) {
        const int i = __builtin_amdgcn_readfirstlane(ii);
        const int buf = i & 1;
        unsigned *marks = smem + buf * RMARK_WORDS;
        unsigned *hitb = marks + RTILE_WORDS;
        int tx = 0, ty = 0;
        if (i < my_tiles) {
            it.next(tx, ty);
            const int X0 = tx * TILE, Y0 = ty * RTH;
            const int X1 = X0 + TILE, Y1 = Y0 + RTH;
            unsigned anyv = 0u;
            unsigned long long fm;
            {
                int ol = lane;
                asm volatile("" : "+v"(ol));
                const int4 gb = gbox[min(ol, nfans - 1)];
                fm = __ballot((int)(ol < nfans) & (int)(gb.z >= X0) & (int)(gb.x < X1) & (int)(gb.w >= Y0) &
                              (int)(gb.y < Y1));
            }
            const int rx0 = x0 - X0, ry0 = y0 - Y0;
            // this wave's groups (fi = wave + 4 k) that meet the tile, one set bit each (scalar find-first-set);
            // the visit exists once, its group's two registers picked and written back by scalar branches
            unsigned long long gm = fm & (RGROUP_MASK << wave);
            while (gm) {
                const int k = __builtin_ctzll(gm) / RWAVES;
                gm &= gm - 1ull;
                unsigned C = Ck[0], S = Sk[0];
#pragma unroll
                for (int kk = 1; kk < RING_GROUPS; ++kk)
                    if (k == kk) {
                        C = Ck[kk];
                        S = Sk[kk];
                    }
                const unsigned b = (unsigned)fan_beam(wave_beam0 + k * RTHREADS, lane);
                ring_visit(C, S, b, rx0, ry0, marks, hitb, anyv, bm);
#pragma unroll
                for (int kk = 0; kk < RING_GROUPS; ++kk)
                    if (k == kk) Sk[kk] = S;
            }
            if (__ballot(anyv != 0u) && lane == 0) s_any[buf] = (unsigned)(i + 1);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see hs_update_kernel
        if (pend_tl) {
            unsigned short *tu = reinterpret_cast<unsigned short *>(pend_tl + ORD_OFF);
            // the quads' offsets are recomputed per tile from an opaque copy of tid (a few VALU): hoisted out of
            // the tile loop they were held in registers the cursors need, and spilled
            int tq = tid;
            asm volatile("" : "+v"(tq));
#pragma unroll
            for (int j = 0; j < RQUADS; ++j) {
                const unsigned mb = qb[j];
                if (!(mb & 15u)) continue;
                const int qi = tq + j * RTHREADS;
                const unsigned o = (unsigned)ring_off(qi >> 4, (qi & 15) << 2, g.tiles_x);
                float4 v = ql[j];
                const float lv[4] = {v.x, v.y, v.z, v.w};
                float nv[4];
                unsigned uv[4];
                if (S2D_APPLY_FAST && !__any((mb >> 8) & 15u)) {
                    // no end cell in this quad slot of the whole wave (three quarters of level 0's, tools'
                    // density model): every marked cell is free only -- updateSetFree alone
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        nv[c] = bit_select(mb, c, lv[c] + lf, lv[c]);
                        uv[c] = mark_free;
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float l = lv[c];
                        const float t = l + lf;                       // updateSetFree
                        const float u = t - lf;                       // ... then updateUnsetFree
                        const float h = bit_select(mb, 4 + c, u, l);  // an earlier beam freed the hit cell
                        const float oc = h < 50.0f ? h + lo : h;      // updateSetOccupied
                        nv[c] = bit_select(mb, c, bit_select(mb, 8 + c, oc, t), l);
                        uv[c] = mark_free + ((mb >> (8 + c)) & 1u);
                    }
                }
                *reinterpret_cast<float4 *>(&pend_tl[o]) = make_float4(nv[0], nv[1], nv[2], nv[3]);
                if ((mb & 15u) == 15u) {
                    *reinterpret_cast<uint2 *>(&tu[o]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        if ((mb >> c) & 1u) tu[o + (unsigned)c] = (unsigned short)uv[c];
                }
                touched += __popc(mb & 15u);
            }
            pend_tl = nullptr;
        }
        if (i < my_tiles) {
            lds_barrier();  // tile i's marks complete
            if (s_any[buf] == (unsigned)(i + 1)) {
                pend_tl = lvw + (size_t)(tx + ty * (RTH / TILE_H) * g.tiles_x) * TILE_BLOCK_WORDS;
                int tq = tid;
                asm volatile("" : "+v"(tq));
#pragma unroll
                for (int j = 0; j < RQUADS; ++j) {
                    const unsigned qi = (unsigned)tq + j * RTHREADS;
                    const int row = (int)(qi >> 4), c4 = (int)((qi & 15u) << 2);
                    const int mw = lds_row(row) + c4;
                    const uint4 m = *reinterpret_cast<const uint4 *>(&marks[mw]);
                    const unsigned h = (hitb[row * (TILE / 32) + (c4 >> 5)] >> (c4 & 31)) & 15u;
                    const unsigned mk = (unsigned)(m.x != W_NONE) | ((unsigned)(m.y != W_NONE) << 1) |
                                        ((unsigned)(m.z != W_NONE) << 2) | ((unsigned)(m.w != W_NONE) << 3);
                    const unsigned od = (m.x & 1u) | ((m.y & 1u) << 1) | ((m.z & 1u) << 2) | ((m.w & 1u) << 3);
                    qb[j] = mk | ((od & mk) << 4) | ((h & mk) << 8);
                    if (mk) ql[j] = *reinterpret_cast<const float4 *>(pend_tl + (unsigned)ring_off(row, c4, g.tiles_x));
                    if (mk) {
                        // "no mark" from an opaque register: a hoisted all-ones quad was held across the loop
                        // and spilled (its reload waited for the quad loads just issued)
                        unsigned none = W_NONE;
                        asm volatile("" : "+v"(none));
                        *reinterpret_cast<uint4 *>(&marks[mw]) = make_uint4(none, none, none, none);
                    }
                    if ((tid & 7) == 0) hitb[row * (TILE / 32) + (c4 >> 5)] = 0u;
                }
            }
        }
    }
    // distinct cells written: summed in LDS (a shuffle reduction here had its lane addresses hoisted to the
    // kernel's start and spilled)
    if (touched) atomicAdd(&s_touched, touched);
    __syncthreads();
    if (tid == 0 && s_touched) atomicAdd(&state[s].tot_touched, (unsigned long long)s_touched);
    clk_stamp(geom.clk, 1, false);
}

// --------------------------------------------------------------------------- utility kernels
__global__ void hs_fill_cells_kernel(float *__restrict__ words, size_t n, size_t stream_words)
{
    // LogOddsCell::resetGridCell  H/map/GridMapLogOdds.h:76-80 : log-odds plane 0.0f, updateIndex -1 (the cold
    // plane -1, the hot ordinal plane 0 = "see the cold plane").  The plane of a word follows from its offset
    // inside its stream (levels start at multiples of a tile block; a per-stream pad, if any, is filled too and
    // never read)
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stream = i / stream_words, w = i - stream * stream_words;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t ds = stride / stream_words, dw = stride - ds * stream_words;
    for (; i < n; i += stride) {
        const unsigned tw = (unsigned)(w % (size_t)TILE_BLOCK_WORDS);
        if (tw >= (unsigned)COLD_OFF) reinterpret_cast<int *>(words)[i] = -1;
        else words[i] = 0.0f;  // log-odds 0.0f, and two zero ordinals per word
        w += dw;  // (stream, w) of i + stride without a division per word
        stream += ds;
        if (w >= stream_words) {
            w -= stream_words;
            ++stream;
        }
    }
}

// Ordinal sweep (hector_internal.h ORD_OFF): every non-zero hot ordinal of streams [stream_begin, +count) becomes
// its cell's updateIndex in the cold plane and is cleared; hs_ord_epoch_kernel then advances the streams' epochs.
// One workgroup per tile block (grid-stride); two ordinals per 4-byte word.
__global__ void __launch_bounds__(256) hs_ord_sweep_kernel(float *__restrict__ cells, const StreamState *__restrict__ state,
                                                           size_t stream_words, int tiles_per_stream, int stream_begin,
                                                           int count)
{
    const size_t nblk = (size_t)count * (size_t)tiles_per_stream;
    for (size_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const int s = stream_begin + (int)(b / (size_t)tiles_per_stream);
        const size_t t = b % (size_t)tiles_per_stream;
        float *tl = cells + (size_t)s * stream_words + t * TILE_BLOCK_WORDS;
        unsigned *hot = reinterpret_cast<unsigned *>(tl + ORD_OFF);
        int *cold = reinterpret_cast<int *>(tl + COLD_OFF);
        const int E = state[s].ord_epoch;
        for (int w = threadIdx.x; w < TILE_CELLS / 2; w += blockDim.x) {
            const unsigned hw = hot[w];
            if (!hw) continue;
            const unsigned h0 = hw & 0xFFFFu, h1 = hw >> 16;
            if (h0) cold[2 * w] = ord_index(h0, E);
            if (h1) cold[2 * w + 1] = ord_index(h1, E);
            hot[w] = 0u;
        }
    }
}

__global__ void hs_ord_epoch_kernel(StreamState *__restrict__ state, int stream_begin, int count)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < count) state[stream_begin + i].ord_epoch = state[stream_begin + i].cur_update_index / 3;
}

// HectorMappingRos::publishMap cell conversion  lesson4/src/hector_mapping/hector_slam.cc:287-304
// (tiled storage -> row-major int8)
__global__ void hs_publish_kernel(const float *__restrict__ lvw, LevelGeom g, int8_t *__restrict__ out)
{
    const size_t n = (size_t)g.sx * g.sy;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        const int x = (int)(i % g.sx), y = (int)(i / g.sx);
        const float l = lvw[cell_word(g, x, y)];
        out[i] = l < 0.0f ? (int8_t)0 : (l > 0.0f ? (int8_t)100 : (int8_t)-1);
    }
}

}  // namespace s2d
