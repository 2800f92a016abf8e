// hector_kernels.hip -- MI355X (gfx950) kernels for the Hector scan-to-map matcher and the
// once-per-scan Bresenham log-odds grid update (reference: lesson4/include/lesson4/hector_mapping/,
// abbreviated H/ below).  Host orchestration + C-ABI live in hector_capi.hip.
//
// Data layout in HBM (per context):
//   cells  : LogOddsCell {float l; int upd} (8 B, H/map/GridMapLogOdds.h:37-87), row-major
//            [stream][level][y][x]; a stream's levels are contiguous (stream_cells per stream).
//   state  : StreamState per stream (pose, last map-update pose, covariance, update indices).
//   points : float2 per beam in level-0 map scale, padded to xy_stride per stream.
//
// One step = one HectorSlamProcessor::update per stream (H/slam_main/HectorSlamProcessor.h:81-108):
//   k1 hs_match_kernel      one 256-thread workgroup per stream: all levels coarse->fine, all
//                           Gauss-Newton iterations, block reduction of H/b, 3x3 solve, gating.
//   k2 hs_update_kernel     one 256-thread workgroup per (stream, level): the scan's bounding box is
//                           walked in 64x64-cell tiles; each ray's cells inside a tile come from the
//                           closed-form Bresenham step range, the once-per-scan semantics of
//                           bresenhamCellFree/Occ (H/map/OccGridMapBase.h:302-330) are resolved in
//                           LDS, then touched cells get ONE coalesced 8-byte read-modify-write.
//                           No global atomics; see DESIGN.md "once-per-scan semantics".
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

// GridMapLogOddsFunctions::getGridProbability  H/map/GridMapLogOdds.h:136-140
__device__ __forceinline__ float cell_prob(float l)
{
    float odds = sdm_expf(l);
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

// --------------------------------------------------------------------------------- k1: match
// Per point: OccGridMapUtil::getCompleteHessianDerivs body (H/map/OccGridMapUtil.h:94-126) with
// interpMapValueWithDerivatives (:139-228).  Accumulates into acc[9] =
// {dTr0, dTr1, dTr2, H00, H11, H22, H01, H02, H12}.
__device__ __forceinline__ void point_terms(const LogOddsCell *__restrict__ cells, const LevelGeom &g, float tx,
                                            float ty, float cs, float sn, float px, float py, float *acc)
{
    float nsn = -sn;
    float x = tx + (cs * px + nsn * py);
    float y = ty + (sn * px + cs * py);
    float v, gx, gy;
    if ((x < 0.0f) || (x > g.lim[0]) || (y < 0.0f) || (y > g.lim[1])) {
        v = 0.0f;
        gx = 0.0f;
        gy = 0.0f;
    } else {
        int ix = (int)x, iy = (int)y;
        float fx = x - (float)ix;
        float fy = y - (float)iy;
        const LogOddsCell *c0 = cells + ((size_t)iy * g.sx + ix);
        const LogOddsCell *c2 = c0 + g.sx;
        float i0 = cell_prob(c0[0].l);
        float i1 = cell_prob(c0[1].l);
        float i2 = cell_prob(c2[0].l);
        float i3 = cell_prob(c2[1].l);
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
    float fun = 1.0f - v;
    // sinRot/cosRot (:87-88) are the same values as the transform's sn/cs
    float rot = ((-sn * px - cs * py) * gx + (cs * px - sn * py) * gy);
    acc[0] = acc[0] + gx * fun;
    acc[1] = acc[1] + gy * fun;
    acc[2] = acc[2] + rot * fun;
    acc[3] = acc[3] + gx * gx;
    acc[4] = acc[4] + gy * gy;
    acc[5] = acc[5] + rot * rot;
    acc[6] = acc[6] + gx * gy;
    acc[7] = acc[7] + gx * rot;
    acc[8] = acc[8] + gy * rot;
}

// One Gauss-Newton step, ScanMatcher::estimateTransformationLogLh (H/matcher/ScanMatcher.h:107-139).
// Every thread ends with the same H, b and estimate (xor-butterfly reductions are symmetric).
__device__ __forceinline__ void gn_step(const LogOddsCell *__restrict__ cells, const LevelGeom &g,
                                        const float2 *__restrict__ pts, int n, float f, float *est, float *H,
                                        float (*red)[MATCH_WAVES][9], int parity, int *clamps)
{
    const int tid = threadIdx.x;
    const float cs = sdm_cosf(est[2]);
    const float sn = sdm_sinf(est[2]);
    float acc[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k] = 0.0f;
    for (int i = tid; i < n; i += MATCH_THREADS) {
        float2 p = pts[i];
        point_terms(cells, g, est[0], est[1], cs, sn, p.x * f, p.y * f, acc);
    }
    // 64-lane xor butterfly, offsets 32..1
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] = acc[k] + __shfl_xor(acc[k], off, 64);
    }
    const int wave = tid >> 6;
    if ((tid & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) red[parity][wave][k] = acc[k];
    }
    __syncthreads();
    float s[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        // xor butterfly over the 4 wave sums: off 2 then off 1
        float a0 = red[parity][0][k] + red[parity][2][k];
        float a1 = red[parity][1][k] + red[parity][3][k];
        s[k] = a0 + a1;
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

__global__ void __launch_bounds__(MATCH_THREADS)
hs_match_kernel(FleetGeom geom, LogOddsCell *__restrict__ cells, StreamState *__restrict__ state,
                const float2 *__restrict__ xy, int xy_stride, const int *__restrict__ counts,
                const float2 *__restrict__ origo, const float *__restrict__ hints, int stream_begin, int mode,
                float *__restrict__ out_pose, float *__restrict__ out_cov)
{
    static_assert(MATCH_THREADS == 64 * MATCH_WAVES && MATCH_WAVES == 4, "reduction tree assumes 4 waves");
    __shared__ float red[2][MATCH_WAVES][9];
    const int local = blockIdx.x;
    const int s = stream_begin + local;
    StreamState &st = state[s];
    const LogOddsCell *scells = cells + (size_t)s * geom.stream_cells;
    const float2 *pts = xy + (size_t)local * xy_stride;
    const int n = counts[local];

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
    float cov[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) cov[k] = st.cov[k];
    int clamps = 0;
    int parity = 0;
    if (mode == MODE_PROCESS || mode == MODE_MATCH_ONLY) {
        // MapRepMultiMap::matchData  H/slam_main/MapRepMultiMap.h:144-167
        float tmp[3] = {hint[0], hint[1], hint[2]};
        for (int lvl = geom.levels - 1; lvl >= 0; --lvl) {
            const LevelGeom &g = geom.lv[lvl];
            const int iters = lvl == 0 ? 5 : 3;
            if (n == 0) continue;  // ScanMatcher::matchData returns the hint (ScanMatcher.h:65, :96)
            const LogOddsCell *lc = scells + g.cell_offset;
            float est[3], H[9];
            map_from_world(g, tmp, est);
            for (int it = 0; it <= iters; ++it) {
                gn_step(lc, g, pts, n, g.pts_scale, est, H, red, parity, &clamps);
                parity ^= 1;
            }
            est[2] = normalize_angle(est[2]);
#pragma unroll
            for (int k = 0; k < 9; ++k) cov[k] = H[k];
            world_from_map(g, est, tmp);
        }
        np_[0] = tmp[0];
        np_[1] = tmp[1];
        np_[2] = tmp[2];
    }
    if (threadIdx.x != 0) return;

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
    if (mode == MODE_PROCESS || mode == MODE_MATCH_ONLY) {
        unsigned long long it = 0;
        for (int lvl = 0; lvl < geom.levels; ++lvl) it += (lvl == 0 ? 6 : 4);
        st.tot_gn_points += it * (unsigned long long)n;
    }
    st.n = n;
    st.origo[0] = origo ? origo[local].x : 0.0f;
    st.origo[1] = origo ? origo[local].y : 0.0f;
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
        st.cur_update_index += 3;            // OccGridMapBase.h:167
        st.map_updates += 1;                 // GridMapBase::setUpdated (GridMapBase.h:333)
        st.step_cells = 0;
        st.tot_updates += 1;
    }
}

// ------------------------------------------------------------------------------- ray geometry
// OccGridMapBase::updateByScan (H/map/OccGridMapBase.h:118-161) + updateLineBresenhami (:220-267).
// Every ray starts at the common begin cell; a ray is stored as its end cell (packed y<<16 | x) or
// RAY_INVALID when updateByScan would skip it (begin == end :157, or begin/end outside :226-238).
constexpr unsigned RAY_INVALID = 0xFFFFFFFFu;
constexpr int TILE = 64;                 // tile edge (cells); a tile row = 64 x 8 B = 512 B
constexpr int TILE_CELLS = TILE * TILE;  // 4096 LDS words = 16 KB
constexpr int UPD_THREADS = 256;
// per-cell LDS word during one tile:
//   W_NONE            untouched
//   W_FREE            freed by >= 1 beam, hit by none
//   h | FF_BIT * f    hit; h = first hitting beam (< 65536); f = freed by some beam b < h first
constexpr unsigned W_NONE = 0xFFFFFFFFu;
constexpr unsigned W_FREE = 0xFFFFFFFEu;
constexpr unsigned FF_BIT = 0x10000u;

struct RayFrame {
    float mx, my, cs, sn;
    int bxi, byi;
};

__device__ __forceinline__ RayFrame ray_frame(const LevelGeom &g, const StreamState &st)
{
    RayFrame fr;
    float mp[3];
    map_from_world(g, st.upd_pose, mp);  // getMapCoordsPose (:124)
    fr.mx = mp[0];
    fr.my = mp[1];
    fr.cs = sdm_cosf(mp[2]);
    fr.sn = sdm_sinf(mp[2]);
    const float f = g.pts_scale;
    float ox = st.origo[0] * f, oy = st.origo[1] * f;
    float nsn = -fr.sn;
    float bx = fr.mx + (fr.cs * ox + nsn * oy);   // poseTransform * origo (:132)
    float by = fr.my + (fr.sn * ox + fr.cs * oy);
    fr.bxi = (int)(bx + 0.5f);                     // (:135)
    fr.byi = (int)(by + 0.5f);
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
    int x1 = (int)ex, y1 = (int)ey;               // (:154)
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
    int ilo, ihi;
    if (w.sa > 0) {
        ilo = A0 - w.a0;
        ihi = A1 - 1 - w.a0;
    } else {
        ilo = w.a0 - (A1 - 1);
        ihi = w.a0 - A0;
    }
    lo = ilo > 0 ? ilo : 0;
    hi = ihi < w.da ? ihi : w.da;
    if (lo > hi) return false;
    int qlo, qhi;
    if (w.sb > 0) {
        qlo = B0 - w.b0;
        qhi = B1 - 1 - w.b0;
    } else {
        qlo = w.b0 - (B1 - 1);
        qhi = w.b0 - B0;
    }
    if (qhi < 0) return false;
    if (w.db == 0) {
        if (qlo > 0) return false;  // q(i) == 0 for every step
        return true;
    }
    if (qlo > 0) {
        int t = (qlo * w.da - w.e0 + w.db - 1) / w.db;
        if (t > lo) lo = t;
    }
    int t2 = ((qhi + 1) * w.da - w.e0 - 1) / w.db;
    if (t2 < hi) hi = t2;
    return lo <= hi;
}

// ------------------------------------------------------------------- k2: tiled grid update
// One workgroup per (stream, level).  For each 64x64 tile of the scan's bounding box:
//   (1) end cells in the tile: LDS atomicMin of the beam index   -> first hitting beam h
//   (2) free steps in the tile: mark W_FREE, or set FF_BIT on a hit cell when b < h
//   (3) one coalesced read-modify-write of every touched cell (8 B) applying the reference's
//       float sequence: free only: l + lf; hit: ((l + lf) - lf) if freed first, then + lo if < 50.
// This equals running bresenhamCellFree / bresenhamCellOcc (:302-330) beam by beam.
__global__ void __launch_bounds__(UPD_THREADS)
hs_update_kernel(FleetGeom geom, LogOddsCell *__restrict__ cells, StreamState *__restrict__ state,
                 const float2 *__restrict__ xy, int xy_stride, int stream_begin, int count, int max_points)
{
    extern __shared__ __attribute__((aligned(16))) unsigned smem[];
    unsigned *tile_w = smem;                 // TILE_CELLS words
    unsigned *rays = smem + TILE_CELLS;      // max_points packed end cells
    __shared__ int s_bbox[4];
    __shared__ int s_any;

    // level-major block order: every stream's level 0 (the largest) is dispatched first
    const int lvl = blockIdx.x / count;
    const int local = blockIdx.x - lvl * count;
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    const LevelGeom &g = geom.lv[lvl];
    const int n = st.n;
    const int tid = threadIdx.x;
    LogOddsCell *lc = cells + (size_t)s * geom.stream_cells + g.cell_offset;

    const RayFrame fr = ray_frame(g, st);
    const int x0 = fr.bxi, y0 = fr.byi;
    if (tid == 0) {
        s_bbox[0] = x0; s_bbox[1] = y0; s_bbox[2] = x0; s_bbox[3] = y0;
        s_any = 0;
    }
    __syncthreads();
    int bx0 = x0, by0 = y0, bx1 = x0, by1 = y0;
    unsigned long long L = 0, R = 0;
    const float2 *pts = xy + (size_t)local * xy_stride;
    for (int b = tid; b < n; b += UPD_THREADS) {
        unsigned r = make_ray(g, fr, pts[b]);
        rays[b] = r;
        if (r != RAY_INVALID) {
            int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
            bx0 = min(bx0, x1); by0 = min(by0, y1); bx1 = max(bx1, x1); by1 = max(by1, y1);
            int adx = abs(x1 - x0), ady = abs(y1 - y0);
            L += (unsigned long long)(max(adx, ady) + 1);
            R += 1;
        }
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
    if ((tid & 63) == 0 && R) {
        atomicAdd(&state[s].step_cells, L);
        atomicAdd(&state[s].tot_cells, L);
        atomicAdd(&state[s].tot_rays, R);
    }
    if (!__syncthreads_or(R != 0)) return;  // no ray drawn on this level
    const int tx0 = s_bbox[0] / TILE, ty0 = s_bbox[1] / TILE;
    const int tx1 = s_bbox[2] / TILE, ty1 = s_bbox[3] / TILE;
    const int mark_free = st.mark_base + 1;  // currMarkFreeIndex (:120)
    const int mark_occ = st.mark_base + 2;   // currMarkOccIndex  (:121)
    const float lf = geom.lf, lo = geom.lo;

    for (int ty = ty0; ty <= ty1; ++ty) {
        for (int tx = tx0; tx <= tx1; ++tx) {
            const int X0 = tx * TILE, Y0 = ty * TILE;
            const int X1 = X0 + TILE, Y1 = Y0 + TILE;
            // clear the tile words
            for (int k = tid; k < TILE_CELLS / 4; k += UPD_THREADS)
                reinterpret_cast<uint4 *>(tile_w)[k] = make_uint4(W_NONE, W_NONE, W_NONE, W_NONE);
            __syncthreads();
            // (1) hits
            bool any = false;
            for (int b = tid; b < n; b += UPD_THREADS) {
                unsigned r = rays[b];
                if (r == RAY_INVALID) continue;
                int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
                if (x1 >= X0 && x1 < X1 && y1 >= Y0 && y1 < Y1) {
                    atomicMin(&tile_w[(y1 - Y0) * TILE + (x1 - X0)], (unsigned)b);
                    any = true;
                }
            }
            __syncthreads();
            // (2) free steps
            for (int b = tid; b < n; b += UPD_THREADS) {
                unsigned r = rays[b];
                if (r == RAY_INVALID) continue;
                int x1 = (int)(r & 0xFFFFu), y1 = (int)(r >> 16);
                if (max(x0, x1) < X0 || min(x0, x1) >= X1 || max(y0, y1) < Y0 || min(y0, y1) >= Y1) continue;
                RayWalk w = ray_walk(x0, y0, x1, y1);
                int lo_i, hi_i;
                bool hit = w.x_major ? walk_range(w, X0, X1, Y0, Y1, lo_i, hi_i) : walk_range(w, Y0, Y1, X0, X1, lo_i, hi_i);
                if (!hit) continue;
                if (hi_i > w.da - 1) hi_i = w.da - 1;  // free steps only
                if (lo_i > hi_i) continue;
                any = true;
                const unsigned num = (unsigned)w.e0 + (unsigned)lo_i * (unsigned)w.db;
                int q = (int)(num / (unsigned)w.da);
                int err = (int)(num - (unsigned)q * (unsigned)w.da);
                int a = w.a0 + w.sa * lo_i;
                int bb = w.b0 + w.sb * q;
                for (int i = lo_i; i <= hi_i; ++i) {
                    int cx = w.x_major ? a : bb;
                    int cy = w.x_major ? bb : a;
                    unsigned *wp = &tile_w[(cy - Y0) * TILE + (cx - X0)];
                    unsigned v = *wp;
                    if (v >= W_FREE) {
                        *wp = W_FREE;
                    } else if ((unsigned)b < (v & 0xFFFFu)) {
                        *wp = v | FF_BIT;  // freed by an earlier beam than the first hit
                    }
                    a += w.sa;
                    err += w.db;
                    if (err >= w.da) {
                        err -= w.da;
                        bb += w.sb;
                    }
                }
            }
            if (any) s_any = 1;
            __syncthreads();
            if (s_any) {
                // (3) apply: wave w handles rows w, w+4, ...; lane = column -> 512 B coalesced rows
                const int col = tid & 63;
                const int gx = X0 + col;
                for (int row = tid >> 6; row < TILE; row += UPD_THREADS / 64) {
                    const int gy = Y0 + row;
                    unsigned v = tile_w[row * TILE + col];
                    if (v == W_NONE || gx >= g.sx || gy >= g.sy) continue;
                    LogOddsCell *cp = lc + (size_t)gy * g.sx + gx;
                    LogOddsCell c = *cp;
                    if (v == W_FREE) {
                        c.l = c.l + lf;        // updateSetFree (GridMapLogOdds.h:120-124)
                        c.upd = mark_free;
                    } else {
                        if (v & FF_BIT) {
                            c.l = c.l + lf;    // bresenhamCellFree by an earlier beam
                            c.l = c.l - lf;    // updateUnsetFree (GridMapLogOdds.h:126-129)
                        }
                        if (c.l < 50.0f) c.l = c.l + lo;  // updateSetOccupied (:108-114)
                        c.upd = mark_occ;
                    }
                    *cp = c;
                }
            }
            __syncthreads();
            if (tid == 0) s_any = 0;
        }
    }
}


// --------------------------------------------------------------------------- utility kernels
__global__ void hs_fill_cells_kernel(LogOddsCell *__restrict__ cells, size_t n)
{
    // LogOddsCell::resetGridCell  H/map/GridMapLogOdds.h:76-80
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        cells[i].l = 0.0f;
        cells[i].upd = -1;
    }
}

// HectorMappingRos::publishMap cell conversion  lesson4/src/hector_mapping/hector_slam.cc:287-304
__global__ void hs_publish_kernel(const LogOddsCell *__restrict__ cells, int8_t *__restrict__ out, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        float l = cells[i].l;
        out[i] = l < 0.0f ? (int8_t)0 : (l > 0.0f ? (int8_t)100 : (int8_t)-1);
    }
}

}  // namespace s2d
