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
//   k2 hs_mark_hits_kernel  one thread per beam: end cell gets the "first hitting beam" marker.
//   k3 hs_free_cells_kernel 64 beams per workgroup, the workgroup's free cells flattened over 256
//                           threads (load balance); first touch applies l += lf exactly once.
//   k4 hs_resolve_hits_kernel the first hitting beam finalises each hit cell.
// k2..k4 reproduce the sequential per-cell float sequence of bresenhamCellFree/Occ
// (H/map/OccGridMapBase.h:302-330) exactly; see DESIGN.md "once-per-scan semantics".
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
    }
}

// ------------------------------------------------------------------------------- ray geometry
// OccGridMapBase::updateByScan (H/map/OccGridMapBase.h:118-161) + updateLineBresenhami (:220-267).
// Bresenham step i (0..abs_da-1 free, abs_da = end) in closed form:
//   cell_i = start + i*off_a + floor((e0 + i*abs_db) / abs_da) * off_b,  e0 = abs_da/2,
// which equals bresenham2D's incremental error walk (:281-298): error stays in [0, abs_da).
struct Ray {
    int valid;
    int start;
    int end;
    int abs_da, abs_db, e0, off_a, off_b;
};

struct RayFrame {
    float mx, my, cs, sn;
    int bxi, byi;
};

__device__ __forceinline__ RayFrame ray_frame(const LevelGeom &g, const StreamState &st)
{
    RayFrame fr;
    float mp[3];
    map_from_world(g, st.upd_pose, mp);
    fr.mx = mp[0];
    fr.my = mp[1];
    fr.cs = sdm_cosf(mp[2]);
    fr.sn = sdm_sinf(mp[2]);
    const float f = g.pts_scale;
    float ox = st.origo[0] * f, oy = st.origo[1] * f;
    float nsn = -fr.sn;
    float bx = fr.mx + (fr.cs * ox + nsn * oy);
    float by = fr.my + (fr.sn * ox + fr.cs * oy);
    fr.bxi = (int)(bx + 0.5f);
    fr.byi = (int)(by + 0.5f);
    return fr;
}

__device__ __forceinline__ Ray make_ray(const LevelGeom &g, const RayFrame &fr, float2 p)
{
    Ray r;
    r.valid = 0;
    const float f = g.pts_scale;
    float px = p.x * f, py = p.y * f;
    float nsn = -fr.sn;
    float ex = fr.mx + (fr.cs * px + nsn * py);
    float ey = fr.my + (fr.sn * px + fr.cs * py);
    ex += 0.5f;
    ey += 0.5f;
    int x1 = (int)ex, y1 = (int)ey;
    int x0 = fr.bxi, y0 = fr.byi;
    if (x0 == x1 && y0 == y1) return r;  // :157
    if ((x0 < 0) || (x0 >= g.sx) || (y0 < 0) || (y0 >= g.sy)) return r;  // :226-229
    if ((x1 < 0) || (x1 >= g.sx) || (y1 < 0) || (y1 >= g.sy)) return r;  // :235-238
    int dx = x1 - x0, dy = y1 - y0;
    int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    int odx = dx > 0 ? 1 : -1;           // util::sign (UtilFunctions.h:55-58)
    int ody = (dy > 0 ? 1 : -1) * g.sx;
    r.valid = 1;
    r.start = y0 * g.sx + x0;
    r.end = y1 * g.sx + x1;
    if (adx >= ady) {
        r.abs_da = adx; r.abs_db = ady; r.off_a = odx; r.off_b = ody;
    } else {
        r.abs_da = ady; r.abs_db = adx; r.off_a = ody; r.off_b = odx;
    }
    r.e0 = r.abs_da / 2;
    return r;
}

// Marker encoding inside LogOddsCell::upd during one scan (values are resolved before the scan ends;
// every pre-scan value is <= markFree - 1 because the previous scan left markFree'/markOcc' < markFree):
//   markFree = U+1                  freed this scan, not hit
//   H(h)  = hb + (n - h)            hit, first hitting beam h, no earlier free   (hb = U+3)
//   FH(h) = hb + (n - h) + n + 1    hit by h and freed by some beam b < h
// atomicMax selects the smallest h; H -> FH conversion is idempotent.

// --------------------------------------------------------------------------- k2: mark hits
__global__ void __launch_bounds__(256)
hs_mark_hits_kernel(FleetGeom geom, LogOddsCell *__restrict__ cells, StreamState *__restrict__ state,
                    const float2 *__restrict__ xy, int xy_stride, int stream_begin)
{
    const int local = blockIdx.z;
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    const int lvl = blockIdx.y;
    const LevelGeom &g = geom.lv[lvl];
    const int n = st.n;
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x * 256 >= n) return;
    LogOddsCell *lc = cells + (size_t)s * geom.stream_cells + g.cell_offset;
    const RayFrame fr = ray_frame(g, st);
    unsigned long long L = 0;
    if (b < n) {
        Ray r = make_ray(g, fr, xy[(size_t)local * xy_stride + b]);
        if (r.valid) {
            const int hb = st.mark_base + 3;
            atomicMax(&lc[r.end].upd, hb + (n - b));
            L = (unsigned long long)r.abs_da + 1ull;
        }
    }
    // Σ(abs_da+1): wave reduce, one atomic per wave
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) L += __shfl_xor(L, off, 64);
    if ((threadIdx.x & 63) == 0 && L) atomicAdd(&state[s].step_cells, L);
}

// --------------------------------------------------------------------------- k3: free cells
__global__ void __launch_bounds__(256)
hs_free_cells_kernel(FleetGeom geom, LogOddsCell *__restrict__ cells, StreamState *__restrict__ state,
                     const float2 *__restrict__ xy, int xy_stride, int stream_begin)
{
    __shared__ int s_pref[FREE_BEAMS + 1];
    __shared__ int s_start[FREE_BEAMS], s_offa[FREE_BEAMS], s_offb[FREE_BEAMS], s_da[FREE_BEAMS],
        s_db[FREE_BEAMS], s_e0[FREE_BEAMS];
    const int local = blockIdx.z;
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    const int n = st.n;
    const int b0 = blockIdx.x * FREE_BEAMS;
    if (b0 >= n) return;
    const int lvl = blockIdx.y;
    const LevelGeom &g = geom.lv[lvl];
    LogOddsCell *lc = cells + (size_t)s * geom.stream_cells + g.cell_offset;
    const int tid = threadIdx.x;
    if (tid < FREE_BEAMS) {
        const RayFrame fr = ray_frame(g, st);
        const int b = b0 + tid;
        int len = 0;
        if (b < n) {
            Ray r = make_ray(g, fr, xy[(size_t)local * xy_stride + b]);
            if (r.valid) {
                len = r.abs_da;  // start cell + abs_da-1 intermediate cells are freed (:277-298)
                s_start[tid] = r.start;
                s_offa[tid] = r.off_a;
                s_offb[tid] = r.off_b;
                s_da[tid] = r.abs_da;
                s_db[tid] = r.abs_db;
                s_e0[tid] = r.e0;
            }
        }
        // inclusive scan over the 64 lengths (one wave)
        int v = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            int t = __shfl_up(v, off, 64);
            if (tid >= off) v += t;
        }
        s_pref[tid + 1] = v;
        if (tid == 0) s_pref[0] = 0;
    }
    __syncthreads();
    const int total = s_pref[FREE_BEAMS];
    const int mark_free = st.mark_base + 1;
    const int hb = st.mark_base + 3;
    const float lf = geom.lf;
    for (int k = tid; k < total; k += 256) {
        // beam j: largest j with s_pref[j] <= k
        int lo = 0, hi = FREE_BEAMS;
#pragma unroll
        for (int it = 0; it < 6; ++it) {
            int mid = (lo + hi) >> 1;
            if (s_pref[mid] <= k) lo = mid;
            else hi = mid;
        }
        const int j = lo;
        const int i = k - s_pref[j];
        const unsigned int da = (unsigned int)s_da[j];
        const unsigned int steps_b = ((unsigned int)s_e0[j] + (unsigned int)i * (unsigned int)s_db[j]) / da;
        const int c = s_start[j] + i * s_offa[j] + (int)steps_b * s_offb[j];
        const int b = b0 + j;
        int *updp = &lc[c].upd;
        int u = __builtin_nontemporal_load(updp) ;
        if (u < mark_free) {
            const int old = atomicMax(updp, mark_free);
            if (old < mark_free) {
                // first touch this scan: updateSetFree (GridMapLogOdds.h:120-124), unique writer
                lc[c].l = lc[c].l + lf;
                continue;
            }
            u = old;
        }
        if (u > hb && u <= hb + n) {
            const int h = n - (u - hb);
            if (b < h) atomicMax(updp, u + n + 1);  // H(h) -> FH(h): freed before the first hit
        }
    }
}

// --------------------------------------------------------------------------- k4: resolve hits
__global__ void __launch_bounds__(256)
hs_resolve_hits_kernel(FleetGeom geom, LogOddsCell *__restrict__ cells, StreamState *__restrict__ state,
                       const float2 *__restrict__ xy, int xy_stride, int stream_begin)
{
    const int local = blockIdx.z;
    const int s = stream_begin + local;
    const StreamState &st = state[s];
    if (!st.do_update) return;
    const int n = st.n;
    if (blockIdx.x * 256 >= n) return;
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n) return;
    const int lvl = blockIdx.y;
    const LevelGeom &g = geom.lv[lvl];
    LogOddsCell *lc = cells + (size_t)s * geom.stream_cells + g.cell_offset;
    const RayFrame fr = ray_frame(g, st);
    Ray r = make_ray(g, fr, xy[(size_t)local * xy_stride + b]);
    if (!r.valid) return;
    const int hb = st.mark_base + 3;
    const int mark_occ = st.mark_base + 2;
    const int u = lc[r.end].upd;
    int h;
    bool freed_first;
    if (u > hb + n) {
        h = n - (u - hb - n - 1);
        freed_first = true;
    } else {
        h = n - (u - hb);
        freed_first = false;
    }
    if (h != b) return;
    // bresenhamCellOcc  H/map/OccGridMapBase.h:315-330
    float l = lc[r.end].l;
    if (freed_first) {
        l = l + geom.lf;   // updateSetFree by the earlier beam
        l = l - geom.lf;   // updateUnsetFree (GridMapLogOdds.h:126-129)
    }
    if (l < 50.0f) l = l + geom.lo;  // updateSetOccupied (GridMapLogOdds.h:108-114)
    lc[r.end].l = l;
    lc[r.end].upd = mark_occ;
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
