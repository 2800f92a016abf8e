/* oracle/hector_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("port") of the reference's Hector scan-matching + occupancy-grid hot path, used
 * as the parity checker for the HIP product.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  It is never linked into, or called by, the product.
 *
 * PARITY STATUS: "parity unpinned" w.r.t. the reference binary.  The reference Hector core
 * (lesson4/include/lesson4/hector_mapping/...) needs Eigen3, which is absent from this image, so it
 * cannot be compiled here (no stand-in headers are written, by rule).  The reference ships no tests,
 * fixtures or known-answer vectors for this path.  This restatement is
 * therefore pinned only by hand-derived known-answer tests (tests/test_oracle_hector.py) and by
 * committed regression vectors it produced itself (tests/golden/hector_*.npz).
 *
 * Every function below cites the reference file:line it follows.  Abbreviation:
 *   H/ = /root/reference/lesson4/include/lesson4/hector_mapping/
 *
 * Floating point: compile with -O2 -ffp-contract=off (no FMA contraction, SSE float => no excess
 * precision).  Eigen's evaluation order (Eigen 3.3, not available here => unpinned) is fixed as:
 *   - Affine2f * Vector2f       : t(i) + (L(i,0)*v0 + L(i,1)*v1)                (transform_right_product_impl)
 *   - Matrix3f * Vector3f       : a0 + (a1 + a2)                                (redux_novec_unroller halving)
 *   - Matrix3f::inverse()       : adjugate of 3x3 cofactors / det, det = c0*m00 + (c1*m10 + c2*m20)
 *   - Scaling*Translation       : linear diag(s,s), translation s*offset
 *   - Transform::inverse(Affine): L^-1 via 2x2 adjugate/det, t' = (-L^-1) * t
 *   - sin/cos/exp               : detmath.h (double, fixed op order, rounded to float once);
 *                                 libm variants selectable (use_libm=1) for the tolerance check.
 *   - util::normalize_angle     : fmod in double (H/util/UtilFunctions.h:36-48)
 *   - abs(float angleDiff)      : fabsf (H/util/UtilFunctions.h:87; overload ambiguity resolved to float)
 *
 * Reduction order of the Hessian sums (H/map/OccGridMapUtil.h:94-126): the reference sums points
 * sequentially (reduce_threads = 0).  reduce_threads = T > 0 restates the HIP kernel's order
 * instead (thread t accumulates points t, t+T, ...; 64-lane xor-butterfly with offsets 32..1;
 * then an xor-butterfly over the T/64 wave sums), so the GPU path can be compared bit-for-bit.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "detmath.h"

#define HO_MAX_LEVELS 8
#define HO_PI 3.14159265358979323846 /* M_PI */

typedef struct {
    float l;   /* LogOddsCell::logOddsVal  H/map/GridMapLogOdds.h:85 */
    int upd;   /* LogOddsCell::updateIndex H/map/GridMapLogOdds.h:86 */
} ho_cell;

typedef struct {
    int sx, sy;
    float cell_len;
    float scale;     /* scaleToMap = 1/cellLength                   GridMapBase.h:276 */
    float map_t[2];  /* mapTworld translation = s * topLeftOffset   GridMapBase.h:278 */
    float inv_l00, inv_l01, inv_l10, inv_l11; /* worldTmap linear    GridMapBase.h:285 */
    float inv_t[2];  /* worldTmap translation */
    float lim[2];    /* mapLimitsf = dims - 2                        MapDimensionProperties.h:66-70 */
    ho_cell *cells;
    int cur_update_index;  /* OccGridMapBase::currUpdateIndex  OccGridMapBase.h:334 */
    int last_update_index; /* GridMapBase::lastUpdateIndex     GridMapBase.h:413 */
    float pts_scale;       /* DataPointContainer::setFrom factor for this level */
} ho_level;

typedef struct {
    int levels;
    ho_level lv[HO_MAX_LEVELS];
    float lf, lo;  /* logOddsFree / logOddsOccupied */
    float min_dist, min_ang;
    float last_map_update_pose[3];
    float last_scan_match_pose[3];
    float last_cov[9];
    int reduce_threads;
    int use_libm;
    unsigned long long sum_L;      /* Σ (abs_da + 1) over the valid rays of the last update */
    unsigned long long sum_free;   /* Σ abs_da */
    int valid_rays;
    int clamp_count;
    float *red;                    /* scratch for tree-order emulation: T*9 floats */
    /* MapRepMultiMap::dataContainers (MapRepMultiMap.h:89): the DataContainer of the last matchData
     * (setFrom at :161), drawn into levels >= 1 by updateByScan (:187).  Kept at level-0 scale; the
     * level's factor is applied at use, the same float product setFrom computes
     * (DataPointContainer.h:46-58).  Empty until the first match; reset() keeps it (:102-110). */
    float *mc_xy;
    int mc_n, mc_cap;
    float mc_origo[2];
    /* per-iteration trace (optional, for fixtures) */
    float *trace;                  /* [max_trace][3+9+3] pose-before, H(9) ... */
    int trace_cap, trace_len;
} ho_ctx;

/* ------------------------------------------------------------------------------------------ */
static inline float ho_sinf(const ho_ctx *c, float x) { return c->use_libm ? sinf(x) : odm_sinf(x); }
static inline float ho_cosf(const ho_ctx *c, float x) { return c->use_libm ? cosf(x) : odm_cosf(x); }
static inline float ho_expf(const ho_ctx *c, float x) { return c->use_libm ? (float)exp((double)x) : odm_expf(x); }

/* (int)v of OccGridMapBase.h:135/:154 for v in int range; NaN or out-of-range (undefined behaviour in
 * the reference, INT_MIN on x86) -> -1, which the bounds check of :226-238 cancels like INT_MIN */
static inline int ho_cell_of(float v)
{
    return (v > -2147483648.0f && v < 2147483648.0f) ? (int)v : -1;
}

/* GridMapLogOddsFunctions::probToLogOdds  H/map/GridMapLogOdds.h:153-157 */
static float ho_prob_to_logodds(float prob)
{
    float odds = prob / (1.0f - prob);
    return (float)log((double)odds);
}

/* GridMapLogOddsFunctions::getGridProbability  H/map/GridMapLogOdds.h:136-140 */
static inline float ho_prob(const ho_ctx *c, float l)
{
    float odds = ho_expf(c, l);
    return odds / (odds + 1.0f);
}

/* util::normalize_angle_pos / normalize_angle  H/util/UtilFunctions.h:36-48 (double fmod) */
static float ho_normalize_angle(float angle)
{
    double two_pi = 2.0f * HO_PI;
    float a = (float)fmod(fmod((double)angle, two_pi) + two_pi, two_pi);
    if ((double)a > HO_PI) a = (float)((double)a - two_pi);
    return a;
}

/* util::poseDifferenceLargerThan  H/util/UtilFunctions.h:72-91 */
static int ho_pose_diff_larger(const float *p1, const float *p2, float dist, float ang)
{
    float dx = p1[0] - p2[0];
    float dy = p1[1] - p2[1];
    float n = sqrtf(dx * dx + dy * dy);
    if (n > dist) return 1;
    float ad = p1[2] - p2[2];
    if ((double)ad > HO_PI) ad = (float)((double)ad - HO_PI * 2.0f);
    else if ((double)ad < -HO_PI) ad = (float)((double)ad + HO_PI * 2.0f);
    if (fabsf(ad) > ang) return 1;
    return 0;
}

/* world->map pose: GridMapBase::getMapCoordsPose  H/map/GridMapBase.h:238-242 */
static inline void ho_map_from_world(const ho_level *L, const float *w, float *m)
{
    m[0] = L->map_t[0] + (L->scale * w[0] + 0.0f * w[1]);
    m[1] = L->map_t[1] + (0.0f * w[0] + L->scale * w[1]);
    m[2] = w[2];
}

/* map->world pose: GridMapBase::getWorldCoordsPose  H/map/GridMapBase.h:229-233 */
static inline void ho_world_from_map(const ho_level *L, const float *m, float *w)
{
    w[0] = L->inv_t[0] + (L->inv_l00 * m[0] + L->inv_l01 * m[1]);
    w[1] = L->inv_t[1] + (L->inv_l10 * m[0] + L->inv_l11 * m[1]);
    w[2] = m[2];
}

/* GridMapBase::setMapTransformation  H/map/GridMapBase.h:270-286 */
static void ho_set_map_transformation(ho_level *L, float off_x, float off_y, float cell_len)
{
    L->cell_len = cell_len;
    L->scale = 1.0f / cell_len;
    L->map_t[0] = L->scale * off_x;
    L->map_t[1] = L->scale * off_y;
    /* inverse of [s 0; 0 s]: 2x2 adjugate / det (Eigen compute_inverse size 2) */
    float m00 = L->scale, m01 = 0.0f, m10 = 0.0f, m11 = L->scale;
    float det = m00 * m11 - m10 * m01;
    float invdet = 1.0f / det;
    L->inv_l00 = m11 * invdet;
    L->inv_l10 = -m10 * invdet;
    L->inv_l01 = -m01 * invdet;
    L->inv_l11 = m00 * invdet;
    /* t' = (-Linv) * t */
    L->inv_t[0] = (-L->inv_l00) * L->map_t[0] + (-L->inv_l01) * L->map_t[1];
    L->inv_t[1] = (-L->inv_l10) * L->map_t[0] + (-L->inv_l11) * L->map_t[1];
}

/* GridMapBase::clear / LogOddsCell::resetGridCell  H/map/GridMapBase.h:102-113, GridMapLogOdds.h:76-80 */
static void ho_level_clear(ho_level *L)
{
    size_t n = (size_t)L->sx * (size_t)L->sy;
    for (size_t i = 0; i < n; ++i) {
        L->cells[i].l = 0.0f;
        L->cells[i].upd = -1;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Construction: MapRepMultiMap ctor  H/slam_main/MapRepMultiMap.h:57-90 ;
 * HectorSlamProcessor ctor  H/slam_main/HectorSlamProcessor.h:57-68 */
ho_ctx *ho_create(float map_resolution, int map_size_x, int map_size_y, float start_x, float start_y,
                  int levels)
{
    if (levels < 1 || levels > HO_MAX_LEVELS || map_size_x < 2 || map_size_y < 2) return NULL;
    ho_ctx *c = (ho_ctx *)calloc(1, sizeof(ho_ctx));
    c->levels = levels;
    int rx = map_size_x, ry = map_size_y;
    float res = map_resolution;
    float total_x = map_resolution * (float)map_size_x;
    float mid_x = total_x * start_x;
    float total_y = map_resolution * (float)map_size_y;
    float mid_y = total_y * start_y;
    for (int i = 0; i < levels; ++i) {
        ho_level *L = &c->lv[i];
        L->sx = rx;
        L->sy = ry;
        L->lim[0] = (float)rx - 2.0f;
        L->lim[1] = (float)ry - 2.0f;
        L->cells = (ho_cell *)malloc(sizeof(ho_cell) * (size_t)rx * (size_t)ry);
        ho_set_map_transformation(L, mid_x, mid_y, res);
        ho_level_clear(L);
        L->cur_update_index = 0;
        L->last_update_index = -1;
        /* dataContainers[i-1].setFrom(container, 1/2^i)  MapRepMultiMap.h:161 */
        L->pts_scale = (float)(1.0 / pow(2.0, (double)i));
        rx /= 2;
        ry /= 2;
        res *= 2.0f;
    }
    /* GridMapLogOddsFunctions ctor defaults  GridMapLogOdds.h:98-102 */
    c->lf = ho_prob_to_logodds(0.4f);
    c->lo = ho_prob_to_logodds(0.6f);
    c->min_dist = 0.4f * 1.0f;
    c->min_ang = 0.13f * 1.0f;
    /* HectorSlamProcessor::reset  HectorSlamProcessor.h:111-117 */
    c->last_map_update_pose[0] = c->last_map_update_pose[1] = c->last_map_update_pose[2] = FLT_MAX;
    memset(c->last_scan_match_pose, 0, sizeof(c->last_scan_match_pose));
    memset(c->last_cov, 0, sizeof(c->last_cov));
    return c;
}

void ho_destroy(ho_ctx *c)
{
    if (!c) return;
    for (int i = 0; i < c->levels; ++i) free(c->lv[i].cells);
    free(c->red);
    free(c->trace);
    free(c->mc_xy);
    free(c);
}

/* HectorSlamProcessor::reset -> MapRepMultiMap::reset -> MapProcContainer::reset (cells only: the grids'
 * update indices, lastScanMatchCov and the stored containers are kept) */
void ho_reset(ho_ctx *c)
{
    c->last_map_update_pose[0] = c->last_map_update_pose[1] = c->last_map_update_pose[2] = FLT_MAX;
    memset(c->last_scan_match_pose, 0, sizeof(c->last_scan_match_pose));
    for (int i = 0; i < c->levels; ++i) ho_level_clear(&c->lv[i]);
}

/* setUpdateFactorFree / Occupied  MapRepMultiMap.h:194-214 -> GridMapLogOdds.h:142-150 */
void ho_set_update_factors(ho_ctx *c, float free_factor, float occ_factor)
{
    c->lf = ho_prob_to_logodds(free_factor);
    c->lo = ho_prob_to_logodds(occ_factor);
}

void ho_set_thresholds(ho_ctx *c, float min_dist, float min_ang)
{
    c->min_dist = min_dist;
    c->min_ang = min_ang;
}

void ho_set_mode(ho_ctx *c, int reduce_threads, int use_libm)
{
    c->reduce_threads = reduce_threads;
    c->use_libm = use_libm;
    free(c->red);
    c->red = reduce_threads > 0 ? (float *)malloc(sizeof(float) * 9 * (size_t)reduce_threads) : NULL;
}

void ho_enable_trace(ho_ctx *c, int cap)
{
    free(c->trace);
    c->trace = (float *)malloc(sizeof(float) * 16 * (size_t)cap);
    c->trace_cap = cap;
    c->trace_len = 0;
}

int ho_trace_len(const ho_ctx *c) { return c->trace_len; }
void ho_get_trace(const ho_ctx *c, float *out) { memcpy(out, c->trace, sizeof(float) * 16 * (size_t)c->trace_len); }

/* ------------------------------------------------------------------------------------------ */
/* OccGridMapUtil::interpMapValueWithDerivatives  H/map/OccGridMapUtil.h:139-228 */
static inline void ho_interp(const ho_ctx *c, const ho_level *L, float x, float y, float *v, float *gx, float *gy)
{
    /* pointOutOfMapBounds  MapDimensionProperties.h:61-64 */
    /* NaN-safe form of the same test: a NaN coordinate (diverged pose) counts as out of map, where the
     * reference would index the grid with (int)NaN (undefined behaviour) */
    if (!(x >= 0.0f) || !(x <= L->lim[0]) || !(y >= 0.0f) || !(y <= L->lim[1])) {
        *v = 0.0f; *gx = 0.0f; *gy = 0.0f;
        return;
    }
    int ix = (int)x, iy = (int)y;
    float fx = x - (float)ix;
    float fy = y - (float)iy;
    int idx = iy * L->sx + ix;
    /* GridMapCacheArray is a value-transparent memo (GridMapCacheArray.h:84-109): evaluate directly */
    float i0 = ho_prob(c, L->cells[idx].l);
    float i1 = ho_prob(c, L->cells[idx + 1].l);
    float i2 = ho_prob(c, L->cells[idx + L->sx].l);
    float i3 = ho_prob(c, L->cells[idx + L->sx + 1].l);
    float dx1 = i0 - i1;
    float dx2 = i2 - i3;
    float dy1 = i0 - i2;
    float dy2 = i1 - i3;
    float xfi = 1.0f - fx;
    float yfi = 1.0f - fy;
    *v = ((i0 * xfi + i1 * fx) * yfi) + ((i2 * xfi + i3 * fx) * fy);
    *gx = -((dx1 * yfi) + (dx2 * fy));
    *gy = -((dy1 * xfi) + (dy2 * fx));
}

/* per-point contribution of OccGridMapUtil::getCompleteHessianDerivs  OccGridMapUtil.h:94-126
 * out[0..8] = dTr0, dTr1, dTr2, H00, H11, H22, H01, H02, H12 */
static inline void ho_point_terms(const ho_ctx *c, const ho_level *L, float tx, float ty, float cs, float sn,
                                  float sinRot, float cosRot, float px, float py, float *out)
{
    /* transform * currPoint : t + (R*p), R = [c -s; s c]  (getTransformForState  :437-440) */
    float nsn = -sn;
    float x = tx + (cs * px + nsn * py);
    float y = ty + (sn * px + cs * py);
    float v, gx, gy;
    ho_interp(c, L, x, y, &v, &gx, &gy);
    float fun = 1.0f - v;
    out[0] = gx * fun;
    out[1] = gy * fun;
    float rot = ((-sinRot * px - cosRot * py) * gx + (cosRot * px - sinRot * py) * gy);
    out[2] = rot * fun;
    out[3] = gx * gx;
    out[4] = gy * gy;
    out[5] = rot * rot;
    out[6] = gx * gy;
    out[7] = gx * rot;
    out[8] = gy * rot;
}

/* OccGridMapUtil::getCompleteHessianDerivs  H/map/OccGridMapUtil.h:77-132
 * H is row-major 3x3 */
static void ho_hessian(ho_ctx *c, const ho_level *L, const float *pose, const float *xy, int n, float f,
                       float *H, float *b)
{
    float cs = ho_cosf(c, pose[2]);
    float sn = ho_sinf(c, pose[2]);
    float sinRot = ho_sinf(c, pose[2]);
    float cosRot = ho_cosf(c, pose[2]);
    float acc[9];
    for (int k = 0; k < 9; ++k) acc[k] = 0.0f;
    int T = c->reduce_threads;
    if (T <= 0) {
        for (int i = 0; i < n; ++i) {
            float t[9];
            ho_point_terms(c, L, pose[0], pose[1], cs, sn, sinRot, cosRot, xy[2 * i] * f, xy[2 * i + 1] * f, t);
            for (int k = 0; k < 9; ++k) acc[k] = acc[k] + t[k];
        }
    } else {
        /* GPU order: per-thread strided partials, then xor butterflies */
        float *r = c->red;
        for (int j = 0; j < T * 9; ++j) r[j] = 0.0f;
        for (int i = 0; i < n; ++i) {
            float t[9];
            ho_point_terms(c, L, pose[0], pose[1], cs, sn, sinRot, cosRot, xy[2 * i] * f, xy[2 * i + 1] * f, t);
            float *rt = r + (size_t)(i % T) * 9;
            for (int k = 0; k < 9; ++k) rt[k] = rt[k] + t[k];
        }
        int W = T / 64;
        float tmp[64 * 9];
        for (int w = 0; w < W; ++w) {
            float *rw = r + (size_t)w * 64 * 9;
            for (int off = 32; off >= 1; off >>= 1) {
                for (int lane = 0; lane < 64; ++lane)
                    for (int k = 0; k < 9; ++k) tmp[lane * 9 + k] = rw[lane * 9 + k] + rw[(lane ^ off) * 9 + k];
                memcpy(rw, tmp, sizeof(float) * 64 * 9);
            }
        }
        /* wave sums: element w = r[w*64*9 .. +9] */
        float ws[16 * 9], wt[16 * 9];
        for (int w = 0; w < W; ++w)
            for (int k = 0; k < 9; ++k) ws[w * 9 + k] = r[(size_t)w * 64 * 9 + k];
        for (int off = W / 2; off >= 1; off >>= 1) {
            for (int w = 0; w < W; ++w)
                for (int k = 0; k < 9; ++k) wt[w * 9 + k] = ws[w * 9 + k] + ws[(w ^ off) * 9 + k];
            memcpy(ws, wt, sizeof(float) * 9 * (size_t)W);
        }
        for (int k = 0; k < 9; ++k) acc[k] = ws[k];
    }
    b[0] = acc[0];
    b[1] = acc[1];
    b[2] = acc[2];
    H[0] = acc[3]; H[4] = acc[4]; H[8] = acc[5];
    H[1] = acc[6]; H[2] = acc[7]; H[5] = acc[8];
    H[3] = H[1]; H[6] = H[2]; H[7] = H[5];
}

/* Matrix3f::inverse() * dTr (Eigen 3.3 compute_inverse size 3; lazy product, halving redux) */
static void ho_solve3(const float *m, const float *b, float *d)
{
#define M(i, j) m[(i)*3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    float c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    float det = c00 * M(0, 0) + (c10 * M(1, 0) + c20 * M(2, 0));
    float invdet = 1.0f / det;
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
    for (int i = 0; i < 3; ++i) d[i] = inv[i * 3] * b[0] + (inv[i * 3 + 1] * b[1] + inv[i * 3 + 2] * b[2]);
#undef COF
#undef M
}

/* ScanMatcher::estimateTransformationLogLh  H/matcher/ScanMatcher.h:107-139 */
static void ho_gn_step(ho_ctx *c, const ho_level *L, float *est, const float *xy, int n, float f, float *H)
{
    float b[3];
    float pose_before[3] = {est[0], est[1], est[2]};
    ho_hessian(c, L, est, xy, n, f, H, b);
    if ((H[0] != 0.0f) && (H[4] != 0.0f)) {
        float d[3];
        ho_solve3(H, b, d);
        if (d[2] > 0.2f) { d[2] = 0.2f; c->clamp_count++; }
        else if (d[2] < -0.2f) { d[2] = -0.2f; c->clamp_count++; }
        est[0] = est[0] + d[0];
        est[1] = est[1] + d[1];
        est[2] = est[2] + d[2];
    }
    if (c->trace && c->trace_len < c->trace_cap) {
        float *t = c->trace + (size_t)16 * c->trace_len++;
        t[0] = pose_before[0]; t[1] = pose_before[1]; t[2] = pose_before[2];
        for (int k = 0; k < 9; ++k) t[3 + k] = H[k];
        t[12] = b[0]; t[13] = b[1]; t[14] = b[2];
        t[15] = 0.0f;
    }
}

/* ScanMatcher::matchData  H/matcher/ScanMatcher.h:60-97 */
static void ho_match_level(ho_ctx *c, int lvl, const float *hint, const float *xy, int n, int max_iter,
                           float *out, float *cov)
{
    ho_level *L = &c->lv[lvl];
    if (n == 0) {
        out[0] = hint[0]; out[1] = hint[1]; out[2] = hint[2];
        return;
    }
    float est[3], H[9];
    ho_map_from_world(L, hint, est);
    ho_gn_step(c, L, est, xy, n, L->pts_scale, H);
    for (int i = 0; i < max_iter; ++i) ho_gn_step(c, L, est, xy, n, L->pts_scale, H);
    est[2] = ho_normalize_angle(est[2]);
    for (int k = 0; k < 9; ++k) cov[k] = H[k];
    ho_world_from_map(L, est, out);
}

/* MapRepMultiMap::matchData  H/slam_main/MapRepMultiMap.h:144-167 */
void ho_match(ho_ctx *c, const float *xy, int n, float ox, float oy, const float *hint, float *pose_out,
              float *cov_out)
{
    /* dataContainers[index-1].setFrom(dataContainer, 1/2^index)  :161 (every level >= 1, every call) */
    if (c->levels > 1) {
        if (n > c->mc_cap) {
            free(c->mc_xy);
            c->mc_cap = n;
            c->mc_xy = (float *)malloc(sizeof(float) * 2 * (size_t)n);
        }
        if (n > 0) memcpy(c->mc_xy, xy, sizeof(float) * 2 * (size_t)n);
        c->mc_n = n;
        c->mc_origo[0] = ox;
        c->mc_origo[1] = oy;
    }
    float tmp[3] = {hint[0], hint[1], hint[2]};
    for (int lvl = c->levels - 1; lvl >= 0; --lvl) {
        float o[3];
        ho_match_level(c, lvl, tmp, xy, n, lvl == 0 ? 5 : 3, o, cov_out);
        tmp[0] = o[0]; tmp[1] = o[1]; tmp[2] = o[2];
    }
    pose_out[0] = tmp[0]; pose_out[1] = tmp[1]; pose_out[2] = tmp[2];
}

/* ------------------------------------------------------------------------------------------ */
/* bresenhamCellFree  H/map/OccGridMapBase.h:302-312 */
static inline void ho_cell_free(ho_ctx *c, ho_level *L, unsigned int off, int mark_free)
{
    ho_cell *cell = &L->cells[off];
    if (cell->upd < mark_free) {
        cell->l += c->lf;           /* updateSetFree  GridMapLogOdds.h:120-124 */
        cell->upd = mark_free;
    }
}

/* bresenhamCellOcc  H/map/OccGridMapBase.h:315-330 */
static inline void ho_cell_occ(ho_ctx *c, ho_level *L, unsigned int off, int mark_free, int mark_occ)
{
    ho_cell *cell = &L->cells[off];
    if (cell->upd < mark_occ) {
        if (cell->upd == mark_free) cell->l -= c->lf;  /* updateUnsetFree  GridMapLogOdds.h:126-129 */
        if (cell->l < 50.0f) cell->l += c->lo;         /* updateSetOccupied GridMapLogOdds.h:108-114 */
        cell->upd = mark_occ;
    }
}

/* bresenham2D  H/map/OccGridMapBase.h:270-299 */
static void ho_bresenham2d(ho_ctx *c, ho_level *L, unsigned int abs_da, unsigned int abs_db, int error_b,
                           int offset_a, int offset_b, unsigned int offset, int mf)
{
    ho_cell_free(c, L, offset, mf);
    unsigned int end = abs_da - 1;
    for (unsigned int i = 0; i < end; ++i) {
        offset += offset_a;
        error_b += abs_db;
        if ((unsigned int)error_b >= abs_da) {
            offset += offset_b;
            error_b -= abs_da;
        }
        ho_cell_free(c, L, offset, mf);
    }
}

/* updateLineBresenhami  H/map/OccGridMapBase.h:220-267 ; returns 1 if the ray was drawn */
static int ho_update_line(ho_ctx *c, ho_level *L, int x0, int y0, int x1, int y1, int mf, int mo)
{
    if ((x0 < 0) || (x0 >= L->sx) || (y0 < 0) || (y0 >= L->sy)) return 0;
    if ((x1 < 0) || (x1 >= L->sx) || (y1 < 0) || (y1 >= L->sy)) return 0;
    int dx = x1 - x0;
    int dy = y1 - y0;
    unsigned int abs_dx = (unsigned int)abs(dx);
    unsigned int abs_dy = (unsigned int)abs(dy);
    int offset_dx = dx > 0 ? 1 : -1;              /* util::sign  UtilFunctions.h:55-58 */
    int offset_dy = (dy > 0 ? 1 : -1) * L->sx;
    unsigned int start = (unsigned int)(y0 * L->sx + x0);
    if (abs_dx >= abs_dy) {
        int error_y = (int)(abs_dx / 2);
        ho_bresenham2d(c, L, abs_dx, abs_dy, error_y, offset_dx, offset_dy, start, mf);
        c->sum_free += abs_dx;
        c->sum_L += abs_dx + 1;
    } else {
        int error_x = (int)(abs_dy / 2);
        ho_bresenham2d(c, L, abs_dy, abs_dx, error_x, offset_dy, offset_dx, start, mf);
        c->sum_free += abs_dy;
        c->sum_L += abs_dy + 1;
    }
    unsigned int end = (unsigned int)(y1 * L->sx + x1);
    ho_cell_occ(c, L, end, mf, mo);
    c->valid_rays++;
    return 1;
}

/* OccGridMapBase::updateByScan  H/map/OccGridMapBase.h:118-168 */
static void ho_update_level(ho_ctx *c, int lvl, const float *xy, int n, float ox, float oy, const float *world_pose)
{
    ho_level *L = &c->lv[lvl];
    float f = L->pts_scale;
    int mf = L->cur_update_index + 1;
    int mo = L->cur_update_index + 2;
    float mp[3];
    ho_map_from_world(L, world_pose, mp);
    float cs = ho_cosf(c, mp[2]);
    float sn = ho_sinf(c, mp[2]);
    float nsn = -sn;
    float ox_l = ox * f, oy_l = oy * f;
    float bx = mp[0] + (cs * ox_l + nsn * oy_l);
    float by = mp[1] + (sn * ox_l + cs * oy_l);
    int bxi = ho_cell_of(bx + 0.5f), byi = ho_cell_of(by + 0.5f);
    for (int i = 0; i < n; ++i) {
        float px = xy[2 * i] * f, py = xy[2 * i + 1] * f;
        float ex = mp[0] + (cs * px + nsn * py);
        float ey = mp[1] + (sn * px + cs * py);
        ex += 0.5f;
        ey += 0.5f;
        int exi = ho_cell_of(ex), eyi = ho_cell_of(ey);
        if (bxi != exi || byi != eyi) ho_update_line(c, L, bxi, byi, exi, eyi, mf, mo);
    }
    L->last_update_index++;          /* setUpdated  GridMapBase.h:333 */
    L->cur_update_index += 3;        /* :167 */
}

/* MapRepMultiMap::updateByScan  H/slam_main/MapRepMultiMap.h:174-191 (+ onMapUpdated: cache epoch, no-op here) */
void ho_update_by_scan(ho_ctx *c, const float *xy, int n, float ox, float oy, const float *world_pose)
{
    c->sum_L = 0;
    c->sum_free = 0;
    c->valid_rays = 0;
    for (int lvl = 0; lvl < c->levels; ++lvl) {
        if (lvl == 0) ho_update_level(c, lvl, xy, n, ox, oy, world_pose);         /* :181-184 */
        else ho_update_level(c, lvl, c->mc_xy, c->mc_n, c->mc_origo[0], c->mc_origo[1], world_pose);  /* :187 */
    }
}

/* HectorSlamProcessor::update  H/slam_main/HectorSlamProcessor.h:81-108 ; returns 1 if the map was updated */
int ho_process(ho_ctx *c, const float *xy, int n, float ox, float oy, const float *hint, int map_without_matching,
               float *pose_out, float *cov_out)
{
    float np[3];
    if (!map_without_matching) {
        ho_match(c, xy, n, ox, oy, hint, np, c->last_cov);
    } else {
        np[0] = hint[0]; np[1] = hint[1]; np[2] = hint[2];
    }
    c->last_scan_match_pose[0] = np[0];
    c->last_scan_match_pose[1] = np[1];
    c->last_scan_match_pose[2] = np[2];
    int did = 0;
    if (ho_pose_diff_larger(np, c->last_map_update_pose, c->min_dist, c->min_ang) || map_without_matching) {
        ho_update_by_scan(c, xy, n, ox, oy, np);
        c->last_map_update_pose[0] = np[0];
        c->last_map_update_pose[1] = np[1];
        c->last_map_update_pose[2] = np[2];
        did = 1;
    }
    if (pose_out) { pose_out[0] = np[0]; pose_out[1] = np[1]; pose_out[2] = np[2]; }
    if (cov_out) memcpy(cov_out, c->last_cov, sizeof(float) * 9);
    return did;
}

/* ------------------------------------------------------------------------------------------ */
/* accessors */
void ho_get_last_pose(const ho_ctx *c, float *pose) { memcpy(pose, c->last_scan_match_pose, sizeof(float) * 3); }
void ho_get_last_cov(const ho_ctx *c, float *cov) { memcpy(cov, c->last_cov, sizeof(float) * 9); }
int ho_levels(const ho_ctx *c) { return c->levels; }
void ho_level_dims(const ho_ctx *c, int lvl, int *sx, int *sy) { *sx = c->lv[lvl].sx; *sy = c->lv[lvl].sy; }
void ho_get_level(const ho_ctx *c, int lvl, float *l_out, int *upd_out)
{
    const ho_level *L = &c->lv[lvl];
    size_t n = (size_t)L->sx * (size_t)L->sy;
    for (size_t i = 0; i < n; ++i) {
        if (l_out) l_out[i] = L->cells[i].l;
        if (upd_out) upd_out[i] = L->cells[i].upd;
    }
}
void ho_set_level(ho_ctx *c, int lvl, const float *l_in, const int *upd_in)
{
    ho_level *L = &c->lv[lvl];
    size_t n = (size_t)L->sx * (size_t)L->sy;
    for (size_t i = 0; i < n; ++i) {
        L->cells[i].l = l_in[i];
        L->cells[i].upd = upd_in[i];
    }
}
int ho_update_index(const ho_ctx *c, int lvl) { return c->lv[lvl].last_update_index; }
int ho_cur_update_index(const ho_ctx *c, int lvl) { return c->lv[lvl].cur_update_index; }
unsigned long long ho_sum_L(const ho_ctx *c) { return c->sum_L; }
unsigned long long ho_sum_free(const ho_ctx *c) { return c->sum_free; }
int ho_valid_rays(const ho_ctx *c) { return c->valid_rays; }
int ho_clamp_count(const ho_ctx *c) { return c->clamp_count; }
void ho_get_factors(const ho_ctx *c, float *lf, float *lo) { *lf = c->lf; *lo = c->lo; }
void ho_get_transform(const ho_ctx *c, int lvl, float *out8)
{
    const ho_level *L = &c->lv[lvl];
    out8[0] = L->scale; out8[1] = L->map_t[0]; out8[2] = L->map_t[1];
    out8[3] = L->inv_l00; out8[4] = L->inv_t[0]; out8[5] = L->inv_t[1];
    out8[6] = L->lim[0]; out8[7] = L->lim[1];
}

/* publishMap conversion  lesson4/src/hector_mapping/hector_slam.cc:287-304 */
void ho_publish_level(const ho_ctx *c, int lvl, int8_t *out)
{
    const ho_level *L = &c->lv[lvl];
    size_t n = (size_t)L->sx * (size_t)L->sy;
    for (size_t i = 0; i < n; ++i) {
        float l = L->cells[i].l;
        out[i] = l < 0.0f ? 0 : (l > 0.0f ? 100 : -1);
    }
}

/* Bresenham cell list of one ray (updateLineBresenhami without the cell updates), for KATs.
 * Writes up to cap linear offsets (free cells then the end cell); returns the count, 0 if cancelled. */
int ho_ray_cells(int sx, int sy, int x0, int y0, int x1, int y1, unsigned int *out, int cap)
{
    if ((x0 < 0) || (x0 >= sx) || (y0 < 0) || (y0 >= sy)) return 0;
    if ((x1 < 0) || (x1 >= sx) || (y1 < 0) || (y1 >= sy)) return 0;
    int dx = x1 - x0, dy = y1 - y0;
    unsigned int adx = (unsigned int)abs(dx), ady = (unsigned int)abs(dy);
    int odx = dx > 0 ? 1 : -1, ody = (dy > 0 ? 1 : -1) * sx;
    unsigned int off = (unsigned int)(y0 * sx + x0);
    unsigned int da, db; int oa, ob;
    if (adx >= ady) { da = adx; db = ady; oa = odx; ob = ody; }
    else { da = ady; db = adx; oa = ody; ob = odx; }
    int err = (int)(da / 2);
    int k = 0;
    if (k < cap) out[k] = off;
    k++;
    for (unsigned int i = 0; i + 1 < da; ++i) {
        off += oa;
        err += db;
        if ((unsigned int)err >= da) { off += ob; err -= da; }
        if (k < cap) out[k] = off;
        k++;
    }
    if (k < cap) out[k] = (unsigned int)(y1 * sx + x1);
    k++;
    return k;
}

/* exposed for the detmath cross-check */
float ho_det_sinf(float x) { return odm_sinf(x); }
float ho_det_cosf(float x) { return odm_cosf(x); }
float ho_det_expf(float x) { return odm_expf(x); }
/* getGridProbability (GridMapLogOdds.h:136-140) as the oracle and the kernels evaluate it; pinned
 * against the compiled reference header by tests/test_oracle_cpu.py::test_grid_probability_pinned */
float ho_det_prob(float l)
{
    const float odds = odm_expf(l);
    return odds / (odds + 1.0f);
}
/* probToLogOdds (GridMapLogOdds.h:153-157) as the oracle evaluates it */
float ho_det_prob_to_logodds(float p) { return ho_prob_to_logodds(p); }

/* ---- scan ingest: LaserScan -> DataContainer ------------------------------------------------------
 * HectorMappingRos::scanCallback (lesson4/src/hector_mapping/hector_slam.cc:186-198):
 *   projector_.projectLaser(scan, laser_point_cloud_, 30.0)  -- laser_geometry (third party, absent
 *   here, not vendored: PARITY UNPINNED for this step).  Restated from its published
 *   LaserProjection::projectLaser_: unit vectors cos / sin(angle_min + (double)i * angle_increment) in
 *   double (getUnitVectors_, cached per scan geometry), output = (double)range * unit, a point is kept
 *   when range < range_cutoff && range >= range_min (range_cutoff < 0 -> range_max), Point32 x / y are
 *   the double products rounded to float, z = 0.
 * then rosPointCloudToDataContainer (hector_slam.cc:320-362), followed statement by statement:
 *   origo = Vector2f(laserPos.x, laserPos.y) * scaleToMap                                   (:329)
 *   dist_sqr = x*x + y*y (float); keep if sqr_min < dist_sqr < sqr_max                      (:334-336)
 *   drop if x < 0 && dist_sqr < 0.5f                                                         (:338-341)
 *   drop if dist_sqr > use_max_scan_range^2 (double comparison)                               (:344-345)
 *   p = laserTransform * (x, y, z): tf dot products ((b0 x + b1 y) + b2 z) + origin, double   (:348)
 *   z_laser = (float)(p.z - laserPos.z); keep if z_min < z_laser < z_max                      (:351-353)
 *   add Vector2f((float)p.x, (float)p.y) * scaleToMap                                          (:356)
 * Returns the number of points written to xy_out (order preserved). */
void ho_unit_vectors(int n, float angle_min, float angle_increment, double *cs_out)
{
    for (int i = 0; i < n; ++i) {
        const double a = (double)angle_min + (double)i * (double)angle_increment;
        cs_out[2 * i] = cos(a);
        cs_out[2 * i + 1] = sin(a);
    }
}

int ho_ingest(int n, const float *ranges, const double *cs, double range_cutoff, float range_min, const double *tf,
              float sqr_min, float sqr_max, double use_max, float z_min, float z_max, float scale, float *xy_out,
              float *origo_out)
{
    origo_out[0] = (float)tf[9] * scale;
    origo_out[1] = (float)tf[10] * scale;
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const float range = ranges[i];
        if (!((range < range_cutoff) && (range >= range_min))) continue;
        const float x = (float)((double)range * cs[2 * i]);
        const float y = (float)((double)range * cs[2 * i + 1]);
        const float z = 0.0f;
        const float dist_sqr = x * x + y * y;
        if (!((dist_sqr > sqr_min) && (dist_sqr < sqr_max))) continue;
        if ((x < 0.0f) && (dist_sqr < 0.50f)) continue;
        if ((double)dist_sqr > use_max * use_max) continue;
        const double vx = (double)x, vy = (double)y, vz = (double)z;
        const double px = ((tf[0] * vx + tf[1] * vy) + tf[2] * vz) + tf[9];
        const double py = ((tf[3] * vx + tf[4] * vy) + tf[5] * vz) + tf[10];
        const double pz = ((tf[6] * vx + tf[7] * vy) + tf[8] * vz) + tf[11];
        const float zl = (float)(pz - tf[11]);
        if (zl > z_min && zl < z_max) {
            xy_out[2 * m] = (float)px * scale;
            xy_out[2 * m + 1] = (float)py * scale;
            ++m;
        }
    }
    return m;
}
