/* oracle/karto_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker of the Karto correlative matcher).
 *
 * PARITY UNPINNED against open_karto itself: the vendored library (lesson6/lib/open_karto) needs boost
 * (K/include/open_karto/Karto.h:37), which this image lacks, so it cannot be compiled here and no
 * reference output exists.  This file restates, sequentially and in the reference's evaluation order,
 * open_karto's ScanMatcher for one MatchScan call (K = lesson6/lib/open_karto):
 *   LocalizedRangeScan::Update          K/include/open_karto/Karto.h:5362-5404  (point readings)
 *   ScanMatcher::Create                 K/src/Mapper.cpp:126-171                 (grid sizes)
 *   CorrelationGrid::CreateGrid/Kernel  K/include/open_karto/Mapper.h:900-1100  (border, smear kernel)
 *   ScanMatcher::MatchScan              K/src/Mapper.cpp:184-300                 (coarse, expansion, fine)
 *   ScanMatcher::CorrelateScan          K/src/Mapper.cpp:309-523
 *   ComputePositionalCovariance         K/src/Mapper.cpp:535-626
 *   ComputeAngularCovariance            K/src/Mapper.cpp:638-690
 *   AddScans / AddScan / FindValidPoints K/src/Mapper.cpp:697-811
 *   CorrelationGrid::SmearPoint         K/include/open_karto/Mapper.h:971-1005
 *   GridIndexLookup::ComputeOffsets     K/include/open_karto/Karto.h:6409-6501
 *   ScanMatcher::GetResponse            K/src/Mapper.cpp:819-856
 *   math::Round / DoubleEqual / NormalizeAngle  K/include/open_karto/Math.h:87-233
 * Two deliberate, documented choices (DESIGN.md "Karto"): the transcendental functions are the
 * deterministic ones of detmath.h (odm_sin / odm_cos / odm_atan2) instead of libm, so the HIP product
 * can reproduce them bit for bit; and the smear kernel values are computed with libm exactly as
 * CalculateKernel does (they are host-side data in both builds).  The sensor pose of a scan is given
 * directly (identity laser offset).  Everything else -- the pose enumeration order, the integer
 * response sums, the penalties, the tie average in pose order, the covariances -- follows the
 * reference's statements one for one.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "detmath.h"

#define KO_PI 3.14159265358979323846
#define KO_2PI 6.28318530717958647692
#define KO_PI_180 0.01745329251994329577
#define KO_TOL 1e-06
#define KO_MAX_VARIANCE 500.0        /* Mapper.cpp:36 */
#define KO_DISTANCE_PENALTY_GAIN 0.2 /* Mapper.cpp:37 */
#define KO_ANGLE_PENALTY_GAIN 0.2    /* Mapper.cpp:38 */
#define KO_OCCUPIED 100              /* GridStates_Occupied, Karto.h:4196 */
#define KO_INVALID_SCAN INT32_MAX    /* Math.h:47 */

/* layout shared with include/slam2d/karto.h (kt_laser / kt_params) */
typedef struct {
    double minimum_angle;
    double angular_resolution;
    double minimum_range;
    double range_threshold;
    int n_readings;
    int pad_;
} ko_laser;

typedef struct {
    double search_size;               /* CorrelationSearchSpaceDimension (or LoopSearchSpaceDimension) */
    double resolution;                /* ...Resolution */
    double smear_deviation;           /* ...SmearDeviation */
    double distance_variance_penalty; /* as stored by Mapper: the square of the parameter */
    double angle_variance_penalty;    /* idem, rad^2 */
    double fine_search_angle_offset;
    double coarse_search_angle_offset;
    double coarse_angle_resolution;
    double minimum_angle_penalty;
    double minimum_distance_penalty;
    int use_response_expansion;
    int pad_;
} ko_params;

/* ---- Math.h ---------------------------------------------------------------------------------- */
static double ko_round(double v) { return v >= 0.0 ? floor(v + 0.5) : ceil(v - 0.5); }
static int ko_deq(double a, double b)
{
    double d = a - b;
    return d < 0.0 ? d >= -KO_TOL : d <= KO_TOL;
}
static double ko_max(double a, double b) { return a > b ? a : b; }
static double ko_sq(double v) { return v * v; }
static double ko_norm_angle(double a)
{
    if (!isfinite(a)) return a; /* the reference would spin; passed through as in the product */
    while (a < -KO_PI) {
        if (a < -KO_2PI) a += (uint32_t)(a / -KO_2PI) * KO_2PI;
        else a += KO_2PI;
    }
    while (a > KO_PI) {
        if (a > KO_2PI) a -= (uint32_t)(a / KO_2PI) * KO_2PI;
        else a -= KO_2PI;
    }
    return a;
}
static double ko_norm_angle_diff(double minuend, double subtrahend)
{
    while (minuend - subtrahend < -KO_PI) minuend += KO_2PI;
    while (minuend - subtrahend > KO_PI) minuend -= KO_2PI;
    return minuend;
}
static int ko_align8(int v) { return (v + 7) & ~7; }

/* ---- geometry (ScanMatcher::Create, CorrelationGrid) ------------------------------------------ */
typedef struct {
    double scale, res;        /* CoordinateConverter scale = 1/resolution; GetResolution() = 1/scale */
    int grid_size, border;    /* ROI side, ROI offset */
    int width, height, ws;    /* full grid, WidthStep = AlignValue(width, 8) */
    int data_size;            /* ws * height */
    int side, probs_ws;       /* search-space probability grid */
    int half, ksize;          /* smear kernel */
    unsigned char *kernel;
} ko_geom;

static int ko_geom_init(const ko_params *p, const ko_laser *L, ko_geom *g)
{
    memset(g, 0, sizeof(*g));
    if (!(p->resolution > 0) || !(p->search_size > 0) || p->smear_deviation < 0 || !(L->range_threshold > 0)) return -1;
    g->side = (int)(uint32_t)(ko_round(p->search_size / p->resolution) + 1);
    int margin = (int)(uint32_t)ceil(L->range_threshold / p->resolution);
    g->grid_size = g->side + 2 * margin;
    g->border = (int)ko_round(2.0 * p->smear_deviation / p->resolution) + 1; /* GetHalfKernelSize + 1 */
    g->width = g->grid_size + 2 * g->border;
    g->height = g->width;
    g->ws = ko_align8(g->width);
    g->data_size = g->ws * g->height;
    g->probs_ws = ko_align8(g->side);
    g->scale = 1.0 / p->resolution;
    g->res = 1.0 / g->scale;
    /* CalculateKernel (Mapper.h:1046-1086), with resolution = GetResolution() */
    if (!(p->smear_deviation >= 0.5 * g->res && p->smear_deviation <= 10 * g->res)) return -2;
    g->half = (int)ko_round(2.0 * p->smear_deviation / g->res);
    g->ksize = 2 * g->half + 1;
    g->kernel = (unsigned char *)malloc((size_t)g->ksize * g->ksize);
    if (!g->kernel) return -3;
    for (int i = -g->half; i <= g->half; i++)
        for (int j = -g->half; j <= g->half; j++) {
            double d = hypot(i * g->res, j * g->res);
            double z = exp(-0.5 * pow(d / p->smear_deviation, 2));
            uint32_t kv = (uint32_t)ko_round(z * KO_OCCUPIED);
            g->kernel[(i + g->half) + g->ksize * (j + g->half)] = (unsigned char)kv;
        }
    return 0;
}

int ko_grid_info(const ko_params *p, const ko_laser *L, int out[10])
{
    ko_geom g;
    int rc = ko_geom_init(p, L, &g);
    if (rc) return rc;
    out[0] = g.grid_size; out[1] = g.border; out[2] = g.width; out[3] = g.ws; out[4] = g.data_size;
    out[5] = g.side; out[6] = g.probs_ws; out[7] = g.half; out[8] = g.ksize; out[9] = 0;
    free(g.kernel);
    return 0;
}

int ko_kernel(const ko_params *p, const ko_laser *L, unsigned char *out, int cap)
{
    ko_geom g;
    int rc = ko_geom_init(p, L, &g);
    if (rc) return rc;
    int n = g.ksize * g.ksize;
    if (n <= cap) memcpy(out, g.kernel, (size_t)n);
    free(g.kernel);
    return n;
}

/* ---- scans (LocalizedRangeScan::Update) ------------------------------------------------------- */
typedef struct {
    double pose[3];
    const double *raw; /* range readings, n_readings */
    int n_raw;
    int npts;
    double *px, *py;
} ko_scan;

static int ko_scan_init(ko_scan *s, const ko_laser *L, const double *raw, const double pose[3])
{
    s->pose[0] = pose[0]; s->pose[1] = pose[1]; s->pose[2] = pose[2];
    s->raw = raw;
    s->n_raw = L->n_readings;
    s->px = (double *)malloc(sizeof(double) * (size_t)(L->n_readings > 0 ? L->n_readings : 1));
    s->py = (double *)malloc(sizeof(double) * (size_t)(L->n_readings > 0 ? L->n_readings : 1));
    if (!s->px || !s->py) return -3;
    s->npts = 0;
    for (int i = 0; i < L->n_readings; i++) {
        double r = raw[i];
        if (!(r >= L->minimum_range && r <= L->range_threshold)) continue; /* InRange */
        double angle = pose[2] + L->minimum_angle + (double)(uint32_t)i * L->angular_resolution;
        s->px[s->npts] = pose[0] + (r * odm_cos(angle));
        s->py[s->npts] = pose[1] + (r * odm_sin(angle));
        s->npts++;
    }
    return 0;
}
static void ko_scan_free(ko_scan *s)
{
    free(s->px);
    free(s->py);
}

/* ---- matcher state ---------------------------------------------------------------------------- */
typedef struct {
    const ko_params *p;
    ko_geom g;
    unsigned char *grid;
    double gox, goy;    /* correlation grid offset */
    double *probs;      /* side * probs_ws */
    double pgox, pgoy;  /* probability grid offset */
    int *lookup;        /* nAngles * npts */
    int lookup_cap;
    int n_angles, npts;
    int error;
    double *dump_resp;  /* test hook: the first coarse CorrelateScan's responses in pose order */
} ko_matcher;

static void ko_w2g(const ko_matcher *m, double x, double y, double ox, double oy, int *gx, int *gy)
{
    *gx = (int)ko_round((x - ox) * m->g.scale);
    *gy = (int)ko_round((y - oy) * m->g.scale);
}

/* CorrelationGrid::GridIndex with boundaryCheck (throws in the reference: flagged here) */
static int ko_roi_index(ko_matcher *m, int gx, int gy)
{
    int x = gx + m->g.border, y = gy + m->g.border;
    if (x < 0 || x >= m->g.width || y < 0 || y >= m->g.height) {
        m->error = 1;
        return 0;
    }
    return x + y * m->g.ws;
}

/* FindValidPoints (Mapper.cpp:755-811): valid[k] = 1 for points on the viewpoint's side */
static void ko_find_valid(const ko_scan *s, double vx, double vy, unsigned char *valid)
{
    const double min_sq = 0.1 * 0.1;
    memset(valid, 0, (size_t)(s->npts > 0 ? s->npts : 1));
    int trailing = 0;
    double fx = 0.0, fy = 0.0;
    int first_time = 1;
    for (int k = 0; k < s->npts; k++) {
        double cx = s->px[k], cy = s->py[k];
        if (first_time && !isnan(cx) && !isnan(cy)) {
            fx = cx;
            fy = cy;
            first_time = 0;
        }
        double dx = fx - cx, dy = fy - cy;
        if (dx * dx + dy * dy > min_sq) {
            double a = vy - fy;
            double b = fx - vx;
            double c = fy * vx - fx * vy;
            double ss = cx * a + cy * b + c;
            fx = cx;
            fy = cy;
            if (ss < 0.0) {
                trailing = k;
            } else {
                for (; trailing != k; ++trailing) valid[trailing] = 1;
            }
        }
    }
}

/* AddScan + SmearPoint (Mapper.cpp:716-748, Mapper.h:971-1005), doSmear = true */
static void ko_add_scan(ko_matcher *m, const ko_scan *s, double vx, double vy, unsigned char *valid)
{
    ko_find_valid(s, vx, vy, valid);
    const ko_geom *g = &m->g;
    for (int k = 0; k < s->npts; k++) {
        if (!valid[k]) continue;
        int gx, gy;
        ko_w2g(m, s->px[k], s->py[k], m->gox, m->goy, &gx, &gy);
        if (!(gx >= 0 && gx < g->grid_size) || !(gy >= 0 && gy < g->grid_size)) continue;
        int idx = (gx + g->border) + (gy + g->border) * g->ws;
        if (m->grid[idx] == KO_OCCUPIED) continue;
        m->grid[idx] = KO_OCCUPIED;
        /* SmearPoint: the centre cell is occupied (just set) */
        for (int j = -g->half; j <= g->half; j++) {
            unsigned char *row = m->grid + (gx + g->border) + (gy + j + g->border) * g->ws;
            int kc = g->half + g->ksize * (j + g->half);
            for (int i = -g->half; i <= g->half; i++) {
                unsigned char kv = g->kernel[i + kc];
                if (kv > row[i]) row[i] = kv;
            }
        }
    }
}

/* rotation part of Transform(sensorPose).InverseTransformPose: FromAxisAngle(0, 0, 1, 0 - h) */
static void ko_inv_rot(double h, double r[6])
{
    double rad = 0.0 - h;
    double c = odm_cos(rad), s = odm_sin(rad);
    double omc = 1.0 - c;
    double zero_omc = (0.0 * 0.0) * omc;
    r[0] = 0.0 * omc + c;        /* m00 = xx*omc + c */
    r[1] = zero_omc - 1.0 * s;   /* m01 = xyMCos - zSin */
    r[2] = zero_omc + 0.0 * s;   /* m02 = xzMCos + ySin */
    r[3] = zero_omc + 1.0 * s;   /* m10 = xyMCos + zSin */
    r[4] = 0.0 * omc + c;        /* m11 */
    r[5] = zero_omc - 0.0 * s;   /* m12 = yzMCos - xSin */
}

/* GridIndexLookup::ComputeOffsets (Karto.h:6409-6501) */
static int ko_compute_offsets(ko_matcher *m, const ko_scan *s, double center, double off, double res)
{
    int n_angles = (int)(uint32_t)(ko_round(off * 2.0 / res) + 1);
    int need = n_angles * (s->npts > 0 ? s->npts : 1);
    if (need > m->lookup_cap) {
        free(m->lookup);
        m->lookup = (int *)malloc(sizeof(int) * (size_t)need);
        if (!m->lookup) return -3;
        m->lookup_cap = need;
    }
    m->n_angles = n_angles;
    m->npts = s->npts;
    double R[6];
    ko_inv_rot(s->pose[2], R);
    double dth = ko_norm_angle(0.0 - s->pose[2]);
    double start = center - off;
    for (int a = 0; a < n_angles; a++) {
        double angle = start + (double)(uint32_t)a * res;
        double cs = odm_cos(angle), sn = odm_sin(angle);
        int *L = m->lookup + (size_t)a * s->npts;
        for (int k = 0; k < s->npts; k++) {
            double r = s->raw[k]; /* the reference indexes the raw readings with the point index */
            if (isnan(r) || isinf(r)) {
                L[k] = KO_INVALID_SCAN;
                continue;
            }
            double dx = s->px[k] - s->pose[0], dy = s->py[k] - s->pose[1];
            double lx = R[0] * dx + R[1] * dy + R[2] * dth;
            double ly = R[3] * dx + R[4] * dy + R[5] * dth;
            double ox = cs * lx - sn * ly;
            double oy = sn * lx + cs * ly;
            int gx, gy;
            ko_w2g(m, ox + m->gox, oy + m->goy, m->gox, m->goy, &gx, &gy);
            L[k] = gx + gy * m->g.ws;
        }
    }
    return 0;
}

/* GetResponse (Mapper.cpp:819-856) */
static double ko_response(const ko_matcher *m, int a, int gpi)
{
    double response = 0.0;
    if (m->npts == 0) return response;
    const int *L = m->lookup + (size_t)a * m->npts;
    for (int k = 0; k < m->npts; k++) {
        int64_t pgi = (int64_t)gpi + L[k];
        if (!(pgi >= 0 && pgi < m->g.data_size) || L[k] == KO_INVALID_SCAN) continue;
        response += m->grid[pgi];
    }
    response /= (double)(uint32_t)(m->npts * KO_OCCUPIED);
    return response;
}

typedef struct {
    double r, x, y, h;
} ko_pose_resp;

static void ko_positional_cov(ko_matcher *m, const double best[3], double best_resp, const double center[3],
                              double offx, double offy, double resx, double resy, double ares, double cov[9])
{
    for (int i = 0; i < 9; i++) cov[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (best_resp < KO_TOL) {
        cov[0] = KO_MAX_VARIANCE;
        cov[4] = KO_MAX_VARIANCE;
        cov[8] = 4 * ko_sq(ares);
        return;
    }
    double axx = 0, axy = 0, ayy = 0, norm = 0;
    double dx = best[0] - center[0], dy = best[1] - center[1];
    uint32_t nX = (uint32_t)(ko_round(offx * 2.0 / resx) + 1);
    double startX = -offx;
    uint32_t nY = (uint32_t)(ko_round(offy * 2.0 / resy) + 1);
    double startY = -offy;
    for (uint32_t iy = 0; iy < nY; iy++) {
        double y = startY + iy * resy;
        for (uint32_t ix = 0; ix < nX; ix++) {
            double x = startX + ix * resx;
            int gx, gy;
            ko_w2g(m, center[0] + x, center[1] + y, m->pgox, m->pgoy, &gx, &gy);
            if (gx < 0 || gx >= m->g.side || gy < 0 || gy >= m->g.side) {
                m->error = 2;
                continue;
            }
            double response = m->probs[gx + gy * m->g.probs_ws];
            if (response >= (best_resp - 0.1)) {
                norm += response;
                axx += (ko_sq(x - dx) * response);
                axy += ((x - dx) * (y - dy) * response);
                ayy += (ko_sq(y - dy) * response);
            }
        }
    }
    if (norm > KO_TOL) {
        double vxx = axx / norm, vxy = axy / norm, vyy = ayy / norm;
        double vtt = 4 * ko_sq(ares);
        double minxx = 0.1 * ko_sq(resx), minyy = 0.1 * ko_sq(resy);
        vxx = ko_max(vxx, minxx);
        vyy = ko_max(vyy, minyy);
        double mult = 1.0 / best_resp;
        cov[0] = vxx * mult;
        cov[1] = vxy * mult;
        cov[3] = vxy * mult;
        cov[4] = vyy * mult;
        cov[8] = vtt;
    }
    if (ko_deq(cov[0], 0.0)) cov[0] = KO_MAX_VARIANCE;
    if (ko_deq(cov[4], 0.0)) cov[4] = KO_MAX_VARIANCE;
}

static void ko_angular_cov(ko_matcher *m, const double best[3], double best_resp, const double center[3],
                           double aoff, double ares, double cov[9])
{
    double best_angle = ko_norm_angle_diff(best[2], center[2]);
    int gx, gy;
    ko_w2g(m, best[0], best[1], m->gox, m->goy, &gx, &gy);
    int gi = ko_roi_index(m, gx, gy);
    uint32_t n = (uint32_t)(ko_round(aoff * 2 / ares) + 1);
    double start = center[2] - aoff;
    double norm = 0.0, acc = 0.0;
    for (uint32_t a = 0; a < n; a++) {
        double angle = start + a * ares;
        double response = ko_response(m, (int)a, gi);
        if (response >= (best_resp - 0.1)) {
            norm += response;
            acc += (ko_sq(angle - best_angle) * response);
        }
    }
    if (norm > KO_TOL) {
        if (acc < KO_TOL) acc = ko_sq(ares);
        acc /= norm;
    } else {
        acc = 1000 * ko_sq(ares);
    }
    cov[8] = acc;
}

/* CorrelateScan (Mapper.cpp:309-523) */
static double ko_correlate(ko_matcher *m, const ko_scan *s, const double center[3], double offx, double offy,
                           double resx, double resy, double aoff, double ares, int penalize, double mean[3],
                           double cov[9], int fine)
{
    if (ko_compute_offsets(m, s, center[2], aoff, ares)) {
        m->error = 3;
        return 0.0;
    }
    const ko_params *p = m->p;
    if (!fine) {
        memset(m->probs, 0, sizeof(double) * (size_t)m->g.side * m->g.probs_ws);
        m->pgox = center[0] - offx;
        m->pgoy = center[1] - offy;
    }
    uint32_t nX = (uint32_t)(ko_round(offx * 2.0 / resx) + 1);
    double startX = -offx;
    uint32_t nY = (uint32_t)(ko_round(offy * 2.0 / resy) + 1);
    double startY = -offy;
    uint32_t nA = (uint32_t)(ko_round(aoff * 2.0 / ares) + 1);
    size_t np = (size_t)nX * nY * nA;
    ko_pose_resp *pr = (ko_pose_resp *)malloc(sizeof(ko_pose_resp) * np);
    if (!pr) {
        m->error = 3;
        return 0.0;
    }
    size_t c = 0;
    for (uint32_t iy = 0; iy < nY; iy++) {
        double y = startY + iy * resy;
        double ny = center[1] + y;
        double sqy = ko_sq(y);
        for (uint32_t ix = 0; ix < nX; ix++) {
            double x = startX + ix * resx;
            double nx = center[0] + x;
            double sqx = ko_sq(x);
            int gx, gy;
            ko_w2g(m, nx, ny, m->gox, m->goy, &gx, &gy);
            int gi = ko_roi_index(m, gx, gy);
            double start = center[2] - aoff;
            for (uint32_t a = 0; a < nA; a++) {
                double angle = start + a * ares;
                double response = ko_response(m, (int)a, gi);
                if (penalize && !ko_deq(response, 0.0)) {
                    double sqd = sqx + sqy;
                    double dp = 1.0 - (KO_DISTANCE_PENALTY_GAIN * sqd / p->distance_variance_penalty);
                    dp = ko_max(dp, p->minimum_distance_penalty);
                    double sqa = ko_sq(angle - center[2]);
                    double ap = 1.0 - (KO_ANGLE_PENALTY_GAIN * sqa / p->angle_variance_penalty);
                    ap = ko_max(ap, p->minimum_angle_penalty);
                    response *= (dp * ap);
                }
                pr[c].r = response;
                pr[c].x = nx;
                pr[c].y = ny;
                pr[c].h = ko_norm_angle(angle);
                c++;
            }
        }
    }
    if (!fine && m->dump_resp) {
        for (size_t i = 0; i < np; i++) m->dump_resp[i] = pr[i].r;
        m->dump_resp = NULL;
    }
    double best = -1;
    for (size_t i = 0; i < np; i++) {
        best = ko_max(best, pr[i].r);
        if (!fine) {
            int gx, gy;
            ko_w2g(m, pr[i].x, pr[i].y, m->pgox, m->pgoy, &gx, &gy);
            if (gx < 0 || gx >= m->g.side || gy < 0 || gy >= m->g.side) {
                m->error = 2;
                continue;
            }
            double *ptr = m->probs + gx + gy * m->g.probs_ws;
            *ptr = ko_max(pr[i].r, *ptr);
        }
    }
    double ax = 0.0, ay = 0.0, tx = 0.0, ty = 0.0;
    int cnt = 0;
    for (size_t i = 0; i < np; i++) {
        if (ko_deq(pr[i].r, best)) {
            ax += pr[i].x;
            ay += pr[i].y;
            tx += odm_cos(pr[i].h);
            ty += odm_sin(pr[i].h);
            cnt++;
        }
    }
    free(pr);
    double avg[3] = {0, 0, 0};
    if (cnt > 0) {
        ax /= cnt;
        ay /= cnt;
        tx /= cnt;
        ty /= cnt;
        avg[0] = ax;
        avg[1] = ay;
        avg[2] = odm_atan2(ty, tx);
    } else {
        m->error = 4; /* "Unable to find best position" */
    }
    if (!fine) ko_positional_cov(m, avg, best, center, offx, offy, resx, resy, ares, cov);
    else ko_angular_cov(m, avg, best, center, aoff, ares, cov);
    mean[0] = avg[0];
    mean[1] = avg[1];
    mean[2] = avg[2];
    if (best > 1.0) best = 1.0;
    return best;
}

/* ScanMatcher::MatchScan (Mapper.cpp:184-300).  Returns 0 or a negative error
 * (-1/-2/-3 parameters / memory, -4 an index the reference would have thrown on). */
static int ko_match_scan_ex(const ko_laser *L, const ko_params *p, const double *q_ranges, const double q_pose[3],
                            int n_base, const double *b_ranges, const double *b_poses, int do_penalize, int do_refine,
                            double mean[3], double cov[9], double *response, double *dump_resp)
{
    ko_matcher m;
    memset(&m, 0, sizeof(m));
    m.p = p;
    m.dump_resp = dump_resp;
    int rc = ko_geom_init(p, L, &m.g);
    if (rc) return rc;
    for (int i = 0; i < 9; i++) cov[i] = 0.0;
    if (L->n_readings == 0) {
        mean[0] = q_pose[0];
        mean[1] = q_pose[1];
        mean[2] = q_pose[2];
        cov[0] = KO_MAX_VARIANCE;
        cov[4] = KO_MAX_VARIANCE;
        cov[8] = 4 * ko_sq(p->coarse_angle_resolution);
        *response = 0.0;
        free(m.g.kernel);
        return 0;
    }
    m.grid = (unsigned char *)calloc((size_t)m.g.data_size, 1);
    m.probs = (double *)calloc((size_t)m.g.side * m.g.probs_ws, sizeof(double));
    ko_scan q;
    memset(&q, 0, sizeof(q));
    unsigned char *valid = (unsigned char *)malloc((size_t)L->n_readings + 1);
    if (!m.grid || !m.probs || !valid || ko_scan_init(&q, L, q_ranges, q_pose)) {
        rc = -3;
        goto out;
    }
    /* MatchScan steps 2-4: centre the grid on the scan pose */
    m.gox = q_pose[0] - (0.5 * (m.g.grid_size - 1) * m.g.res);
    m.goy = q_pose[1] - (0.5 * (m.g.grid_size - 1) * m.g.res);
    /* AddScans(rBaseScans, scanPose.GetPosition()) */
    for (int b = 0; b < n_base; b++) {
        ko_scan s;
        memset(&s, 0, sizeof(s));
        if (ko_scan_init(&s, L, b_ranges + (size_t)b * L->n_readings, b_poses + 3 * b)) {
            ko_scan_free(&s);
            rc = -3;
            goto out;
        }
        ko_add_scan(&m, &s, q_pose[0], q_pose[1], valid);
        ko_scan_free(&s);
    }
    {
        double sd = (double)m.g.side;
        double coff = 0.5 * (sd - 1) * m.g.res;
        double cres = 2 * m.g.res;
        double best = ko_correlate(&m, &q, q_pose, coff, coff, cres, cres, p->coarse_search_angle_offset,
                                   p->coarse_angle_resolution, do_penalize, mean, cov, 0);
        if (p->use_response_expansion) {
            if (ko_deq(best, 0.0)) {
                double aoff = p->coarse_search_angle_offset;
                for (int i = 0; i < 3; i++) {
                    aoff += 20 * KO_PI_180; /* DegreesToRadians(20) */
                    best = ko_correlate(&m, &q, q_pose, coff, coff, cres, cres, aoff, p->coarse_angle_resolution,
                                        do_penalize, mean, cov, 0);
                    if (!ko_deq(best, 0.0)) break;
                }
            }
        }
        if (do_refine) {
            double fo = cres * 0.5;
            double center[3] = {mean[0], mean[1], mean[2]};
            best = ko_correlate(&m, &q, center, fo, fo, m.g.res, m.g.res, 0.5 * p->coarse_angle_resolution,
                                p->fine_search_angle_offset, do_penalize, mean, cov, 1);
        }
        *response = best;
    }
    if (m.error) rc = -4;
out:
    ko_scan_free(&q);
    free(valid);
    free(m.grid);
    free(m.probs);
    free(m.lookup);
    free(m.g.kernel);
    return rc;
}

int ko_match_scan(const ko_laser *L, const ko_params *p, const double *q_ranges, const double q_pose[3], int n_base,
                  const double *b_ranges, const double *b_poses, int do_penalize, int do_refine, double mean[3],
                  double cov[9], double *response)
{
    return ko_match_scan_ex(L, p, q_ranges, q_pose, n_base, b_ranges, b_poses, do_penalize, do_refine, mean, cov,
                            response, NULL);
}

/* Test hook: the coarse window's responses (nY * nX * nAngles doubles, CorrelateScan's pose order
 * y, x, angle, Mapper.cpp:371-425) of one MatchScan, for the sharded-window exchange tests. */
int ko_coarse_responses(const ko_laser *L, const ko_params *p, const double *q_ranges, const double q_pose[3],
                        int n_base, const double *b_ranges, const double *b_poses, int do_penalize, double *resp_out)
{
    double mean[3], cov[9], r;
    return ko_match_scan_ex(L, p, q_ranges, q_pose, n_base, b_ranges, b_poses, do_penalize, 0, mean, cov, &r,
                            resp_out);
}

/* The correlation grid AddScans builds for a query pose (test hook: compared with the device grid). */
int ko_build_grid(const ko_laser *L, const ko_params *p, const double q_pose[3], int n_base, const double *b_ranges,
                  const double *b_poses, unsigned char *out)
{
    ko_matcher m;
    memset(&m, 0, sizeof(m));
    m.p = p;
    int rc = ko_geom_init(p, L, &m.g);
    if (rc) return rc;
    m.grid = out;
    memset(out, 0, (size_t)m.g.data_size);
    unsigned char *valid = (unsigned char *)malloc((size_t)L->n_readings + 1);
    m.gox = q_pose[0] - (0.5 * (m.g.grid_size - 1) * m.g.res);
    m.goy = q_pose[1] - (0.5 * (m.g.grid_size - 1) * m.g.res);
    for (int b = 0; b < n_base && valid; b++) {
        ko_scan s;
        memset(&s, 0, sizeof(s));
        if (ko_scan_init(&s, L, b_ranges + (size_t)b * L->n_readings, b_poses + 3 * b) == 0)
            ko_add_scan(&m, &s, q_pose[0], q_pose[1], valid);
        ko_scan_free(&s);
    }
    free(valid);
    free(m.g.kernel);
    return valid ? 0 : -3;
}
