/* oracle/plicp_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker of the PL-ICP path).
 *
 * PARITY UNPINNED.  lesson3's PL-ICP odometry (lesson3/src/plicp_odometry.cc:327-436) calls CSM's
 * `sm_icp` (lesson3/src/plicp_odometry.cc:391; CSM = apt ros-kinetic-csm, version not pinned by the
 * repo, install_dependence.sh:4, not vendored and absent from this image).  This file restates the
 * published algorithm of CSM's icp_loop (A. Censi, "An ICP variant using a point-to-line metric",
 * ICRA 2008) for the parameters the node sets (plicp_odometry.cc:58-186):
 *   per iteration: world coordinates of the new scan under the current estimate;
 *   correspondences: for each valid point the closest valid reference point j1 inside the polar
 *     search interval (max_angular_correction_deg, max_linear_correction; extrema rejected), j2 the
 *     closer of j1's next valid neighbours, dist^2 <= max_correspondence_dist^2 (exact search: the
 *     node's use_corr_tricks only accelerates the same search);
 *   fail if fewer than 5 % of the rays have a correspondence;
 *   trimming: point-to-segment distance e_i; keep e_i <= min(e_(k*maxPerc), mult * e_(k*adaptive_order))
 *     (order statistics of the k valid errors); outliers_remove_doubles: drop i when
 *     dist2_j1(i) > 9 * min over i' sharing j1;
 *   estimate: point-to-line GPC -- minimise sum (R p + t - q)^T C (R p + t - q), C = n n^T (n the
 *     normal of segment j1-j2), over x = (tx, ty, cos, sin) with cos^2 + sin^2 = 1: Lagrange
 *     multiplier = the largest root of |(S + l I)^-1 h| = 1 (bisection, 200 steps);
 *   stop on |delta| < epsilon (delta = x_old^-1 (+) x_new), on a repeated correspondence hash
 *     (oscillation), or after max_iterations.
 * The GPU kernel (csrc/plicp_kernels.hip) evaluates the same double-precision op sequence (no FMA,
 * deterministic atan / sin / cos of detmath.h, the same summation order with reduce_threads = 256),
 * so the two agree bit for bit; agreement with the absent CSM binary is not claimed.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "detmath.h"

typedef struct {
    double max_angular_correction_deg;  /* 45 */
    double max_linear_correction;       /* 1.0 m */
    double epsilon_xy;                  /* 1e-6 */
    double epsilon_theta;               /* 1e-6 */
    double max_correspondence_dist;     /* 1.0 m */
    double outliers_maxPerc;            /* 0.90 */
    double outliers_adaptive_order;     /* 0.7 */
    double outliers_adaptive_mult;      /* 2.0 */
    int max_iterations;                 /* 10 */
    int use_point_to_line_distance;     /* 1 */
    int outliers_remove_doubles;        /* 1 */
    int pad_;
} plo_params;

#define PLO_MAX_RAYS 8192

typedef struct {
    int n;
    double px[PLO_MAX_RAYS], py[PLO_MAX_RAYS];
    int valid[PLO_MAX_RAYS];
    int up[PLO_MAX_RAYS], down[PLO_MAX_RAYS];  /* next valid index above / below, -1 if none */
} plo_scan;

static void plo_cartesian(plo_scan *s, int n, double angle_min, double angle_inc, const double *theta, const double *r)
{
    s->n = n;
    for (int i = 0; i < n; ++i) {
        const double th = theta ? theta[i] : angle_min + i * angle_inc;  /* LaserScanToLDP (plicp_odometry.cc:306) */
        s->valid[i] = r[i] > 0.0;                              /* readings = -1 for invalid (:302) */
        s->px[i] = s->valid[i] ? r[i] * odm_cos(th) : 0.0;     /* ld_compute_cartesian */
        s->py[i] = s->valid[i] ? r[i] * odm_sin(th) : 0.0;
    }
    int last = -1;
    for (int i = 0; i < n; ++i) { s->down[i] = last; if (s->valid[i]) last = i; }
    last = -1;
    for (int i = n - 1; i >= 0; --i) { s->up[i] = last; if (s->valid[i]) last = i; }
}

/* projection_on_line / projection_on_segment / distance (CSM math_utils) */
static double plo_dist_to_segment(double ax, double ay, double bx, double by, double x, double y)
{
    const double t0 = ax - bx, t1 = ay - by;
    const double one_on_r = 1.0 / sqrt(t0 * t0 + t1 * t1);
    const double nx = t1 * one_on_r, ny = -t0 * one_on_r;
    const double rho = nx * ax + ny * ay;
    const double lx = (nx * rho + ny * ny * x) - nx * ny * y;
    const double ly = (ny * rho - nx * ny * x) + nx * nx * y;
    double qx, qy;
    if ((lx - ax) * (lx - bx) + (ly - ay) * (ly - by) < 0.0) {
        qx = lx; qy = ly;
    } else {
        const double da = (ax - x) * (ax - x) + (ay - y) * (ay - y);
        const double db = (bx - x) * (bx - x) + (by - y) * (by - y);
        if (da < db) { qx = ax; qy = ay; } else { qx = bx; qy = by; }
    }
    return sqrt((qx - x) * (qx - x) + (qy - y) * (qy - y));
}

/* possible_interval (CSM icp_corr_dumb.c) */
static void plo_interval(const plo_params *p, double wx, double wy, int n, double min_theta, double max_theta,
                         int *from, int *to)
{
    const double angle_res = (max_theta - min_theta) / n;
    const double norm = sqrt(wx * wx + wy * wy);
    const double delta = fabs(p->max_angular_correction_deg * (ODM_PI / 180.0)) + fabs(odm_atan(p->max_linear_correction / norm));
    const int range = (int)ceil(delta / angle_res);
    double start_theta = odm_atan2(wy, wx);
    if (start_theta < min_theta) start_theta += 2.0 * ODM_PI;
    if (start_theta > max_theta) start_theta -= 2.0 * ODM_PI;
    const int start_cell = (int)((start_theta - min_theta) / (max_theta - min_theta) * n);
    int f = start_cell - range, t = start_cell + range;
    *from = f < 0 ? 0 : (f > n - 1 ? n - 1 : f);
    *to = t < 0 ? 0 : (t > n - 1 ? n - 1 : t);
}

/* 14 GPC terms of one correspondence: bigM upper triangle (10) and g (4) */
static void plo_terms(double px, double py, double qx, double qy, double c00, double c01, double c11, double *o)
{
    o[0] = c00;
    o[1] = c01;
    o[2] = c00 * px + c01 * py;
    o[3] = -c00 * py + c01 * px;
    o[4] = c11;
    o[5] = c01 * px + c11 * py;
    o[6] = -c01 * py + c11 * px;
    o[7] = (c00 * px * px + 2.0 * c01 * px * py) + c11 * py * py;
    o[8] = ((-c00 * px * py + c01 * px * px) - c01 * py * py) + c11 * px * py;
    o[9] = (c00 * py * py - 2.0 * c01 * px * py) + c11 * px * px;
    const double a0 = c00 * qx + c01 * qy, a1 = c01 * qx + c11 * qy;
    o[10] = -2.0 * a0;
    o[11] = -2.0 * a1;
    o[12] = -2.0 * (px * a0 + py * a1);
    o[13] = -2.0 * (-py * a0 + px * a1);
}

/* sum of per-ray 14-vectors over valid entries: reduce_threads = 0 sequential; T > 0 the GPU order
 * (thread t sums i = t, t+T, ...; 64-lane xor butterfly; waves ((w0+w2)+(w1+w3)) for T = 256) */
static void plo_reduce(const double (*v)[14], const int *ok, int n, int T, double *out)
{
    for (int k = 0; k < 14; ++k) out[k] = 0.0;
    if (T <= 0) {
        for (int i = 0; i < n; ++i)
            if (ok[i])
                for (int k = 0; k < 14; ++k) out[k] = out[k] + v[i][k];
        return;
    }
    double *acc = (double *)calloc((size_t)T * 14, sizeof(double));
    for (int t = 0; t < T; ++t)
        for (int i = t; i < n; i += T)
            if (ok[i])
                for (int k = 0; k < 14; ++k) acc[t * 14 + k] = acc[t * 14 + k] + v[i][k];
    double *tmp = (double *)malloc(sizeof(double) * (size_t)T * 14);
    for (int off = 32; off >= 1; off >>= 1) {
        for (int t = 0; t < T; ++t)
            for (int k = 0; k < 14; ++k) tmp[t * 14 + k] = acc[t * 14 + k] + acc[(((t & 63) ^ off) + (t & ~63)) * 14 + k];
        memcpy(acc, tmp, sizeof(double) * (size_t)T * 14);
    }
    const int W = T / 64;
    for (int k = 0; k < 14; ++k) {
        if (W == 4) out[k] = (acc[0 * 64 * 14 + k] + acc[2 * 64 * 14 + k]) + (acc[1 * 64 * 14 + k] + acc[3 * 64 * 14 + k]);
        else {
            double s = 0.0;
            for (int w = 0; w < W; ++w) s = s + acc[w * 64 * 14 + k];
            out[k] = s;
        }
    }
    free(acc);
    free(tmp);
}

/* GPC solve: x = (tx, ty, theta); returns 0 if degenerate */
static int plo_gpc_solve(const double *m, double *x)
{
    const double m00 = m[0], m01 = m[1], m02 = m[2], m03 = m[3], m11 = m[4], m12 = m[5], m13 = m[6];
    const double m22 = m[7], m23 = m[8], m33 = m[9];
    const double g0 = m[10], g1 = m[11], g2 = m[12], g3 = m[13];
    const double detA = m00 * m11 - m01 * m01;
    if (!(detA > 0.0)) return 0;
    const double ia00 = m11 / detA, ia01 = -m01 / detA, ia11 = m00 / detA;
    /* Ainv B (2x2), B = [[m02, m03], [m12, m13]] */
    const double ab00 = ia00 * m02 + ia01 * m12, ab01 = ia00 * m03 + ia01 * m13;
    const double ab10 = ia01 * m02 + ia11 * m12, ab11 = ia01 * m03 + ia11 * m13;
    /* S = D - B^T Ainv B */
    const double s00 = m22 - (m02 * ab00 + m12 * ab10);
    const double s01 = m23 - (m02 * ab01 + m12 * ab11);
    const double s11 = m33 - (m03 * ab01 + m13 * ab11);
    /* h = -g_r / 2 + B^T Ainv g_t / 2 */
    const double agt0 = ia00 * g0 + ia01 * g1, agt1 = ia01 * g0 + ia11 * g1;
    const double h0 = -0.5 * g2 + 0.5 * (m02 * agt0 + m12 * agt1);
    const double h1 = -0.5 * g3 + 0.5 * (m03 * agt0 + m13 * agt1);
    const double hn = sqrt(h0 * h0 + h1 * h1);
    if (!(hn > 0.0)) return 0;
    const double mid = 0.5 * (s00 + s11);
    const double rad = sqrt(0.25 * (s00 - s11) * (s00 - s11) + s01 * s01);
    const double lmin = mid - rad;
    double lo = -lmin, hi = -lmin + hn;
    for (int it = 0; it < 200; ++it) {
        const double l = 0.5 * (lo + hi);
        const double a = s00 + l, d = s11 + l;
        const double det = a * d - s01 * s01;
        const double r0 = (d * h0 - s01 * h1) / det, r1 = (a * h1 - s01 * h0) / det;
        if (r0 * r0 + r1 * r1 > 1.0) lo = l; else hi = l;
    }
    const double l = 0.5 * (lo + hi);
    const double a = s00 + l, d = s11 + l;
    const double det = a * d - s01 * s01;
    const double r0 = (d * h0 - s01 * h1) / det, r1 = (a * h1 - s01 * h0) / det;
    /* t = -Ainv (B r + g_t / 2) */
    const double br0 = (m02 * r0 + m03 * r1) + 0.5 * g0, br1 = (m12 * r0 + m13 * r1) + 0.5 * g1;
    x[0] = -(ia00 * br0 + ia01 * br1);
    x[1] = -(ia01 * br0 + ia11 * br1);
    x[2] = odm_atan2(r1, r0);
    return isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]);
}

/* correspondence-set hash for oscillation detection (the role of CSM's ld_corr_hash): an
 * order-free sum of mixed (i, j1, j2) words, so the GPU computes it with one integer reduction */
static unsigned plo_mix(unsigned x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

static unsigned plo_hash(const int *j1, const int *j2, const int *ok, int n)
{
    unsigned h = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned v = ok[i] ? (unsigned)(j1[i] + 1000 * j2[i]) : 0xFFFFFFFFu;
        h += plo_mix((unsigned)i * 0x9E3779B9U ^ v);
    }
    return h & 0x7FFFFFFFu;
}

static double plo_angle_diff(double a, double b)
{
    double d = a - b;
    while (d > ODM_PI) d -= 2.0 * ODM_PI;
    while (d <= -ODM_PI) d += 2.0 * ODM_PI;
    return d;
}

static double plo_kth(double *v, int k, int idx)  /* idx-th smallest of v[0..k) (v is sorted in place) */
{
    for (int i = 1; i < k; ++i) {  /* insertion sort: k <= 8192, test sizes only */
        double x = v[i];
        int j = i - 1;
        while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; --j; }
        v[j + 1] = x;
    }
    return v[idx];
}

/* sm_icp for one scan pair; returns valid (all_is_okay).  info: iterations, nvalid; error. */
int plo_icp_theta(const plo_params *p, int n, double angle_min, double angle_inc, const double *theta,
                  const double *ref_r, const double *sens_r, const double *first_guess, int reduce_threads,
                  double *x_out, int *iterations_out, int *nvalid_out, double *error_out, int *trace_hashes)
{
    if (n < 2 || n > PLO_MAX_RAYS) return 0;
    plo_scan *ref = (plo_scan *)malloc(sizeof(plo_scan));
    plo_scan *sens = (plo_scan *)malloc(sizeof(plo_scan));
    plo_cartesian(ref, n, angle_min, angle_inc, theta, ref_r);
    plo_cartesian(sens, n, angle_min, angle_inc, theta, sens_r);
    /* ldp->min_theta / max_theta = theta[0] / theta[n-1] (LaserScanToLDP, plicp_odometry.cc:312-313) */
    const double min_theta = theta ? theta[0] : angle_min, max_theta = theta ? theta[n - 1] : angle_min + (n - 1) * angle_inc;
    int *j1 = (int *)malloc(sizeof(int) * n), *j2 = (int *)malloc(sizeof(int) * n), *ok = (int *)malloc(sizeof(int) * n);
    double *d2 = (double *)malloc(sizeof(double) * n), *e = (double *)malloc(sizeof(double) * n);
    double *sorted = (double *)malloc(sizeof(double) * n), *best_j = (double *)malloc(sizeof(double) * n);
    double (*terms)[14] = (double (*)[14])malloc(sizeof(double) * 14 * (size_t)n);
    unsigned hashes[64];
    double x_old[3] = {first_guess[0], first_guess[1], first_guess[2]}, x_new[3] = {x_old[0], x_old[1], x_old[2]};
    int all_ok = 1, it = 0, nvalid = 0;
    double total_error = 0.0;
    const double maxd2 = p->max_correspondence_dist * p->max_correspondence_dist;
    const int max_it = p->max_iterations < 64 ? p->max_iterations : 64;
    for (it = 0; it < max_it; ++it) {
        const double c = odm_cos(x_old[2]), s = odm_sin(x_old[2]);
        int ncorr = 0;
        for (int i = 0; i < n; ++i) {
            ok[i] = 0;
            j1[i] = j2[i] = -1;
            if (!sens->valid[i]) continue;
            /* ld_compute_world_coords */
            const double wx = (c * sens->px[i] - s * sens->py[i]) + x_old[0];
            const double wy = (s * sens->px[i] + c * sens->py[i]) + x_old[1];
            int from, to;
            plo_interval(p, wx, wy, n, min_theta, max_theta, &from, &to);
            int b1 = -1;
            double best = 0.0;
            for (int j = from; j <= to; ++j) {
                if (!ref->valid[j]) continue;
                const double dx = wx - ref->px[j], dy = wy - ref->py[j];
                const double dist = dx * dx + dy * dy;
                if (dist > maxd2) continue;
                if (b1 == -1 || dist < best) { b1 = j; best = dist; }
            }
            if (b1 == -1 || b1 == 0 || b1 == n - 1) continue;   /* no match / extrema */
            const int up = ref->up[b1], dn = ref->down[b1];
            if (up == -1 && dn == -1) continue;
            int b2;
            if (up == -1) b2 = dn;
            else if (dn == -1) b2 = up;
            else {
                const double du = (wx - ref->px[up]) * (wx - ref->px[up]) + (wy - ref->py[up]) * (wy - ref->py[up]);
                const double dd = (wx - ref->px[dn]) * (wx - ref->px[dn]) + (wy - ref->py[dn]) * (wy - ref->py[dn]);
                b2 = du < dd ? up : dn;
            }
            j1[i] = b1;
            j2[i] = b2;
            d2[i] = best;
            ok[i] = 1;
            ++ncorr;
            e[i] = plo_dist_to_segment(ref->px[b1], ref->py[b1], ref->px[b2], ref->py[b2], wx, wy);
        }
        if (ncorr < 0.05 * n) { all_ok = 0; break; }
        /* kill_outliers_trim */
        int k = 0;
        for (int i = 0; i < n; ++i) if (ok[i]) sorted[k++] = e[i];
        int order = (int)floor(k * p->outliers_maxPerc);
        order = order < 0 ? 0 : (order > k - 1 ? k - 1 : order);
        int order2 = (int)floor(k * p->outliers_adaptive_order);
        order2 = order2 < 0 ? 0 : (order2 > k - 1 ? k - 1 : order2);
        const double lim1 = plo_kth(sorted, k, order);
        const double lim2 = p->outliers_adaptive_mult * sorted[order2];
        const double limit = lim1 < lim2 ? lim1 : lim2;
        nvalid = 0;
        for (int i = 0; i < n; ++i) {
            if (!ok[i]) continue;
            if (e[i] > limit) ok[i] = 0;
            else ++nvalid;
        }
        {   /* total error in the same summation order as the 14 GPC sums */
            for (int i = 0; i < n; ++i) {
                terms[i][0] = ok[i] ? e[i] : 0.0;
                for (int q = 1; q < 14; ++q) terms[i][q] = 0.0;
            }
            double tmp[14];
            plo_reduce((const double (*)[14])terms, ok, n, reduce_threads, tmp);
            total_error = tmp[0];
        }
        /* kill_outliers_double */
        if (p->outliers_remove_doubles) {
            for (int j = 0; j < n; ++j) best_j[j] = 1000000.0;
            for (int i = 0; i < n; ++i) if (ok[i] && d2[i] < best_j[j1[i]]) best_j[j1[i]] = d2[i];
            for (int i = 0; i < n; ++i) if (ok[i] && d2[i] > 9.0 * best_j[j1[i]]) ok[i] = 0;
        }
        /* compute_next_estimate (point-to-line GPC) */
        for (int i = 0; i < n; ++i) {
            if (!ok[i]) continue;
            const double qx = ref->px[j1[i]], qy = ref->py[j1[i]];
            double c00, c01, c11;
            if (p->use_point_to_line_distance) {
                const double dfx = ref->px[j1[i]] - ref->px[j2[i]], dfy = ref->py[j1[i]] - ref->py[j2[i]];
                const double one_on_norm = 1.0 / sqrt(dfx * dfx + dfy * dfy);
                const double nx = dfy * one_on_norm, ny = -dfx * one_on_norm;
                c00 = nx * nx; c01 = nx * ny; c11 = ny * ny;
            } else {
                c00 = 1.0; c01 = 0.0; c11 = 1.0;
            }
            plo_terms(sens->px[i], sens->py[i], qx, qy, c00, c01, c11, terms[i]);
        }
        double m[14];
        plo_reduce((const double (*)[14])terms, ok, n, reduce_threads, m);
        if (!plo_gpc_solve(m, x_new)) { all_ok = 0; break; }
        /* pose_diff_d(x_new, x_old) */
        const double co = odm_cos(x_old[2]), so = odm_sin(x_old[2]);
        const double ddx = x_new[0] - x_old[0], ddy = x_new[1] - x_old[1];
        const double dl0 = co * ddx + so * ddy, dl1 = -so * ddx + co * ddy, dl2 = plo_angle_diff(x_new[2], x_old[2]);
        hashes[it] = plo_hash(j1, j2, ok, n);
        if (trace_hashes) trace_hashes[it] = (int)hashes[it];
        int loop = 0;
        for (int a = 0; a < it; ++a) if (hashes[a] == hashes[it]) loop = 1;
        if (loop) break;
        if (fabs(dl0) < p->epsilon_xy && fabs(dl1) < p->epsilon_xy && fabs(dl2) < p->epsilon_theta) break;
        x_old[0] = x_new[0]; x_old[1] = x_new[1]; x_old[2] = x_new[2];
    }
    x_out[0] = x_new[0]; x_out[1] = x_new[1]; x_out[2] = x_new[2];
    if (iterations_out) *iterations_out = it + (it < max_it ? 1 : 0);
    if (nvalid_out) *nvalid_out = nvalid;
    if (error_out) *error_out = total_error;
    free(ref); free(sens); free(j1); free(j2); free(ok); free(d2); free(e); free(sorted); free(best_j); free(terms);
    return all_ok;
}

/* sm_icp with the uniform angles angle_min + i * angle_inc */
int plo_icp(const plo_params *p, int n, double angle_min, double angle_inc, const double *ref_r, const double *sens_r,
            const double *first_guess, int reduce_threads, double *x_out, int *iterations_out, int *nvalid_out,
            double *error_out, int *trace_hashes)
{
    return plo_icp_theta(p, n, angle_min, angle_inc, NULL, ref_r, sens_r, first_guess, reduce_threads, x_out,
                         iterations_out, nvalid_out, error_out, trace_hashes);
}

void plo_default_params(plo_params *p)
{
    /* ScanMatchPLICP::InitParams (lesson3/src/plicp_odometry.cc:74-186) */
    p->max_angular_correction_deg = 45.0;
    p->max_linear_correction = 1.0;
    p->max_iterations = 10;
    p->epsilon_xy = 0.000001;
    p->epsilon_theta = 0.000001;
    p->max_correspondence_dist = 1.0;
    p->use_point_to_line_distance = 1;
    p->outliers_maxPerc = 0.90;
    p->outliers_adaptive_order = 0.7;
    p->outliers_adaptive_mult = 2.0;
    p->outliers_remove_doubles = 1;
    p->pad_ = 0;
}
