/* oracle/gmapping_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * C restatement ("port") of the reference's single-scan GMapping grid (lesson4 make_gmapping_map):
 * GMapping::ComputeMap  lesson4/src/gmapping/gmapping.cc:171-242 over the reference grid headers
 * (G/ = lesson4/include/lesson4/gmapping/).  Pinned against oracle/_ref/libgmapping_ref.so, which
 * compiles those reference headers unmodified (tests/test_oracle_gmapping.py, and the committed
 * fixtures tests/golden/gmapping_*.npz produced by oracle/make_golden.py from the reference build).
 *
 * Dense row-major outputs [y*sx + x]: n (hits), visits, acc (2 floats).  Storage in the reference
 * is x-major patches (G/grid/harray2d.h, array2d.h); only the published values matter.
 * Pose extension (build-defined): see gmapping_ref_harness.cc.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ScanMatcherMap ctor geometry  G/grid/map.h:133-143 ; HierarchicalArray2D patch size 32 (harray2d.h:36) */
void gmo_map_geometry(double xmin, double ymin, double xmax, double ymax, double delta, int *sx, int *sy,
                      int *sx2, int *sy2, double *cx, double *cy)
{
    *cx = (xmin + xmax) / 2.0;
    *cy = (ymin + ymax) / 2.0;
    int px = ((int)ceil((xmax - xmin) / delta)) >> 5;
    int py = ((int)ceil((ymax - ymin) / delta)) >> 5;
    *sx = px << 5;
    *sy = py << 5;
    *sx2 = (int)round((*cx - xmin) / delta);
    *sy2 = (int)round((*cy - ymin) / delta);
}

/* Map::world2map  G/grid/map.h:171-174 */
static inline void gmo_world2map(double wx, double wy, double cx, double cy, double delta, int sx2, int sy2,
                                 int *mx, int *my)
{
    *mx = (int)round((wx - cx) / delta) + sx2;
    *my = (int)round((wy - cy) / delta) + sy2;
}

/* GridLineTraversal::gridLineCore + gridLine  G/grid/gridlinetraversal.h:27-207.
 * Returns num_points; writes points (x,y) into out (capacity must be >= max(|dx|,|dy|)+1). */
int gmo_grid_line(int sxp, int syp, int exp_, int eyp, int *out)
{
    int dx = abs(exp_ - sxp), dy = abs(eyp - syp);
    int incr1, incr2, d, x, y, xend, yend, xdir, ydir, cnt = 0;
    if (dy <= dx) {
        d = 2 * dy - dx;
        incr1 = 2 * dy;
        incr2 = 2 * (dy - dx);
        if (sxp > exp_) { x = exp_; y = eyp; ydir = -1; xend = sxp; }
        else { x = sxp; y = syp; ydir = 1; xend = exp_; }
        out[2 * cnt] = x; out[2 * cnt + 1] = y; cnt++;
        int up = ((eyp - syp) * ydir) > 0;
        while (x < xend) {
            x++;
            if (d < 0) d += incr1;
            else { y += up ? 1 : -1; d += incr2; }
            out[2 * cnt] = x; out[2 * cnt + 1] = y; cnt++;
        }
    } else {
        d = 2 * dx - dy;
        incr1 = 2 * dx;
        incr2 = 2 * (dx - dy);
        if (syp > eyp) { y = eyp; x = exp_; yend = syp; xdir = -1; }
        else { y = syp; x = sxp; yend = eyp; xdir = 1; }
        out[2 * cnt] = x; out[2 * cnt + 1] = y; cnt++;
        int right = ((exp_ - sxp) * xdir) > 0;
        while (y < yend) {
            y++;
            if (d < 0) d += incr1;
            else { x += right ? 1 : -1; d += incr2; }
            out[2 * cnt] = x; out[2 * cnt + 1] = y; cnt++;
        }
    }
    /* gridLine: reverse so that points[0] == start  (:196-206) */
    if (sxp != out[0] || syp != out[1]) {
        int half = cnt / 2;
        for (int i = 0, j = cnt - 1; i < half; i++, j--) {
            int tx = out[2 * i], ty = out[2 * i + 1];
            out[2 * i] = out[2 * j]; out[2 * i + 1] = out[2 * j + 1];
            out[2 * j] = tx; out[2 * j + 1] = ty;
        }
    }
    return cnt;
}

/* GMapping::ComputeMap  gmapping.cc:171-242 (fresh map per call, gmapping.cc:135).
 * Returns Σ(num_points - 1) (free-cell updates). Cells outside the map are an assert() in the
 * reference (G/grid/map.h:188-191); they are skipped here and counted in *oob. */
long long gmo_compute_map(double px, double py, double ct, double st, const float *ranges, int nbeams,
                          const double *a_cos, const double *a_sin, double max_range, double max_urange,
                          double xmin, double ymin, double xmax, double ymax, double delta, int32_t *n_out,
                          int32_t *visits_out, float *acc_out, int *num_hits, int *oob)
{
    int sx, sy, sx2, sy2;
    double cx, cy;
    gmo_map_geometry(xmin, ymin, xmax, ymax, delta, &sx, &sy, &sx2, &sy2, &cx, &cy);
    memset(n_out, 0, sizeof(int32_t) * (size_t)sx * sy);
    memset(visits_out, 0, sizeof(int32_t) * (size_t)sx * sy);
    if (acc_out) memset(acc_out, 0, sizeof(float) * 2 * (size_t)sx * sy);
    int p0x, p0y;
    gmo_world2map(px, py, cx, cy, delta, sx2, sy2, &p0x, &p0y);
    int cap = 2 * (sx + sy + 8);
    int *pts = (int *)malloc(sizeof(int) * 2 * (size_t)cap);
    long long nfree = 0;
    int nh = 0, bad = 0;
    /* free pass (all lines first, then hits: gmapping.cc:227-241) */
    double *hx = (double *)malloc(sizeof(double) * (size_t)(nbeams > 0 ? nbeams : 1));
    double *hy = (double *)malloc(sizeof(double) * (size_t)(nbeams > 0 ? nbeams : 1));
    for (int i = 0; i < nbeams; i++) {
        double d = ranges[i];
        if (d > max_range || d == 0.0 || !isfinite(d)) continue;
        if (d > max_urange) d = max_urange;
        double ca = a_cos[i], sa = a_sin[i];
        double dirx = ct * ca - st * sa;
        double diry = st * ca + ct * sa;
        double wx = px, wy = py;
        wx += d * dirx;
        wy += d * diry;
        int p1x, p1y;
        gmo_world2map(wx, wy, cx, cy, delta, sx2, sy2, &p1x, &p1y);
        int np = gmo_grid_line(p0x, p0y, p1x, p1y, pts);
        for (int k = 0; k < np - 1; k++) {
            int x = pts[2 * k], y = pts[2 * k + 1];
            if (x < 0 || y < 0 || x >= sx || y >= sy) { bad++; continue; }
            visits_out[(size_t)y * sx + x]++;
            nfree++;
        }
        if (d < max_urange) { hx[nh] = wx; hy[nh] = wy; nh++; }
    }
    for (int k = 0; k < nh; k++) {
        int x, y;
        gmo_world2map(hx[k], hy[k], cx, cy, delta, sx2, sy2, &x, &y);
        if (x < 0 || y < 0 || x >= sx || y >= sy) { bad++; continue; }
        size_t o = (size_t)y * sx + x;
        if (acc_out) {
            acc_out[2 * o] += (float)hx[k];
            acc_out[2 * o + 1] += (float)hy[k];
        }
        n_out[o]++;
        visits_out[o]++;
    }
    free(pts); free(hx); free(hy);
    *num_hits = nh;
    if (oob) *oob = bad;
    return nfree;
}

/* GMapping::PublishMap threshold loop  gmapping.cc:141-159 (occ = n/visits, -1 if unvisited) */
void gmo_publish(const int32_t *n, const int32_t *visits, int sx, int sy, double occ_thresh, int8_t *out)
{
    for (size_t o = 0; o < (size_t)sx * sy; o++) {
        double occ = visits[o] ? (double)n[o] * 1 / (double)visits[o] : -1;
        out[o] = occ < 0 ? -1 : (occ > occ_thresh ? 100 : 0);
    }
}
