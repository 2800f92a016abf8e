// oracle/gmapping_ref_harness.cc -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libgmapping_ref.so).
//
// Compiles the REFERENCE GMapping grid core unmodified, where it lies under /root/reference
// (lesson4/include/lesson4/gmapping/grid/{map,harray2d,array2d,gridlinetraversal}.h and
// utils/point.h, std-only).  No reference source is copied into this repository.
//
// The ROS node glue GMapping::ComputeMap (lesson4/src/gmapping/gmapping.cc:171-242) needs ROS only
// for `scan_msg->ranges`, so it is restated here over a plain float array.  Every line/cell/count
// operation is done by the reference headers: Map::world2map, GridLineTraversal::gridLine,
// HierarchicalArray2D::setActiveArea/allocActiveArea, PointAccumulator::update.
//
// Extension (build-defined): the reference fixes the laser pose lp = (0,0,0)
// (gmapping.cc:177) and ignores theta (gmapping.cc:196-198).  The harness accepts a pose
// (x, y, theta) and per-particle (cos theta, sin theta); the beam direction is
// (ct*ca - st*sa, st*ca + ct*sa), which for theta = 0 (ct = 1, st = 0) reduces exactly to the
// reference's (ca, sa).  Parity with the reference is therefore pinned for theta = 0 poses.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "lesson4/gmapping/grid/gridlinetraversal.h"
#include "lesson4/gmapping/grid/map.h"

using namespace gmapping;

extern "C" {

// Returns the map size in *sx/*sy for the given bounds (ScanMatcherMap ctor, G/grid/map.h:133-143).
void gmr_map_size(double xmin, double ymin, double xmax, double ymax, double delta, int *sx, int *sy)
{
    Point center((xmin + xmax) / 2.0, (ymin + ymax) / 2.0);
    ScanMatcherMap m(center, xmin, ymin, xmax, ymax, delta);
    *sx = m.getMapSizeX();
    *sy = m.getMapSizeY();
}

// One ComputeMap on a fresh map (gmapping.cc:135, :171-242).
// Outputs are dense row-major [y*sx + x]:  n_out (hits), visits_out, acc_out (2 floats per cell), any
// may be NULL (all NULL: ComputeMap alone, as bench.py times the reference's CPU path).
// Returns the number of free-cell updates (Σ (num_points-1)).
long long gmr_compute_map(double px, double py, double ct, double st,
                          const float *ranges, int nbeams, const double *a_cos, const double *a_sin,
                          double max_range, double max_urange,
                          double xmin, double ymin, double xmax, double ymax, double delta,
                          int32_t *n_out, int32_t *visits_out, float *acc_out, int *num_hits)
{
    Point center((xmin + xmax) / 2.0, (ymin + ymax) / 2.0);
    ScanMatcherMap map(center, xmin, ymin, xmax, ymax, delta);
    std::vector<GridLineTraversalLine> line_lists;
    std::vector<Point> hit_lists;

    OrientedPoint lp(px, py, 0.0);
    IntPoint p0 = map.world2map(lp);
    HierarchicalArray2D<PointAccumulator>::PointSet activeArea;
    for (int i = 0; i < nbeams; i++) {
        double d = ranges[i];
        if (d > max_range || d == 0.0 || !std::isfinite(d))
            continue;
        if (d > max_urange)
            d = max_urange;
        Point phit = lp;
        double ca = a_cos[i], sa = a_sin[i];
        double dirx = ct * ca - st * sa;
        double diry = st * ca + ct * sa;
        phit.x += d * dirx;
        phit.y += d * diry;
        IntPoint p1 = map.world2map(phit);
        GridLineTraversalLine line;
        GridLineTraversal::gridLine(p0, p1, &line);
        line_lists.push_back(line);
        for (int k = 0; k < line.num_points - 1; k++)
            activeArea.insert(map.storage().patchIndexes(line.points[k]));
        if (d < max_urange) {
            IntPoint cp = map.storage().patchIndexes(p1);
            activeArea.insert(cp);
            hit_lists.push_back(phit);
        }
    }
    map.storage().setActiveArea(activeArea, true);
    map.storage().allocActiveArea();
    long long nfree = 0;
    for (auto &line : line_lists) {
        for (int k = 0; k < line.num_points - 1; k++) {
            map.cell(line.points[k]).update(false, Point(0, 0));
            nfree++;
        }
    }
    for (auto &hit : hit_lists) {
        IntPoint p1 = map.world2map(hit);
        map.cell(p1).update(true, hit);
    }
    *num_hits = (int)hit_lists.size();
    if (!n_out && !visits_out && !acc_out) return nfree;  // ComputeMap only (CPU-baseline timing)
    int sx = map.getMapSizeX(), sy = map.getMapSizeY();
    const ScanMatcherMap &cm = map;
    for (int y = 0; y < sy; y++) {
        for (int x = 0; x < sx; x++) {
            IntPoint p(x, y);
            const PointAccumulator &c = cm.cell(p);
            size_t o = (size_t)y * sx + x;
            if (n_out) n_out[o] = c.n;
            if (visits_out) visits_out[o] = c.visits;
            if (acc_out) {
                acc_out[2 * o] = c.acc.x;
                acc_out[2 * o + 1] = c.acc.y;
            }
        }
    }
    return nfree;
}

// GridLineTraversal::gridLine for KATs: writes (x,y) pairs, returns num_points.
int gmr_grid_line(int x0, int y0, int x1, int y1, int *out_xy, int cap)
{
    GridLineTraversalLine line;
    GridLineTraversal::gridLine(IntPoint(x0, y0), IntPoint(x1, y1), &line);
    for (int k = 0; k < line.num_points && k < cap; k++) {
        out_xy[2 * k] = line.points[k].x;
        out_xy[2 * k + 1] = line.points[k].y;
    }
    return line.num_points;
}

// Map::world2map (G/grid/map.h:171-174)
void gmr_world2map(double xmin, double ymin, double xmax, double ymax, double delta, double wx, double wy,
                   int *mx, int *my)
{
    Point center((xmin + xmax) / 2.0, (ymin + ymax) / 2.0);
    ScanMatcherMap m(center, xmin, ymin, xmax, ymax, delta);
    IntPoint p = m.world2map(Point(wx, wy));
    *mx = p.x;
    *my = p.y;
}

}  // extern "C"
