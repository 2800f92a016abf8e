// gmapping_internal.h -- device data layout of the GMapping particle-map path (config 4).
//
// Reference: GMapping::ComputeMap (lesson4/src/gmapping/gmapping.cc:171-242) builds a FRESH
// ScanMatcherMap per scan (:128-135) and counts, per cell, n (hits) and visits
// (PointAccumulator, lesson4/include/lesson4/gmapping/grid/map.h:17-48).  The build evaluates it for
// P candidate poses ("particles") of the same scan.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace s2d {

constexpr int GM_TILE = 64;                 // tile width (cells)
constexpr int GM_TILE_H = 32;               // tile height (cells)
constexpr int GM_TILE_CELLS = GM_TILE * GM_TILE_H;
// Per particle map: one packed word per cell, n << 16 | visits (both <= max_beams <= 8192: a beam
// visits a cell at most once), in 64 x 32-cell tiles of 8 KB; a tile stamp per tile (the step that
// last wrote it: older tiles read as the untouched cells of a fresh map); and a compact list of the
// cells hit this step with their accumulators (acc is zero everywhere else).
constexpr int GM_TILE_BLOCK_WORDS = GM_TILE_CELLS;
struct GmHitCell {
    int cell;       // y * sx + x
    float ax, ay;   // PointAccumulator::acc (map.h:37-48)
};
constexpr int GM_THREADS = 256;
constexpr unsigned GM_RAY_INVALID = 0xFFFFFFFFu;
constexpr unsigned GM_RAY_HIT = 0x80000000u;  // packed ray: hit flag | y << 16 | x

// ScanMatcherMap geometry (G/grid/map.h:133-143, world2map :171-174) + ComputeMap parameters
struct GmGeom {
    int sx, sy;          // map size (multiple of the 32-cell patch, harray2d.h)
    int sx2, sy2;        // map cell of the map centre
    double cx, cy;       // map centre (world)
    double delta;        // resolution
    double max_range;    // maxRange: beams beyond are dropped (gmapping.cc:183)
    double max_urange;   // maxUrange: beams beyond are clamped and not hits (:185-187, :209-214)
    double occ_thresh;   // PublishMap occupancy threshold (gmapping.cc:150), used by the score
    int tiles_x, tiles_y;
    size_t particle_words;  // 4-byte words per particle map (tiles)
    int max_beams;
    int ntiles;             // tiles_x * tiles_y (one stamp each)
};

// Per-particle state: the tile box written by the last ComputeMap (cells outside it read as an
// untouched fresh map: n = visits = 0, acc = 0) and the last step's counters.
struct alignas(16) GmState {
    int tx0, ty0, tx1, ty1;  // tile box of the last ComputeMap (tx1 < tx0: none)
    int score;               // hits of this scan on occupied cells of the particle's previous map
    int hits;                // hit beams (d < max_urange) of this scan
    long long free_updates;  // Σ (num_points - 1): the free-cell visit updates of this scan
    int step;                // ComputeMap calls so far: tiles stamped `step` belong to the current map
    int hit_cells;           // slots of the particle's hit-cell list (one per beam; cell < 0: no entry)
    int pad_[2];
};

}  // namespace s2d
