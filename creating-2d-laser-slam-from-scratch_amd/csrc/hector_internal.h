// hector_internal.h -- device data layout shared by the Hector kernels and the host runtime.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace s2d {

constexpr double S2D_PI = 3.14159265358979323846;  // M_PI
constexpr int MAX_LEVELS = 8;
constexpr int MATCH_THREADS = 256;
constexpr int MATCH_WAVES = MATCH_THREADS / 64;
// Cell storage is tiled: a level is a grid of TILE x TILE_H tiles (padded up), each tile one
// contiguous 20 KB block of three planes, cells in the same order in each (4 x 4-cell blocks, see tile_cell):
//   [0, TILE_CELLS)             log-odds floats (LogOddsCell::logOddsVal)
//   [ORD_OFF, +TILE_CELLS / 2)  16-bit update ordinals ("hot" updateIndex, written by every grid update)
//   [COLD_OFF, +TILE_CELLS)     32-bit updateIndex ints ("cold": written only by the ordinal sweep and hs_set_map)
// LogOddsCell::updateIndex (GridMapLogOdds.h:85-86) of a cell is read from the hot plane when its ordinal h is
// non-zero -- the last update k that touched it, h = 2 (k - E) + 1 + hit, E the stream's ordinal epoch, so the
// index is 3 (E + (h - 1) / 2) + 1 + (h - 1) % 2 = currMarkFreeIndex / currMarkOccIndex of update k
// (OccGridMapBase.h:120-121, 167: currUpdateIndex = 3 k) -- and from the cold plane otherwise.  Every
// ORD_SWEEP_MAX steps at most, hs_ord_sweep_kernel moves every non-zero ordinal into the cold plane and advances
// E, so h never overflows 16 bits.  The grid update thus writes 2 B of index per marked cell instead of 4
// (round 5: the 4-B index stores were a quarter of hs_update_kernel's time).
// A tile is exactly the unit the grid-update kernel reads and writes.
#ifndef S2D_TILE_H
#define S2D_TILE_H 32
#endif
constexpr int TILE = 64;
constexpr int TILE_H = S2D_TILE_H;
constexpr int TILE_CELLS = TILE * TILE_H;   // 2048 at 64 x 32
constexpr int ORD_OFF = TILE_CELLS;                    // 4-byte word offset of the 16-bit ordinal plane
constexpr int COLD_OFF = TILE_CELLS + TILE_CELLS / 2;   // 4-byte word offset of the 32-bit index plane
constexpr int TILE_BLOCK_WORDS = COLD_OFF + TILE_CELLS;
constexpr int ORD_SWEEP_MAX = 32000;  // steps between ordinal sweeps at most (h <= 2 * 32000 + 1 < 2^16)
// updateIndex of a cell from its hot ordinal h (!= 0) and the stream's ordinal epoch E
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int ord_index(unsigned h, int epoch)
{
    return 3 * (epoch + (int)((h - 1u) >> 1)) + 1 + (int)((h - 1u) & 1u);
}

enum StepMode : int {
    MODE_PROCESS = 0,        // HectorSlamProcessor::update
    MODE_MATCH_ONLY = 1,     // MapRepMultiMap::matchData
    MODE_NO_MATCH_FORCE = 2, // HectorSlamProcessor::update(map_without_matching = true)
    MODE_UPDATE_ONLY = 3,    // MapRepMultiMap::updateByScan with a given pose
};

// LogOddsCell (lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h:37-87): {logOddsVal,
// updateIndex}; stored split into the two planes of a tile block (see above).

// One pyramid level: GridMapBase transforms (GridMapBase.h:270-286) + MapDimensionProperties limits.
struct LevelGeom {
    int sx, sy;
    float scale;      // scaleToMap
    float map_t[2];   // mapTworld translation
    float inv_l[4];   // worldTmap linear (row-major 2x2)
    float inv_t[2];   // worldTmap translation
    float lim[2];     // mapLimitsf = dims - 2
    float pts_scale;  // DataPointContainer::setFrom factor 1/2^level
    float cell_len;
    int tiles_x, tiles_y;  // storage tiles (sx, sy rounded up to TILE, TILE_H)
    size_t word_offset;    // offset of this level inside a stream's block, in 4-byte words
};

// Inside a tile, cells are stored in CELL_BLK x CELL_BLK blocks (4 x 4 cells = 64 B per plane), the
// blocks row-major: a ray's cells -- a line in any direction -- then share DRAM sectors and cache lines
// (the once-per-scan update moves ~13 % fewer bytes than with row-major tiles: a 4 x 4 block holds ~4 cells
// of a line whatever its angle, a 64-cell row only ~1 of a steep one), and a quad of 4 cells of one row
// (x % 4 == 0) is still 16 contiguous bytes.
constexpr int CELL_BLK = 4;
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int tile_cell(int lx, int ly)  // (lx, ly) inside the tile (>= 0) -> its word inside a plane
{
    // unsigned: shifts and masks, whatever the compiler knows of the signs
    const unsigned x = (unsigned)lx, y = (unsigned)ly;
    return (int)(((y / CELL_BLK) * (TILE / CELL_BLK) + (x / CELL_BLK)) * (CELL_BLK * CELL_BLK) + (y % CELL_BLK) * CELL_BLK +
                 (x % CELL_BLK));
}

// word index of cell (x, y)'s log-odds inside its level (its ordinal and index: ORD_OFF / COLD_OFF planes, above)
#if defined(__HIPCC__)
__host__ __device__
#endif
inline size_t cell_word(const LevelGeom &g, int x, int y)
{
    return ((size_t)((y / TILE_H) * g.tiles_x + (x / TILE)) * TILE_BLOCK_WORDS) + (size_t)tile_cell(x % TILE, y % TILE_H);
}

struct FleetGeom {
    int levels;
    float lf, lo;              // logOddsFree / logOddsOccupied
    float min_dist, min_ang;   // map update thresholds
    size_t stream_words;       // 4-byte words per stream (all levels, tiled, both planes; + the stream pad)
    size_t cells_words;        // of which cells (the levels)
    int upd_parts[MAX_LEVELS]; // hs_update_kernel workgroups per (stream, level)
    int upd_minp[MAX_LEVELS];  // list-driven split: at least this many workgroups per level (0: upd_split's)
    // clock probe (hs_set_clock_probe; NULL = off): [kernel * 4 + {0: shader cycles, 1: 100-MHz ticks,
    // 2: workgroups}] summed over every CLK_SAMPLE-th workgroup's lifetime (kernel 0 match, 1 update)
    unsigned long long *clk;
    LevelGeom lv[MAX_LEVELS];
};
constexpr int CLK_SAMPLE = 16;

// Per-stream processor state (HectorSlamProcessor members + per-grid update indices).
struct alignas(16) StreamState {
    float pose[3];           // lastScanMatchPose
    float last_upd_pose[3];  // lastMapUpdatePose
    float cov[9];            // lastScanMatchCov
    float upd_pose[3];       // pose used by this step's raycast
    float origo[2];          // this step's DataContainer origo (level-0 map scale)
    int cur_update_index;    // OccGridMapBase::currUpdateIndex (all levels advance together)
    int map_updates;         // GridMapBase::lastUpdateIndex + 1
    int do_update;           // this step updates the map
    int mark_base;           // currUpdateIndex used for this step's marks
    int n;                   // this step's point count
    int clamp_count;         // "SearchDir angle change too large" events (ScanMatcher.h:123-132)
    unsigned long long step_cells;  // Σ (abs_da + 1) of this step's valid rays, all levels
    // cumulative counters since the last hs_reset_counters (algorithmic-byte accounting)
    unsigned long long tot_cells;     // Σ (abs_da + 1)  (cells visited by the raycast)
    unsigned long long tot_rays;      // valid rays drawn
    unsigned long long tot_gn_points; // Σ over GN iterations of the points evaluated
    unsigned long long tot_updates;   // map updates (steps with do_update)
    unsigned long long tot_steps;     // steps
    unsigned long long tot_touched;   // distinct cells written by the grid update (Σ levels, per scan)
    int step_index;                   // steps since hs_reset (pose-log row)
    int ord_epoch;                    // E: update ordinal of the last ordinal sweep (see ORD_OFF)
    int ord_base;                     // this step's hot ordinal of a freed cell, 2 (k - E) + 1 (+1: occupied)
    // sticky: an update's hot ordinal passed 0xFFFF, i.e. more than ORD_SWEEP_MAX updates went by without the
    // library's ordinal sweep (e.g. replayed graph captures of *_device calls): hs_get_map refuses to decode the
    // stream's updateIndex until hs_reset; the log-odds are unaffected
    int ord_overflow;
    // MapRepMultiMap::dataContainers (MapRepMultiMap.h:89, :161): the DataContainer of the last
    // matchData, which updateByScan draws into levels >= 1 (:187).  Its points (level-0 scale) live in
    // the context's per-stream container buffer; empty (mc_n = 0) until the first match.
    int mc_n;
    float mc_origo[2];
};

// Binned grid-update work queue (hs_bin_kernel -> hs_tile_kernel).
struct WorkItem {
    int s;                 // stream
    int lvl_kind;          // level | kind << 8 (0 = one tile + its segment list, 1 = whole level)
    unsigned tile_xy;      // first tile (x | y << 16), in tiles
    unsigned begin_xy;     // ray start cell (x | y << 16)
    unsigned seg_begin;    // tile: first segment; whole: ntx | nty << 16
    unsigned seg_count;    // tile: number of segments
    unsigned mark_base;    // stream's currUpdateIndex for this step (marks = +1 / +2)
    unsigned n;            // points of the scan (whole items)
};
struct WorkQueue {
    unsigned seg_used, item_used, whole_used, overflow;  // zeroed by hs_match_kernel every step
    unsigned item_cap, seg_cap, pad_[2];
};

// Streams whose map is updated this step, appended by hs_match_kernel (order-free: the per-stream work
// is independent), consumed by hs_update_kernel.  Two lists alternate: the update kernel reads one and
// clears the other, which the next step's match kernel fills.
struct UpdList {
    int count;
    int pad_[3];
    int stream[1];  // [B] local stream indices
};

// Workgroups per (stream, level) of hs_update_kernel for U updating streams on ncu CUs: about 4 level-0
// workgroups per CU for small batches (2 for U <= 32), at least 2 for level 0 (8 for a single-level
// map, which has no coarser levels to fill the tail of the grid: c2, 1024 streams, 2 / 3 / 4 / 6 / 8 /
// 12 / 16 parts = 1.48 / 1.50 / 1.53 / 1.57 / 1.61 / 1.58 / 1.51 M scans/s), halved per level
// (measured).
inline __host__ __device__ void upd_split(int U, int ncu, int levels, int *parts, const int *minp)
{
    const int target = U <= 32 ? 2 : 4;
    int p0 = U > 0 ? (target * ncu + U - 1) / U : 1;
    if (p0 < 2) p0 = 2;
    if (levels == 1 && p0 < 8) p0 = 8;
    for (int l = 0; l < levels; ++l) {
        int v = p0 >> l;
        if (v < minp[l]) v = minp[l];
        parts[l] = v < 1 ? 1 : (v > 64 ? 64 : v);
    }
}

// Optional device pose log: the match kernel appends every step's pose of streams [0, streams).
struct PoseLog {
    float *buf;          // [capacity][streams][3]
    int streams;         // slots per row
    int capacity;
    const int *slot_of;  // device [B]: slot of stream s (< 0: not logged); NULL: stream s -> slot s
};

}  // namespace s2d
