// hector_internal.h -- device data layout shared by the Hector kernels and the host runtime.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace s2d {

constexpr double S2D_PI = 3.14159265358979323846;  // M_PI
constexpr int MAX_LEVELS = 8;
constexpr int MATCH_THREADS = 256;
constexpr int MATCH_WAVES = MATCH_THREADS / 64;
constexpr int FREE_BEAMS = 64;  // beams per free-cells workgroup

enum StepMode : int {
    MODE_PROCESS = 0,        // HectorSlamProcessor::update
    MODE_MATCH_ONLY = 1,     // MapRepMultiMap::matchData
    MODE_NO_MATCH_FORCE = 2, // HectorSlamProcessor::update(map_without_matching = true)
    MODE_UPDATE_ONLY = 3,    // MapRepMultiMap::updateByScan with a given pose
};

// LogOddsCell (lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h:37-87), same 8-byte layout.
struct LogOddsCell {
    float l;
    int upd;
};
static_assert(sizeof(LogOddsCell) == 8, "LogOddsCell must be 8 bytes");

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
    size_t cell_offset;  // offset of this level inside a stream's cell block
};

struct FleetGeom {
    int levels;
    float lf, lo;              // logOddsFree / logOddsOccupied
    float min_dist, min_ang;   // map update thresholds
    size_t stream_cells;       // cells per stream (all levels)
    LevelGeom lv[MAX_LEVELS];
};

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
};

}  // namespace s2d
