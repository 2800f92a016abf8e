/* include/slam2d/hector_map_backend.hpp -- Eigen-free C++ core of the MapRepHip drop-in.
 *
 * Owns one hs_ctx with ONE stream (the ROS drop-in) and the host mirrors of the map levels that
 * MapRepresentationInterface::getGridMap (lesson4/include/lesson4/hector_mapping/slam_main/
 * MapRepresentationInterface.h:54) hands to the node's publish thread.  include/slam2d/MapRepHip.h
 * maps the reference's types (Eigen vectors, DataContainer, GridMap, MapLockerInterface) onto it; the
 * backend itself needs only the C-ABI (include/slam2d/hector.h), so it is compiled and tested here
 * (tests/cpp/hector_threads_test.cpp) without Eigen or ROS.
 *
 * Threads.  The reference runs matchData / updateByScan on the ROS spin thread and publishMap on a
 * second thread (hector_slam.cc:201, :254-317).  Every hs_* call is serialised by the context's own
 * mutex and returns a consistent state, so refresh() -- one hs_get_map of log-odds, updateIndex and the
 * map update index together -- never sees a half-applied scan.  The mirrors are guarded by the
 * backend's own mutex.
 */
#ifndef SLAM2D_HECTOR_MAP_BACKEND_HPP
#define SLAM2D_HECTOR_MAP_BACKEND_HPP

#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "hector.h"

namespace slam2d {

class HectorMapBackend {
public:
    // One level of the pyramid as the host sees it (GridMapBase.h:85-87, :301-304, :333-334).
    struct Level {
        int size_x = 0, size_y = 0;
        float cell_length = 0.0f;
        float origin[2] = {0.0f, 0.0f};   // world coordinates of cell (0, 0)
        std::vector<float> logodds;       // row-major, LogOddsCell::logOddsVal
        std::vector<int32_t> update;      // row-major, LogOddsCell::updateIndex
        int update_index = -2;            // GridMapBase::getUpdateIndex of the mirrored state (-2: never read)
    };

    // MapRepMultiMap(mapResolution, mapSizeX, mapSizeY, numDepth, startCoords) (MapRepMultiMap.h:57-90)
    HectorMapBackend(float map_resolution, int map_size_x, int map_size_y, int levels, float start_x, float start_y,
                     int max_points = 2048)
    {
        check(hs_create(&ctx_, 1, map_resolution, map_size_x, map_size_y, start_x, start_y, levels, max_points),
              "hs_create");  // no CPU fallback: without a HIP device this throws
        levels_.resize(levels);
        for (int l = 0; l < levels; ++l) {
            Level &L = levels_[l];
            check(hs_get_map_info(ctx_, l, &L.size_x, &L.size_y, &L.cell_length, L.origin), "hs_get_map_info");
        }
    }
    ~HectorMapBackend() { hs_destroy(ctx_); }
    HectorMapBackend(const HectorMapBackend &) = delete;
    HectorMapBackend &operator=(const HectorMapBackend &) = delete;

    // MapRepresentationInterface::reset (:49), getScaleToMap / getMapLevels (:51-53)
    void reset() { check(hs_reset(ctx_), "hs_reset"); }
    float scaleToMap() const
    {
        float s = 0.0f;
        check(hs_get_scale_to_map(ctx_, &s), "hs_get_scale_to_map");
        return s;
    }
    int levels() const { return (int)levels_.size(); }

    // setUpdateFactorFree / setUpdateFactorOccupied (:67-68): the C-ABI takes both at once
    void setUpdateFactorFree(float f)
    {
        free_ = f;
        check(hs_set_update_factors(ctx_, free_, occ_), "hs_set_update_factors");
    }
    void setUpdateFactorOccupied(float f)
    {
        occ_ = f;
        check(hs_set_update_factors(ctx_, free_, occ_), "hs_set_update_factors");
    }
    void setMapUpdateThresholds(float min_dist, float min_angle)
    {
        check(hs_set_map_update_thresholds(ctx_, min_dist, min_angle), "hs_set_map_update_thresholds");
    }

    // matchData (:62): xy = the DataContainer's points in map scale (2 floats each), origo in map scale
    void match(const float *xy, int n, float ox, float oy, const float hint[3], float pose[3], float cov[9])
    {
        check(hs_match(ctx_, 0, xy, n, ox, oy, hint, pose, cov), "hs_match");
    }
    // updateByScan (:65) of every level, then onMapUpdated (:59)
    void updateByScan(const float *xy, int n, float ox, float oy, const float pose[3])
    {
        check(hs_update_by_scan(ctx_, 0, xy, n, ox, oy, pose), "hs_update_by_scan");
    }
    // HectorSlamProcessor::update (HectorSlamProcessor.h:81-108) in one call; returns did-update
    bool process(const float *xy, int n, float ox, float oy, const float *hint, bool map_without_matching,
                 float pose[3], float cov[9])
    {
        int did = 0;
        check(hs_update(ctx_, 0, xy, n, ox, oy, hint, map_without_matching ? 1 : 0, pose, cov, &did), "hs_update");
        return did != 0;
    }

    // getGridMap (:54) support: re-read `level` from the device when its update index moved.  Returns
    // true when the mirror changed (the adapter then advances its GridMap's update index so that
    // publishMap, hector_slam.cc:277, republishes).
    bool refresh(int level)
    {
        std::lock_guard<std::mutex> lk(mirror_mu_);
        Level &L = levels_.at(level);
        int idx = 0;
        check(hs_get_map(ctx_, 0, level, nullptr, nullptr, nullptr, &idx), "hs_get_map");
        if (idx == L.update_index) return false;
        const size_t n = (size_t)L.size_x * L.size_y;
        L.logodds.resize(n);
        L.update.resize(n);
        // log-odds, cell indices and the map's update index of ONE device state (one locked call)
        check(hs_get_map(ctx_, 0, level, nullptr, L.logodds.data(), L.update.data(), &idx), "hs_get_map");
        L.update_index = idx;
        return true;
    }
    // The mirror of `level` (valid after refresh); the caller holds no lock while another thread may
    // refresh, so copy what it needs under lock() or refresh from the same thread (the publish thread).
    const Level &level(int l) const { return levels_.at(l); }
    std::mutex &mirrorMutex() { return mirror_mu_; }
    hs_ctx *context() { return ctx_; }

private:
    static void check(int rc, const char *what)
    {
        if (rc != HS_OK) throw std::runtime_error(std::string(what) + ": " + hs_last_error());
    }
    hs_ctx *ctx_ = nullptr;
    float free_ = 0.4f, occ_ = 0.6f;  // GridMapLogOddsFunctions ctor defaults (GridMapLogOdds.h:98-102)
    std::vector<Level> levels_;
    std::mutex mirror_mu_;
};

}  // namespace slam2d

#endif
