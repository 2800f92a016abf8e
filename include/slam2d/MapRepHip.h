/* include/slam2d/MapRepHip.h -- the drop-in MapRepresentationInterface of the reference's Hector node,
 * backed by the MI355X C-ABI.
 *
 * Seam: hectorslam::MapRepresentationInterface (lesson4/include/lesson4/hector_mapping/slam_main/
 * MapRepresentationInterface.h:44-69), constructed at HectorSlamProcessor.h:61.  The swap is one line
 * there:
 *     mapRep = new MapRepHip(mapResolution, mapSizeX, mapSizeY, multi_res_size, startCoords);
 *
 * This header is built in the maintainer's ROS workspace, next to the reference headers it includes (they need
 * Eigen3, which this repository's image lacks).  Here it is compile-checked against the reference's own headers
 * with an API-only Eigen stand-in (tests/cpp/maprep_compile_check.cpp, `make -C tests/cpp maprep_check`: every
 * pure virtual overridden, the members instantiated; spelling and signatures only, nothing run).  Every call it
 * makes goes through slam2d::HectorMapBackend (hector_map_backend.hpp), which is compiled and tested here
 * (tests/cpp/hector_threads_test.cpp: a spin thread updating while a publish thread refreshes).
 *
 * Behaviour kept from MapRepMultiMap (MapRepMultiMap.h) / MapProcContainer (MapProcContainer.h):
 *   - updateByScan locks the mutex of EVERY level around the update (MapProcContainer.h:125-139 locks
 *     each level around its own gridMap->updateByScan; the device updates all levels in one call, so
 *     all level locks are held for it, in level order);
 *   - getGridMap(level) returns a host GridMap refreshed from the device whenever the device map's
 *     update index moved, and then advances that GridMap's own update index (GridMapBase::setUpdated,
 *     GridMapBase.h:333), so publishMap's `lastGetMapUpdateIndex != gridMap.getUpdateIndex()` test
 *     (hector_slam.cc:277) sees every new map and republishes;
 *   - getGridMap runs on the publish thread while matchData / updateByScan run on the spin thread: the
 *     C-ABI serialises the two on the context's mutex and hands back one consistent device state.
 */
#ifndef SLAM2D_MAPREPHIP_H
#define SLAM2D_MAPREPHIP_H

#include <memory>
#include <vector>

// Include order as HectorSlamProcessor.h:32-40: MapRepresentationInterface.h has no includes of its own and
// forward-declares GridMap / DataContainer at global scope, so hectorslam::GridMap, DataContainer,
// MapLockerInterface and Eigen must be declared before it, or its pure virtuals name other types than the
// overrides below.
#include "../map/GridMap.h"                  // -> Eigen, OccGridMapBase, DataPointContainer
#include "../scan/DataPointContainer.h"
#include "../util/MapLockerInterface.h"
#include "MapRepresentationInterface.h"      // lesson4/include/lesson4/hector_mapping/slam_main/
#include <slam2d/hector_map_backend.hpp>

namespace hectorslam {

class MapRepHip : public MapRepresentationInterface {
public:
    MapRepHip(float mapResolution, int mapSizeX, int mapSizeY, unsigned int numDepth,
              const Eigen::Vector2f &startCoords, int maxPoints = 2048)
        : be_(mapResolution, mapSizeX, mapSizeY, (int)numDepth, startCoords.x(), startCoords.y(), maxPoints)
    {
        // host mirrors with MapRepMultiMap's geometry (MapRepMultiMap.h:61-85)
        Eigen::Vector2i res(mapSizeX, mapSizeY);
        const float totalX = mapResolution * static_cast<float>(mapSizeX);
        const float totalY = mapResolution * static_cast<float>(mapSizeY);
        const Eigen::Vector2f mid(totalX * startCoords.x(), totalY * startCoords.y());
        float cell = mapResolution;
        for (unsigned int i = 0; i < numDepth; ++i) {
            mirrors_.emplace_back(new GridMap(cell, res, mid));
            mutexes_.push_back(nullptr);
            res /= 2;
            cell *= 2.0f;
        }
    }
    ~MapRepHip() override
    {
        // MapProcContainer::cleanup owns and deletes the lockers (MapProcContainer.h:65-67) through the interface,
        // which has no virtual destructor in the reference (MapLockerInterface.h:31-36): the same deletion is kept
        for (MapLockerInterface *m : mutexes_) delete m;
    }

    void reset() override
    {
        be_.reset();
        for (auto &g : mirrors_) g->reset();
    }
    float getScaleToMap() const override { return be_.scaleToMap(); }
    int getMapLevels() const override { return be_.levels(); }

    const GridMap &getGridMap(int mapLevel) const override
    {
        GridMap &g = *mirrors_.at(mapLevel);
        if (be_.refresh(mapLevel)) {
            std::lock_guard<std::mutex> lk(be_.mirrorMutex());
            const slam2d::HectorMapBackend::Level &L = be_.level(mapLevel);
            const int n = L.size_x * L.size_y;
            for (int i = 0; i < n; ++i) {
                LogOddsCell &c = g.getCell(i);
                c.logOddsVal = L.logodds[i];
                c.updateIndex = L.update[i];
            }
            g.setUpdated();  // publishMap compares getUpdateIndex (hector_slam.cc:277)
        }
        return g;
    }

    void addMapMutex(int i, MapLockerInterface *mapMutex) override
    {
        delete mutexes_.at(i);
        mutexes_[i] = mapMutex;
    }
    MapLockerInterface *getMapMutex(int i) override { return mutexes_.at(i); }
    void onMapUpdated() override {}  // value-transparent: the device keeps no cache across scans

    Eigen::Vector3f matchData(const Eigen::Vector3f &beginEstimateWorld, const DataContainer &dataContainer,
                              Eigen::Matrix3f &covMatrix) override
    {
        pack(dataContainer);
        float pose[3], cov[9];
        be_.match(xy_.data(), dataContainer.getSize(), dataContainer.getOrigo().x(), dataContainer.getOrigo().y(),
                  beginEstimateWorld.data(), pose, cov);
        covMatrix = Eigen::Map<Eigen::Matrix<float, 3, 3, Eigen::RowMajor>>(cov);
        return Eigen::Vector3f(pose[0], pose[1], pose[2]);
    }

    void updateByScan(const DataContainer &dataContainer, const Eigen::Vector3f &robotPoseWorld) override
    {
        pack(dataContainer);
        for (MapLockerInterface *m : mutexes_)
            if (m) m->lockMap();
        try {
            be_.updateByScan(xy_.data(), dataContainer.getSize(), dataContainer.getOrigo().x(),
                             dataContainer.getOrigo().y(), robotPoseWorld.data());
        } catch (...) {
            unlockAll();
            throw;
        }
        unlockAll();
    }

    void setUpdateFactorFree(float free_factor) override { be_.setUpdateFactorFree(free_factor); }
    void setUpdateFactorOccupied(float occupied_factor) override { be_.setUpdateFactorOccupied(occupied_factor); }

private:
    void unlockAll()
    {
        for (auto it = mutexes_.rbegin(); it != mutexes_.rend(); ++it)
            if (*it) (*it)->unlockMap();
    }
    void pack(const DataContainer &dc)  // DataContainer: map-scale Vector2f points (hector_slam.cc:356)
    {
        xy_.resize(2 * (size_t)dc.getSize());
        for (int i = 0; i < dc.getSize(); ++i) {
            xy_[2 * i] = dc.getVecEntry(i).x();
            xy_[2 * i + 1] = dc.getVecEntry(i).y();
        }
    }

    mutable slam2d::HectorMapBackend be_;
    std::vector<std::unique_ptr<GridMap>> mirrors_;
    std::vector<MapLockerInterface *> mutexes_;
    std::vector<float> xy_;
};

}  // namespace hectorslam

#endif
