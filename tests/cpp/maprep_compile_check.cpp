// tests/cpp/maprep_compile_check.cpp -- TEST INFRASTRUCTURE: compiles include/slam2d/MapRepHip.h, the drop-in
// hectorslam::MapRepresentationInterface (MapRepresentationInterface.h:44-69; the one-line swap at
// HectorSlamProcessor.h:61), against the reference's own Hector headers under /root/reference and
// the API-only Eigen stand-in in tests/cpp/eigen_api_stub/ (Eigen3 is absent from this image).  It checks spelling
// and signatures only: every pure virtual is overridden (the class is concrete), the constructor, getGridMap's
// host mirror (GridMap::getCell, setUpdated: GridMapBase.h:152, 333; OccGridMapBase.h:49) and matchData /
// updateByScan instantiate.  Nothing is run and no parity is claimed.
#include <type_traits>

#include <slam2d/MapRepHip.h>

static_assert(!std::is_abstract<hectorslam::MapRepHip>::value, "MapRepHip overrides every pure virtual of the interface");
static_assert(std::is_base_of<hectorslam::MapRepresentationInterface, hectorslam::MapRepHip>::value, "drop-in type");

// instantiates the adapter's members exactly as HectorSlamProcessor drives them (HectorSlamProcessor.h:61-108)
hectorslam::MapRepresentationInterface *maprep_make(float res, int sx, int sy, unsigned int levels, const Eigen::Vector2f &start)
{
    return new hectorslam::MapRepHip(res, sx, sy, levels, start);
}
void maprep_drive(hectorslam::MapRepresentationInterface *m, const hectorslam::DataContainer &dc)
{
    Eigen::Matrix3f cov;
    const Eigen::Vector3f p = m->matchData(Eigen::Vector3f(0.0f, 0.0f, 0.0f), dc, cov);
    m->updateByScan(dc, p);
    const hectorslam::GridMap &g = m->getGridMap(0);
    (void)g.getUpdateIndex();
    m->setUpdateFactorFree(0.4f);
    m->setUpdateFactorOccupied(0.9f);
    (void)m->getScaleToMap();
    (void)m->getMapLevels();
    m->onMapUpdated();
    m->reset();
    delete m;
}
