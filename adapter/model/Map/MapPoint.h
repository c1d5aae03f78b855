// Test model only — stands in for Modules/Map/MapPoint.h with the members the adapter uses
// (MapPoint.h: getWorldPosition, setWorldPosition(Eigen::Vector3f&), getId, clone).
#pragma once

#include <memory>

#include "minimal_eigen_sophus.h"

class MapPoint {
public:
    explicit MapPoint(Eigen::Vector3f &p3d) : position3D_(p3d), nId_(nNextId_++) {}
    MapPoint(const MapPoint &other) = default;
    MapPoint *clone() const { return new MapPoint(*this); }
    Eigen::Vector3f getWorldPosition() { return position3D_; }
    void setWorldPosition(Eigen::Vector3f &p3d) { position3D_ = p3d; }
    long unsigned int getId() { return nId_; }
    static void resetIdCounter() { nNextId_ = 0; }   // model only: fresh maps in one test process

private:
    Eigen::Vector3f position3D_;
    long unsigned int nId_;
    static inline long unsigned int nNextId_ = 0;   // MapPoint.cc:22
};
