// Test model only — stands in for Modules/Visualization/MapVisualizer.h (Pangolin is absent): the
// constructor and update(bool) the optimizer calls; updates are counted instead of drawn.
#pragma once

#include <memory>

#include "Map/Map.h"
#include "Utils/CommonTypes.h"

class MapVisualizer {
public:
    MapVisualizer() = delete;
    MapVisualizer(std::shared_ptr<Map> pMap, const PoseData initialPose = PoseData(), const bool showScene = true)
        : pMap_(pMap), initialPose_(initialPose), showScene_(showScene) {}
    void update(bool drawRaysSelection = false) {
        updates_++;
        lastDrawRays_ = drawRaysSelection;
    }
    int updates() const { return updates_; }   // model only

private:
    std::shared_ptr<Map> pMap_;
    PoseData initialPose_;
    bool showScene_;
    int updates_ = 0;
    bool lastDrawRays_ = false;
};
