// Test model only — stands in for Modules/Map/Map.h (Map.cc) with the members the adapter uses:
// the keyframe / map point tables (std::unordered_map, iterated exactly as the reference's), the
// observation and covisibility tables, the global-transformation store and clone().
#pragma once

#include <cassert>
#include <memory>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

#include "Map/KeyFrame.h"
#include "Map/MapPoint.h"

typedef long unsigned int ID;

class Map {
public:
    Map() = default;
    explicit Map(float minCommonObs) : minCommonObs_(minCommonObs) {}

    void insertMapPoint(std::shared_ptr<MapPoint> pMP) {
        mMapPoints_[pMP->getId()] = pMP;
        mMapPointObs_[pMP->getId()].clear();
    }
    void insertKeyFrame(std::shared_ptr<KeyFrame> pKF) {
        mKeyFrames_[pKF->getId()] = pKF;
        mKeyFrameObs_[pKF->getId()].clear();
        mCovisibilityGraph_[pKF->getId()].clear();
    }
    std::shared_ptr<KeyFrame> getKeyFrame(ID id) { return mKeyFrames_.count(id) ? mKeyFrames_[id] : nullptr; }
    std::shared_ptr<MapPoint> getMapPoint(ID id) { return mMapPoints_.count(id) ? mMapPoints_[id] : nullptr; }

    // Map.cc:100-132 (the descriptor / normal update is not modelled)
    void addObservation(ID kfId, ID mpId, size_t idx) {
        assert(mKeyFrameObs_[kfId].count(mpId) == 0);
        mKeyFrameObs_[kfId][mpId] = idx;
        mMapPointObs_[mpId][kfId] = idx;
        for (const auto &p : mMapPointObs_[mpId]) {
            if (p.first == kfId) continue;
            mCovisibilityGraph_[kfId][p.first]++;
            mCovisibilityGraph_[p.first][kfId]++;
        }
    }
    // Map.cc:134-149
    void removeObservation(ID kfId, ID mpId) {
        mKeyFrameObs_[kfId].erase(mpId);
        mMapPointObs_[mpId].erase(kfId);
        for (const auto &p : mMapPointObs_[mpId]) {
            mCovisibilityGraph_[kfId][p.first]--;
            mCovisibilityGraph_[p.first][kfId]--;
        }
    }
    std::unordered_map<ID, std::shared_ptr<MapPoint>> &getMapPoints() { return mMapPoints_; }
    std::unordered_map<ID, std::shared_ptr<KeyFrame>> &getKeyFrames() { return mKeyFrames_; }

    // Map.cc:178-209
    void getLocalMapOfKeyFrame(ID kfId, std::set<ID> &sLocalMapPointsIds, std::set<ID> &sLocalKeyFramesIds,
                               std::set<ID> &sLocalFixedKeyFramesIds) {
        std::set<ID> sAllKFs;
        sLocalKeyFramesIds.insert(kfId);
        for (const auto &p : mKeyFrameObs_[kfId]) sLocalMapPointsIds.insert(p.first);
        for (const auto &p : mCovisibilityGraph_[kfId]) {
            if (p.second > minCommonObs_) {
                sLocalKeyFramesIds.insert(p.first);
                for (const auto &q : mKeyFrameObs_[p.first]) sLocalMapPointsIds.insert(q.first);
            }
        }
        for (ID mp : sLocalMapPointsIds)
            for (const auto &p : mMapPointObs_[mp]) sAllKFs.insert(p.first);
        for (ID k : sAllKFs)
            if (!sLocalKeyFramesIds.count(k)) sLocalFixedKeyFramesIds.insert(k);
    }

    int isMapPointInKeyFrame(ID mp, ID kf) {
        int idx = -1;
        if (mKeyFrameObs_[kf].count(mp) != 0) idx = (int)mKeyFrameObs_[kf][mp];
        return idx;
    }
    int getNumberOfObservations(ID mp) { return (int)mMapPointObs_[mp].size(); }

    // Map.cc:323-343
    void insertGlobalKeyFramesTransformation(ID kf1, ID kf2, const Sophus::SE3f &transformation) {
        mGTransformation_[kf1][kf2] = transformation;
        mGTransformation_[kf2][kf1] = transformation.inverse();
    }
    Sophus::SE3f getGlobalKeyFramesTransformation(ID kf1, ID kf2) {
        Sophus::SE3f globalT;
        if (mGTransformation_.count(kf1) && mGTransformation_[kf1].count(kf2)) globalT = mGTransformation_[kf1][kf2];
        return globalT;
    }

    // Map.cc:30-58: MapPoints and KeyFrames cloned and inserted in this map's iteration order,
    // observations re-added, covisibility copied; the global-transformation store is NOT copied
    std::shared_ptr<Map> clone() const {
        auto newMap = std::make_shared<Map>(minCommonObs_);
        for (const auto &kv : mMapPoints_)
            if (kv.second) newMap->insertMapPoint(std::shared_ptr<MapPoint>(kv.second->clone()));
        for (const auto &kv : mKeyFrames_)
            if (kv.second) newMap->insertKeyFrame(std::shared_ptr<KeyFrame>(kv.second->clone()));
        for (const auto &kv : mKeyFrameObs_)
            for (const auto &o : kv.second) newMap->addObservation(kv.first, o.first, o.second);
        for (const auto &kv : mCovisibilityGraph_)
            for (const auto &c : kv.second) newMap->mCovisibilityGraph_[kv.first][c.first] = c.second;
        return newMap;
    }

private:
    std::unordered_map<ID, std::shared_ptr<MapPoint>> mMapPoints_;
    std::unordered_map<ID, std::shared_ptr<KeyFrame>> mKeyFrames_;
    std::unordered_map<ID, std::unordered_map<ID, size_t>> mKeyFrameObs_;
    std::unordered_map<ID, std::unordered_map<ID, size_t>> mMapPointObs_;
    std::unordered_map<ID, std::unordered_map<ID, int>> mCovisibilityGraph_;
    std::unordered_map<ID, std::unordered_map<ID, Sophus::SE3f>> mGTransformation_;
    float minCommonObs_ = 0.f;
};
