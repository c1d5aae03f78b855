// Test model only — stands in for Modules/Map/KeyFrame.h with the members the adapter uses
// (getId, getPose/setPose, getKeyPoint(s), getDepthMeasure, get/setEstimatedDepthScale,
// getMapPoints/setMapPoint, getCalibration, getInvSigma2, getNumberOfScales, clone).
#pragma once

#include <memory>
#include <stdexcept>
#include <vector>

#include "Mapping/Frame.h"

class KeyFrame {
public:
    explicit KeyFrame(Frame &f)
        : vKeys_(f.getKeyPoints()), vDepthMeasurements_(f.getDepthMeasurements()), vMapPoints_(f.getMapPoints()),
          calibration_(f.getCalibration()), phcalibration_(f.getPHCalibration()),
          imageDepthScale_(f.getDepthScale()), estimatedDepthScale_(f.getEstimatedDepthScale()),
          Tcw_(f.getPose()), nId_(nNextId_++) {
        const int n = f.getNumberOfScales();
        for (int i = 0; i < n; i++) {
            vScaleFactor_.push_back(f.getScaleFactor(i));
            vInvSigma2_.push_back(f.getInvSigma2(i));
        }
    }
    // KeyFrame.cc:68-99: every MapPoint of the slots cloned (distinct from the Map's objects)
    KeyFrame(const KeyFrame &other)
        : vKeys_(other.vKeys_), vDepthMeasurements_(other.vDepthMeasurements_), calibration_(other.calibration_),
          phcalibration_(other.phcalibration_), imageDepthScale_(other.imageDepthScale_),
          estimatedDepthScale_(other.estimatedDepthScale_), Tcw_(other.Tcw_), nId_(other.nId_),
          vScaleFactor_(other.vScaleFactor_), vInvSigma2_(other.vInvSigma2_) {
        for (const auto &pMP : other.vMapPoints_)
            vMapPoints_.emplace_back(pMP ? std::shared_ptr<MapPoint>(pMP->clone()) : nullptr);
    }
    KeyFrame *clone() const { return new KeyFrame(*this); }

    Sophus::SE3f getPose() { return Tcw_; }
    void setPose(Sophus::SE3f &Tcw) { Tcw_ = Tcw; }
    cv::KeyPoint getKeyPoint(size_t idx) { return vKeys_[idx]; }
    std::vector<cv::KeyPoint> &getKeyPoints() { return vKeys_; }
    float getDepthMeasure(size_t idx) { return vDepthMeasurements_[idx]; }
    std::vector<float> &getDepthMeasurements() { return vDepthMeasurements_; }
    // KeyFrame.cc:181-202: the depth image lookup; the simulation sets no image
    double getDepthMeasure(float x, float y, bool scaled = true) {
        (void)x; (void)y; (void)scaled;
        throw std::runtime_error("Depth image is not initialized.");
    }
    double getEstimatedDepthScale() { return estimatedDepthScale_; }
    void setEstimatedDepthScale(double scale) { estimatedDepthScale_ = scale; }
    std::vector<std::shared_ptr<MapPoint>> &getMapPoints() { return vMapPoints_; }
    void setMapPoint(size_t idx, std::shared_ptr<MapPoint> pMP) { vMapPoints_[idx] = pMP; }
    std::shared_ptr<MapPoint> getMapPoint(size_t idx) { return vMapPoints_[idx]; }
    std::shared_ptr<CameraModel> getCalibration() { return calibration_; }
    std::shared_ptr<CameraModel> getPHCalibration() { return phcalibration_; }
    long unsigned int getId() { return nId_; }
    float getScaleFactor(int octave) { return vScaleFactor_[octave]; }
    float getInvSigma2(int octave) { return vInvSigma2_[octave]; }
    int getNumberOfScales() { return (int)vScaleFactor_.size(); }
    static void resetIdCounter() { nNextId_ = 0; }   // model only

private:
    std::vector<cv::KeyPoint> vKeys_;
    std::vector<float> vDepthMeasurements_;
    std::vector<std::shared_ptr<MapPoint>> vMapPoints_;
    std::shared_ptr<CameraModel> calibration_, phcalibration_;
    double imageDepthScale_ = 1.0, estimatedDepthScale_ = 1.0;
    Sophus::SE3f Tcw_;
    long unsigned int nId_;
    std::vector<float> vScaleFactor_, vInvSigma2_;
    static inline long unsigned int nNextId_ = 0;   // KeyFrame.cc:25
};
