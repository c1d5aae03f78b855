// Test model only — stands in for Modules/Mapping/Frame.h with the members the adapter
// (poseOnlyOptimization) and the KeyFrame constructor use.  The constructor has the reference's
// parameter list (Frame.h:46-52); grid, image boundaries and descriptors are not modelled.
#pragma once

#include <memory>
#include <vector>

#include "Calibration/CameraModel.h"
#include "Map/MapPoint.h"
#include "minimal_eigen_sophus.h"

class Frame {
public:
    Frame() = default;
    Frame(const int nFeatures, const int nGridCols, const int nGridRows, const int nImCols, const int nImRows,
          int nScales, float fScaleFactor, const std::shared_ptr<CameraModel> calibration,
          const std::shared_ptr<CameraModel> phcalibration, const std::vector<float> &vDistortion = {},
          const double dScale = 0.0, const float depthError = 0.0)
        : vKeys_(nFeatures), vDepthMeasurements_(nFeatures), vMapPoints_(nFeatures, nullptr),
          calibration_(calibration), phcalibration_(phcalibration), imageDepthScale_(dScale),
          depthError_(depthError) {
        (void)nGridCols; (void)nGridRows; (void)nImCols; (void)nImRows; (void)vDistortion;
        // scale pyramid and uncertainties (Frame.cc:57-75)
        vScaleFactor_.assign(nScales, 1.0f);
        vInvScaleFactor_.assign(nScales, 1.0f);
        vSigma2_.assign(nScales, 1.0f);
        vInvSigma2_.assign(nScales, 1.0f);
        for (int i = 1; i < nScales; i++) {
            vScaleFactor_[i] = vScaleFactor_[i - 1] * fScaleFactor;
            vSigma2_[i] = vScaleFactor_[i] * vScaleFactor_[i];
        }
        for (int i = 0; i < nScales; i++) {
            vInvScaleFactor_[i] = 1.0f / vScaleFactor_[i];
            vInvSigma2_[i] = 1.0f / vSigma2_[i];
        }
    }

    void setPose(Sophus::SE3f &Tcw) { Tcw_ = Tcw; }
    const Sophus::SE3f getPose() const { return Tcw_; }
    std::vector<cv::KeyPoint> &getKeyPoints() { return vKeys_; }
    cv::KeyPoint getKeyPoint(const size_t idx) { return vKeys_[idx]; }
    void setKeyPoint(cv::KeyPoint pKP, const size_t idx) { vKeys_[idx] = pKP; }
    float getDepthMeasure(const size_t idx) { return vDepthMeasurements_[idx]; }
    std::vector<float> &getDepthMeasurements() { return vDepthMeasurements_; }
    void setDepthMeasure(float depth, const size_t idx) { vDepthMeasurements_[idx] = depth; }
    std::vector<std::shared_ptr<MapPoint>> &getMapPoints() { return vMapPoints_; }
    std::shared_ptr<MapPoint> getMapPoint(const size_t idx) { return vMapPoints_[idx]; }
    void setMapPoint(size_t idx, std::shared_ptr<MapPoint> pMP) { vMapPoints_[idx] = pMP; }
    std::shared_ptr<CameraModel> getCalibration() { return calibration_; }
    std::shared_ptr<CameraModel> getPHCalibration() { return phcalibration_; }
    int getNumberOfScales() { return (int)vScaleFactor_.size(); }
    float getScaleFactor(int octave) { return vScaleFactor_[octave]; }
    float getInvScaleFactor(int octave) { return vInvScaleFactor_[octave]; }
    float getSigma2(int octave) { return vSigma2_[octave]; }
    float getInvSigma2(int octave) { return vInvSigma2_[octave]; }
    double getDepthScale() { return imageDepthScale_; }
    double getEstimatedDepthScale() { return estimatedDepthScale_; }
    void setEstimatedDepthScale(double scale) { estimatedDepthScale_ = scale; }
    float getDepthError() { return depthError_; }

private:
    std::vector<cv::KeyPoint> vKeys_;
    std::vector<float> vDepthMeasurements_;
    std::vector<std::shared_ptr<MapPoint>> vMapPoints_;
    std::shared_ptr<CameraModel> calibration_, phcalibration_;
    double imageDepthScale_ = 0.0, estimatedDepthScale_ = 1.0;
    float depthError_ = 0.0f;
    Sophus::SE3f Tcw_;
    std::vector<float> vScaleFactor_, vInvScaleFactor_, vSigma2_, vInvSigma2_;
};
