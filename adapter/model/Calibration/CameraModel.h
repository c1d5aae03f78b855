// Test model only — stands in for Modules/Calibration/CameraModel.h (see model/minimal_eigen_sophus.h).
// The adapter reads the calibration through getParameter(i) (CameraModel.h:77): for the
// KannalaBrandt8 model every keyframe carries, fx fy cx cy k0 k1 k2 k3.
#pragma once

#include <memory>
#include <vector>

#include "minimal_eigen_sophus.h"

class CameraModel {
public:
    CameraModel() = default;
    explicit CameraModel(const std::vector<float> &vParameters) : vParameters_(vParameters) {}
    virtual ~CameraModel() = default;
    float getParameter(const int i) { return vParameters_[i]; }
    void setParameter(const float p, const size_t i) { vParameters_[i] = p; }
    size_t getNumberOfParameters() const { return vParameters_.size(); }

protected:
    std::vector<float> vParameters_;
};

// KannalaBrandt8 (Modules/Calibration/KannalaBrandt8.h): 8 parameters
class KannalaBrandt8 : public CameraModel {
public:
    explicit KannalaBrandt8(const std::vector<float> &vParameters) : CameraModel(vParameters) {}
};
