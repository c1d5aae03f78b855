// Test model only — stands in for Modules/System/Settings.h: the same getters (Settings.h:49-120),
// read from the YAML subset the reference's cv::FileStorage parses (Settings.cc:27-190; a missing
// numeric key reads 0, a missing string "").
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "Calibration/CameraModel.h"

class Settings {
public:
    Settings();
    Settings(const std::string &configFile);

    std::shared_ptr<CameraModel> getCalibration();
    std::shared_ptr<CameraModel> getPHCalibration();
    std::vector<float> getDistortionParameters();
    int getImCols();
    int getImRows();

    std::string getBorderMask();
    int getFeaturesPerImage();
    int getNumberOfScales();
    float getScaleFactor();

    int getGridCols();
    int getGridRows();

    float getEpipolarTh();

    int getMatchingInitTh();
    int getMatchingGuidedTh();
    int getMatchingByProjectionTh();
    int getMatchingForTriangulationTh();
    int getMatchingFuseTh();

    float getMatchingInitRadius();

    int getMinCommonObs();

    float getMinMatches();
    float getMinCos();
    bool getCheckingSelection();
    float getDepthLimit();

    Eigen::Vector3f getFirstCameraPos();
    Eigen::Vector3f getSecondCameraPos();

    float getSimulatedRepError();
    int getDecimalsRepError();
    float getSimulatedDepthError();
    float getSimulatedDepthWeight();
    float getSimulatedDepthScaleC1();
    float getSimulatedDepthScaleC2();
    double getDepthMeasurementsScale();

    double getOptRepWeight();
    double getOptArapWeight();
    double getOptGlobalWeight();
    double getOptAlphaWeight();
    double getOptBetaWeight();

    std::string getOptSelection();
    std::string getOptWeightsSelection();
    std::string getTrianMethod();
    std::string getTrianLocation();

    int getnOptimizations();
    int getnOptIterations();

    int getNloptnOptimizations();
    double getNloptRelTolerance();
    double getNloptAbsTolerance();
    double getNloptRepLowerBound();
    double getNloptRepUpperBound();
    double getNloptGlobalLowerBound();
    double getNloptGlobalUpperBound();
    double getNloptArapLowerBound();
    double getNloptArapUpperBound();

    std::string getExpFilePath();

    bool getShowScene();
    bool getDrawRaysSelection();
    bool getShowSolution();
    bool getStopExecutionOption();

private:
    double num(const char *key) const;
    std::string str(const char *key) const;
    std::map<std::string, std::string> kv_;
};
