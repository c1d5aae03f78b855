// Test model only — definitions for the stand-in Settings and Measurements (see
// minimal_eigen_sophus.h).  Not part of the adapter.
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "System/Settings.h"
#include "Utils/Measurements.h"

namespace {
std::string trim(const std::string &s) {
    const size_t a = s.find_first_not_of(" \t\r\n");
    if (a == std::string::npos) return "";
    const size_t b = s.find_last_not_of(" \t\r\n");
    return s.substr(a, b - a + 1);
}
}  // namespace

Settings::Settings() = default;

Settings::Settings(const std::string &configFile) {
    std::ifstream in(configFile);
    std::string line;
    while (std::getline(in, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty() || line[0] == '%') continue;
        const size_t colon = line.find(':');
        if (colon == std::string::npos) continue;
        std::string k = trim(line.substr(0, colon)), v = trim(line.substr(colon + 1));
        if (v.size() >= 2 && v.front() == '"' && v.back() == '"') v = v.substr(1, v.size() - 2);
        kv_[k] = v;
    }
}

double Settings::num(const char *key) const {
    auto it = kv_.find(key);
    if (it == kv_.end()) return 0.0;
    char *end = nullptr;
    const double v = std::strtod(it->second.c_str(), &end);
    return (end && *end == '\0') ? v : 0.0;
}

std::string Settings::str(const char *key) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? std::string() : it->second;
}

std::shared_ptr<CameraModel> Settings::getCalibration() {
    return std::make_shared<KannalaBrandt8>(std::vector<float>{
        (float)num("Camera.fx"), (float)num("Camera.fy"), (float)num("Camera.cx"), (float)num("Camera.cy"),
        (float)num("Camera.d0"), (float)num("Camera.d1"), (float)num("Camera.d2"), (float)num("Camera.d3")});
}
std::shared_ptr<CameraModel> Settings::getPHCalibration() { return getCalibration(); }
std::vector<float> Settings::getDistortionParameters() { return {}; }
int Settings::getImCols() { return (int)num("Camera.cols"); }
int Settings::getImRows() { return (int)num("Camera.rows"); }
std::string Settings::getBorderMask() { return str("FeatureExtractor.imageBoderMask"); }
int Settings::getFeaturesPerImage() { return (int)num("FeatureExtractor.nFeatures"); }
int Settings::getNumberOfScales() { return (int)num("FeatureExtractor.nScales"); }
float Settings::getScaleFactor() { return (float)num("FeatureExtractor.fScaleFactor"); }
int Settings::getGridCols() { return (int)num("FeatureGrid.nGridCols"); }
int Settings::getGridRows() { return (int)num("FeatureGrid.nGridRows"); }
float Settings::getEpipolarTh() { return (float)num("Epipolar.th"); }
int Settings::getMatchingInitTh() { return (int)num("Matching.initialization"); }
int Settings::getMatchingGuidedTh() { return (int)num("Matching.guidedMatching"); }
int Settings::getMatchingByProjectionTh() { return (int)num("Matching.searchByProjection"); }
int Settings::getMatchingForTriangulationTh() { return (int)num("Matching.searchForTriangulation"); }
int Settings::getMatchingFuseTh() { return (int)num("Matching.fuse"); }
float Settings::getMatchingInitRadius() { return (float)num("Matching.initialization.radius"); }
int Settings::getMinCommonObs() { return (int)num("Map.minObs"); }
float Settings::getMinMatches() { return (float)num("Triangulation.minMatches"); }
float Settings::getMinCos() { return (float)num("Triangulation.minCos"); }
bool Settings::getCheckingSelection() { return str("Triangulation.checks") == "true"; }
float Settings::getDepthLimit() { return (float)num("Triangulation.depthLimit"); }
Eigen::Vector3f Settings::getFirstCameraPos() {
    return Eigen::Vector3f((float)num("Camera.FirstPose.x"), (float)num("Camera.FirstPose.y"), (float)num("Camera.FirstPose.z"));
}
Eigen::Vector3f Settings::getSecondCameraPos() {
    return Eigen::Vector3f((float)num("Camera.SecondPose.x"), (float)num("Camera.SecondPose.y"), (float)num("Camera.SecondPose.z"));
}
float Settings::getSimulatedRepError() { return (float)num("Keypoints.RepError"); }
int Settings::getDecimalsRepError() { return (int)num("Keypoints.decimalsApproximation"); }
float Settings::getSimulatedDepthError() { return (float)num("Measurements.DepthError"); }
float Settings::getSimulatedDepthWeight() { return (float)num("Measurements.DepthWeight"); }
float Settings::getSimulatedDepthScaleC1() { return (float)num("Measurements.DepthScale.C1"); }
float Settings::getSimulatedDepthScaleC2() { return (float)num("Measurements.DepthScale.C2"); }
double Settings::getDepthMeasurementsScale() { return num("Measurements.Depth.Scale"); }
double Settings::getOptRepWeight() { return num("Optimization.rep"); }
double Settings::getOptArapWeight() { return num("Optimization.arap"); }
double Settings::getOptGlobalWeight() { return num("Optimization.global"); }
double Settings::getOptAlphaWeight() { return num("Optimization.alpha"); }
double Settings::getOptBetaWeight() { return num("Optimization.beta"); }
std::string Settings::getOptSelection() { return str("Optimization.selection"); }
std::string Settings::getOptWeightsSelection() { return str("Optimization.weightsSelection"); }
std::string Settings::getTrianMethod() { return str("Triangulation.method"); }
std::string Settings::getTrianLocation() { return str("Triangulation.seed.location"); }
int Settings::getnOptimizations() { return (int)num("Optimization.numberOfOptimizations"); }
int Settings::getnOptIterations() { return (int)num("Optimization.numberOfIterations"); }
int Settings::getNloptnOptimizations() { return (int)num("Optimization.nlopt.numberOfIterations"); }
double Settings::getNloptRelTolerance() { return num("Optimization.nlopt.relTolerance"); }
double Settings::getNloptAbsTolerance() { return num("Optimization.nlopt.absTolerance"); }
double Settings::getNloptRepLowerBound() { return num("Optimization.nlopt.rep.lowerBound"); }
double Settings::getNloptRepUpperBound() { return num("Optimization.nlopt.rep.upperBound"); }
double Settings::getNloptGlobalLowerBound() { return num("Optimization.nlopt.global.lowerBound"); }
double Settings::getNloptGlobalUpperBound() { return num("Optimization.nlopt.global.upperBound"); }
double Settings::getNloptArapLowerBound() { return num("Optimization.nlopt.arap.lowerBound"); }
double Settings::getNloptArapUpperBound() { return num("Optimization.nlopt.arap.upperBound"); }
std::string Settings::getExpFilePath() { return str("Experiment.Filepath"); }
bool Settings::getShowScene() { return str("MapVisualizer.showScene") == "true"; }
bool Settings::getDrawRaysSelection() { return str("MapVisualizer.drawRays") == "true"; }
bool Settings::getShowSolution() { return str("Visualizer.showSolution") == "true"; }
bool Settings::getStopExecutionOption() { return str("Execution.stop") == "true"; }

// The reference's Measurements.cc computes and writes the map errors (es_ES locale); the model
// appends one line naming the call so that a test can check when deformationOptimization makes it.
namespace {
void note(const std::string &filePath, const std::string &what) {
    if (filePath.empty()) return;
    std::ofstream out(filePath, std::ios::app);
    out << what << "\n";
}
}  // namespace

void measureSimAbsoluteMapErrors(const std::shared_ptr<Map> pMap, const std::vector<Eigen::Vector3f> originalPoints,
                                 const std::vector<Eigen::Vector3f> movedPoints, const std::string filePath) {
    note(filePath, "measureSimAbsoluteMapErrors " + std::to_string(pMap->getMapPoints().size()) + " " +
                       std::to_string(originalPoints.size()) + " " + std::to_string(movedPoints.size()));
}

void measureRealAbsoluteMapErrors(const std::shared_ptr<Map> pMap, const std::string filePath) {
    note(filePath, "measureRealAbsoluteMapErrors " + std::to_string(pMap->getMapPoints().size()));
}

void measureRelativeMapErrors(std::shared_ptr<Map> pMap, std::string filePath) {
    note(filePath, "measureRelativeMapErrors " + std::to_string(pMap->getKeyFrames().size()));
}
