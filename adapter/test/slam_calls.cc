// slam_calls — compile-and-call check of the adapter from the reference's call sites.
//
// SLAMCaller holds the members Modules/System/SLAM.h gives SLAM (pMap_, settings_, mapVisualizer_,
// originalPoints_, movedPoints_) with the same types, and its two methods make the calls of
// SLAM.cc:127 and SLAM.cc:145 with the same expressions.  main() builds a small two-keyframe map with
// the model, calls every entry point of g2oBundleAdjustment.h and calculatePixelsStandDev, and prints
// one line per call with the largest MapPoint displacement.  Without a usable GPU every call reports
// on stderr and leaves the map unchanged (the adapter's error behaviour); with one, the solves run.
#include <cmath>
#include <cstdio>
#include <memory>
#include <vector>

#include "Optimization/g2oBundleAdjustment.h"
#include "Utils/Geometry.h"

class SLAMCaller {
public:
    SLAMCaller(const std::string &settingsFile, std::shared_ptr<Map> pMap, std::vector<Eigen::Vector3f> original,
               std::vector<Eigen::Vector3f> moved)
        : settings_(settingsFile), pMap_(pMap), originalPoints_(original), movedPoints_(moved) {
        mapVisualizer_ = std::make_shared<MapVisualizer>(pMap_);
    }
    void processImage() {
        deformationOptimization(pMap_, settings_, mapVisualizer_);                                // SLAM.cc:127
    }
    void processSimulatedImage() {
        deformationOptimization(pMap_, settings_, mapVisualizer_, originalPoints_ , movedPoints_);  // SLAM.cc:145
    }
    std::shared_ptr<MapVisualizer> &visualizer() { return mapVisualizer_; }

private:
    Settings settings_;
    std::shared_ptr<Map> pMap_;
    std::shared_ptr<MapVisualizer> mapVisualizer_;
    std::vector<Eigen::Vector3f> originalPoints_, movedPoints_;
};

namespace {

std::vector<Eigen::Vector3f> snapshot(Map &m) {
    std::vector<Eigen::Vector3f> out;
    for (ID id = 0; id < m.getMapPoints().size(); id++) out.push_back(m.getMapPoint(id)->getWorldPosition());
    return out;
}

double max_move(Map &m, const std::vector<Eigen::Vector3f> &before) {
    double mx = 0;
    for (ID id = 0; id < before.size(); id++) mx = std::fmax(mx, (m.getMapPoint(id)->getWorldPosition() - before[id]).norm());
    return mx;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: slam_calls settings.yaml\n");
        return 2;
    }
    // two keyframes looking at a 6x6 grid of points (KF 0 at the origin, KF 1 shifted along x);
    // the observations are the exact equidistant projections, rounded to 0.1 px
    const int n = 36;
    const std::vector<float> kb8 = {458.654f, 457.296f, 367.215f, 248.375f, 0.f, 0.f, 0.f, 0.f};
    auto cam = std::make_shared<KannalaBrandt8>(kb8);
    auto pMap = std::make_shared<Map>(15.0f);
    std::vector<Eigen::Vector3f> original, moved;
    std::vector<std::shared_ptr<KeyFrame>> kfs;
    std::vector<std::shared_ptr<MapPoint>> mps;
    for (int i = 0; i < n; i++) {
        Eigen::Vector3f a(0.01f * (i % 6) - 0.025f, 0.01f * (i / 6) - 0.025f, 0.2f + 0.002f * std::sin(1.3f * i));
        Eigen::Vector3f b = a + Eigen::Vector3f(0.f, 0.0025f, 0.f);
        original.push_back(a);
        moved.push_back(b);
    }
    for (int k = 0; k < 2; k++) {
        Frame f(n, 0, 0, 640, 480, 8, 1.2f, cam, cam);
        Sophus::SE3f T(Eigen::Quaternionf(1.f, 0.f, 0.f, 0.f), Eigen::Vector3f(k ? -0.02f : 0.f, 0.f, 0.f));
        f.setPose(T);
        for (int i = 0; i < n; i++) {
            const Eigen::Vector3f pw = k ? moved[i] : original[i];
            const Eigen::Vector3f pc = T * pw;
            const float r = std::atan2(std::sqrt(pc.x() * pc.x() + pc.y() * pc.y()), pc.z());
            const float psi = std::atan2(pc.y(), pc.x());
            cv::KeyPoint kp;
            kp.pt.x = std::round(10.f * (kb8[0] * r * std::cos(psi) + kb8[2])) / 10.f;
            kp.pt.y = std::round(10.f * (kb8[1] * r * std::sin(psi) + kb8[3])) / 10.f;
            f.setKeyPoint(kp, i);
            f.setDepthMeasure(pc.z() * (k ? 1.7f : 0.4f), i);
        }
        kfs.push_back(std::make_shared<KeyFrame>(f));
        pMap->insertKeyFrame(kfs.back());
    }
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 2; k++) {
            Eigen::Vector3f p = k ? moved[i] : original[i];
            p = p + Eigen::Vector3f(0.0004f, -0.0003f, 0.0005f);
            mps.push_back(std::make_shared<MapPoint>(p));
            pMap->insertMapPoint(mps.back());
            kfs[k]->setMapPoint(i, mps.back());
            pMap->addObservation(kfs[k]->getId(), mps.back()->getId(), i);
        }

    SLAMCaller slam(argv[1], pMap, original, moved);
    auto before = snapshot(*pMap);
    slam.processImage();
    std::printf("deformationOptimization(127) max_move %.9g updates %d\n", max_move(*pMap, before),
                slam.visualizer()->updates());
    before = snapshot(*pMap);
    slam.processSimulatedImage();
    std::printf("deformationOptimization(145) max_move %.9g updates %d\n", max_move(*pMap, before),
                slam.visualizer()->updates());
    before = snapshot(*pMap);
    double update = -1.0;
    arapOptimization(pMap.get(), 1.0, 50.0, 2e5, 0.0, 0.0, 0.003f, 5, &update);
    std::printf("arapOptimization max_move %.9g update %.9g\n", max_move(*pMap, before), update);
    PixelsError pe{-1, -1, -1, -1, -1, -1};
    calculatePixelsStandDev(pMap, pe);
    std::printf("calculatePixelsStandDev desvc1 %.9g desvc2 %.9g\n", pe.desvc1, pe.desvc2);
    before = snapshot(*pMap);
    bundleAdjustment(pMap.get());
    std::printf("bundleAdjustment max_move %.9g\n", max_move(*pMap, before));
    before = snapshot(*pMap);
    localBundleAdjustment(pMap.get(), 1);
    std::printf("localBundleAdjustment max_move %.9g\n", max_move(*pMap, before));
    Frame frame(n, 0, 0, 640, 480, 8, 1.2f, cam, cam);
    Sophus::SE3f T1 = kfs[1]->getPose();
    frame.setPose(T1);
    for (int i = 0; i < n; i++) {
        frame.setKeyPoint(kfs[1]->getKeyPoint(i), i);
        frame.setMapPoint(i, kfs[1]->getMapPoint(i));
    }
    const int nGood = poseOnlyOptimization(frame);
    std::printf("poseOnlyOptimization inliers %d\n", nGood);
    std::printf("ok\n");
    return 0;
}
