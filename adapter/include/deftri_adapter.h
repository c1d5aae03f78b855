// deftri_adapter.h — the part of the adapter that is not the reference's API: which GPU the
// calling thread's solver context uses, the Map <-> deftri_map marshalling shared by the optimizer
// and metric definitions, and the last call's solver report (for callers that log it).
#ifndef DEFTRI_ADAPTER_H
#define DEFTRI_ADAPTER_H

#include <cstdint>
#include <memory>
#include <vector>

#include "Map/Map.h"
#include "deftri.h"

namespace deftri_adapter {

// HIP device of the calling thread's contexts (default 0).  Takes effect for contexts created
// afterwards: call it before the thread's first optimizer call.  One context per host thread, as
// the reference's optimizer is single-threaded per Map.
void set_device(int device);
// the calling thread's ARAP / BA contexts, created on first use; nullptr (and a message on stderr)
// when no gfx950 device is usable
deftri_ctx *context();
deftri_ba_ctx *ba_context();

// g2o::SE3Quat(T.unit_quaternion().cast<double>(), T.translation().cast<double>()) with
// normalizeRotation (w >= 0, unit norm): qx qy qz qw tx ty tz — how every reference graph reads a pose
void se3quat7(const Sophus::SE3f &T, double out[7]);
// Sophus::SE3f of a solved SE3Quat estimate (7-vector): the quaternion cast to float and normalized
Sophus::SE3f se3f_from7(const double t7[7]);

// A deftri_map view of a Map: the keyframes in the Map's own iteration order (the order every
// reference loop takes), their slots, observations, keypoints, simulated depths and calibration,
// and the global-transformation store queried for every ordered keyframe pair.
class MapView {
public:
    explicit MapView(Map *pMap);
    deftri_map *map() { return &m_; }
    // arapOptimization's write-back (g2oBundleAdjustment.cc:967-1007): depth scales, fp32 positions of
    // every slot's MapPoint, and insertGlobalKeyFramesTransformation(0, 1, T_g)
    void write_back(Map *pMap);

private:
    struct Arrays {
        std::vector<int64_t> id;
        std::vector<float> pos;
        std::vector<int32_t> obs;
        std::vector<float> uv, dep, isig;
        std::vector<int32_t> oct;
    };
    std::vector<std::shared_ptr<KeyFrame>> order_;
    std::vector<Arrays> arr_;
    std::vector<deftri_keyframe> kfs_;
    std::vector<deftri_global_entry> globals_;
    deftri_map m_{};
};

// the solver report of this thread's last arapOptimization, or of the last optimize() of its last
// bundle-adjustment call (zeroed before each call); report_slot() is where the adapter writes it
const deftri_report &last_report();
deftri_report &report_slot();
// the report of this thread's last deformationOptimization round
const deftri_deformation_report &last_deformation_report();

}  // namespace deftri_adapter

#endif  // DEFTRI_ADAPTER_H
