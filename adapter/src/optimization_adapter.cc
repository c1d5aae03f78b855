// optimization_adapter.cc — definitions of the reference's ARAP entry points over the C-ABI:
//   arapOptimization        g2oBundleAdjustment.cc:608-1008
//   deformationOptimization g2oBundleAdjustment.cc:446-606 (+ outerObjective, nloptOptimization.cc:4-37)
//   arapOpen3DOptimization  g2oBundleAdjustment.cc:1010- (Open3D; out of scope: reports, map unchanged)
//   calculatePixelsStandDev Modules/Utils/Geometry.cc:370-498
// The Map is read through its public members only (KeyFrame / MapPoint getters, the observation
// and global-transformation tables) and written back through the setters the reference uses.  The
// graph build, the LM solve, the weight search and the metric run inside libdeftri.so.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>

#include "Optimization/g2oBundleAdjustment.h"
#include "Utils/Geometry.h"
#include "Utils/Measurements.h"
#include "deftri_adapter.h"

namespace deftri_adapter {

namespace {
int g_device = 0;

struct ThreadContexts {
    deftri_ctx *arap = nullptr;
    deftri_ba_ctx *ba = nullptr;
    bool arap_failed = false, ba_failed = false;
    ~ThreadContexts() {
        if (arap) deftri_ctx_destroy(arap);
        if (ba) deftri_ba_destroy(ba);
    }
};
thread_local ThreadContexts t_ctx;
thread_local deftri_report t_report;
thread_local deftri_deformation_report t_def_report;
}  // namespace

void set_device(int device) { g_device = device; }

deftri_ctx *context() {
    if (!t_ctx.arap && !t_ctx.arap_failed) {
        const int rc = deftri_ctx_create(g_device, &t_ctx.arap);
        if (rc) {
            std::cerr << "deftri: no usable gfx950 device " << g_device << " (error " << rc << ")" << std::endl;
            t_ctx.arap = nullptr;
            t_ctx.arap_failed = true;
        }
    }
    return t_ctx.arap;
}

deftri_ba_ctx *ba_context() {
    if (!t_ctx.ba && !t_ctx.ba_failed) {
        const int rc = deftri_ba_create(g_device, &t_ctx.ba);
        if (rc) {
            std::cerr << "deftri: no usable gfx950 device " << g_device << " (error " << rc << ")" << std::endl;
            t_ctx.ba = nullptr;
            t_ctx.ba_failed = true;
        }
    }
    return t_ctx.ba;
}

const deftri_report &last_report() { return t_report; }
deftri_report &report_slot() { return t_report; }
const deftri_deformation_report &last_deformation_report() { return t_def_report; }

void se3quat7(const Sophus::SE3f &T, double out[7]) {
    const auto &q = T.unit_quaternion();
    double d[4] = {q.x(), q.y(), q.z(), q.w()};
    if (d[3] < 0)
        for (double &v : d) v = -v;
    const double nrm = std::sqrt(((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) + d[3] * d[3]);
    for (int k = 0; k < 4; k++) out[k] = d[k] / nrm;
    const auto &t = T.translation();
    out[4] = t.x();
    out[5] = t.y();
    out[6] = t.z();
}

Sophus::SE3f se3f_from7(const double t7[7]) {
    const Eigen::Quaterniond q(t7[3], t7[0], t7[1], t7[2]);
    const Eigen::Vector3d t(t7[4], t7[5], t7[6]);
    return Sophus::SE3f(q.cast<float>(), t.cast<float>());
}

MapView::MapView(Map *pMap) {
    for (auto &kv : pMap->getKeyFrames()) order_.push_back(kv.second);   // the reference's loop order (:640-645)
    const size_t K = order_.size();
    arr_.resize(K);
    kfs_.resize(K);
    for (size_t k = 0; k < K; k++) {
        KeyFrame &kf = *order_[k];
        Arrays &A = arr_[k];
        std::vector<std::shared_ptr<MapPoint>> &slots = kf.getMapPoints();
        const size_t nSlots = slots.size();
        A.id.assign(nSlots, -1);
        A.pos.assign(3 * nSlots, 0.f);
        A.obs.assign(nSlots, -1);
        for (size_t i = 0; i < nSlots; i++) {
            if (!slots[i]) continue;
            A.id[i] = (int64_t)slots[i]->getId();
            const Eigen::Vector3f p = slots[i]->getWorldPosition();
            A.pos[3 * i] = p.x();
            A.pos[3 * i + 1] = p.y();
            A.pos[3 * i + 2] = p.z();
            A.obs[i] = pMap->isMapPointInKeyFrame(slots[i]->getId(), kf.getId());   // (:765-768)
        }
        std::vector<cv::KeyPoint> &keys = kf.getKeyPoints();
        const size_t nObs = keys.size();
        A.uv.resize(2 * nObs);
        A.oct.resize(nObs);
        A.dep.resize(nObs);
        for (size_t j = 0; j < nObs; j++) {
            A.uv[2 * j] = keys[j].pt.x;
            A.uv[2 * j + 1] = keys[j].pt.y;
            A.oct[j] = keys[j].octave;
            // the per-index simulated depth (KeyFrame.cc:123-125); the image lookup of :816,846 throws
            // in the simulation
            A.dep[j] = kf.getDepthMeasure(j);
        }
        const int nScales = kf.getNumberOfScales();
        for (int o = 0; o < nScales; o++) A.isig.push_back(kf.getInvSigma2(o));
        deftri_keyframe &D = kfs_[k];
        D = deftri_keyframe{};
        D.id = (int64_t)kf.getId();
        se3quat7(kf.getPose(), D.pose);
        std::shared_ptr<CameraModel> cam = kf.getCalibration();
        for (int i = 0; i < 8; i++) D.kb8[i] = cam->getParameter(i);
        D.n_scales = (int32_t)A.isig.size();
        D.inv_sigma2 = A.isig.data();
        D.depth_scale = kf.getEstimatedDepthScale();
        D.n_slots = (int32_t)nSlots;
        D.point_id = A.id.data();
        D.point_pos = A.pos.data();
        D.obs_index = A.obs.data();
        D.kp_uv = A.uv.data();
        D.kp_octave = A.oct.data();
        D.depth = A.dep.data();
        D.n_obs = (int32_t)nObs;
    }
    // every pair's T_g starts from getGlobalKeyFramesTransformation(k2, k1) (:664): the store queried
    // for every ordered pair, only the stored entries passed (an absent pair reads the identity)
    for (size_t a = 0; a < K; a++)
        for (size_t b = 0; b < K; b++) {
            if (a == b) continue;
            const ID ia = order_[a]->getId(), ib = order_[b]->getId();
            const Sophus::SE3f G = pMap->getGlobalKeyFramesTransformation(ia, ib);
            double g7[7];
            se3quat7(G, g7);
            const bool identity = g7[0] == 0 && g7[1] == 0 && g7[2] == 0 && g7[4] == 0 && g7[5] == 0 && g7[6] == 0;
            if (identity) continue;
            deftri_global_entry e{};
            e.kf1 = (int64_t)ia;
            e.kf2 = (int64_t)ib;
            std::copy(g7, g7 + 7, e.t);
            globals_.push_back(e);
        }
    m_.n_keyframes = (int32_t)K;
    m_.keyframes = kfs_.data();
    const double identity7[7] = {0, 0, 0, 1, 0, 0, 0};
    std::copy(identity7, identity7 + 7, m_.global_t);
    m_.n_global = (int32_t)globals_.size();
    m_.globals = globals_.data();
}

void MapView::write_back(Map *pMap) {
    for (size_t k = 0; k < order_.size(); k++) {
        KeyFrame &kf = *order_[k];
        kf.setEstimatedDepthScale(kfs_[k].depth_scale);                    // (:967-972)
        std::vector<std::shared_ptr<MapPoint>> &slots = kf.getMapPoints();
        for (size_t i = 0; i < slots.size(); i++) {
            if (!slots[i]) continue;
            Eigen::Vector3f p(arr_[k].pos[3 * i], arr_[k].pos[3 * i + 1], arr_[k].pos[3 * i + 2]);
            slots[i]->setWorldPosition(p);                                 // (:978-990)
        }
    }
    const Sophus::SE3f Tg = se3f_from7(m_.global_t);                      // (:999-1007)
    pMap->insertGlobalKeyFramesTransformation(0, 1, Tg);
}

}  // namespace deftri_adapter

using deftri_adapter::MapView;

void arapOptimization(Map *pMap, double repBalanceWeight, double globalBalanceWeight, double arapBalanceWeight,
                      double alphaWeight, double betaWeight, float DepthError, int nOptIterations,
                      double *optimizationUpdate) {
    deftri_ctx *ctx = deftri_adapter::context();
    if (!ctx) return;                                                      // map unchanged
    MapView view(pMap);
    double update = 0.0;
    deftri_report &rep = deftri_adapter::report_slot();
    rep = deftri_report{};
    const int rc = deftri_arap_optimization(ctx, view.map(), repBalanceWeight, globalBalanceWeight, arapBalanceWeight,
                                            alphaWeight, betaWeight, DepthError, nOptIterations, &update, &rep);
    if (rc) {
        std::cerr << "deftri: arapOptimization: " << deftri_last_error(ctx) << " (error " << rc << ")" << std::endl;
        return;                                                            // map unchanged
    }
    view.write_back(pMap);
    if (optimizationUpdate) *optimizationUpdate = update;                 // reset, then summed (:974-986)
}

void arapOpen3DOptimization(Map *pMap) {
    (void)pMap;
    std::cerr << "deftri: arapOpen3DOptimization (Open3D DeformAsRigidAsPossible) is not part of the device path; "
                 "map unchanged"
              << std::endl;
}

double getInvUncertainty(std::shared_ptr<open3d::geometry::TriangleMesh> mesh, std::vector<Eigen::Vector3d> v1Positions,
                         std::vector<Eigen::Vector3d> v2Positions, size_t i) {
    (void)mesh; (void)v1Positions; (void)v2Positions; (void)i;
    throw std::logic_error("getInvUncertainty needs Open3D's TriangleMesh; the device path does not use it");
}

void calculatePixelsStandDev(std::shared_ptr<Map> Map, PixelsError &pixelsErrors) {
    deftri_ctx *ctx = deftri_adapter::context();
    if (!ctx) return;
    MapView view(Map.get());
    deftri_pixels_error pe{};
    const int rc = deftri_pixels_stand_dev(ctx, view.map(), &pe);
    if (rc) {
        std::cerr << "deftri: calculatePixelsStandDev: " << deftri_last_error(ctx) << " (error " << rc << ")" << std::endl;
        return;
    }
    pixelsErrors = PixelsError{pe.avgc1, pe.avgc2, pe.avg, pe.desvc1, pe.desvc2, pe.desv};
}

namespace {
void append_line(const std::string &filePath, const std::string &text) {
    // the reference imbues es_ES.UTF-8 (absent on these hosts); these lines hold small integers only
    std::ofstream out(filePath, std::ios::app);
    if (out.is_open())
        out << text;
    else
        std::cerr << "Unable to open file for writing" << std::endl;
}
}  // namespace

void deformationOptimization(std::shared_ptr<Map> pMap, Settings &settings, std::shared_ptr<MapVisualizer> &mapVisualizer,
                             const std::vector<Eigen::Vector3f> originalPoints,
                             const std::vector<Eigen::Vector3f> movedPoints) {
    const float simulatedDepthErrorStanDesv = settings.getSimulatedDepthWeight() / 1000;   // (:449)
    double repBalanceWeight = settings.getOptRepWeight();
    double arapBalanceWeight = settings.getOptArapWeight();
    double globalBalanceWeight = settings.getOptGlobalWeight();
    const double alphaWeight = settings.getOptAlphaWeight();
    const double betaWeight = settings.getOptBetaWeight();
    const std::string optSelection = settings.getOptSelection();
    const std::string optWeightsSelection = settings.getOptWeightsSelection();
    const int nOptimizations = settings.getnOptimizations();
    const int nOptIterations = settings.getnOptIterations();
    const bool drawRaysSelection = settings.getDrawRaysSelection();
    const std::string filePath = settings.getExpFilePath();

    // "twoOptimizations" + "nlopt": the NLopt Nelder-Mead search on map clones, then arapOptimization
    // with its optimum (:487-530).  "twoOptimizations" + anything else is the Eigen LM (:531-564),
    // whose minimize() returns ImproperInputParameters before evaluating (the functor declares 2
    // values for the 3 weights: m < n), so that round is arapOptimization at the unchanged weights —
    // the same as every other selection's round (:565-568).
    deftri_deformation_params prm{};
    prm.selection = (optSelection == "twoOptimizations" && optWeightsSelection == "nlopt") ? 1 : 0;
    prm.alpha = alphaWeight;
    prm.beta = betaWeight;
    prm.depth_error = simulatedDepthErrorStanDesv;
    prm.n_iterations = nOptIterations;
    prm.n_optimizations = 1;                      // one round per call: this loop is the reference's
    prm.lb[0] = settings.getNloptRepLowerBound();
    prm.ub[0] = settings.getNloptRepUpperBound();
    prm.lb[1] = settings.getNloptGlobalLowerBound();
    prm.ub[1] = settings.getNloptGlobalUpperBound();
    prm.lb[2] = settings.getNloptArapLowerBound();
    prm.ub[2] = settings.getNloptArapUpperBound();
    prm.xtol_rel = settings.getNloptRelTolerance();
    prm.xtol_abs = settings.getNloptAbsTolerance();
    prm.maxeval = settings.getNloptnOptimizations();

    const size_t nMapPoints = pMap->getMapPoints().size();
    prm.n_map_points = (int32_t)nMapPoints;
    double optimizationUpdate = 100;
    for (int i = 1; i <= nOptimizations && optimizationUpdate >= (0.0001 * nMapPoints); i++) {
        if (optSelection == "open3DArap") {
            arapOpen3DOptimization(pMap.get());
        } else {
            deftri_ctx *ctx = deftri_adapter::context();
            if (!ctx) return;
            prm.rep = repBalanceWeight;
            prm.global = globalBalanceWeight;
            prm.arap = arapBalanceWeight;
            MapView view(pMap.get());
            deftri_deformation_report &rep = const_cast<deftri_deformation_report &>(deftri_adapter::last_deformation_report());
            rep = deftri_deformation_report{};
            const int rc = deftri_deformation_optimization(ctx, view.map(), &prm, &rep);
            if (rc == DEFTRI_E_SEARCH)                 // nlopt::opt::optimize throws on a failure code
                throw std::runtime_error("nlopt failure");
            if (rc) {
                std::cerr << "deftri: deformationOptimization: " << deftri_last_error(ctx) << " (error " << rc << ")"
                          << std::endl;
                return;
            }
            view.write_back(pMap.get());
            optimizationUpdate = rep.update;
            if (prm.selection == 1) {                  // the optimum is the next round's start (:528-530)
                repBalanceWeight = rep.weights[0];
                globalBalanceWeight = rep.weights[1];
                arapBalanceWeight = rep.weights[2];
            }
        }
        std::cout << "\nOptimization COMPLETED... " << i << " / " << nOptimizations << " iterations." << std::endl;
        std::cout << "\nOptimization change: " << optimizationUpdate << std::endl;
        mapVisualizer->update(drawRaysSelection);
        if (i != nOptimizations) {
            append_line(filePath, std::to_string(i) + " / " + std::to_string(nOptimizations) + " MEASUREMENTS: \n");
            measureRelativeMapErrors(pMap, filePath);
            if (originalPoints.empty() || movedPoints.empty())
                measureRealAbsoluteMapErrors(pMap, filePath);
            else
                measureSimAbsoluteMapErrors(pMap, originalPoints, movedPoints, filePath);
        }
    }
    append_line(filePath, "FINAL MEASUREMENTS: \n");
    mapVisualizer->update(drawRaysSelection);
}
