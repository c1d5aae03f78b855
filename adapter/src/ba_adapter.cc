// ba_adapter.cc — the reference's bundle-adjustment entry points over the C-ABI (deftri_ba_*):
//   bundleAdjustment(Map*)               g2oBundleAdjustment.cc:38-138
//   poseOnlyOptimization(Frame&)         g2oBundleAdjustment.cc:140-243
//   localBundleAdjustment(Map*, ID)      g2oBundleAdjustment.cc:245-444
// Each builds the reference's graph (pose vertices in KeyFrame iteration order, KeyFrame 0 fixed,
// MapPoints marginalized, EdgeSE3ProjectXYZ with information invSigma2(octave) I2 and Huber
// (float)sqrt(5.99)) as flat arrays, hands it to the device, and replays the reference's control
// flow around optimize(): outlier levels, robust-kernel removal, write-back in fp32.  The same flows
// run in deftri/ba.py (the parity tests' host mirror).
#include <cmath>
#include <iostream>
#include <set>
#include <unordered_map>
#include <vector>

#include "Optimization/g2oBundleAdjustment.h"
#include "deftri_adapter.h"

namespace {

constexpr double kChi2Outlier = 5.991;

struct BAGraph {
    std::vector<double> poses, points, obs, info;
    std::vector<float> kb8;
    std::vector<uint8_t> pose_fixed, point_fixed;
    std::vector<int32_t> edge_point, edge_pose;
    // per edge: the KeyFrame / Frame slot and MapPoint it came from (outlier removal)
    std::vector<size_t> edge_slot;
    std::vector<int> edge_kf;
    std::vector<std::shared_ptr<MapPoint>> mps;       // point vertices in creation order
    std::unordered_map<MapPoint *, int32_t> mp_index;

    void add_pose(const Sophus::SE3f &T, const std::shared_ptr<CameraModel> &cam, bool fixed) {
        double p7[7];
        deftri_adapter::se3quat7(T, p7);
        poses.insert(poses.end(), p7, p7 + 7);
        for (int i = 0; i < 8; i++) kb8.push_back(cam->getParameter(i));
        pose_fixed.push_back(fixed ? 1 : 0);
    }
    int32_t point_of(const std::shared_ptr<MapPoint> &mp) {
        auto it = mp_index.find(mp.get());
        if (it != mp_index.end()) return it->second;
        const int32_t id = (int32_t)mps.size();
        mp_index.emplace(mp.get(), id);
        mps.push_back(mp);
        const Eigen::Vector3f p = mp->getWorldPosition();
        points.insert(points.end(), {(double)p.x(), (double)p.y(), (double)p.z()});
        return id;
    }
    void add_edge(int32_t point, int32_t pose, const cv::KeyPoint &kp, float invSigma2, int kf, size_t slot) {
        edge_point.push_back(point);
        edge_pose.push_back(pose);
        obs.insert(obs.end(), {(double)kp.pt.x, (double)kp.pt.y});
        info.push_back(invSigma2);
        edge_kf.push_back(kf);
        edge_slot.push_back(slot);
    }
    deftri_ba_desc desc() const {
        deftri_ba_desc d{};
        d.n_poses = (int32_t)pose_fixed.size();
        d.n_points = (int32_t)mps.size();
        d.n_edges = (int32_t)edge_point.size();
        d.poses = poses.data();
        d.pose_fixed = pose_fixed.data();
        d.pose_kb8 = kb8.data();
        d.points = points.data();
        d.point_fixed = point_fixed.empty() ? nullptr : point_fixed.data();
        d.edge_point = edge_point.data();
        d.edge_pose = edge_pose.data();
        d.edge_obs = obs.data();
        d.edge_info = info.data();
        d.huber_delta = (double)(float)std::sqrt(5.99);   // const float thHuber2D = sqrt(5.99)
        return d;
    }
};

deftri_lm_params lm_params(int n_iterations) {
    deftri_lm_params p{};
    p.n_iterations = n_iterations;
    p.max_trials = 10;
    p.tau = 1e-5;
    p.analytic_jacobians = 1;
    return p;
}

bool report(deftri_ba_ctx *ba, int rc, const char *what) {
    if (rc) std::cerr << "deftri: " << what << ": " << deftri_ba_last_error(ba) << " (error " << rc << ")" << std::endl;
    return rc == 0;
}

// fp32 write-back: Sophus::SE3f of the estimate, estimate().cast<float>() for points
void write_poses(const std::vector<std::shared_ptr<KeyFrame>> &kfs, size_t n, const std::vector<double> &poses) {
    for (size_t k = 0; k < n; k++) {
        Sophus::SE3f T = deftri_adapter::se3f_from7(&poses[7 * k]);
        kfs[k]->setPose(T);
    }
}
void write_points(const BAGraph &g, const std::vector<double> &pts) {
    for (size_t i = 0; i < g.mps.size(); i++) {
        Eigen::Vector3f p((float)pts[3 * i], (float)pts[3 * i + 1], (float)pts[3 * i + 2]);
        g.mps[i]->setWorldPosition(p);
    }
}

}  // namespace

void bundleAdjustment(Map *pMap) {
    deftri_ba_ctx *ba = deftri_adapter::ba_context();
    if (!ba) return;
    BAGraph g;
    std::vector<std::shared_ptr<KeyFrame>> kfs;
    for (auto &kv : pMap->getKeyFrames()) {                                 // (:58-117)
        std::shared_ptr<KeyFrame> kf = kv.second;
        const int32_t pose = (int32_t)kfs.size();
        g.add_pose(kf->getPose(), kf->getCalibration(), kf->getId() == 0);
        std::vector<std::shared_ptr<MapPoint>> &slots = kf->getMapPoints();
        for (size_t s = 0; s < slots.size(); s++) {
            if (!slots[s]) continue;
            const cv::KeyPoint kp = kf->getKeyPoint(s);
            g.add_edge(g.point_of(slots[s]), pose, kp, kf->getInvSigma2(kp.octave), pose, s);
        }
        kfs.push_back(kf);
    }
    const deftri_ba_desc d = g.desc();
    deftri_lm_params p = lm_params(20);                                    // optimizer.optimize(20)
    deftri_report &r = deftri_adapter::report_slot();
    r = deftri_report{};
    std::vector<double> poses(g.poses.size()), pts(g.points.size());
    if (!report(ba, deftri_ba_upload(ba, &d), "bundleAdjustment") ||
        !report(ba, deftri_ba_solve_lm(ba, &p, 0, &r), "bundleAdjustment") ||
        !report(ba, deftri_ba_download(ba, poses.data(), pts.data()), "bundleAdjustment"))
        return;                                                            // map unchanged
    write_poses(kfs, kfs.size(), poses);                                   // (:119-136)
    write_points(g, pts);
}

void localBundleAdjustment(Map *pMap, ID currKeyFrameId) {
    deftri_ba_ctx *ba = deftri_adapter::ba_context();
    if (!ba) return;
    std::set<ID> sLocalMapPoints, sLocalKeyFrames, sFixedKeyFrames;
    pMap->getLocalMapOfKeyFrame(currKeyFrameId, sLocalMapPoints, sLocalKeyFrames, sFixedKeyFrames);
    BAGraph g;
    std::vector<std::shared_ptr<KeyFrame>> kfs;
    // local KeyFrames (every observed point), then the fixed ones (edges to local points only) (:276-387)
    for (int fixedSet = 0; fixedSet < 2; fixedSet++) {
        for (ID kfId : fixedSet ? sFixedKeyFrames : sLocalKeyFrames) {
            std::shared_ptr<KeyFrame> kf = pMap->getKeyFrame(kfId);
            const int32_t pose = (int32_t)kfs.size();
            g.add_pose(kf->getPose(), kf->getCalibration(), fixedSet || kfId == 0);
            std::vector<std::shared_ptr<MapPoint>> &slots = kf->getMapPoints();
            for (size_t s = 0; s < slots.size(); s++) {
                if (!slots[s]) continue;
                if (fixedSet && !sLocalMapPoints.count(slots[s]->getId())) continue;
                const cv::KeyPoint kp = kf->getKeyPoint(s);
                g.add_edge(g.point_of(slots[s]), pose, kp, kf->getInvSigma2(kp.octave), pose, s);
            }
            kfs.push_back(kf);
        }
    }
    const size_t nLocal = sLocalKeyFrames.size();
    const deftri_ba_desc d = g.desc();
    const size_t E = g.edge_point.size();
    deftri_report &r = deftri_adapter::report_slot();
    r = deftri_report{};
    deftri_lm_params p5 = lm_params(5), p10 = lm_params(10);
    std::vector<double> chi(E);
    std::vector<uint8_t> dpos(E), level(E), robust(E, 0);
    if (!report(ba, deftri_ba_upload(ba, &d), "localBundleAdjustment") ||
        !report(ba, deftri_ba_solve_lm(ba, &p5, 0, &r), "localBundleAdjustment") ||   // optimize(5)
        !report(ba, deftri_ba_edge_chi2(ba, chi.data(), dpos.data()), "localBundleAdjustment"))
        return;
    // outliers (chi2 > 5.991 or depth <= 0) to level 1, robust kernels off, optimize(10) (:389-412)
    for (size_t e = 0; e < E; e++) level[e] = (chi[e] > kChi2Outlier || !dpos[e]) ? 1 : 0;
    if (!report(ba, deftri_ba_set_edge_flags(ba, level.data(), robust.data()), "localBundleAdjustment") ||
        !report(ba, deftri_ba_solve_lm(ba, &p10, 0, &r), "localBundleAdjustment") ||
        !report(ba, deftri_ba_edge_chi2(ba, chi.data(), dpos.data()), "localBundleAdjustment"))
        return;
    std::vector<double> poses(g.poses.size()), pts(g.points.size());
    if (!report(ba, deftri_ba_download(ba, poses.data(), pts.data()), "localBundleAdjustment")) return;
    // outlier observations removed from the map (:414-428)
    for (size_t e = 0; e < E; e++) {
        if (!(chi[e] > kChi2Outlier || !dpos[e])) continue;
        std::shared_ptr<KeyFrame> kf = kfs[g.edge_kf[e]];
        const ID mpId = g.mps[g.edge_point[e]]->getId();
        kf->setMapPoint(g.edge_slot[e], nullptr);
        pMap->removeObservation(kf->getId(), mpId);
    }
    write_poses(kfs, nLocal, poses);                                        // local KeyFrames only (:430-437)
    write_points(g, pts);
}

int poseOnlyOptimization(Frame &currFrame) {
    deftri_ba_ctx *ba = deftri_adapter::ba_context();
    if (!ba) return 0;
    std::vector<std::shared_ptr<MapPoint>> &slots = currFrame.getMapPoints();
    const size_t nSlots = slots.size();
    BAGraph g;
    g.add_pose(currFrame.getPose(), currFrame.getCalibration(), false);
    std::vector<size_t> edgeSlot;
    for (size_t s = 0; s < nSlots; s++) {                                  // (:157-187): Xworld fixed
        if (!slots[s]) continue;
        const cv::KeyPoint kp = currFrame.getKeyPoint(s);
        g.add_edge(g.point_of(slots[s]), 0, kp, currFrame.getInvSigma2(kp.octave), 0, s);
        edgeSlot.push_back(s);
    }
    g.point_fixed.assign(g.mps.size(), 1);
    const size_t E = edgeSlot.size();
    const deftri_ba_desc d = g.desc();
    if (!report(ba, deftri_ba_upload(ba, &d), "poseOnlyOptimization")) return 0;
    std::vector<uint8_t> vInlier(nSlots, 0), level(E, 0), robust(E, 1), maskLo(E), maskHi(E);
    std::vector<int> edgeOfSlot(nSlots, -1);
    for (size_t e = 0; e < E; e++) {
        vInlier[edgeSlot[e]] = 1;
        edgeOfSlot[edgeSlot[e]] = (int)e;
    }
    std::vector<double> chi(E);
    deftri_lm_params p10 = lm_params(10);
    deftri_report &r = deftri_adapter::report_slot();
    r = deftri_report{};
    // 4 rounds: reset the pose, initializeOptimization(0), optimize(10), reclassify (:189-228).  The
    // guard before computeError() reads vInlier[round] instead of vInlier[j] (:196-197): edges j <=
    // round are checked against vInlier[round] as it was before edge `round` is reclassified, later
    // edges against its new value
    for (size_t rnd = 0; rnd < 4; rnd++) {
        if (!report(ba, deftri_ba_set_state(ba, g.poses.data(), nullptr), "poseOnlyOptimization") ||
            !report(ba, deftri_ba_set_edge_flags(ba, level.data(), robust.data()), "poseOnlyOptimization") ||
            !report(ba, deftri_ba_solve_lm(ba, &p10, 0, &r), "poseOnlyOptimization"))
            return 0;
        bool anyLo = false, anyHi = false;
        for (size_t e = 0; e < E; e++) {
            maskLo[e] = edgeSlot[e] <= rnd;
            maskHi[e] = !maskLo[e];
            anyLo = anyLo || maskLo[e];
            anyHi = anyHi || maskHi[e];
        }
        const bool outlierBefore = rnd < nSlots ? !vInlier[rnd] : false;
        if (outlierBefore && anyLo && !report(ba, deftri_ba_compute_errors(ba, maskLo.data()), "poseOnlyOptimization"))
            return 0;
        if (!report(ba, deftri_ba_edge_chi2(ba, chi.data(), nullptr), "poseOnlyOptimization")) return 0;
        bool inlierRnd;
        if (rnd < nSlots && edgeOfSlot[rnd] >= 0)
            inlierRnd = !(chi[edgeOfSlot[rnd]] > kChi2Outlier);
        else
            inlierRnd = rnd < nSlots ? vInlier[rnd] != 0 : false;
        if (!inlierRnd && anyHi) {
            if (!report(ba, deftri_ba_compute_errors(ba, maskHi.data()), "poseOnlyOptimization") ||
                !report(ba, deftri_ba_edge_chi2(ba, chi.data(), nullptr), "poseOnlyOptimization"))
                return 0;
        }
        for (size_t e = 0; e < E; e++) {
            const bool out = chi[e] > kChi2Outlier;
            vInlier[edgeSlot[e]] = out ? 0 : 1;
            level[e] = out ? 1 : 0;
            if (rnd == 2) robust[e] = 0;
        }
    }
    int nGood = 0;
    for (size_t s = 0; s < nSlots; s++) {                                  // (:230-240)
        if (!vInlier[s])
            currFrame.setMapPoint(s, nullptr);
        else
            nGood++;
    }
    std::vector<double> pose(7);
    if (!report(ba, deftri_ba_download(ba, pose.data(), nullptr), "poseOnlyOptimization")) return nGood;
    Sophus::SE3f T = deftri_adapter::se3f_from7(pose.data());
    currFrame.setPose(T);
    return nGood;
}
