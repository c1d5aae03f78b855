// map_io.h — test harness only: a Map of the model (adapter/model) rebuilt from the binary dump
// tests/adapter_io.py writes from the Python host model (deftri/mapmodel.py), and the results
// written back in the same spirit.  Layout (little-endian), all counts int32:
//   "DTMAP001" | n_kf | per keyframe, in insertion order: id i64, q[4] f32 (x y z w), t[3] f32,
//   kb8[8] f32, n_scales, scale_factor f32, inv_sigma2[n_scales] f32, depth_scale f64, n_slots,
//   uv[2 n_slots] f32, octave[n_slots] i32, depth[n_slots] f32, point_id[n_slots] i64 (-1 = null)
//   | n_mp | per MapPoint, in insertion order: id i64, pos[3] f32
//   | n_obs | per observation, in Map::addObservation order: kf i64, mp i64, idx i64
//   | n_gt | per stored global transformation: kf1 i64, kf2 i64, q[4] f32, t[3] f32
//   | n_pts | original[3 n_pts] f32, moved[3 n_pts] f32
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "Map/Map.h"

struct MapDump {
    std::shared_ptr<Map> map;
    std::vector<std::shared_ptr<KeyFrame>> kfs;          // insertion order
    std::vector<std::shared_ptr<MapPoint>> mps;          // insertion order
    std::vector<Eigen::Vector3f> original, moved;
    std::map<long unsigned int, std::shared_ptr<Frame>> frames;
};

class Reader {
public:
    explicit Reader(const std::string &path) : f_(std::fopen(path.c_str(), "rb")) {
        if (!f_) throw std::runtime_error("cannot open " + path);
    }
    ~Reader() { std::fclose(f_); }
    template <typename T>
    T get() {
        T v;
        if (std::fread(&v, sizeof(T), 1, f_) != 1) throw std::runtime_error("short read");
        return v;
    }
    template <typename T>
    std::vector<T> vec(size_t n) {
        std::vector<T> v(n);
        if (n && std::fread(v.data(), sizeof(T), n, f_) != n) throw std::runtime_error("short read");
        return v;
    }

private:
    std::FILE *f_;
};

inline MapDump read_map(const std::string &path) {
    Reader r(path);
    const auto magic = r.vec<char>(8);
    if (std::string(magic.begin(), magic.end()) != "DTMAP001") throw std::runtime_error("not a map dump");
    MapPoint::resetIdCounter();
    KeyFrame::resetIdCounter();
    MapDump d;
    d.map = std::make_shared<Map>(15.0f);
    struct KfData {
        int64_t id;
        std::vector<int64_t> pid;
    };
    std::vector<KfData> kd;
    const int32_t nkf = r.get<int32_t>();
    for (int k = 0; k < nkf; k++) {
        const int64_t id = r.get<int64_t>();
        const auto q = r.vec<float>(4);
        const auto t = r.vec<float>(3);
        const auto kb8 = r.vec<float>(8);
        const int32_t nScales = r.get<int32_t>();
        const float factor = r.get<float>();
        const auto isig = r.vec<float>(nScales);
        const double depthScale = r.get<double>();
        const int32_t nSlots = r.get<int32_t>();
        const auto uv = r.vec<float>(2 * (size_t)nSlots);
        const auto oct = r.vec<int32_t>(nSlots);
        const auto dep = r.vec<float>(nSlots);
        auto cam = std::make_shared<KannalaBrandt8>(kb8);
        auto f = std::make_shared<Frame>(nSlots, 0, 0, 0, 0, nScales, factor, cam, cam);
        for (int o = 0; o < nScales; o++)
            if (f->getInvSigma2(o) != isig[o]) throw std::runtime_error("invSigma2 table differs from Frame's");
        Sophus::SE3f T(Eigen::Quaternionf(q[3], q[0], q[1], q[2]), Eigen::Vector3f(t[0], t[1], t[2]));
        f->setPose(T);
        for (int s = 0; s < nSlots; s++) {
            cv::KeyPoint kp;
            kp.pt.x = uv[2 * s];
            kp.pt.y = uv[2 * s + 1];
            kp.octave = oct[s];
            f->setKeyPoint(kp, s);
            f->setDepthMeasure(dep[s], s);
        }
        f->setEstimatedDepthScale(depthScale);
        auto kf = std::make_shared<KeyFrame>(*f);
        if ((int64_t)kf->getId() != id) throw std::runtime_error("keyframe ids must be 0.. in insertion order");
        d.frames[kf->getId()] = f;
        d.kfs.push_back(kf);
        kd.push_back({id, r.vec<int64_t>(nSlots)});
    }
    const int32_t nmp = r.get<int32_t>();
    std::map<int64_t, std::shared_ptr<MapPoint>> byId;
    for (int i = 0; i < nmp; i++) {
        const int64_t id = r.get<int64_t>();
        auto p = r.vec<float>(3);
        Eigen::Vector3f pos(p[0], p[1], p[2]);
        auto mp = std::make_shared<MapPoint>(pos);
        if ((int64_t)mp->getId() != id) throw std::runtime_error("map point ids must be 0.. in insertion order");
        d.mps.push_back(mp);
        byId[id] = mp;
    }
    for (auto &kf : d.kfs) d.map->insertKeyFrame(kf);
    for (auto &mp : d.mps) d.map->insertMapPoint(mp);
    for (size_t k = 0; k < d.kfs.size(); k++)
        for (size_t s = 0; s < kd[k].pid.size(); s++)
            if (kd[k].pid[s] >= 0) d.kfs[k]->setMapPoint(s, byId.at(kd[k].pid[s]));
    const int32_t nobs = r.get<int32_t>();
    for (int i = 0; i < nobs; i++) {
        const int64_t kf = r.get<int64_t>(), mp = r.get<int64_t>(), idx = r.get<int64_t>();
        d.map->addObservation((ID)kf, (ID)mp, (size_t)idx);
    }
    const int32_t ngt = r.get<int32_t>();
    for (int i = 0; i < ngt; i++) {
        const int64_t a = r.get<int64_t>(), b = r.get<int64_t>();
        const auto q = r.vec<float>(4);
        const auto t = r.vec<float>(3);
        // inserted as the reference does: T for (a, b), its inverse for (b, a)
        d.map->insertGlobalKeyFramesTransformation((ID)a, (ID)b,
                                                   Sophus::SE3f(Eigen::Quaternionf(q[3], q[0], q[1], q[2]),
                                                                Eigen::Vector3f(t[0], t[1], t[2])));
    }
    const int32_t npts = r.get<int32_t>();
    const auto o = r.vec<float>(3 * (size_t)npts), m = r.vec<float>(3 * (size_t)npts);
    for (int i = 0; i < npts; i++) {
        d.original.emplace_back(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
        d.moved.emplace_back(m[3 * i], m[3 * i + 1], m[3 * i + 2]);
    }
    return d;
}
