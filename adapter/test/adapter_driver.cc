// adapter_driver — test harness only: runs one reference API call through the adapter on a map
// dumped by tests/adapter_io.py, and writes the map's state afterwards for the Python side to
// compare with its own host mirror (deftri/optimization.py) on the same map.
//
//   adapter_driver <map.bin> <out.bin> deformation <settings.yaml> [sim]
//       deformationOptimization(pMap, settings, mapVisualizer) as SLAM.cc:127 calls it, or with the
//       dump's original / moved points as SLAM.cc:145 does ("sim")
//   adapter_driver <map.bin> <out.bin> arap <rep> <global> <arap> <depthError> <nIt>
//   adapter_driver <map.bin> <out.bin> pixels
//   adapter_driver <map.bin> <out.bin> ba | localba <kfId> | poseonly <kfId>
//
// Output (little-endian): "DTOUT001" | n_kf | per keyframe (insertion order): id i64,
// depth_scale f64, pose[7] f64 (se3quat7) | n_mp | per MapPoint (insertion order): id i64, pos[3]
// f32, present u8 (still in a slot) | global (0,1) and (1,0) [14] f64 | n_extra | extra[n] f64.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <set>
#include <string>

#include "../test/map_io.h"
#include "Optimization/g2oBundleAdjustment.h"
#include "Utils/Geometry.h"
#include "deftri_adapter.h"

namespace {

struct Writer {
    std::FILE *f;
    explicit Writer(const std::string &p) : f(std::fopen(p.c_str(), "wb")) {
        if (!f) throw std::runtime_error("cannot write " + p);
    }
    ~Writer() { std::fclose(f); }
    template <typename T>
    void put(const T &v) { std::fwrite(&v, sizeof(T), 1, f); }
    template <typename T>
    void put(const T *v, size_t n) { std::fwrite(v, sizeof(T), n, f); }
};

void write_state(const std::string &path, MapDump &d, const std::vector<double> &extra) {
    Writer w(path);
    w.put("DTOUT001", 8);
    w.put((int32_t)d.kfs.size());
    std::set<MapPoint *> present;
    for (auto &kf : d.kfs) {
        w.put((int64_t)kf->getId());
        w.put(kf->getEstimatedDepthScale());
        double p7[7];
        deftri_adapter::se3quat7(kf->getPose(), p7);
        w.put(p7, 7);
        for (auto &mp : kf->getMapPoints())
            if (mp) present.insert(mp.get());
    }
    w.put((int32_t)d.mps.size());
    for (auto &mp : d.mps) {
        w.put((int64_t)mp->getId());
        const Eigen::Vector3f p = mp->getWorldPosition();
        w.put(p.data(), 3);
        w.put((uint8_t)(present.count(mp.get()) ? 1 : 0));
    }
    double g[14] = {};
    if (d.kfs.size() >= 2) {
        deftri_adapter::se3quat7(d.map->getGlobalKeyFramesTransformation(0, 1), g);
        deftri_adapter::se3quat7(d.map->getGlobalKeyFramesTransformation(1, 0), g + 7);
    }
    w.put(g, 14);
    w.put((int32_t)extra.size());
    w.put(extra.data(), extra.size());
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::cerr << "usage: adapter_driver map.bin out.bin mode [args]" << std::endl;
        return 2;
    }
    MapDump d = read_map(argv[1]);
    const std::string mode = argv[3];
    std::vector<double> extra;
    if (mode == "deformation") {
        if (argc < 5) return 2;
        Settings settings(argv[4]);
        auto viz = std::make_shared<MapVisualizer>(d.map);
        if (argc > 5 && std::string(argv[5]) == "sim")
            deformationOptimization(d.map, settings, viz, d.original, d.moved);   // SLAM.cc:145
        else
            deformationOptimization(d.map, settings, viz);                        // SLAM.cc:127
        const deftri_deformation_report &r = deftri_adapter::last_deformation_report();
        extra = {(double)viz->updates(), r.weights[0], r.weights[1], r.weights[2], r.update, r.minf,
                 (double)r.nlopt_result};
    } else if (mode == "arap") {
        if (argc < 9) return 2;
        double upd = -1.0;
        arapOptimization(d.map.get(), std::atof(argv[4]), std::atof(argv[5]), std::atof(argv[6]), 0.0, 0.0,
                         (float)std::atof(argv[7]), std::atoi(argv[8]), &upd);
        const deftri_report &r = deftri_adapter::last_report();
        extra = {upd, r.chi2_initial, r.chi2_final, (double)r.iterations, (double)r.trials_total};
    } else if (mode == "pixels") {
        PixelsError pe{-1, -1, -1, -1, -1, -1};
        calculatePixelsStandDev(d.map, pe);
        extra = {pe.avgc1, pe.avgc2, pe.avg, pe.desvc1, pe.desvc2, pe.desv};
    } else if (mode == "ba") {
        bundleAdjustment(d.map.get());
        const deftri_report &r = deftri_adapter::last_report();
        extra = {r.chi2_initial, r.chi2_final, (double)r.iterations, (double)r.trials_total};
    } else if (mode == "localba") {
        if (argc < 5) return 2;
        localBundleAdjustment(d.map.get(), (ID)std::atol(argv[4]));
        const deftri_report &r = deftri_adapter::last_report();
        extra = {r.chi2_initial, r.chi2_final, (double)r.iterations, (double)r.trials_total};
    } else if (mode == "poseonly") {
        if (argc < 5) return 2;
        Frame &f = *d.frames.at((ID)std::atol(argv[4]));
        // the Frame's slots as the KeyFrame holds them (the dump filled the KeyFrame's)
        auto kf = d.map->getKeyFrame((ID)std::atol(argv[4]));
        for (size_t s = 0; s < kf->getMapPoints().size(); s++) f.setMapPoint(s, kf->getMapPoints()[s]);
        const int nGood = poseOnlyOptimization(f);
        double p7[7];
        deftri_adapter::se3quat7(f.getPose(), p7);
        extra = {(double)nGood};
        extra.insert(extra.end(), p7, p7 + 7);
        for (size_t s = 0; s < f.getMapPoints().size(); s++) extra.push_back(f.getMapPoints()[s] ? 1.0 : 0.0);
    } else {
        std::cerr << "unknown mode " << mode << std::endl;
        return 2;
    }
    write_state(argv[2], d, extra);
    return 0;
}
