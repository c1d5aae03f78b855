// graph_builder.h — the graph construction of the reference's arapOptimization
// (Modules/Optimization/g2oBundleAdjustment.cc:640-953) over the deftri_map view.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/deftri.h"

namespace deftri {

struct GraphResult {
    deftri_problem_desc desc{};
    // owned arrays behind desc
    std::vector<double> points, tg, scales, cam_pose, rep_obs, rep_info, dep_meas, dep_info, arap_w, rot, pair_area,
        pair_info, order_xy;
    std::vector<float> cam_kb8;
    std::vector<int32_t> rep_point, rep_cam, dep_point, dep_scale, dep_cam, arap_pts, arap_pair, arap_rot;
    // writeback metadata
    std::vector<int64_t> point_mpid;          // point index -> MapPoint id
    std::vector<float> point_orig;            // fp32 original positions
    std::vector<int32_t> kf_scale;            // keyframe (map order) -> last scale vertex (-1: none)
    std::vector<int32_t> pair_kf1, pair_kf2;  // per pair: keyframe indices (map order)
    std::vector<int32_t> pair_T;              // facets.count() per pair
    std::vector<int32_t> pair_hull;           // convex hull size per pair
    std::vector<double> rep_base;             // per reprojection edge: invSigma2 of its octave
    // memo: the serialized inputs (everything but the weights) of the graph held here
    std::vector<unsigned char> memo_key;
    bool memo_valid = false;
    int64_t memo_hits = 0;                    // calls answered from the memo (kept across rebuilds)
    // structure memo (deformationOptimization's next round: the written-back map, positions / depth
    // scales / T_g moved, everything else equal): the per-pair meshes and where every
    // position-dependent value came from.  A later call with the same structure key whose every pair's
    // previous triangulation is still THE Delaunay triangulation of the moved points (and whose vector
    // map is still the identity) refreshes the values in place — the same descriptor, bit for bit, as a
    // full build of that map, except order_xy (the ordering hint): it keeps the coordinates of the
    // build that established the structure, so the device plan is reused
    // (tests/test_graph.py::test_next_round_fast_path_is_a_full_build)
    // a pair's mesh depends only on its keyframe 1's positions (v1Positions, :653-662): the pairs
    // that share keyframe 1 (every all-pairs graph) share one mesh
    struct MeshData {
        std::vector<int32_t> tris, off, adj, pos_idx, inv;
        std::vector<double> pos1, w;          // positions (x y z) and host cot weights (empty: device pass)
        int n1 = 0, T = 0, hull = 0;
        int skipped = 0;                      // duplicate points the triangulation left out
        int flips = -1;                       // >= 0: repaired from the previous round's mesh (flips)
        double area = 0;
        bool identity_map = false;
    };
    struct PairMesh {
        std::shared_ptr<const MeshData> mesh;
        int n2 = 0, kf1 = 0, kf2 = 0;
        int64_t w_off = 0;
    };
    std::vector<unsigned char> struct_key;
    bool struct_valid = false;
    std::vector<PairMesh> meshes;
    std::vector<double> wcat;                 // the pairs' CSR cot weights, concatenated
    std::vector<int64_t> arap_wk;             // per ARAP edge: its weight's entry in wcat
    std::vector<int32_t> point_kf, point_slot;   // per point: the keyframe (map order) and slot of its position
    std::vector<int32_t> order_kf, order_slot;   // ... and of its ordering coordinates
    int64_t struct_hits = 0;                  // calls answered by the structure memo
    int64_t mesh_repairs = 0, mesh_flips = 0; // full builds' meshes flip-repaired from the previous round (kept)
    double ms_last = 0;                       // host time of the last build (either path)
};

// The per-pair geometry on the device (graph_dev.hip): the cot weights of the pair's CSR mesh (one
// thread per triangle corner, the edge's two corner terms added in the finishing pass) and computeR
// (one thread per vertex); the same arithmetic as the host loops (procrustes.h), so both give the
// same weights and rotations bit for bit
class GraphDevice {
 public:
    GraphDevice(int device, hipStream_t st) : dev_(device), st_(st) {}
    ~GraphDevice();
    // 0 done; 1 a non-manifold edge (more than two opposite corners): nothing usable, the caller
    // runs the host loops for this pair; -1 a HIP error (err)
    int mesh_pass(int n1, int n2, const int32_t *tris, int ntri, const int32_t *off, const int32_t *adj, int64_t nadj,
                  const int32_t *pos_idx, const int32_t *inv, const double *pos1, const double *pos2, double *w,
                  double *R, std::string &err);
    double ms_last = 0;          // device time of the last mesh_pass (kernels only)

 private:
    int dev_;
    hipStream_t st_;
    void *buf_ = nullptr;
    size_t cap_ = 0;
};

// pair_window > 0: only keyframe pairs (a, b) with b - a <= pair_window in map order (the
// sliding-window deviation of BASELINE C5; 0 = every pair, the reference's loop :640-645)
bool build_arap_graph(const deftri_map &map, double rep_weight, double arap_weight, float depth_error,
                      GraphResult &g, std::string &err, int pair_window = 0, GraphDevice *gdev = nullptr);

void writeback_arap(deftri_map &map, const GraphResult &g, const std::vector<double> &points,
                    const std::vector<double> &scales, const std::vector<double> &tg, double *optimization_update);

// Delaunay mesh of the positions' (x, y) (ComputeDelaunayTriangulation3D + ComputeAdjacencyList,
// Geometry.cc:317-368): sorted neighbour lists, GetSurfaceArea, createVectorMap (vertex -> position)
bool mesh_adjacency(const std::vector<double> &pos, int n, std::vector<std::vector<int32_t>> &adj,
                    std::vector<int32_t> &pos_index, double &area, std::string &err);

// 3x3 helpers exported for tests
void procrustes_rotation(const double S[9], double R[9]);

}  // namespace deftri
