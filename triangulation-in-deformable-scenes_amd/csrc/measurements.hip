// measurements.hip — the map-error measurements of Modules/Utils/Measurements.cc on the device
// (SURVEY §8 f3): measureSimAbsoluteMapErrors (:8-98) and measureRelativeMapErrors (:350-518).
// The host walks the map in the reference's order and builds the index lists (the Delaunay mesh of
// each keyframe pair, the slot / position index quirks); the device evaluates every per-point and
// per-mesh-edge term and reduces them in a fixed order (per-block partial sums, then an ordered
// final pass: deterministic, no atomics).  The reference accumulates in float (absolute errors)
// and double (relative errors) sequentially; the device sums in double in its fixed tree, so the
// absolute figures agree with the reference's float accumulation to its rounding (tests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/deftri.h"
#include "graph_builder.h"
#include "kernels.h"

namespace deftri {
namespace dev {

#define TID (blockIdx.x * blockDim.x + threadIdx.x)

// measureSimAbsoluteMapErrors per correspondence j (fp32 as the reference): |orig - moved|,
// |opt1 - orig|, |opt2 - moved| and the two squared norms (Eigen norm = sqrt(squaredNorm),
// squaredNorm = (x^2 + y^2) + z^2)
__global__ void k_abs_terms(int n, const float *__restrict__ opt1, const float *__restrict__ opt2,
                            const float *__restrict__ orig, const float *__restrict__ moved, double *__restrict__ out) {
    int j = TID;
    if (j >= n) return;
    float m[3], e1[3], e2[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        m[k] = orig[3 * j + k] - moved[3 * j + k];
        e1[k] = opt1[3 * j + k] - orig[3 * j + k];
        e2[k] = opt2[3 * j + k] - moved[3 * j + k];
    }
    const float sm = __fadd_rn(__fadd_rn(__fmul_rn(m[0], m[0]), __fmul_rn(m[1], m[1])), __fmul_rn(m[2], m[2]));
    const float s1 = __fadd_rn(__fadd_rn(__fmul_rn(e1[0], e1[0]), __fmul_rn(e1[1], e1[1])), __fmul_rn(e1[2], e1[2]));
    const float s2 = __fadd_rn(__fadd_rn(__fmul_rn(e2[0], e2[0]), __fmul_rn(e2[1], e2[1])), __fmul_rn(e2[2], e2[2]));
    out[j] = (double)sqrtf(sm);                        // movement
    out[n + j] = (double)sqrtf(s1);                    // original error
    out[2 * n + j] = (double)sqrtf(s2);                // moved error
    out[3 * n + j] = (double)s1;                       // squared original error
    out[4 * n + j] = (double)s2;                       // squared moved error
}

// measureRelativeMapErrors, one mesh neighbour (i, j) of a keyframe pair: ||(pi2 - pj2) - (pi1 - pj1)||^2
// and ||(Rg pi2 - t - pi1) + (Rg pj2 - t - pj1)||^2 (Rg, t: the pair's global transformation)
__global__ void k_rel_terms(int n, const int32_t *__restrict__ ij, const double *__restrict__ p1,
                            const double *__restrict__ p2, const double *__restrict__ Rt, double *__restrict__ out) {
    int k = TID;
    if (k >= n) return;
    const int i = ij[2 * k], j = ij[2 * k + 1];
    double rel = 0, glob = 0;
    double gi[3], gj[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double d1 = p1[3 * i + r] - p1[3 * j + r], d2 = p2[3 * i + r] - p2[3 * j + r];
        const double diff = d2 - d1;
        rel += diff * diff;
        gi[r] = Rt[3 * r] * p2[3 * i] + Rt[3 * r + 1] * p2[3 * i + 1] + Rt[3 * r + 2] * p2[3 * i + 2];
        gj[r] = Rt[3 * r] * p2[3 * j] + Rt[3 * r + 1] * p2[3 * j + 1] + Rt[3 * r + 2] * p2[3 * j + 2];
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double v = ((gi[r] - Rt[9 + r]) - p1[3 * i + r]) + ((gj[r] - Rt[9 + r]) - p1[3 * j + r]);
        glob += v * v;
    }
    out[k] = rel;
    out[n + k] = glob;
}

// depth term of one matched slot: (d1 - z1 s1)^2 + (d2 - z2 s2)^2, z = (T_cw p)_z (g2o SE3Quat::map)
__global__ void k_depth_terms(int n, const float *__restrict__ pw, const double *__restrict__ dm,
                              const double *__restrict__ cam, double s1, double s2, double *__restrict__ out) {
    int k = TID;
    if (k >= n) return;
    double t = 0;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const double *R = cam + 12 * c;
        const double x = pw[6 * k + 3 * c], y = pw[6 * k + 3 * c + 1], z = pw[6 * k + 3 * c + 2];
        const double zc = R[6] * x + R[7] * y + R[8] * z + R[11];
        const double e = dm[2 * k + c] - zc * (c == 0 ? s1 : s2);
        t += e * e;
    }
    out[k] = t;
}

}  // namespace dev

namespace {

static inline unsigned nblk(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// fixed-order sums of `cnt` consecutive arrays of n doubles (device) -> host
int sums(const double *d_terms, int64_t n, int cnt, double *part, double *d_out, double *h_out, hipStream_t st) {
    for (int c = 0; c < cnt; c++) launch_sum(n, d_terms + c * n, nullptr, 0, 0, part, 256, d_out + c, st);
    if (hipMemcpyAsync(h_out, d_out, sizeof(double) * cnt, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

void quat_to_R(const double *q, double *R) {     // unit quaternion (x y z w) -> row-major R
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

}  // namespace
}  // namespace deftri

using namespace deftri;

// device scratch of one measurement call (freed before returning)
struct Scratch {
    std::vector<void *> p;
    ~Scratch() { for (void *q : p) hipFree(q); }
    template <class T>
    T *put(const std::vector<T> &v) {
        void *d = nullptr;
        if (hipMalloc(&d, sizeof(T) * std::max<size_t>(v.size(), 1)) != hipSuccess) return nullptr;
        p.push_back(d);
        if (!v.empty()) hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice);
        return (T *)d;
    }
    double *alloc(size_t n) {
        void *d = nullptr;
        if (hipMalloc(&d, sizeof(double) * std::max<size_t>(n, 1)) != hipSuccess) return nullptr;
        p.push_back(d);
        return (double *)d;
    }
};

extern "C" int deftri_measure_sim_absolute_map_errors(int32_t device, const deftri_map *map, int32_t n_points,
                                                      const float *original, const float *moved,
                                                      deftri_abs_errors *out) {
    if (!map || !out || n_points < 0 || (n_points > 0 && (!original || !moved)) || map->n_keyframes < 0)
        return DEFTRI_E_ARG;
    std::memset(out, 0, sizeof(*out));
    // Map::getMapPoints(): every MapPoint held by a keyframe slot, by id
    std::vector<std::pair<int64_t, const float *>> mps;
    for (int k = 0; k < map->n_keyframes; k++) {
        const deftri_keyframe &kf = map->keyframes[k];
        for (int s = 0; s < kf.n_slots; s++)
            if (kf.point_id[s] >= 0) mps.emplace_back(kf.point_id[s], kf.point_pos + 3 * (int64_t)s);
    }
    std::sort(mps.begin(), mps.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    mps.erase(std::unique(mps.begin(), mps.end(), [](const auto &a, const auto &b) { return a.first == b.first; }),
              mps.end());
    const int64_t point_count = (int64_t)mps.size();
    const int64_t pairs = point_count / 2;          // j < mapPoints.size() / 2, points i = 2j and 2j + 1 by id
    out->point_count = point_count;
    if (point_count == 0) return 0;
    if (pairs > n_points) return DEFTRI_E_ARG;
    auto by_id = [&](int64_t id) -> const float * {
        auto it = std::lower_bound(mps.begin(), mps.end(), id, [](const auto &a, int64_t v) { return a.first < v; });
        return (it != mps.end() && it->first == id) ? it->second : nullptr;
    };
    std::vector<float> o1(3 * pairs), o2(3 * pairs), og(3 * pairs), mv(3 * pairs);
    for (int64_t j = 0; j < pairs; j++) {
        const float *a = by_id(2 * j), *b = by_id(2 * j + 1);
        if (!a || !b) return DEFTRI_E_ARG;              // the reference dereferences them unchecked
        for (int c = 0; c < 3; c++) {
            o1[3 * j + c] = a[c]; o2[3 * j + c] = b[c];
            og[3 * j + c] = original[3 * j + c]; mv[3 * j + c] = moved[3 * j + c];
        }
    }
    if (hipSetDevice(device) != hipSuccess) return DEFTRI_E_NODEVICE;
    Scratch sc;
    hipStream_t st = nullptr;
    const float *d1 = sc.put(o1), *d2 = sc.put(o2), *dg = sc.put(og), *dm = sc.put(mv);
    double *terms = sc.alloc(5 * (size_t)pairs), *part = sc.alloc(256), *dout = sc.alloc(8);
    if (!d1 || !d2 || !dg || !dm || !terms || !part || !dout) return DEFTRI_E_HIP;
    if (pairs > 0)
        hipLaunchKernelGGL(dev::k_abs_terms, dim3(nblk(pairs, 256)), dim3(256), 0, st, (int)pairs, d1, d2, dg, dm, terms);
    double s[5] = {0, 0, 0, 0, 0};
    if (sums(terms, pairs, 5, part, dout, s, st)) return DEFTRI_E_HIP;
    // Deviation (documented): the reference accumulates these sums in float, one point at
    // a time (Measurements.cc:17-53); here the per-point terms are summed in fp64 in a fixed order and
    // only the totals are cast to float before the reference's float divisions (:65-79) — a closer
    // sum, equal to the float one to its rounding at test sizes.  point_count_in_kf = size / 2.0 -> int
    const float tm = (float)s[0], te1 = (float)s[1], te2 = (float)s[2];
    const float te = (float)(s[1] + s[2]), tsq = (float)(s[3] + s[4]);
    const int in_kf = (int)(point_count / 2.0);
    out->average_movement = (double)(tm / in_kf) * 1000;
    out->average_error_original = (double)(te1 / in_kf) * 1000;
    out->average_error_moved = (double)(te2 / in_kf) * 1000;
    out->average_error = (double)(te / (float)point_count) * 1000;
    out->rmse = (double)std::sqrt(tsq / (float)point_count) * 1000;
    return 0;
}

extern "C" int deftri_measure_relative_map_errors(int32_t device, const deftri_map *map, deftri_rel_errors *out,
                                                  int32_t max_pairs, int32_t *n_pairs) {
    if (!map || !n_pairs || map->n_keyframes < 0 || (max_pairs > 0 && !out)) return DEFTRI_E_ARG;
    *n_pairs = 0;
    const int K = map->n_keyframes;
    if (hipSetDevice(device) != hipSuccess) return DEFTRI_E_NODEVICE;
    hipStream_t st = nullptr;
    // accumulators carried across the pairs, as in the reference
    double depthError = 0, globalT = 0, meanSq = 0;
    int64_t validPairs = 0, nMatches = 0;
    for (int a = 0; a < K; a++)
        for (int b = a + 1; b < K; b++) {
            const deftri_keyframe &kf1 = map->keyframes[b], &kf2 = map->keyframes[a];
            // getGlobalKeyFramesTransformation(k2->first, k1->first): table entry or identity
            double tq[7] = {0, 0, 0, 1, 0, 0, 0};
            for (int32_t e = 0; e < map->n_global; e++)
                if (map->globals[e].kf1 == kf1.id && map->globals[e].kf2 == kf2.id) {
                    for (int i = 0; i < 7; i++) tq[i] = map->globals[e].t[i];
                    break;
                }
            // Rs_global = so3().matrix() and Ts in fp32, cast to double
            double Rt[12];
            {
                float q[4] = {(float)tq[0], (float)tq[1], (float)tq[2], (float)tq[3]};
                float x = q[0], y = q[1], z = q[2], w = q[3];
                float tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
                float txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
                float R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                              txz - twy, tyz + twx, 1 - (txx + tyy)};
                for (int i = 0; i < 9; i++) Rt[i] = (double)R[i];
                for (int i = 0; i < 3; i++) Rt[9 + i] = (double)(float)tq[4 + i];
            }
            const double s1 = kf1.depth_scale, s2 = kf2.depth_scale;
            // extractPositions
            std::vector<double> v1, v2;
            for (int s = 0; s < kf1.n_slots; s++)
                if (kf1.point_id[s] >= 0) for (int c = 0; c < 3; c++) v1.push_back((double)kf1.point_pos[3 * s + c]);
            for (int s = 0; s < kf2.n_slots; s++)
                if (kf2.point_id[s] >= 0) for (int c = 0; c < 3; c++) v2.push_back((double)kf2.point_pos[3 * s + c]);
            const int n1 = (int)v1.size() / 3, n2 = (int)v2.size() / 3;
            std::vector<std::vector<int32_t>> adj;
            std::vector<int32_t> posIdx;
            double area = 0;
            std::string err;
            if (!mesh_adjacency(v1, n1, adj, posIdx, area, err)) return DEFTRI_E_GRAPH;
            std::vector<int32_t> inv(n1, -1);                 // invertedPosIndexes
            for (int v = 0; v < n1; v++) inv[posIdx[v]] = v;
            // camera poses (g2o SE3Quat from the fp32 unit quaternion): rows of R, t
            std::vector<double> cam(24);
            const deftri_keyframe *ks[2] = {&kf1, &kf2};
            for (int c = 0; c < 2; c++) {
                double qn[4], n = 0;
                for (int i = 0; i < 4; i++) { qn[i] = ks[c]->pose[i]; n += qn[i] * qn[i]; }
                n = std::sqrt(n);
                for (int i = 0; i < 4; i++) qn[i] /= n;
                quat_to_R(qn, &cam[12 * c]);
                for (int i = 0; i < 3; i++) cam[12 * c + 9 + i] = ks[c]->pose[4 + i];
            }
            std::vector<float> dpw;
            std::vector<double> dm;
            std::vector<int32_t> ij;
            int64_t pairMatches = 0, pairValid = 0;
            const int ns = std::min(kf1.n_slots, kf2.n_slots);
            for (int i = 0; i < ns; i++) {
                if (kf1.point_id[i] < 0 || kf2.point_id[i] < 0) continue;
                const int idx1 = kf1.obs_index[i], idx2 = kf2.obs_index[i];
                if (idx1 < 0 || idx2 < 0) continue;
                if (idx1 >= kf1.n_obs || idx2 >= kf2.n_obs) return DEFTRI_E_ARG;
                for (int c = 0; c < 3; c++) dpw.push_back(kf1.point_pos[3 * i + c]);
                for (int c = 0; c < 3; c++) dpw.push_back(kf2.point_pos[3 * i + c]);
                // getDepthMeasure(u, v, false) reads a depth image the simulation never sets (it throws
                // there): the per-index simulated depth, as the solver's depth edges
                dm.push_back((double)kf1.depth[idx1]);
                dm.push_back((double)kf2.depth[idx2]);
                if (i >= n1 || inv[i] < 0) continue;             // slot i used as a position index
                const int meshIndex = inv[i];
                if (adj[meshIndex].empty()) continue;
                for (int j : adj[meshIndex]) {
                    const int pj = posIdx[j];
                    if (i >= n2 || pj >= n2) continue;
                    ij.push_back(i); ij.push_back(pj);
                    pairValid++;
                }
                pairMatches++;
            }
            const int64_t nr = (int64_t)ij.size() / 2, nd = (int64_t)dm.size() / 2;
            Scratch sc;
            const int32_t *d_ij = sc.put(ij);
            const double *d_p1 = sc.put(v1), *d_p2 = sc.put(v2), *d_Rt = sc.put(std::vector<double>(Rt, Rt + 12));
            const float *d_pw = sc.put(dpw);
            const double *d_dm = sc.put(dm), *d_cam = sc.put(cam);
            double *rel = sc.alloc(2 * (size_t)nr), *dep = sc.alloc((size_t)nd), *part = sc.alloc(256), *dout = sc.alloc(4);
            if (!d_ij || !d_p1 || !d_p2 || !d_Rt || !d_pw || !d_dm || !d_cam || !rel || !dep || !part || !dout)
                return DEFTRI_E_HIP;
            if (nr > 0)
                hipLaunchKernelGGL(dev::k_rel_terms, dim3(nblk(nr, 256)), dim3(256), 0, st, (int)nr, d_ij, d_p1, d_p2, d_Rt, rel);
            if (nd > 0)
                hipLaunchKernelGGL(dev::k_depth_terms, dim3(nblk(nd, 256)), dim3(256), 0, st, (int)nd, d_pw, d_dm, d_cam, s1,
                                   s2, dep);
            double sr[2] = {0, 0}, sd = 0;
            if (sums(rel, nr, 2, part, dout, sr, st) || sums(dep, nd, 1, part, dout + 2, &sd, st)) return DEFTRI_E_HIP;
            depthError += sd;
            meanSq += sr[0];
            globalT += sr[1];
            validPairs += pairValid;
            nMatches += pairMatches;
            if (*n_pairs < max_pairs) {
                deftri_rel_errors &o = out[*n_pairs];
                o.kf1 = kf1.id; o.kf2 = kf2.id;
                o.reported = validPairs > 1 ? 1 : 0;          // the reference prints only then
                o.rel_error = meanSq / area;
                o.depth_error = depthError;
                o.global_t_error = globalT / area;
                o.area = area;
                o.valid_pairs = validPairs;
                o.n_matches = nMatches;
            }
            (*n_pairs)++;
        }
    return 0;
}
