// graph_builder.cpp — host construction of the non-rigid BA graph, following the reference's
// arapOptimization graph build (Modules/Optimization/g2oBundleAdjustment.cc:640-953) and helpers
// in Modules/Utils/Geometry.cc:
//   extractPositions        :258-270  (drops null slots -> compacted "positions")
//   ComputeEdgeWeightsCot   :272-298  (mean of a.b/|a x b| over opposite vertices, clamped >= 0)
//   createVectorMap         :300-315  (vertex -> first position with isApprox(1e-6))
//   ComputeDelaunay...3D    :317-368  (lower-Delaunay triangles of (x, y); T = facets.count())
//   computeR                :549-604  (per-vertex Procrustes R_i = V U^T with det fix)
// and Open3D's TriangleMesh ComputeAdjacencyList / GetEdgeToVerticesMap / GetSurfaceArea.
// O(n log n) replacements for the reference's O(n^2) createVectorMap / getInvUncertainty loops;
// the getInvUncertainty result is unused by the reference (:887) and is not computed.
// Index semantics kept bit-for-bit, including the slot-vs-position quirk:
//   i = invertedPosIndexes[mpIndex]  (slot used as a position index)
//   neighbour slot = posIndexes[j]   (position index used as a slot index)
#include "graph_builder.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <numeric>
#include <unordered_map>

#include "delaunay.h"

namespace deftri {

namespace {

// Eigen::JacobiSVD<Matrix3d>(S, ComputeFullU | ComputeFullV) restated (two-sided Jacobi with
// real_2x2_jacobi_svd + JacobiRotation::makeJacobi, precision 2*eps, then sign fix and a
// descending selection sort) — computeR (Geometry.cc:590) decomposes with it, and for
// rank-deficient S_i the rotation depends on exactly these steps.
struct Rot { double c, s; };
inline void rot_left(double *M, int p, int q, Rot j) {     // M.applyOnTheLeft(p, q, j)
    for (int i = 0; i < 3; i++) {
        double x = M[3 * p + i], y = M[3 * q + i];
        M[3 * p + i] = j.c * x + j.s * y;
        M[3 * q + i] = -j.s * x + j.c * y;
    }
}
inline void rot_right(double *M, int p, int q, Rot j) {    // M.applyOnTheRight(p, q, j)
    Rot t{j.c, -j.s};
    for (int i = 0; i < 3; i++) {
        double x = M[3 * i + p], y = M[3 * i + q];
        M[3 * i + p] = t.c * x + t.s * y;
        M[3 * i + q] = -t.s * x + t.c * y;
    }
}
void eigen_jacobi_svd3(const double Min[9], double U[9], double sv[3], double V[9]) {
    const double precision = 2.0 * std::numeric_limits<double>::epsilon();
    const double considerAsZero = std::numeric_limits<double>::min();
    double scale = 0;
    for (int i = 0; i < 9; i++) scale = std::max(scale, std::fabs(Min[i]));
    if (scale == 0.0) scale = 1.0;
    double W[9];
    for (int i = 0; i < 9; i++) W[i] = Min[i] / scale;
    for (int i = 0; i < 9; i++) U[i] = V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    double maxDiag = std::max(std::fabs(W[0]), std::max(std::fabs(W[4]), std::fabs(W[8])));
    bool finished = false;
    int guard = 0;
    while (!finished && guard++ < 1000) {
        finished = true;
        for (int p = 1; p < 3; p++)
            for (int q = 0; q < p; q++) {
                double threshold = std::max(considerAsZero, precision * maxDiag);
                if (std::fabs(W[3 * p + q]) > threshold || std::fabs(W[3 * q + p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd(W, p, q)
                    double m00 = W[3 * p + p], m01 = W[3 * p + q], m10 = W[3 * q + p], m11 = W[3 * q + q];
                    Rot rot1;
                    double t = m00 + m11, d = m10 - m01;
                    if (std::fabs(d) < std::numeric_limits<double>::min()) { rot1.s = 0; rot1.c = 1; }
                    else {
                        double u = t / d, tmp = std::sqrt(1.0 + u * u);
                        rot1.s = 1.0 / tmp; rot1.c = u / tmp;
                    }
                    // m.applyOnTheLeft(0, 1, rot1)
                    double a0 = rot1.c * m00 + rot1.s * m10, a1 = rot1.c * m01 + rot1.s * m11;
                    double b0 = -rot1.s * m00 + rot1.c * m10, b1 = -rot1.s * m01 + rot1.c * m11;
                    m00 = a0; m01 = a1; m10 = b0; m11 = b1;
                    // j_right.makeJacobi(m, 0, 1): x = m00, y = m01, z = m11
                    Rot jr;
                    double deno = 2.0 * std::fabs(m01);
                    if (deno < std::numeric_limits<double>::min()) { jr.c = 1; jr.s = 0; }
                    else {
                        double tau = (m00 - m11) / deno;
                        double w = std::sqrt(tau * tau + 1.0);
                        double tt = tau > 0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
                        double sign_t = tt > 0 ? 1.0 : -1.0;
                        double n = 1.0 / std::sqrt(tt * tt + 1.0);
                        jr.s = -sign_t * (m01 / std::fabs(m01)) * std::fabs(tt) * n;
                        jr.c = n;
                    }
                    // j_left = rot1 * j_right.transpose()
                    Rot jrt{jr.c, -jr.s};
                    Rot jl{rot1.c * jrt.c - rot1.s * jrt.s, rot1.c * jrt.s + rot1.s * jrt.c};
                    rot_left(W, p, q, jl);
                    rot_right(U, p, q, Rot{jl.c, -jl.s});
                    rot_right(W, p, q, jr);
                    rot_right(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(std::fabs(W[3 * p + p]), std::fabs(W[3 * q + q])));
                }
            }
    }
    for (int i = 0; i < 3; i++) {
        double a = W[3 * i + i];
        sv[i] = std::fabs(a);
        if (a < 0) for (int r = 0; r < 3; r++) U[3 * r + i] = -U[3 * r + i];
    }
    for (int i = 0; i < 3; i++) sv[i] *= scale;
    for (int i = 0; i < 3; i++) {
        int pos = i;
        double mx = sv[i];
        for (int k = i + 1; k < 3; k++) if (sv[k] > mx) { mx = sv[k]; pos = k; }
        if (mx == 0.0) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int r = 0; r < 3; r++) { std::swap(U[3 * r + i], U[3 * r + pos]); std::swap(V[3 * r + i], V[3 * r + pos]); }
        }
    }
}

double det3(const double M[9]) {     // Eigen determinant_impl<3>
    auto h = [&](int a, int b, int c) { return M[a] * (M[3 + b] * M[6 + c] - M[3 + c] * M[6 + b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

void quat_from_mat(const double m[9], double q[4]) {   // Eigen Quaternion(Matrix3), x y z w
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t; q[1] = (m[2] - m[6]) * t; q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}

void mat_from_quat(const double q[4], double R[9]) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    double twx = tx * w, twy = ty * w, twz = tz * w;
    double txx = tx * x, txy = ty * x, txz = tz * x;
    double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// createVectorMap(vertices = pos, positions = pos, 1e-6): vertex k -> first position p with
// (v_k - p).squaredNorm() <= 1e-12 * min(|v_k|^2, |p|^2)   (Eigen isApprox)
std::vector<int32_t> vector_map(const std::vector<double> &pos, int n) {
    std::vector<int32_t> out(n);
    std::iota(out.begin(), out.end(), 0);
    std::vector<int32_t> byx(n);
    std::iota(byx.begin(), byx.end(), 0);
    std::sort(byx.begin(), byx.end(), [&](int a, int b) { return pos[3 * a] < pos[3 * b] || (pos[3 * a] == pos[3 * b] && a < b); });
    std::vector<int32_t> rank(n);
    for (int i = 0; i < n; i++) rank[byx[i]] = i;
    const double prec2 = 1e-12;
    for (int k = 0; k < n; k++) {
        const double *v = &pos[3 * k];
        double nk = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        double rad = std::sqrt(prec2 * nk);
        int best = k;
        for (int dir = -1; dir <= 1; dir += 2) {
            for (int r = rank[k] + dir; r >= 0 && r < n; r += dir) {
                int p = byx[r];
                if (std::fabs(pos[3 * p] - v[0]) > rad) break;
                if (p >= best) continue;
                const double *w = &pos[3 * p];
                double dx = v[0] - w[0], dy = v[1] - w[1], dz = v[2] - w[2];
                double np = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
                if (dx * dx + dy * dy + dz * dz <= prec2 * std::min(nk, np)) best = p;
            }
        }
        out[k] = best;
    }
    return out;
}

struct Mesh {
    std::vector<int32_t> tris;
    std::vector<std::vector<int32_t>> adj;    // sorted
    std::unordered_map<uint64_t, double> w;   // ordered edge -> cot weight
    double area = 0;
    int T = 0, hull = 0;
};

inline uint64_t ekey(int a, int b) { int lo = std::min(a, b), hi = std::max(a, b); return ((uint64_t)lo << 32) | (uint32_t)hi; }

bool build_mesh(const std::vector<double> &pos, int n, Mesh &M, std::string &err) {
    if (n < 3) { err = "Not enough points to create a triangular mesh."; return false; }
    std::vector<double> xy(2 * (size_t)n);
    for (int i = 0; i < n; i++) { xy[2 * i] = pos[3 * i]; xy[2 * i + 1] = pos[3 * i + 1]; }
    int skipped = 0;
    if (!delaunay2d(xy.data(), n, M.tris, M.hull, skipped)) { err = "Delaunay triangulation failed (collinear input)"; return false; }
    int ntri = (int)M.tris.size() / 3;
    M.T = ntri + std::max(0, M.hull - 2);       // qhull facets.count(): lower + upper Delaunay facets
    M.adj.assign(n, {});
    std::vector<std::pair<uint64_t, int32_t>> e2v;
    e2v.reserve(3 * (size_t)ntri);
    for (int t = 0; t < ntri; t++) {
        int a = M.tris[3 * t], b = M.tris[3 * t + 1], c = M.tris[3 * t + 2];
        M.adj[a].push_back(b); M.adj[a].push_back(c);
        M.adj[b].push_back(a); M.adj[b].push_back(c);
        M.adj[c].push_back(a); M.adj[c].push_back(b);
        e2v.emplace_back(ekey(a, b), c);
        e2v.emplace_back(ekey(b, c), a);
        e2v.emplace_back(ekey(c, a), b);
        const double *p0 = &pos[3 * a], *p1 = &pos[3 * b], *p2 = &pos[3 * c];
        double x[3] = {p0[0] - p1[0], p0[1] - p1[1], p0[2] - p1[2]};
        double y[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};
        double cr[3] = {x[1] * y[2] - x[2] * y[1], x[2] * y[0] - x[0] * y[2], x[0] * y[1] - x[1] * y[0]};
        M.area += 0.5 * std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    }
    for (auto &a : M.adj) { std::sort(a.begin(), a.end()); a.erase(std::unique(a.begin(), a.end()), a.end()); }
    std::stable_sort(e2v.begin(), e2v.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    M.w.reserve(e2v.size());
    for (size_t i = 0; i < e2v.size();) {
        size_t j = i;
        double sum = 0;
        int cnt = 0;
        int e0 = (int)(e2v[i].first >> 32), e1 = (int)(e2v[i].first & 0xFFFFFFFFu);
        while (j < e2v.size() && e2v[j].first == e2v[i].first) {
            int v2 = e2v[j].second;
            const double *A = &pos[3 * e0], *B = &pos[3 * e1], *V = &pos[3 * v2];
            double a[3] = {A[0] - V[0], A[1] - V[1], A[2] - V[2]};
            double b[3] = {B[0] - V[0], B[1] - V[1], B[2] - V[2]};
            double cr[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
            sum += (a[0] * b[0] + a[1] * b[1] + a[2] * b[2]) / std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
            cnt++;
            j++;
        }
        double wt = cnt > 0 ? sum / cnt : 0;
        M.w[e2v[i].first] = wt < 0.0 ? 0.0 : wt;
        i = j;
    }
    return true;
}

}  // namespace

bool mesh_adjacency(const std::vector<double> &pos, int n, std::vector<std::vector<int32_t>> &adj,
                    std::vector<int32_t> &pos_index, double &area, std::string &err) {
    Mesh M;
    if (!build_mesh(pos, n, M, err)) return false;
    adj = std::move(M.adj);
    area = M.area;
    pos_index = vector_map(pos, n);
    return true;
}

void procrustes_rotation(const double S[9], double R[9]) {
    double U[9], s[3], V[9];
    eigen_jacobi_svd3(S, U, s, V);
    auto vut = [&](double *O) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) O[3 * i + j] = V[3 * i] * U[3 * j] + V[3 * i + 1] * U[3 * j + 1] + V[3 * i + 2] * U[3 * j + 2];
    };
    vut(R);
    if (det3(R) < 0) {
        for (int i = 0; i < 3; i++) U[3 * i + 2] *= -1;
        vut(R);
    }
    double q[4];
    quat_from_mat(R, q);                  // Sophus::SO3d keeps the unit quaternion
    mat_from_quat(q, R);
}

bool build_arap_graph(const deftri_map &map, double rep_weight, double arap_weight, float depth_error,
                      GraphResult &g, std::string &err, int pair_window) {
    g = GraphResult();
    int K = map.n_keyframes;
    if (K < 0 || (K > 0 && !map.keyframes)) { err = "bad map"; return false; }
    std::vector<int32_t> cam_of(K, -1);
    std::unordered_map<int64_t, int32_t> pidx;
    auto cam_index = [&](int k) {
        if (cam_of[k] < 0) {
            cam_of[k] = (int32_t)(g.cam_pose.size() / 7);
            const deftri_keyframe &kf = map.keyframes[k];
            for (int i = 0; i < 7; i++) g.cam_pose.push_back(kf.pose[i]);
            for (int i = 0; i < 8; i++) g.cam_kb8.push_back(kf.kb8[i]);
        }
        return cam_of[k];
    };
    g.kf_scale.assign(K, -1);
    const double info_dep = 1.0 / ((double)depth_error * (double)depth_error);
    int32_t rot_base = 0;
    for (int a = 0; a < K; a++) {
        for (int b = a + 1; b < K; b++) {
            if (pair_window > 0 && b - a > pair_window) continue;
            const deftri_keyframe &kf1 = map.keyframes[b];   // pKF1 = k2->second
            const deftri_keyframe &kf2 = map.keyframes[a];   // pKF2 = k1->second
            int32_t q = (int32_t)g.pair_area.size();
            // extractPositions
            std::vector<double> pos1, pos2;
            for (int s = 0; s < kf1.n_slots; s++)
                if (kf1.point_id[s] >= 0)
                    for (int k = 0; k < 3; k++) pos1.push_back((double)kf1.point_pos[3 * s + k]);
            for (int s = 0; s < kf2.n_slots; s++)
                if (kf2.point_id[s] >= 0)
                    for (int k = 0; k < 3; k++) pos2.push_back((double)kf2.point_pos[3 * s + k]);
            int n1 = (int)pos1.size() / 3, n2 = (int)pos2.size() / 3;
            static const bool timing = std::getenv("DEFTRI_GRAPH_TIMING") != nullptr;
            auto tnow = [] { return std::chrono::steady_clock::now(); };
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            auto t0 = tnow();
            Mesh M;
            if (!build_mesh(pos1, n1, M, err)) return false;
            auto t1 = tnow();
            // T_global: map transformation for (kf1, kf2) or identity (:664-677)
            // getGlobalKeyFramesTransformation(k2->first, k1->first) = (kf1.id, kf2.id): the table
            // entry for that ordered pair, a default (identity) SE3f when absent (Map.cc:332-343)
            double Tg[7] = {0, 0, 0, 1, 0, 0, 0};
            if (map.n_global > 0) {
                for (int32_t e = 0; e < map.n_global; e++)
                    if (map.globals[e].kf1 == kf1.id && map.globals[e].kf2 == kf2.id) {
                        for (int i = 0; i < 7; i++) Tg[i] = map.globals[e].t[i];
                        break;
                    }
            } else if (a == 0 && b == 1) {
                for (int i = 0; i < 7; i++) Tg[i] = map.global_t[i];
            }
            {
                float tn = std::sqrt((float)Tg[4] * (float)Tg[4] + (float)Tg[5] * (float)Tg[5] + (float)Tg[6] * (float)Tg[6]);
                double qn = std::sqrt(Tg[0] * Tg[0] + Tg[1] * Tg[1] + Tg[2] * Tg[2] + Tg[3] * Tg[3]);
                bool rot_id = qn > 0 && std::fabs(std::fabs(Tg[3] / qn) - 1.0) < 1e-10;
                if (tn == 0.0f && rot_id) { Tg[0] = Tg[1] = Tg[2] = 0; Tg[3] = 1; Tg[4] = Tg[5] = Tg[6] = 0; }
            }
            std::vector<int32_t> posIdx = vector_map(pos1, n1);
            std::unordered_map<int32_t, int32_t> inv;
            for (int v = 0; v < n1; v++) inv[posIdx[v]] = v;
            auto t2 = tnow();
            // computeR
            std::vector<double> Rs(9 * (size_t)n1, 0.0);
            for (int v = 0; v < n1; v++) { Rs[9 * v] = Rs[9 * v + 4] = Rs[9 * v + 8] = 1.0; }
            for (int p = 0; p < n1; p++) {
                auto it = inv.find(p);
                if (it == inv.end()) continue;
                int i = it->second;
                double S[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (int j : M.adj[i]) {
                    double wt = M.w[ekey(i, j)];
                    int pi = posIdx[i], pj = posIdx[j];
                    if (pi >= n2 || pj >= n2) continue;
                    double e1[3], e2[3];
                    for (int k = 0; k < 3; k++) { e1[k] = pos1[3 * pi + k] - pos1[3 * pj + k]; e2[k] = pos2[3 * pi + k] - pos2[3 * pj + k]; }
                    for (int r = 0; r < 3; r++)
                        for (int c = 0; c < 3; c++) S[3 * r + c] += wt * e1[r] * e2[c];
                }
                procrustes_rotation(S, &Rs[9 * i]);
            }
            auto t3 = tnow();
            g.rot.insert(g.rot.end(), Rs.begin(), Rs.end());
            for (int i = 0; i < 7; i++) g.tg.push_back(Tg[i]);
            int32_t s1 = (int32_t)g.scales.size();
            g.scales.push_back(kf1.depth_scale); g.kf_scale[b] = s1;
            int32_t s2 = (int32_t)g.scales.size();
            g.scales.push_back(kf2.depth_scale); g.kf_scale[a] = s2;
            int32_t c1 = cam_index(b), c2 = cam_index(a);
            g.pair_area.push_back(M.area);
            g.pair_info.push_back(arap_weight * std::pow((double)M.T, 2));
            g.pair_kf1.push_back(b); g.pair_kf2.push_back(a);
            g.pair_T.push_back(M.T); g.pair_hull.push_back(M.hull);
            auto add_point = [&](int64_t id, const float *p, int ord_slot) {
                auto it = pidx.find(id);
                if (it != pidx.end()) return it->second;
                int32_t k = (int32_t)g.point_mpid.size();
                pidx[id] = k;
                g.point_mpid.push_back(id);
                for (int c = 0; c < 3; c++) { g.points.push_back((double)p[c]); g.point_orig.push_back(p[c]); }
                g.order_xy.push_back((double)kf1.point_pos[3 * ord_slot]);
                g.order_xy.push_back((double)kf1.point_pos[3 * ord_slot + 1]);
                return k;
            };
            int nslots = kf1.n_slots;
            for (int mp = 0; mp < nslots; mp++) {
                if (mp >= kf2.n_slots) break;
                int64_t id1 = kf1.point_id[mp], id2 = kf2.point_id[mp];
                if (id1 < 0 || id2 < 0) continue;
                int32_t p1 = add_point(id1, kf1.point_pos + 3 * mp, mp);
                int32_t p2 = add_point(id2, kf2.point_pos + 3 * mp, mp);
                int32_t o1 = kf1.obs_index[mp], o2 = kf2.obs_index[mp];
                if (o1 < 0 || o2 < 0) continue;
                if (o1 >= kf1.n_obs || o2 >= kf2.n_obs) { err = "observation index out of range"; return false; }
                // reprojection edges (:765-812)
                g.rep_point.push_back(p1); g.rep_cam.push_back(c1);
                g.rep_obs.push_back((double)kf1.kp_uv[2 * o1]); g.rep_obs.push_back((double)kf1.kp_uv[2 * o1 + 1]);
                g.rep_info.push_back((double)kf1.inv_sigma2[kf1.kp_octave[o1]] * rep_weight);
                g.rep_point.push_back(p2); g.rep_cam.push_back(c2);
                g.rep_obs.push_back((double)kf2.kp_uv[2 * o2]); g.rep_obs.push_back((double)kf2.kp_uv[2 * o2 + 1]);
                g.rep_info.push_back((double)kf2.inv_sigma2[kf2.kp_octave[o2]] * rep_weight);
                // depth edges (:816-856), simulated per-index depth
                g.dep_point.push_back(p1); g.dep_scale.push_back(s1); g.dep_cam.push_back(c1);
                g.dep_meas.push_back((double)kf1.depth[o1]); g.dep_info.push_back(info_dep);
                g.dep_point.push_back(p2); g.dep_scale.push_back(s2); g.dep_cam.push_back(c2);
                g.dep_meas.push_back((double)kf2.depth[o2]); g.dep_info.push_back(info_dep);
                // ARAP edges (:871-953)
                auto it = inv.find(mp);
                if (it == inv.end()) continue;
                int i = it->second;
                if (M.adj[i].empty()) continue;
                for (int j : M.adj[i]) {
                    int slot = posIdx[j];
                    if (slot >= kf1.n_slots || slot >= kf2.n_slots) continue;
                    int64_t j1 = kf1.point_id[slot], j2 = kf2.point_id[slot];
                    if (j1 < 0 || j2 < 0) continue;
                    int32_t pj1 = add_point(j1, kf1.point_pos + 3 * slot, slot);
                    int32_t pj2 = add_point(j2, kf2.point_pos + 3 * slot, slot);
                    g.arap_pts.push_back(p1); g.arap_pts.push_back(p2);
                    g.arap_pts.push_back(pj1); g.arap_pts.push_back(pj2);
                    g.arap_pair.push_back(q);
                    g.arap_rot.push_back(rot_base + i); g.arap_rot.push_back(rot_base + j);
                    g.arap_w.push_back(M.w[ekey(i, j)]);
                }
            }
            rot_base += n1;
            if (timing)
                std::fprintf(stderr, "[deftri graph] pair %d: mesh %.1f ms, vector map %.1f, computeR %.1f, edges %.1f\n", q,
                             ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, tnow()));
        }
    }
    deftri_problem_desc &d = g.desc;
    d = deftri_problem_desc{};
    d.n_points = (int32_t)g.point_mpid.size();
    d.n_pairs = (int32_t)g.pair_area.size();
    d.n_scales = (int32_t)g.scales.size();
    d.n_cams = (int32_t)(g.cam_pose.size() / 7);
    d.n_rep = (int32_t)g.rep_point.size();
    d.n_depth = (int32_t)g.dep_point.size();
    d.n_arap = (int32_t)g.arap_pair.size();
    d.n_rot = (int32_t)(g.rot.size() / 9);
    d.points = g.points.data(); d.tg = g.tg.data(); d.scales = g.scales.data();
    d.cam_kb8 = g.cam_kb8.data(); d.cam_pose = g.cam_pose.data();
    d.rep_point = g.rep_point.data(); d.rep_cam = g.rep_cam.data(); d.rep_obs = g.rep_obs.data();
    d.rep_info = g.rep_info.data();
    d.huber_delta = (double)(float)std::sqrt(100.991);          // const float deltaMono = sqrt(100.991)
    d.dep_point = g.dep_point.data(); d.dep_scale = g.dep_scale.data(); d.dep_cam = g.dep_cam.data();
    d.dep_meas = g.dep_meas.data(); d.dep_info = g.dep_info.data();
    d.arap_pts = g.arap_pts.data(); d.arap_pair = g.arap_pair.data(); d.arap_rot = g.arap_rot.data();
    d.arap_w = g.arap_w.data(); d.rot = g.rot.data(); d.pair_area = g.pair_area.data(); d.pair_info = g.pair_info.data();
    d.order_xy = g.order_xy.data();
    return true;
}

void writeback_arap(deftri_map &map, const GraphResult &g, const std::vector<double> &points,
                    const std::vector<double> &scales, const std::vector<double> &tg, double *optimization_update) {
    // scales: the last vertex created for each KeyFrame (mKeyFrameId overwrite, :967-972)
    for (int k = 0; k < map.n_keyframes; k++)
        if (g.kf_scale[k] >= 0) map.keyframes[k].depth_scale = scales[g.kf_scale[k]];
    // points: fp32 writeback + sum ||p_old - p_new|| (:974-990)
    std::unordered_map<int64_t, int32_t> pidx;
    pidx.reserve(g.point_mpid.size() * 2);
    for (size_t i = 0; i < g.point_mpid.size(); i++) pidx[g.point_mpid[i]] = (int32_t)i;
    double upd = 0;
    for (size_t i = 0; i < g.point_mpid.size(); i++) {
        float nf[3] = {(float)points[3 * i], (float)points[3 * i + 1], (float)points[3 * i + 2]};
        float dx = g.point_orig[3 * i] - nf[0], dy = g.point_orig[3 * i + 1] - nf[1], dz = g.point_orig[3 * i + 2] - nf[2];
        upd += (double)std::sqrt(dx * dx + dy * dy + dz * dz);
    }
    for (int k = 0; k < map.n_keyframes; k++) {
        deftri_keyframe &kf = map.keyframes[k];
        for (int s = 0; s < kf.n_slots; s++) {
            if (kf.point_id[s] < 0) continue;
            auto it = pidx.find(kf.point_id[s]);
            if (it == pidx.end()) continue;
            for (int c = 0; c < 3; c++) kf.point_pos[3 * s + c] = (float)points[3 * (size_t)it->second + c];
        }
    }
    if (optimization_update) *optimization_update = upd;
    // global transformation of the last pair (insertGlobalKeyFramesTransformation(0, 1, T), :999-1007)
    if (!g.pair_area.empty()) {
        size_t q = g.pair_area.size() - 1;
        for (int i = 0; i < 7; i++) map.global_t[i] = tg[7 * q + i];
    }
}

}  // namespace deftri
