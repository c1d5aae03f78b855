// sim_host.cpp — the reference's simulated observations, on the host (upstream producer, SURVEY
// §8 f4): SLAM::setCameraPoses (Modules/System/SLAM.cc:223-235), getSimulatedDepthMeasurements
// (:321-338) and createKeyPoints (:281-319).
//
// The noise streams are the reference's own: a fresh std::default_random_engine (libstdc++:
// minstd_rand0, seed 1) with std::normal_distribution<float> per function — the same <random>
// implementation the reference links, so the draws are the same numbers in the same order (4 per
// correspondence for the keypoints: x1, y1, x2, y2; 2 for the depths: d1, d2).  The camera poses are
// Sophus::SE3f built from (R, t): the rotation kept as the unit quaternion Eigen computes from the
// matrix (Quaternion(Matrix3) — trace / largest-diagonal branch), points moved by the quaternion
// rotation Sophus applies (uv = 2 q.vec x p; p + w uv + q.vec x uv) plus t.  Sophus and Eigen are
// not in this image, so their arithmetic is restated from their published sources (version
// unpinned: the reference vendors neither).  All float arithmetic, one rounding per operation
// (built with -ffp-contract=off).
#include <cmath>
#include <cstdint>
#include <random>

#include "../../include/deftri.h"

namespace {

struct V3 { float x, y, z; };
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V3 normalized(V3 v) {                       // Eigen: v / sqrt(squaredNorm), squaredNorm = (x^2 + y^2) + z^2
    const float n2 = (v.x * v.x + v.y * v.y) + v.z * v.z;
    if (!(n2 > 0.0f)) return v;
    const float n = std::sqrt(n2);
    return {v.x / n, v.y / n, v.z / n};
}

// SLAM::lookAt (SLAM.cc:340-351), up = UnitY; columns (right, up, forward); R[r][c] row-major
void look_at(V3 cam, V3 target, float R[9]) {
    const V3 f = normalized({target.x - cam.x, target.y - cam.y, target.z - cam.z});
    const V3 r = normalized(cross({0.0f, 1.0f, 0.0f}, f));
    const V3 u = normalized(cross(f, r));
    const V3 cols[3] = {r, u, f};
    for (int c = 0; c < 3; c++) { R[0 * 3 + c] = cols[c].x; R[1 * 3 + c] = cols[c].y; R[2 * 3 + c] = cols[c].z; }
}

// Eigen::Quaternion<float>(Matrix3f) (quaternionbase_assign_impl): q = (x, y, z, w)
void quat_from_matrix(const float m[9], float q[4]) {
    auto M = [&](int r, int c) { return m[r * 3 + c]; };
    float t = (M(0, 0) + M(1, 1)) + M(2, 2);
    if (t > 0.0f) {
        t = std::sqrt(t + 1.0f);
        q[3] = 0.5f * t;
        t = 0.5f / t;
        q[0] = (M(2, 1) - M(1, 2)) * t;
        q[1] = (M(0, 2) - M(2, 0)) * t;
        q[2] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(((M(i, i) - M(j, j)) - M(k, k)) + 1.0f);
        q[i] = 0.5f * t;
        t = 0.5f / t;
        q[3] = (M(k, j) - M(j, k)) * t;
        q[j] = (M(j, i) + M(i, j)) * t;
        q[k] = (M(k, i) + M(i, k)) * t;
    }
}

// Sophus SE3f * p: SO3 (unit quaternion) * p + t
V3 se3_apply(const float q[4], const float t[3], V3 p) {
    const V3 qv = {q[0], q[1], q[2]};
    V3 uv = cross(qv, p);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const V3 c = cross(qv, uv);
    const float w = q[3];
    const V3 r = {(p.x + w * uv.x) + c.x, (p.y + w * uv.y) + c.y, (p.z + w * uv.z) + c.z};
    return {r.x + t[0], r.y + t[1], r.z + t[2]};
}

// KannalaBrandt8::project (KannalaBrandt8.cc:32-49), fp32 with the libm float functions
void kb8_project(const float k[8], V3 p, float &u, float &v) {
    const float x2_plus_y2 = p.x * p.x + p.y * p.y;
    const float theta = atan2f(sqrtf(x2_plus_y2), p.z);
    const float psi = atan2f(p.y, p.x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = (((theta + k[4] * theta3) + k[5] * theta5) + k[6] * theta7) + k[7] * theta9;
    u = k[0] * r * std::cos(psi) + k[2];
    v = k[1] * r * std::sin(psi) + k[3];
}

// Conversions.cc:64-67 roundToDecimals(double, int): round(value * 10^d) / 10^d
double round_to_decimals(double value, int decimals) {
    const double factor = std::pow(10.0, decimals);
    return std::round(value * factor) / factor;
}

}  // namespace

extern "C" int deftri_sim_two_view(int32_t n, const float *orig, const float *moved, const float c1[3],
                                   const float c2[3], const float kb8_1[8], const float kb8_2[8], float rep_error,
                                   int32_t decimals, float depth_error_mm, float depth_scale_1, float depth_scale_2,
                                   float *uv1, float *uv2, float *depth1, float *depth2, float pose1[7],
                                   float pose2[7]) {
    if (n < 0 || (n > 0 && (!orig || !moved || !uv1 || !uv2 || !depth1 || !depth2)) || !c1 || !c2 || !kb8_1 ||
        !kb8_2 || !pose1 || !pose2)
        return DEFTRI_E_ARG;
    // setCameraPoses: T1w = (I, c1), T2w = (lookAt(c2, moved[0]), c2)
    float R1[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, R2[9];
    if (n > 0) look_at({c2[0], c2[1], c2[2]}, {moved[0], moved[1], moved[2]}, R2);
    else for (int i = 0; i < 9; i++) R2[i] = R1[i];
    float q1[4], q2[4];
    quat_from_matrix(R1, q1);
    quat_from_matrix(R2, q2);
    for (int i = 0; i < 4; i++) { pose1[i] = q1[i]; pose2[i] = q2[i]; }
    for (int i = 0; i < 3; i++) { pose1[4 + i] = c1[i]; pose2[4 + i] = c2[i]; }
    // getSimulatedDepthMeasurements
    {
        std::default_random_engine generator;
        std::normal_distribution<float> distribution(0.0f, depth_error_mm / 1000);
        for (int32_t i = 0; i < n; i++) {
            const V3 pc1 = se3_apply(q1, c1, {orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]});
            const V3 pc2 = se3_apply(q2, c2, {moved[3 * i], moved[3 * i + 1], moved[3 * i + 2]});
            const float d1 = pc1.z * depth_scale_1 + distribution(generator);
            const float d2 = pc2.z * depth_scale_2 + distribution(generator);
            depth1[i] = d1;
            depth2[i] = d2;
        }
    }
    // createKeyPoints
    {
        std::default_random_engine generator;
        std::normal_distribution<float> distribution(0.0f, rep_error);
        for (int32_t i = 0; i < n; i++) {
            const V3 pc1 = se3_apply(q1, c1, {orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]});
            const V3 pc2 = se3_apply(q2, c2, {moved[3 * i], moved[3 * i + 1], moved[3 * i + 2]});
            float ox, oy, mx, my;
            kb8_project(kb8_1, pc1, ox, oy);
            kb8_project(kb8_2, pc2, mx, my);
            float e = distribution(generator);
            uv1[2 * i] = (float)round_to_decimals(ox + e, decimals);
            e = distribution(generator);
            uv1[2 * i + 1] = (float)round_to_decimals(oy + e, decimals);
            e = distribution(generator);
            uv2[2 * i] = (float)round_to_decimals(mx + e, decimals);
            e = distribution(generator);
            uv2[2 * i + 1] = (float)round_to_decimals(my + e, decimals);
        }
    }
    return 0;
}

// The raw stream of one fresh std::default_random_engine + std::normal_distribution<float>(mean,
// stddev): n draws (parity tests pin it against a restatement of libstdc++'s algorithm).
extern "C" int deftri_sim_normal_stream(int64_t n, float mean, float stddev, float *out) {
    if (n < 0 || (n > 0 && !out)) return DEFTRI_E_ARG;
    std::default_random_engine generator;
    std::normal_distribution<float> distribution(mean, stddev);
    for (int64_t i = 0; i < n; i++) out[i] = distribution(generator);
    return 0;
}
