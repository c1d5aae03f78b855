// device_math.h — SE3Quat / quaternion / Kannala–Brandt8 math shared by the gfx950 kernels.
//
// Formulas restate (for parity):
//   g2o SE3Quat::map / exp / operator* / normalizeRotation (types_six_dof_expmap)
//   Eigen QuaternionBase::toRotationMatrix, Quaternion(Matrix3) and _transformVector
//   KannalaBrandt8::project / projectJac (reference Modules/Calibration/KannalaBrandt8.cc:32-49,
//   85-114) — evaluated in fp32 exactly as the reference (it projects p.cast<float>()).
#pragma once
#include <hip/hip_runtime.h>

namespace deftri {
namespace dev {

// The SE3 / quaternion helpers restate the reference's double arithmetic operation for operation:
// no FMA contraction (the reference's x86-64 build has no FMA), so a depth or reprojection error and
// the numeric Jacobians built from it (a difference of two evaluations 2e-9 apart, which amplifies an
// ulp into ~1e-7 of the derivative) carry the reference's bits.

struct Quat { double x, y, z, w; };

__device__ __forceinline__ void quat_normalize_rot(Quat &q) {
#pragma clang fp contract(off)
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

__device__ __forceinline__ void quat_to_mat(const Quat &q, double R[9]) {
#pragma clang fp contract(off)
    double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ Quat quat_from_mat(const double m[9]) {
#pragma clang fp contract(off)
    Quat q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        double c[3];
        t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}

__device__ __forceinline__ void quat_rotate(const Quat &q, const double v[3], double o[3]) {
#pragma clang fp contract(off)
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
    o[0] = v[0] + q.w * uv[0] + c[0];
    o[1] = v[1] + q.w * uv[1] + c[1];
    o[2] = v[2] + q.w * uv[2] + c[2];
}

__device__ __forceinline__ Quat quat_mul(const Quat &a, const Quat &b) {
#pragma clang fp contract(off)
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

struct SE3 { Quat r; double t[3]; };

__device__ __forceinline__ SE3 se3_load(const double *a) {
    SE3 T;
    T.r.x = a[0]; T.r.y = a[1]; T.r.z = a[2]; T.r.w = a[3];
    T.t[0] = a[4]; T.t[1] = a[5]; T.t[2] = a[6];
    return T;
}
__device__ __forceinline__ void se3_store(const SE3 &T, double *a) {
    a[0] = T.r.x; a[1] = T.r.y; a[2] = T.r.z; a[3] = T.r.w;
    a[4] = T.t[0]; a[5] = T.t[1]; a[6] = T.t[2];
}

__device__ __forceinline__ void se3_map(const SE3 &T, const double p[3], double o[3]) {
#pragma clang fp contract(off)
    quat_rotate(T.r, p, o);
    o[0] += T.t[0]; o[1] += T.t[1]; o[2] += T.t[2];
}

// g2o SE3Quat::exp(omega, upsilon)
__device__ __forceinline__ SE3 se3_exp(const double u[6]) {
#pragma clang fp contract(off)
    const double *w = u, *ups = u + 3;
    double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double O2[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double a, b, c, dd;
    if (theta < 0.00001) { a = 1; b = 0.5; c = 0.5; dd = 1.0 / 6.0; }
    else {
        double st = sin(theta), ct = cos(theta);
        a = st / theta;
        b = (1 - ct) / (theta * theta);
        c = b;
        dd = (theta - st) / pow(theta, 3.0);
    }
    double R[9], V[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        double I = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = I + a * O[i] + b * O2[i];
        V[i] = I + c * O[i] + dd * O2[i];
    }
    SE3 T;
    T.r = quat_from_mat(R);
    for (int i = 0; i < 3; i++) T.t[i] = V[3 * i] * ups[0] + V[3 * i + 1] * ups[1] + V[3 * i + 2] * ups[2];
    quat_normalize_rot(T.r);
    return T;
}

// A * B (SE3Quat::operator*)
__device__ __forceinline__ SE3 se3_mul(const SE3 &A, const SE3 &B) {
#pragma clang fp contract(off)
    SE3 r = A;
    double tb[3];
    quat_rotate(A.r, B.t, tb);
    r.t[0] += tb[0]; r.t[1] += tb[1]; r.t[2] += tb[2];
    r.r = quat_mul(A.r, B.r);
    quat_normalize_rot(r.r);
    return r;
}

// ---- Kannala–Brandt 8, fp32 ---------------------------------------------------------------
// fp32 without FMA contraction, like the reference's x86-64 build (no -march): only the ocml vs
// glibc transcendental (atan2f, sinf, cosf) ulp differences remain against the oracle.
__device__ __forceinline__ void kb8_project(const float *k, const float p[3], float uv[2]) {
#pragma clang fp contract(off)
    const float x2_plus_y2 = p[0] * p[0] + p[1] * p[1];
    const float theta = atan2f(sqrtf(x2_plus_y2), p[2]);
    const float psi = atan2f(p[1], p[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + k[4] * theta3 + k[5] * theta5 + k[6] * theta7 + k[7] * theta9;
    uv[0] = k[0] * r * cosf(psi) + k[2];
    uv[1] = k[1] * r * sinf(psi) + k[3];
}

__device__ __forceinline__ void kb8_project_jac(const float *k, const float p[3], float J[6]) {
#pragma clang fp contract(off)
    float x2 = p[0] * p[0], y2 = p[1] * p[1], z2 = p[2] * p[2];
    float r2 = x2 + y2;
    float r = sqrtf(r2);
    float r3 = r2 * r;
    float theta = atan2f(r, p[2]);
    float theta2 = theta * theta, theta3 = theta2 * theta;
    float theta4 = theta2 * theta2, theta5 = theta4 * theta;
    float theta6 = theta2 * theta4, theta7 = theta6 * theta;
    float theta8 = theta4 * theta4, theta9 = theta8 * theta;
    float f = theta + theta3 * k[4] + theta5 * k[5] + theta7 * k[6] + theta9 * k[7];
    float fd = 1 + 3 * k[4] * theta2 + 5 * k[5] * theta4 + 7 * k[6] * theta6 + 9 * k[7] * theta8;
    J[0] = k[0] * (fd * p[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
    J[1] = k[0] * (fd * p[2] * p[1] * p[0] / (r2 * (r2 + z2)) - f * p[1] * p[0] / r3);
    J[2] = -k[0] * fd * p[0] / (r2 + z2);
    J[3] = k[1] * (fd * p[2] * p[1] * p[0] / (r2 * (r2 + z2)) - f * p[1] * p[0] / r3);
    J[4] = k[1] * (fd * p[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
    J[5] = -k[1] * fd * p[1] / (r2 + z2);
}

}  // namespace dev
}  // namespace deftri
