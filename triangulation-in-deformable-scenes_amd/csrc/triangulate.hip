// triangulate.hip — the map-point producer in front of the solver, one thread per correspondence
// (SURVEY §8(f) row 4): Mapping::triangulateSimulatedMapPoints (reference
// Modules/Mapping/Mapping.cc:280-349) with the Simulation.yaml settings Triangulation.method
// "NRSLAM" and seed.location "FarPoints":
//   xn = normalize(KannalaBrandt8::unproject(uv))            KannalaBrandt8.cc:51-83 (Newton on theta,
//                                                             10 steps, stop at |fix| < 1e-6)
//   triangulateNRSLAM(xn1, xn2, T1w, T2w, "FarPoints")       Geometry.cc:103-153
//   isValidParallax: both depths >= 0, cos(ray1, ray2) <= minCos   Mapping.cc:351-366
// Everything in fp32 without FMA contraction, as the reference's Eigen/Sophus float code.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace deftri {
namespace dev {

#pragma clang fp contract(off)
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 scl(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float nrm(V3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
__device__ __forceinline__ V3 normalized(V3 a) { const float n = nrm(a); return v3(a.x / n, a.y / n, a.z / n); }
// T = [R | t] row-major 3x4
__device__ __forceinline__ V3 rot(const float *T, V3 p) {
    return v3(T[0] * p.x + T[1] * p.y + T[2] * p.z, T[4] * p.x + T[5] * p.y + T[6] * p.z,
              T[8] * p.x + T[9] * p.y + T[10] * p.z);
}
__device__ __forceinline__ V3 rotT(const float *T, V3 p) {     // R^T p
    return v3(T[0] * p.x + T[4] * p.y + T[8] * p.z, T[1] * p.x + T[5] * p.y + T[9] * p.z,
              T[2] * p.x + T[6] * p.y + T[10] * p.z);
}
__device__ __forceinline__ V3 xform(const float *T, V3 p) { return add(rot(T, p), v3(T[3], T[7], T[11])); }

// KannalaBrandt8::unproject (KannalaBrandt8.cc:51-83)
__device__ __forceinline__ V3 kb8_unproject(const float *k, float u, float v) {
    const float px = (u - k[2]) / k[0], py = (v - k[3]) / k[1];
    const float theta_d = sqrtf(px * px + py * py);
    float th = 0.0f;
    if (theta_d > 1e-8f) {
        float theta = theta_d;
        for (int j = 0; j < 10; j++) {
            const float t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
            const float k0t2 = k[4] * t2, k1t4 = k[5] * t4, k2t6 = k[6] * t6, k3t8 = k[7] * t8;
            const float fix = (theta * (1 + k0t2 + k1t4 + k2t6 + k3t8) - theta_d) /
                              (1 + 3 * k0t2 + 5 * k1t4 + 7 * k2t6 + 9 * k3t8);
            theta = theta - fix;
            if (fabsf(fix) < 1e-6f) break;
        }
        th = theta;
    }
    return v3(sinf(th) * px / theta_d, sinf(th) * py / theta_d, cosf(th));
}

// Tp: T1w, T2w, T21 = T2w T1w^-1, T2w^-1 (3x4 each, formed on the host as Sophus does)
__global__ void k_triangulate_nrslam(int n, const float *__restrict__ uv1, const float *__restrict__ uv2,
                                     const float *__restrict__ kb1, const float *__restrict__ kb2,
                                     const float *__restrict__ Tp, float min_cos, float *__restrict__ x1out,
                                     float *__restrict__ x2out, uint8_t *__restrict__ valid) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const float *T1w = Tp, *T2w = Tp + 12, *T21 = Tp + 24, *T2i = Tp + 36;
    const V3 xn1 = normalized(kb8_unproject(kb1, uv1[2 * i], uv1[2 * i + 1]));   // Mapping.cc:297-298
    const V3 xn2 = normalized(kb8_unproject(kb2, uv2[2 * i], uv2[2 * i + 1]));
    // triangulateNRSLAM (Geometry.cc:103-153), FarPoints
    const V3 f0 = normalized(xn1), f1 = normalized(xn2);
    const V3 t = v3(T21[3], T21[7], T21[11]);
    const V3 Rf0 = rot(T21, f0);
    const V3 p = cross(Rf0, f1), q = cross(Rf0, t), r = cross(f1, t);
    const float pn = nrm(p), qn = nrm(q), rn = nrm(r);
    const float lambda0 = rn / pn, lambda1 = qn / pn;
    V3 point0 = scl(lambda0, Rf0);
    const V3 point1 = scl(lambda1, f1);
    const V3 x1 = scl(qn / (qn + rn), add(t, scl(rn / pn, add(Rf0, f1))));
    point0 = add(t, point0);
    const V3 p3D1 = add(point0, sub(point0, x1));
    const V3 p3D2 = add(point1, sub(point1, x1));
    const V3 X1 = xform(T2i, p3D1), X2 = xform(T2i, p3D2);                    // T2w.inverse() * p
    // isValidParallax (Mapping.cc:351-366)
    const V3 c1 = xform(T1w, X1), c2 = xform(T2w, X2);
    const V3 ray1 = normalized(rotT(T1w, xn1)), ray2 = normalized(rotT(T2w, xn2));
    const float cosp = dot(ray1, ray2) / (nrm(ray1) * nrm(ray2));
    const bool fin = isfinite(X1.x) && isfinite(X1.y) && isfinite(X1.z) && isfinite(X2.x) && isfinite(X2.y) &&
                     isfinite(X2.z);
    valid[i] = (c1.z >= 0.0f && c2.z >= 0.0f && cosp <= min_cos && fin) ? 1 : 0;
    x1out[3 * i] = X1.x; x1out[3 * i + 1] = X1.y; x1out[3 * i + 2] = X1.z;
    x2out[3 * i] = X2.x; x2out[3 * i + 1] = X2.y; x2out[3 * i + 2] = X2.z;
}
#pragma clang fp contract(on)

}  // namespace dev

void launch_triangulate_nrslam(int n, const float *uv1, const float *uv2, const float *kb1, const float *kb2,
                               const float *Tp, float min_cos, float *x1, float *x2, uint8_t *valid, hipStream_t st) {
    if (n > 0)
        hipLaunchKernelGGL(dev::k_triangulate_nrslam, dim3((n + 255) / 256), dim3(256), 0, st, n, uv1, uv2, kb1, kb2,
                           Tp, min_cos, x1, x2, valid);
}

}  // namespace deftri
