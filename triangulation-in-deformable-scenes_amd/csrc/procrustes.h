// procrustes.h — computeR's per-vertex rotation (Modules/Utils/Geometry.cc:549-604), shared by the
// host graph builder and the device kernel (graph_dev.hip) so both produce the same bits:
//   S_i = sum_j w_ij e1_ij e2_ij^T,  Eigen::JacobiSVD<Matrix3d>(S_i, ComputeFullU | ComputeFullV),
//   R_i = V U^T (last column of U negated when det < 0), kept as Sophus::SO3d (unit quaternion).
// The SVD is Eigen's two-sided Jacobi restated (real_2x2_jacobi_svd + JacobiRotation::makeJacobi,
// precision 2*eps, sign fix, descending selection sort): for rank-deficient S_i the rotation depends
// on exactly these steps.  Callers compile this with FMA contraction off (the host build has no FMA;
// graph_dev.hip is built with -ffp-contract=off), one rounding per operation on both sides.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace deftri {
namespace pr {

constexpr double kEps = 2.220446049250313080847e-16;       // numeric_limits<double>::epsilon()
constexpr double kMin = 2.225073858507201383090e-308;      // numeric_limits<double>::min()

struct Rot { double c, s; };
__host__ __device__ inline double dmax(double a, double b) { return a < b ? b : a; }   // std::max

__host__ __device__ inline void rot_left(double *M, int p, int q, Rot j) {     // M.applyOnTheLeft(p, q, j)
    for (int i = 0; i < 3; i++) {
        double x = M[3 * p + i], y = M[3 * q + i];
        M[3 * p + i] = j.c * x + j.s * y;
        M[3 * q + i] = -j.s * x + j.c * y;
    }
}
__host__ __device__ inline void rot_right(double *M, int p, int q, Rot j) {    // M.applyOnTheRight(p, q, j)
    Rot t{j.c, -j.s};
    for (int i = 0; i < 3; i++) {
        double x = M[3 * i + p], y = M[3 * i + q];
        M[3 * i + p] = t.c * x + t.s * y;
        M[3 * i + q] = -t.s * x + t.c * y;
    }
}

__host__ __device__ inline void jacobi_svd3(const double Min[9], double U[9], double sv[3], double V[9]) {
    const double precision = 2.0 * kEps;
    const double considerAsZero = kMin;
    double scale = 0;
    for (int i = 0; i < 9; i++) scale = dmax(scale, fabs(Min[i]));
    if (scale == 0.0) scale = 1.0;
    double W[9];
    for (int i = 0; i < 9; i++) W[i] = Min[i] / scale;
    for (int i = 0; i < 9; i++) U[i] = V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    double maxDiag = dmax(fabs(W[0]), dmax(fabs(W[4]), fabs(W[8])));
    bool finished = false;
    int guard = 0;
    while (!finished && guard++ < 1000) {
        finished = true;
        for (int p = 1; p < 3; p++)
            for (int q = 0; q < p; q++) {
                double threshold = dmax(considerAsZero, precision * maxDiag);
                if (fabs(W[3 * p + q]) > threshold || fabs(W[3 * q + p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd(W, p, q)
                    double m00 = W[3 * p + p], m01 = W[3 * p + q], m10 = W[3 * q + p], m11 = W[3 * q + q];
                    Rot rot1;
                    double t = m00 + m11, d = m10 - m01;
                    if (fabs(d) < kMin) { rot1.s = 0; rot1.c = 1; }
                    else {
                        double u = t / d, tmp = sqrt(1.0 + u * u);
                        rot1.s = 1.0 / tmp; rot1.c = u / tmp;
                    }
                    // m.applyOnTheLeft(0, 1, rot1)
                    double a0 = rot1.c * m00 + rot1.s * m10, a1 = rot1.c * m01 + rot1.s * m11;
                    double b0 = -rot1.s * m00 + rot1.c * m10, b1 = -rot1.s * m01 + rot1.c * m11;
                    m00 = a0; m01 = a1; m10 = b0; m11 = b1;
                    // j_right.makeJacobi(m, 0, 1): x = m00, y = m01, z = m11
                    Rot jr;
                    double deno = 2.0 * fabs(m01);
                    if (deno < kMin) { jr.c = 1; jr.s = 0; }
                    else {
                        double tau = (m00 - m11) / deno;
                        double w = sqrt(tau * tau + 1.0);
                        double tt = tau > 0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
                        double sign_t = tt > 0 ? 1.0 : -1.0;
                        double n = 1.0 / sqrt(tt * tt + 1.0);
                        jr.s = -sign_t * (m01 / fabs(m01)) * fabs(tt) * n;
                        jr.c = n;
                    }
                    // j_left = rot1 * j_right.transpose()
                    Rot jrt{jr.c, -jr.s};
                    Rot jl{rot1.c * jrt.c - rot1.s * jrt.s, rot1.c * jrt.s + rot1.s * jrt.c};
                    rot_left(W, p, q, jl);
                    rot_right(U, p, q, Rot{jl.c, -jl.s});
                    rot_right(W, p, q, jr);
                    rot_right(V, p, q, jr);
                    maxDiag = dmax(maxDiag, dmax(fabs(W[3 * p + p]), fabs(W[3 * q + q])));
                }
            }
    }
    for (int i = 0; i < 3; i++) {
        double a = W[3 * i + i];
        sv[i] = fabs(a);
        if (a < 0) for (int r = 0; r < 3; r++) U[3 * r + i] = -U[3 * r + i];
    }
    for (int i = 0; i < 3; i++) sv[i] *= scale;
    for (int i = 0; i < 3; i++) {
        int pos = i;
        double mx = sv[i];
        for (int k = i + 1; k < 3; k++) if (sv[k] > mx) { mx = sv[k]; pos = k; }
        if (mx == 0.0) break;
        if (pos != i) {
            double t = sv[i]; sv[i] = sv[pos]; sv[pos] = t;
            for (int r = 0; r < 3; r++) {
                t = U[3 * r + i]; U[3 * r + i] = U[3 * r + pos]; U[3 * r + pos] = t;
                t = V[3 * r + i]; V[3 * r + i] = V[3 * r + pos]; V[3 * r + pos] = t;
            }
        }
    }
}

__host__ __device__ inline double det3(const double M[9]) {     // Eigen determinant_impl<3>
    const double h0 = M[0] * (M[4] * M[8] - M[5] * M[7]);
    const double h1 = M[1] * (M[3] * M[8] - M[5] * M[6]);
    const double h2 = M[2] * (M[3] * M[7] - M[4] * M[6]);
    return h0 - h1 + h2;
}

__host__ __device__ inline void quat_from_mat(const double m[9], double q[4]) {   // Eigen Quaternion(Matrix3), x y z w
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t; q[1] = (m[2] - m[6]) * t; q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}

__host__ __device__ inline void mat_from_quat(const double q[4], double R[9]) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    double twx = tx * w, twy = ty * w, twz = tz * w;
    double txx = tx * x, txy = ty * x, txz = tz * x;
    double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

}  // namespace pr

// ComputeEdgeWeightsCot's term for the edge (A, B) seen from its opposite vertex V (Geometry.cc:
// 272-298): a.b / |a x b| with a = A - V, b = B - V (A the lower vertex index)
__host__ __device__ inline double cot_term(const double *A, const double *B, const double *V) {
    const double a[3] = {A[0] - V[0], A[1] - V[1], A[2] - V[2]};
    const double b[3] = {B[0] - V[0], B[1] - V[1], B[2] - V[2]};
    const double cr[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    return (a[0] * b[0] + a[1] * b[1] + a[2] * b[2]) / sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
}
// the edge's weight: the mean over its (at most two) opposite vertices, clamped at 0
__host__ __device__ inline double cot_weight(double sum, int num) {
    const double wt = num > 0 ? sum / num : 0;
    return wt < 0.0 ? 0.0 : wt;
}

// R = the computeR rotation of the 3x3 cross-covariance S (row-major)
__host__ __device__ inline void procrustes_rotation_hd(const double S[9], double R[9]) {
    double U[9], s[3], V[9];
    pr::jacobi_svd3(S, U, s, V);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[3 * i + j] = V[3 * i] * U[3 * j] + V[3 * i + 1] * U[3 * j + 1] + V[3 * i + 2] * U[3 * j + 2];
    if (pr::det3(R) < 0) {
        for (int i = 0; i < 3; i++) U[3 * i + 2] *= -1;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = V[3 * i] * U[3 * j] + V[3 * i + 1] * U[3 * j + 1] + V[3 * i + 2] * U[3 * j + 2];
    }
    double q[4];
    pr::quat_from_mat(R, q);                  // Sophus::SO3d keeps the unit quaternion
    pr::mat_from_quat(q, R);
}

// one vertex of computeR over the pair's mesh (CSR adjacency with per-entry cot weights):
// identity unless a position maps to the vertex (invertedPosIndexes), neighbours whose positions
// are past KF2's count skipped (Geometry.cc:567-585)
__host__ __device__ inline void compute_r_vertex(int i, int n2, const int32_t *off, const int32_t *adj, const double *w,
                                                 const int32_t *posIdx, const int32_t *inv, const double *pos1,
                                                 const double *pos2, double *R) {
    if (inv[posIdx[i]] != i) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double S[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int pi = posIdx[i];
    for (int32_t k = off[i]; k < off[i + 1]; k++) {
        const int pj = posIdx[adj[k]];
        if (pi >= n2 || pj >= n2) continue;
        const double wt = w[k];
        double e1[3], e2[3];
        for (int c = 0; c < 3; c++) { e1[c] = pos1[3 * pi + c] - pos1[3 * pj + c]; e2[c] = pos2[3 * pi + c] - pos2[3 * pj + c]; }
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) S[3 * r + c] += wt * e1[r] * e2[c];
    }
    procrustes_rotation_hd(S, R);
}

}  // namespace deftri
