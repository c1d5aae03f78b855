// kernels.hip — gfx950 kernels of the deformable-triangulation LM hot path.
//
// Stage                    replaces (reference / g2o)                                   kernel(s)
// ----------------------   -----------------------------------------------------------  -------------------------
// residuals + Jacobians    computeActiveErrors + linearizeOplus of the three edge types  k_lin_rep/k_lin_dep/k_lin_arap
//                          (g2oTypes.h:267-298, 300-349, 390-421; g2oTypes.cc:270-283)
// H, b assembly            BlockSolver::buildSystem / constructQuadraticForm             k_hchunk/k_hfinal, k_bchunk/k_bfinal
// H + lambda I             BlockSolver::setLambda                                        k_scatter
// LDL^T                    LinearSolverEigen (SimplicialLDLT) factorization              k_ea, k_diag, k_trsm, k_update
// solve                    SimplicialLDLT::solve                                         k_fwd, k_fwd_gemv, k_bwd_gemv, k_bwd
// x <- x (+) dx            OptimizableGraph::update (vertex oplusImpl)                   k_update_state
// chi2 / scale reductions  activeRobustChi2, OptimizationAlgorithmLevenberg::computeScale k_sum_partial/k_sum_final, ...
//
// All reductions are deterministic (fixed-order per-chunk partials, then an ordered final pass):
// no floating-point atomics anywhere on the path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>

#include "device_math.h"
#include "diag_panel.h"
#include "kernels.h"
#include "symbolic.h"
#include "ticket.h"

namespace deftri {
namespace dev {

#define TID (blockIdx.x * blockDim.x + threadIdx.x)

// ------------------------------------------------------------------------------------------
// edge errors / Jacobians
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void huber_rho(double delta, double e2, double &rho0, double &rho1) {
#pragma clang fp contract(off)
    if (delta <= 0) { rho0 = e2; rho1 = 1.0; return; }
    double dsqr = delta * delta;
    if (e2 <= dsqr) { rho0 = e2; rho1 = 1.0; }
    else { double se = sqrt(e2); rho0 = 2 * se * delta - dsqr; rho1 = delta / se; }
}

__device__ __forceinline__ double lin_rep_edge(int e, int R, const int32_t *__restrict__ rp, const int32_t *__restrict__ rc,
                          const double *__restrict__ obs, const double *__restrict__ info, double hdelta,
                          const double *__restrict__ points, const double *__restrict__ cam_pose,
                          const double *__restrict__ cam_R, const float *__restrict__ kb8,
                          double *__restrict__ J, double *__restrict__ W, double *__restrict__ E,
                          double *__restrict__ chi, int want_jac) {
#pragma clang fp contract(off)
    if (e >= R) return 0.0;
    int c = rc[e];
    const double *pp = points + 3 * (int64_t)rp[e];
    double p[3] = {pp[0], pp[1], pp[2]}, pc[3];
    SE3 T = se3_load(cam_pose + 7 * c);
    se3_map(T, p, pc);
    float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]}, uv[2];
    kb8_project(kb8 + 8 * c, pf, uv);
    double e0 = obs[2 * e] - (double)uv[0], e1 = obs[2 * e + 1] - (double)uv[1];
    double om = info[e];
    double c2 = e0 * (om * e0) + e1 * (om * e1);
    double rho0, rho1;
    huber_rho(hdelta, c2, rho0, rho1);
    if (chi) chi[e] = rho0;
    if (!want_jac) return rho0;
    float jf[6];
    kb8_project_jac(kb8 + 8 * c, pf, jf);
    const double *Rm = cam_R + 9 * c;
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int k = 0; k < 3; k++)
            J[6 * (int64_t)e + 3 * r + k] = -(double)jf[3 * r] * Rm[k] - (double)jf[3 * r + 1] * Rm[3 + k] -
                                           (double)jf[3 * r + 2] * Rm[6 + k];
    W[e] = rho1 * om;
    E[2 * (int64_t)e] = e0;
    E[2 * (int64_t)e + 1] = e1;
    return rho0;
}

__device__ __forceinline__ double depth_err(const SE3 &T, const double p[3], double meas, double s) {
#pragma clang fp contract(off)
    double pc[3];
    se3_map(T, p, pc);
    double x = meas / s - pc[2];
    double error = x * x;                         // pow(x, 2)
    if (s <= 0.0) error = error * 500;
    return error;
}

__device__ __forceinline__ double lin_dep_edge(int e, int D, const int32_t *__restrict__ dpt, const int32_t *__restrict__ dsc,
                          const int32_t *__restrict__ dcam, const double *__restrict__ meas,
                          const double *__restrict__ info, const double *__restrict__ points,
                          const double *__restrict__ scales, const double *__restrict__ cam_pose,
                          const double *__restrict__ cam_R, double *__restrict__ J, double *__restrict__ W,
                          double *__restrict__ E, double *__restrict__ chi, int want_jac, int analytic) {
#pragma clang fp contract(off)
    if (e >= D) return 0.0;
    int c = dcam[e];
    const double *pp = points + 3 * (int64_t)dpt[e];
    double p[3] = {pp[0], pp[1], pp[2]};
    double s = scales[dsc[e]], mv = meas[e];
    SE3 T = se3_load(cam_pose + 7 * c);
    double err = depth_err(T, p, mv, s);
    double om = info[e];
    const double c2 = err * (om * err);
    if (chi) chi[e] = c2;
    if (!want_jac) return c2;
    double Jv[4];
    if (analytic) {
        double pc[3];
        se3_map(T, p, pc);
        double r = mv / s - pc[2];
        double f = (s <= 0.0) ? 500.0 : 1.0;
        const double *Rm = cam_R + 9 * c;
        for (int k = 0; k < 3; k++) Jv[k] = f * 2.0 * r * (-Rm[6 + k]);
        Jv[3] = f * 2.0 * r * (-mv / (s * s));
    } else {                                       // g2o BaseBinaryEdge numeric, delta 1e-9
        const double delta = 1e-9, scalar = 1.0 / (2 * delta);
        for (int k = 0; k < 3; k++) {
            double bak = p[k];
            p[k] = bak + delta; double ep = depth_err(T, p, mv, s);
            p[k] = bak - delta; double em = depth_err(T, p, mv, s);
            p[k] = bak;
            Jv[k] = scalar * (ep - em);
        }
        Jv[3] = scalar * (depth_err(T, p, mv, s + delta) - depth_err(T, p, mv, s - delta));
    }
    for (int k = 0; k < 4; k++) J[4 * (int64_t)e + k] = Jv[k];
    W[e] = om;
    E[e] = err;
    return c2;
}

// x / area by the pair's reciprocal: q0 = x RN(1/area), the residual x - q0 area exact by FMA, one
// correction q0 + res RN(1/area) — Markstein's sequence, the correctly rounded quotient (the bits of
// x / area) for operands far from overflow / underflow, as the ARAP terms are (point differences
// over a mesh area; tools/micro/div_markstein.c: 4e8 random operand pairs, no difference;
// tests/test_markstein.py runs it on every CPU suite).  An exact
// quotient (zero residual) returns q0 itself, so the sign of a zero quotient is kept.  One division
// per edge instead of up to 108 (the numeric Jacobian's perturbed energies)
struct AreaDiv {
    double v, r;
};
__device__ __forceinline__ AreaDiv area_div(double area) { return AreaDiv{area, 1.0 / area}; }
__device__ __forceinline__ double adiv(double x, const AreaDiv &a) {
#pragma clang fp contract(off)
    const double q0 = x * a.r;
    const double res = __fma_rn(-q0, a.v, x);
    return res == 0.0 ? q0 : __fma_rn(res, a.r, q0);
}

// The ARAP energy's arithmetic, written out as explicit products, FMAs and sums (contraction off):
// arap_err_rt and the numeric Jacobian's piece reuse (arap_base / arap_pert) form the same operations,
// so an energy assembled from pieces of the unperturbed evaluation has the bits of a full one.
__device__ __forceinline__ double arap_mrow(const double *R, const double *v) {
#pragma clang fp contract(off)
    return __fma_rn(R[2], v[2], __fma_rn(R[1], v[1], R[0] * v[0]));
}
// (w (fn + gn) + eg) - 0
__device__ __forceinline__ double arap_sum(const double *dg, const double *f, const double *g, double w) {
#pragma clang fp contract(off)
    const double eg = __fma_rn(dg[2], dg[2], __fma_rn(dg[1], dg[1], dg[0] * dg[0]));
    const double fn = __fma_rn(f[2], f[2], __fma_rn(f[1], f[1], f[0] * f[0]));
    const double gn = __fma_rn(g[2], g[2], __fma_rn(g[1], g[1], g[0] * g[0]));
    return __fma_rn(w, fn + gn, eg) - 0.0;
}
__device__ __forceinline__ double arap_fg(const double *f, const double *g) {
#pragma clang fp contract(off)
    const double fn = __fma_rn(f[2], f[2], __fma_rn(f[1], f[1], f[0] * f[0]));
    const double gn = __fma_rn(g[2], g[2], __fma_rn(g[1], g[1], g[0] * g[0]));
    return fn + gn;
}
__device__ __forceinline__ double arap_sum_fg(const double *dg, double fg, double w) {
#pragma clang fp contract(off)
    const double eg = __fma_rn(dg[2], dg[2], __fma_rn(dg[1], dg[1], dg[0] * dg[0]));
    return __fma_rn(w, fg, eg) - 0.0;
}

// the ARAP energy with the global transformation given as (rotation matrix, translation)
__device__ __forceinline__ double arap_err_rt(const double *v1i, const double *v2i, const double *v1j,
                                              const double *v2j, const double *Rg, const double *tt,
                                              const double *Ri, const double *Rj, double w, const AreaDiv &area) {
    // every product and sum written out (no compiler contraction): the numeric Jacobian's reuse of
    // pieces (arap_base / arap_pert) forms the same operations and so the same bits
#pragma clang fp contract(off)
    double dg[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const double a = arap_mrow(Rg + 3 * k, v2i), b = arap_mrow(Rg + 3 * k, v2j);
        dg[k] = ((a - tt[k]) - v1i[k]) + ((b - tt[k]) - v1j[k]);
    }
    double d1i[3], d2i[3], d1j[3], d2j[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        d1i[k] = v1i[k] - v1j[k]; d2i[k] = v2i[k] - v2j[k];
        d1j[k] = v1j[k] - v1i[k]; d2j[k] = v2j[k] - v2i[k];
    }
    double f[3], g[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        f[k] = adiv(d2i[k] - arap_mrow(Ri + 3 * k, d1i), area);
        g[k] = adiv(d2j[k] - arap_mrow(Rj + 3 * k, d1j), area);
    }
    return arap_sum(dg, f, g, w);
}

__device__ __forceinline__ double arap_err(const double *v1i, const double *v2i, const double *v1j,
                                           const double *v2j, const SE3 &T, const double *Ri,
                                           const double *Rj, double w, const AreaDiv &area) {
    double Rg[9];
    quat_to_mat(T.r, Rg);
    return arap_err_rt(v1i, v2i, v1j, v2j, Rg, T.t, Ri, Rj, w, area);
}

struct ArapBase {                  // one point configuration's pieces
    double A[3], B[3];             // (Rg v2i - t) - v1i, (Rg v2j - t) - v1j
    double d1i[3], d1j[3];         // v1i - v1j, v1j - v1i
    double rf[3], rg[3];           // rows of Ri d1i, Rj d1j
    double f[3], g[3];
};
__device__ __forceinline__ void arap_base(const double *v1i, const double *v2i, const double *v1j, const double *v2j,
                                          const double *Rg, const double *tt, const double *Ri, const double *Rj,
                                          const AreaDiv &area, ArapBase &o) {
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const double a = arap_mrow(Rg + 3 * k, v2i), b = arap_mrow(Rg + 3 * k, v2j);
        o.A[k] = (a - tt[k]) - v1i[k];
        o.B[k] = (b - tt[k]) - v1j[k];
        o.d1i[k] = v1i[k] - v1j[k];
        o.d1j[k] = v1j[k] - v1i[k];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        o.rf[k] = arap_mrow(Ri + 3 * k, o.d1i);
        o.rg[k] = arap_mrow(Rj + 3 * k, o.d1j);
        o.f[k] = adiv((v2i[k] - v2j[k]) - o.rf[k], area);
        o.g[k] = adiv((v2j[k] - v2i[k]) - o.rg[k], area);
    }
}
// the energy with coordinate DD of point VI (0 v1i, 1 v2i, 2 v1j, 3 v2j) set to x; the others as in
// the base `o` of the points Q (the perturbed evaluation's other coordinates)
template <int VI, int DD>
__device__ __forceinline__ double arap_pert(const ArapBase &o, const double (*Q)[3], double x, const double *Rg,
                                            const double *tt, const double *Ri, const double *Rj, double w,
                                            const AreaDiv &area) {
#pragma clang fp contract(off)
    double dg[3], f[3], g[3];
    if constexpr (VI == 0 || VI == 2) {
        // v1i / v1j: d1i, d1j change in one coordinate -> every row of Ri d1i, Rj d1j
        double v1i[3], v1j[3], d1i[3], d1j[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            v1i[k] = (VI == 0 && k == DD) ? x : Q[0][k];
            v1j[k] = (VI == 2 && k == DD) ? x : Q[2][k];
            d1i[k] = v1i[k] - v1j[k];
            d1j[k] = v1j[k] - v1i[k];
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            f[k] = adiv((Q[1][k] - Q[3][k]) - arap_mrow(Ri + 3 * k, d1i), area);
            g[k] = adiv((Q[3][k] - Q[1][k]) - arap_mrow(Rj + 3 * k, d1j), area);
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if (k != DD) dg[k] = o.A[k] + o.B[k];
            else {
                const double a = arap_mrow(Rg + 3 * k, Q[1]), b = arap_mrow(Rg + 3 * k, Q[3]);
                dg[k] = ((a - tt[k]) - v1i[k]) + ((b - tt[k]) - v1j[k]);
            }
        }
    } else {
        // v2i / v2j: Rg v2 changes in every row; d2i, d2j in one coordinate -> f, g in one row
        double v2i[3], v2j[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            v2i[k] = (VI == 1 && k == DD) ? x : Q[1][k];
            v2j[k] = (VI == 3 && k == DD) ? x : Q[3][k];
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if constexpr (VI == 1) dg[k] = ((arap_mrow(Rg + 3 * k, v2i) - tt[k]) - Q[0][k]) + o.B[k];
            else dg[k] = o.A[k] + ((arap_mrow(Rg + 3 * k, v2j) - tt[k]) - Q[2][k]);
            if (k == DD) {
                f[k] = adiv((v2i[k] - v2j[k]) - o.rf[k], area);
                g[k] = adiv((v2j[k] - v2i[k]) - o.rg[k], area);
            } else {
                f[k] = o.f[k];
                g[k] = o.g[k];
            }
        }
    }
    return arap_sum(dg, f, g, w);
}

// g2o's numeric Jacobian of an ARAP edge perturbs the pair's T_g by exp(+-delta e_d) * T_g; those
// 12 transformations (and T_g itself) are the same for every edge of the pair, so they are formed
// once per pair here: per pair kArapPre x (rotation matrix 9, translation 3), transformation 0 the
// unperturbed one, 1 + 2d / 2 + 2d the +delta / -delta perturbations of twist coordinate d.
constexpr int kArapPre = 13;
__device__ __forceinline__ void arap_pre_one(int t, int Q, const double *__restrict__ tg, double *__restrict__ pre) {
    if (t >= Q * kArapPre) return;
    const int q = t / kArapPre, k = t % kArapPre;
    const SE3 T = se3_load(tg + 7 * q);
    SE3 X = T;
    if (k > 0) {
        const double delta = 1e-9;
        double uu[6] = {0, 0, 0, 0, 0, 0};
        uu[(k - 1) >> 1] = (k & 1) ? delta : -delta;
        X = se3_mul(se3_exp(uu), T);
    }
    double *o = pre + 12 * (int64_t)t;
    quat_to_mat(X.r, o);
    o[9] = X.t[0]; o[10] = X.t[1]; o[11] = X.t[2];
}
__global__ void k_arap_pre(int Q, const double *__restrict__ tg, double *__restrict__ pre, const int *gate) {
    if (gate && !*gate) return;
    arap_pre_one(TID, Q, tg, pre);
}

// MODE 0: error and chi2 only; 1: + analytic Jacobian; 2: + g2o numeric Jacobian, pieces reused; 3: the
// same, every evaluation in full (one kernel per mode: each gets the registers of its own path)
template <int MODE>
__device__ __forceinline__ double lin_arap_edge(int e, int E_, const int32_t *__restrict__ apts, const int32_t *__restrict__ apair,
                           const int32_t *__restrict__ arot, const double *__restrict__ aw,
                           const double *__restrict__ rot, const double *__restrict__ parea,
                           const double *__restrict__ pinfo, const double *__restrict__ points,
                           const double *__restrict__ tg, const double *__restrict__ tg_pre,
                           double *__restrict__ J, double *__restrict__ W,
                           double *__restrict__ E, double *__restrict__ chi, int want_jac, int analytic,
                           int64_t jld) {
    if (e >= E_) return 0.0;
    const int32_t *v = apts + 4 * (int64_t)e;
    double P[4][3];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const double *pp = points + 3 * (int64_t)v[k];
        P[k][0] = pp[0]; P[k][1] = pp[1]; P[k][2] = pp[2];
    }
    int q = apair[e];
    SE3 T = se3_load(tg + 7 * q);
    const double *Ri = rot + 9 * (int64_t)arot[2 * (int64_t)e];
    const double *Rj = rot + 9 * (int64_t)arot[2 * (int64_t)e + 1];
    double w = aw[e], om = pinfo[q];
    const AreaDiv area = area_div(parea[q]);
    double err = arap_err(P[0], P[1], P[2], P[3], T, Ri, Rj, w, area);
    const double c2 = err * (om * err);
    if (chi) chi[e] = c2;
    if (MODE == 0) return c2;
    double Jv[18];
    if (MODE == 1) {
        double Rg[9];
        quat_to_mat(T.r, Rg);
        double d1[3], d2[3], a[3], c[3], g[3], u[3], s2[3];
        for (int k = 0; k < 3; k++) { d1[k] = P[0][k] - P[2][k]; d2[k] = P[1][k] - P[3][k]; s2[k] = P[1][k] + P[3][k]; }
        for (int k = 0; k < 3; k++) {
            a[k] = d2[k] - (Ri[3 * k] * d1[0] + Ri[3 * k + 1] * d1[1] + Ri[3 * k + 2] * d1[2]);
            c[k] = d2[k] - (Rj[3 * k] * d1[0] + Rj[3 * k + 1] * d1[1] + Rj[3 * k + 2] * d1[2]);
            double rs = Rg[3 * k] * s2[0] + Rg[3 * k + 1] * s2[1] + Rg[3 * k + 2] * s2[2];
            u[k] = rs - 2 * T.t[k];
            g[k] = u[k] - (P[0][k] + P[2][k]);
        }
        double co = 2.0 * w / (area.v * area.v);
        double qv[3], rv[3], rg[3];
        for (int k = 0; k < 3; k++) {
            qv[k] = co * (a[k] + c[k]);
            rv[k] = co * ((Ri[k] * a[0] + Ri[3 + k] * a[1] + Ri[6 + k] * a[2]) +
                          (Rj[k] * c[0] + Rj[3 + k] * c[1] + Rj[6 + k] * c[2]));
            rg[k] = 2.0 * (Rg[k] * g[0] + Rg[3 + k] * g[1] + Rg[6 + k] * g[2]);
        }
        for (int k = 0; k < 3; k++) {
            Jv[0 + k] = -rv[k] - 2.0 * g[k];
            Jv[3 + k] = qv[k] + rg[k];
            Jv[6 + k] = rv[k] - 2.0 * g[k];
            Jv[9 + k] = -qv[k] + rg[k];
        }
        Jv[12] = 2.0 * (u[1] * g[2] - u[2] * g[1]);
        Jv[13] = 2.0 * (u[2] * g[0] - u[0] * g[2]);
        Jv[14] = 2.0 * (u[0] * g[1] - u[1] * g[0]);
        Jv[15] = -4.0 * g[0]; Jv[16] = -4.0 * g[1]; Jv[17] = -4.0 * g[2];
    } else if (MODE == 2) {
#pragma clang fp contract(off)
        // g2o BaseMultiEdge numeric, delta 1e-9, with the pieces an evaluation shares with the
        // unperturbed one reused (the bits of MODE 3's full evaluations, tests/test_gpu_sp.py): a
        // T_g perturbation leaves the rows' terms f, g unchanged (no division), a v2i / v2j one changes
        // one row of each (2 of 6 divisions).  g2o's + evaluations see the other coordinates as
        // x + 0.0, the - ones as x - 0.0 = x: the same bits unless a coordinate is -0.0, and an edge
        // with one takes the full evaluations.  Each column is stored when formed.
        auto jst = [&](int k, double v) {
            if (jld) J[k * jld + e] = v;
            else J[18 * (int64_t)e + k] = v;
        };
        bool negz = false;
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int k = 0; k < 3; k++) negz |= __double_as_longlong(P[a][k]) == (long long)0x8000000000000000ull;
        if (negz) {
            // MODE 3's evaluations, inline (a call would give every wave a stack)
            const double delta = 1e-9, scalar = 1.0 / (2 * delta);
            const double *X = tg_pre + 12 * kArapPre * (int64_t)q;
#pragma unroll
            for (int vi = 0; vi < 4; vi++)
#pragma unroll 1
                for (int dd = 0; dd < 3; dd++) {
                    double Pp[4][3], Pm[4][3];
#pragma unroll
                    for (int a = 0; a < 4; a++)
#pragma unroll
                        for (int k = 0; k < 3; k++) {
                            const double d = (a == vi && k == dd) ? delta : 0.0;
                            Pp[a][k] = P[a][k] + d;
                            Pm[a][k] = P[a][k] - d;
                        }
                    const double ep = arap_err_rt(Pp[0], Pp[1], Pp[2], Pp[3], X, X + 9, Ri, Rj, w, area);
                    const double em = arap_err_rt(Pm[0], Pm[1], Pm[2], Pm[3], X, X + 9, Ri, Rj, w, area);
                    jst(3 * vi + dd, scalar * (ep - em));
                }
#pragma unroll 1
            for (int dd = 0; dd < 6; dd++) {
                const double *Xp = X + 12 * (1 + 2 * dd), *Xm = Xp + 12;
                const double ep = arap_err_rt(P[0], P[1], P[2], P[3], Xp, Xp + 9, Ri, Rj, w, area);
                const double em = arap_err_rt(P[0], P[1], P[2], P[3], Xm, Xm + 9, Ri, Rj, w, area);
                jst(12 + dd, scalar * (ep - em));
            }
        } else {
            const double delta = 1e-9, scalar = 1.0 / (2 * delta);
            const double *X = tg_pre + 12 * kArapPre * (int64_t)q;
            double Rg[12];
#pragma unroll
            for (int k = 0; k < 12; k++) Rg[k] = X[k];
            ArapBase bm;
            arap_base(P[0], P[1], P[2], P[3], Rg, Rg + 9, Ri, Rj, area, bm);
            const double fgm = arap_fg(bm.f, bm.g);
#pragma unroll 1
            for (int dd = 0; dd < 6; dd++) {
                const double *Xp = X + 12 * (1 + 2 * dd), *Xm = Xp + 12;
                double dp[3], dm[3];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    dp[k] = ((arap_mrow(Xp + 3 * k, P[1]) - Xp[9 + k]) - P[0][k]) + ((arap_mrow(Xp + 3 * k, P[3]) - Xp[9 + k]) - P[2][k]);
                    dm[k] = ((arap_mrow(Xm + 3 * k, P[1]) - Xm[9 + k]) - P[0][k]) + ((arap_mrow(Xm + 3 * k, P[3]) - Xm[9 + k]) - P[2][k]);
                }
                jst(12 + dd, scalar * (arap_sum_fg(dp, fgm, w) - arap_sum_fg(dm, fgm, w)));
            }
            auto point = [&](auto VI_, auto DD_) {
                constexpr int VI = decltype(VI_)::value, DD = decltype(DD_)::value;
                const double ep = arap_pert<VI, DD>(bm, P, P[VI][DD] + delta, Rg, Rg + 9, Ri, Rj, w, area);
                const double em = arap_pert<VI, DD>(bm, P, P[VI][DD] - delta, Rg, Rg + 9, Ri, Rj, w, area);
                jst(3 * VI + DD, scalar * (ep - em));
            };
            using std::integral_constant;
            point(integral_constant<int, 0>{}, integral_constant<int, 0>{});
            point(integral_constant<int, 0>{}, integral_constant<int, 1>{});
            point(integral_constant<int, 0>{}, integral_constant<int, 2>{});
            point(integral_constant<int, 1>{}, integral_constant<int, 0>{});
            point(integral_constant<int, 1>{}, integral_constant<int, 1>{});
            point(integral_constant<int, 1>{}, integral_constant<int, 2>{});
            point(integral_constant<int, 2>{}, integral_constant<int, 0>{});
            point(integral_constant<int, 2>{}, integral_constant<int, 1>{});
            point(integral_constant<int, 2>{}, integral_constant<int, 2>{});
            point(integral_constant<int, 3>{}, integral_constant<int, 0>{});
            point(integral_constant<int, 3>{}, integral_constant<int, 1>{});
            point(integral_constant<int, 3>{}, integral_constant<int, 2>{});
        }
    } else {                                       // MODE 3: g2o BaseMultiEdge numeric, delta 1e-9,
#pragma clang fp contract(off)
        const double delta = 1e-9, scalar = 1.0 / (2 * delta);   // every evaluation in full
        const double *X = tg_pre + 12 * kArapPre * (int64_t)q;
        double Rg[12];
#pragma unroll
        for (int k = 0; k < 12; k++) Rg[k] = X[k];
        // one coordinate at a time: x + delta (the others + 0.0, which leaves them unchanged), the
        // coordinate loop kept rolled so a single evaluation's registers are live
#pragma unroll
        for (int vi = 0; vi < 4; vi++)
#pragma unroll 1
            for (int dd = 0; dd < 3; dd++) {
                double Pp[4][3], Pm[4][3];
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const double d = (a == vi && k == dd) ? delta : 0.0;
                        Pp[a][k] = P[a][k] + d;
                        Pm[a][k] = P[a][k] - d;
                    }
                double ep = arap_err_rt(Pp[0], Pp[1], Pp[2], Pp[3], Rg, Rg + 9, Ri, Rj, w, area);
                double em = arap_err_rt(Pm[0], Pm[1], Pm[2], Pm[3], Rg, Rg + 9, Ri, Rj, w, area);
                const double jv = scalar * (ep - em);
                if (dd == 0) Jv[3 * vi] = jv;
                else if (dd == 1) Jv[3 * vi + 1] = jv;
                else Jv[3 * vi + 2] = jv;
            }
        for (int dd = 0; dd < 6; dd++) {
            const double *Xp = X + 12 * (1 + 2 * dd), *Xm = Xp + 12;
            double ep = arap_err_rt(P[0], P[1], P[2], P[3], Xp, Xp + 9, Ri, Rj, w, area);
            double em = arap_err_rt(P[0], P[1], P[2], P[3], Xm, Xm + 9, Ri, Rj, w, area);
            Jv[12 + dd] = scalar * (ep - em);
        }
    }
    if (MODE != 2) {
        if (jld) {
#pragma unroll
            for (int k = 0; k < 18; k++) J[k * jld + e] = Jv[k];
        } else {
            for (int k = 0; k < 18; k++) J[18 * (int64_t)e + k] = Jv[k];
        }
    }
    W[e] = om;
    E[e] = err;
    return c2;
}

// a 128-thread workgroup's sum (the linearization's chi2 partials): a butterfly per wave, then the two
// waves; the value in thread 0
__device__ __forceinline__ double block128_sum(double v) {
    __shared__ double r2[2];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) r2[threadIdx.x >> 6] = v;
    __syncthreads();
    return r2[0] + r2[1];
}

__global__ void k_lin_rep(int R, const int32_t *__restrict__ rp, const int32_t *__restrict__ rc,
                          const double *__restrict__ obs, const double *__restrict__ info, double hdelta,
                          const double *__restrict__ points, const double *__restrict__ cam_pose,
                          const double *__restrict__ cam_R, const float *__restrict__ kb8,
                          double *__restrict__ J, double *__restrict__ W, double *__restrict__ E,
                          double *__restrict__ chi, int want_jac, const int *gate) {
    if (gate && !*gate) return;
    lin_rep_edge(TID, R, rp, rc, obs, info, hdelta, points, cam_pose, cam_R, kb8, J, W, E, chi, want_jac);
}

__global__ void k_lin_dep(int D, const int32_t *__restrict__ dpt, const int32_t *__restrict__ dsc,
                          const int32_t *__restrict__ dcam, const double *__restrict__ meas,
                          const double *__restrict__ info, const double *__restrict__ points,
                          const double *__restrict__ scales, const double *__restrict__ cam_pose,
                          const double *__restrict__ cam_R, double *__restrict__ J, double *__restrict__ W,
                          double *__restrict__ E, double *__restrict__ chi, int want_jac, int analytic, const int *gate) {
    if (gate && !*gate) return;
    lin_dep_edge(TID, D, dpt, dsc, dcam, meas, info, points, scales, cam_pose, cam_R, J, W, E, chi, want_jac, analytic);
}

// MODE 0: error and chi2 only; 1: + analytic Jacobian; 2: + g2o numeric Jacobian (one kernel per
// mode: each gets the registers of its own path)
template <int MODE>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(MODE == 2 ? 2 : 1, 8))) k_lin_arap(int E_, const int32_t *__restrict__ apts, const int32_t *__restrict__ apair,
                           const int32_t *__restrict__ arot, const double *__restrict__ aw,
                           const double *__restrict__ rot, const double *__restrict__ parea,
                           const double *__restrict__ pinfo, const double *__restrict__ points,
                           const double *__restrict__ tg, const double *__restrict__ tg_pre,
                           double *__restrict__ J, double *__restrict__ W,
                           double *__restrict__ E, double *__restrict__ chi, int want_jac, int analytic,
                           int64_t jld, const int *gate, double *__restrict__ lpart, int64_t nsum) {
    if (gate && !*gate) return;
    const double c = lin_arap_edge<MODE>(TID, E_, apts, apair, arot, aw, rot, parea, pinfo, points, tg, tg_pre, J, W, E,
                                         lpart ? nullptr : chi, want_jac, analytic, jld);
    if (lpart && (int64_t)blockIdx.x * 128 < nsum) {
        const double v = block128_sum(TID < nsum ? c : 0.0);
        if (threadIdx.x == 0) lpart[blockIdx.x] = v;
    }
}

// the errors and chi2 of every reprojection, depth and ARAP edge in one launch (the trial's
// evaluation): the same per-edge code as k_lin_rep / k_lin_dep / k_lin_arap<0>, block ranges by type
// the linearization's single-point edges and the pair table of the numeric ARAP Jacobian in one
// launch (block ranges: reprojection, depth, then the pairs' perturbed T_g): k_lin_arap reads the
// table, so it follows in its own launch
__global__ void __launch_bounds__(128) k_lin_pts(const DevProblem P, int nbr, int nbd, int want_jac, int analytic) {
    if (P.gate_lin && !*P.gate_lin) return;
    const int b = blockIdx.x, t = threadIdx.x;
    double c = 0.0;
    if (b < nbr)
        c = lin_rep_edge(b * 128 + t, P.R, P.rep_point, P.rep_cam, P.rep_obs, P.rep_info, P.huber_delta, P.points,
                         P.cam_pose, P.cam_R, P.cam_kb8, P.Jrep, P.Wrep, P.Erep, P.lin_part ? nullptr : P.chi_rep,
                         want_jac);
    else if (b < nbr + nbd)
        c = lin_dep_edge((b - nbr) * 128 + t, P.D, P.dep_point, P.dep_scale, P.dep_cam, P.dep_meas, P.dep_info, P.points,
                         P.scales, P.cam_pose, P.cam_R, P.Jdep, P.Wdep, P.Edep, P.lin_part ? nullptr : P.chi_dep,
                         want_jac, analytic);
    else
        arap_pre_one((b - nbr - nbd) * 128 + t, P.Q, P.tg, P.tg_pre);
    if (P.lin_part && b < nbr + nbd) {             // (a workgroup-uniform branch)
        const double v = block128_sum(c);
        if (t == 0) P.lin_part[b] = v;
    }
}

__global__ void __launch_bounds__(128) k_lin_chi(const DevProblem P, int nbr, int nbd) {
    if (P.gate_trial && !*P.gate_trial) return;
    const int b = blockIdx.x, t = threadIdx.x;
    if (b < nbr)
        lin_rep_edge(b * 128 + t, P.R, P.rep_point, P.rep_cam, P.rep_obs, P.rep_info, P.huber_delta, P.points, P.cam_pose,
                     P.cam_R, P.cam_kb8, P.Jrep, P.Wrep, P.Erep, P.chi_rep, 0);
    else if (b < nbr + nbd)
        lin_dep_edge((b - nbr) * 128 + t, P.D, P.dep_point, P.dep_scale, P.dep_cam, P.dep_meas, P.dep_info, P.points,
                     P.scales, P.cam_pose, P.cam_R, P.Jdep, P.Wdep, P.Edep, P.chi_dep, 0, 0);
    else
        lin_arap_edge<0>((b - nbr - nbd) * 128 + t, P.E, P.arap_pts, P.arap_pair, P.arap_rot, P.arap_w, P.rot,
                         P.pair_area, P.pair_info, P.points, P.tg, nullptr, P.Jarap, P.Warap, P.Earap, P.chi_arap, 0, 0,
                         P.jarap_ld);
}

// the four sums of a partial layout (nb0 rep, nb1 dep, nb2 arap, nb3 den workgroups) by one 256-thread
// workgroup: wave w adds kind w's partials (lane-strided, eight loads in flight, added in order), then
// a butterfly; s[w] set for every thread on return (trial_eval_host_sums is the same order on the host)
__device__ __forceinline__ void part_sums_block(const double *part, int nb0, int nb1, int nb2, int nb3, double *s) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lo = w == 0 ? 0 : w == 1 ? nb0 : w == 2 ? nb0 + nb1 : nb0 + nb1 + nb2;
    const int hi = w == 0 ? nb0 : w == 1 ? nb0 + nb1 : w == 2 ? nb0 + nb1 + nb2 : nb0 + nb1 + nb2 + nb3;
    double a = 0.0;
    int i = lo + lane;
    for (; i + 7 * 64 < hi; i += 8 * 64) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = ld_sc1(part + i + 64 * u);
#pragma unroll
        for (int u = 0; u < 8; u++) a += v[u];
    }
    for (; i < hi; i += 64) a += ld_sc1(part + i);
    for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
    if (lane == 0) s[w] = a;
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_part_sums(const double *__restrict__ part, int nb0, int nb1, int nb2, int nb3,
                                                  double *out, double *den_out, double *total, const int *gate) {
    if (gate && !*gate) return;
    __shared__ double s[4];
    part_sums_block(part, nb0, nb1, nb2, nb3, s);
    if (threadIdx.x == 0) {
        out[0] = s[0];
        out[1] = s[1];
        out[2] = s[2];
        if (den_out) *den_out = s[3];
        if (total) *total = (s[0] + s[2]) + s[1];
    }
}

// a trial's evaluation (kernels.h EvalJob): workgroups [0, nbr) reprojection edges, then nbd depth,
// nba owned ARAP edges, then runs of dx.(lambda dx + b); each a run of 256 ept, thread t taking
// entries t, t + 256, ... of it in order.  The per-edge arithmetic is k_lin_chi's; no per-edge chi2
// is stored.
__global__ void __launch_bounds__(256) k_trial_eval(const DevProblem P, const EvalJob J, int ept, int nbr, int nbd, int nba,
                                                   double *__restrict__ part, int *cnt, const ReadBack rb) {
    if (J.gate && !*J.gate) return;
    const int b = blockIdx.x, t = threadIdx.x;
    const int64_t run = 256 * (int64_t)ept;
    double acc = 0.0;
    if (b < nbr) {
        const int64_t e0 = b * run + t;
        for (int u = 0; u < ept; u++)
            acc += lin_rep_edge((int)(e0 + 256 * u), P.R, P.rep_point, P.rep_cam, P.rep_obs, P.rep_info, P.huber_delta, P.points,
                                P.cam_pose, P.cam_R, P.cam_kb8, nullptr, nullptr, nullptr, nullptr, 0);
    } else if (b < nbr + nbd) {
        const int64_t e0 = (b - nbr) * run + t;
        for (int u = 0; u < ept; u++)
            acc += lin_dep_edge((int)(e0 + 256 * u), P.D, P.dep_point, P.dep_scale, P.dep_cam, P.dep_meas, P.dep_info, P.points,
                                P.scales, P.cam_pose, P.cam_R, nullptr, nullptr, nullptr, nullptr, 0, 0);
    } else if (b < nbr + nbd + nba) {
        const int64_t e0 = (b - nbr - nbd) * run + t;
        for (int u = 0; u < ept; u++)
            acc += lin_arap_edge<0>((int)(e0 + 256 * u), (int)J.n_arap, P.arap_pts, P.arap_pair, P.arap_rot, P.arap_w, P.rot,
                                    P.pair_area, P.pair_info, P.points, P.tg, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0,
                                    P.jarap_ld);
    } else {
        const double lam = J.lambda_dev ? *J.lambda_dev : J.lambda;
        const int64_t i0 = (b - nbr - nbd - nba) * run + t;
        for (int u = 0; u < ept; u++) {
            const int64_t i = i0 + 256 * u;
            if (i < J.n_den) {
                const double v = J.dx[i];
                acc += v * (lam * v + J.b[i]);
            }
        }
    }
    // the workgroup's partial: a butterfly per wave, then the four waves
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __shared__ double red[4], s[4];
    __shared__ int last;
    const int w = t >> 6, lane = t & 63;
    if (lane == 0) red[w] = acc;
    __syncthreads();
    if (J.h_part) {                                // the host finishes the sums: no ticket
        if (t == 0) J.h_part[b] = (red[0] + red[1]) + (red[2] + red[3]);
        if (b == 0 && rb.h_rec) {
            const bool final_st = J.rec_clear && rb.rec[0] != 0.0;
            if (t < rb.nrec) rb.h_rec[t] = rb.rec[t];
            if (t == 0) *rb.h_flag = *rb.flag;
            __syncthreads();                       // (every read of the record done)
            if (final_st) {
                for (int64_t i = t; i < J.nclear; i += 256) J.rec_clear[i] = 0.0;
                if (t == 0) *J.flag_clear = 0;
            }
        }
        return;
    }
    if (t == 0) {
        st_sc1(part + b, (red[0] + red[1]) + (red[2] + red[3]));
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        last = ticket_last(cnt, (int)gridDim.x, b);
    }
    __syncthreads();
    if (!last) return;
    part_sums_block(part, nbr, nbd, nba, (int)gridDim.x - nbr - nbd - nba, s);
    if (t == 0) {
        J.out[0] = s[0];
        J.out[1] = s[1];
        J.out[2] = s[2];
        if (J.den_out) *J.den_out = s[3];
        if (J.total) *J.total = (s[0] + s[2]) + s[1];
    }
    __syncthreads();
    if (rb.h_scal) {
        if (t < rb.ns) rb.h_scal[t] = rb.scal[t];
        if (t == 0) *rb.h_flag = *rb.flag;
        if (rb.rec && t < rb.nrec) rb.h_rec[t] = rb.rec[t];
    }
}

// ------------------------------------------------------------------------------------------
// deterministic H / b assembly
// ------------------------------------------------------------------------------------------
struct EdgeJ {
    const double *Jrep, *Wrep, *Erep, *Jdep, *Wdep, *Edep, *Jarap, *Warap, *Earap;
};

// Jacobian slice of vertex `role` of edge (kind, e): pointer, vertex dim, residual dim, row stride
__device__ __forceinline__ void jac_slice(const EdgeJ &ej, int kind, int64_t e, int role, const double *&ptr,
                                          int &dim, int &m, int &stride, double &w, const double *&err) {
    if (kind == 0) { ptr = ej.Jrep + 6 * e; dim = 3; m = 2; stride = 3; w = ej.Wrep[e]; err = ej.Erep + 2 * e; }
    else if (kind == 1) {
        ptr = ej.Jdep + 4 * e + (role == 0 ? 0 : 3); dim = (role == 0) ? 3 : 1; m = 1; stride = 0;
        w = ej.Wdep[e]; err = ej.Edep + e;
    } else {
        ptr = ej.Jarap + 18 * e + (role < 4 ? 3 * role : 12); dim = (role < 4) ? 3 : 6; m = 1; stride = 0;
        w = ej.Warap[e]; err = ej.Earap + e;
    }
}

__global__ void k_hchunk(int64_t nchunks, const uint64_t *__restrict__ contrib, const int64_t *__restrict__ cbeg,
                         const int32_t *__restrict__ clen, EdgeJ ej, double *__restrict__ part) {
    int64_t c = TID;
    if (c >= nchunks) return;
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = 0.0;
    int rows = 0, cols = 0;
    int64_t b0 = cbeg[c];
    int n = clen[c];
    // the next record is fetched while the current one is accumulated (breaks the
    // record -> Jacobian load chain of consecutive contributions)
    uint64_t rec_next = n > 0 ? contrib[b0] : 0;
    for (int t = 0; t < n; t++) {
        const uint64_t rec = rec_next;
        if (t + 1 < n) rec_next = contrib[b0 + t + 1];
        int64_t e = (int64_t)(rec & 0xFFFFFFFFFFull);
        int kind = (int)((rec >> 40) & 0xF), rcol = (int)((rec >> 44) & 0xF), rrow = (int)((rec >> 48) & 0xF);
        const double *Jc, *Jr, *er;
        int dc, dr, m, st;
        double w;
        jac_slice(ej, kind, e, rcol, Jc, dc, m, st, w, er);
        jac_slice(ej, kind, e, rrow, Jr, dr, m, st, w, er);
        rows = dr; cols = dc;
        for (int r = 0; r < m; r++) {
#pragma unroll
            for (int i = 0; i < 6; i++) {
                if (i >= dr) break;
                double a = Jr[r * st + i] * w;
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    if (j >= dc) break;
                    acc[i * 6 + j] += a * Jc[r * st + j];
                }
            }
        }
    }
    double *o = part + 36 * c;
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++)
            if (i < rows && j < cols) o[i * cols + j] = acc[i * 6 + j];
}

__global__ void k_hfinal(int64_t nblocks, const int64_t *__restrict__ blk_chunk_begin,
                         const int64_t *__restrict__ val_off, const int32_t *__restrict__ brows,
                         const int32_t *__restrict__ bcols, const double *__restrict__ part,
                         double *__restrict__ hval) {
    int64_t b = TID;
    if (b >= nblocks) return;
    int64_t c0 = blk_chunk_begin[b], c1 = blk_chunk_begin[b + 1];
    if (c1 - c0 > kHeavyChunks) return;                 // k_hfinal_heavy
    const int n = brows[b] * bcols[b];
    double *o = hval + val_off[b];
    // partials summed in chunk order in registers (one store per entry)
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = 0.0;
    for (int64_t c = c0; c < c1; c++) {
        const double *pc = part + 36 * c;
#pragma unroll
        for (int k = 0; k < 36; k++)
            if (k < n) acc[k] += pc[k];
    }
#pragma unroll
    for (int k = 0; k < 36; k++)
        if (k < n) o[k] = acc[k];
}

// blocks fed by thousands of chunks (the global T_g / depth-scale rows): each of kHeavySplit
// workgroups takes a contiguous slice of the chunks, strided per-thread sums then an in-order sum
// over the 256 partials; the slices are then added in order — fixed order, no atomics
constexpr int kHeavySplit = 32;
template <int W>
__device__ __forceinline__ void heavy_sum(int64_t c0, int64_t c1, int n, const double *__restrict__ part,
                                          double *__restrict__ o) {
    __shared__ double red[256][W + 1];
    double acc[W];
#pragma unroll
    for (int k = 0; k < W; k++) acc[k] = 0.0;
    for (int64_t c = c0 + threadIdx.x; c < c1; c += 256)
#pragma unroll
        for (int k = 0; k < W; k++)
            if (k < n) acc[k] += part[W * c + k];
#pragma unroll
    for (int k = 0; k < W; k++) red[threadIdx.x][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < n) {
        double s = 0.0;
        for (int t = 0; t < 256; t++) s += red[t][threadIdx.x];
        o[threadIdx.x] = s;
    }
}

// heavy blocks split over kHeavySplit workgroups each: workgroup g sums its contiguous slice of
// the block's chunks (heavy_sum order) into scratch; k_heavy_final adds the slices in slice order
template <int W>
__global__ void __launch_bounds__(256) k_heavy_split(const int64_t *__restrict__ heavy,
                                                     const int64_t *__restrict__ chunk_begin,
                                                     const double *__restrict__ part, double *__restrict__ scratch) {
    const int64_t h = blockIdx.x / kHeavySplit, g = blockIdx.x % kHeavySplit;
    const int64_t v = heavy[h];
    const int64_t c0 = chunk_begin[v], len = chunk_begin[v + 1] - c0;
    heavy_sum<W>(c0 + g * len / kHeavySplit, c0 + (g + 1) * len / kHeavySplit, W, part,
                 scratch + (h * kHeavySplit + g) * W);
}

template <int W>
__global__ void k_heavy_final(const int64_t *__restrict__ heavy, const int64_t *__restrict__ off,
                              const int32_t *__restrict__ nr, const int32_t *__restrict__ nc,
                              const double *__restrict__ scratch, double *__restrict__ out) {
    const int64_t h = blockIdx.x, v = heavy[h];
    const int n = nc ? nr[v] * nc[v] : nr[v];
    const int k = threadIdx.x;
    if (k >= n) return;
    double s = 0.0;
    for (int g = 0; g < kHeavySplit; g++) s += scratch[(h * kHeavySplit + g) * W + k];
    out[off[v] + k] = s;
}

__global__ void k_bchunk(int64_t nchunks, const uint64_t *__restrict__ contrib, const int64_t *__restrict__ cbeg,
                         const int32_t *__restrict__ clen, EdgeJ ej, double *__restrict__ part) {
    int64_t c = TID;
    if (c >= nchunks) return;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    int64_t b0 = cbeg[c];
    int n = clen[c];
    for (int t = 0; t < n; t++) {
        uint64_t rec = contrib[b0 + t];
        int64_t e = (int64_t)(rec & 0xFFFFFFFFFFull);
        int kind = (int)((rec >> 40) & 0xF), role = (int)((rec >> 44) & 0xF);
        const double *Jv, *er;
        int dim, m, st;
        double w;
        jac_slice(ej, kind, e, role, Jv, dim, m, st, w, er);
        for (int r = 0; r < m; r++) {
            double we = w * er[r];
#pragma unroll
            for (int i = 0; i < 6; i++)
                if (i < dim) acc[i] -= Jv[r * st + i] * we;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) part[6 * c + i] = acc[i];
}

__global__ void k_bfinal(int64_t nv, const int64_t *__restrict__ v_chunk_begin, const int64_t *__restrict__ voff,
                         const int32_t *__restrict__ vdim, const double *__restrict__ part, double *__restrict__ b) {
    int64_t v = TID;
    if (v >= nv) return;
    if (v_chunk_begin[v + 1] - v_chunk_begin[v] > kHeavyChunks) return;   // k_bfinal_heavy
    int dim = vdim[v];
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t c = v_chunk_begin[v]; c < v_chunk_begin[v + 1]; c++)
        for (int i = 0; i < 6; i++) acc[i] += part[6 * c + i];
    for (int i = 0; i < dim; i++) b[voff[v] + i] = acc[i];
}

// H (+ lambda I) -> fronts
__global__ void k_scatter(int64_t nblocks, const int64_t *__restrict__ val_off, const int32_t *__restrict__ brows,
                          const int32_t *__restrict__ bcols, const int64_t *__restrict__ barena,
                          const int32_t *__restrict__ bld, const int32_t *__restrict__ bdiag,
                          const double *__restrict__ hval, const LaneOff lo, const double *__restrict__ lam_dev,
                          double *__restrict__ arena) {
    int64_t b = TID;
    if (b >= nblocks) return;
    // lam_dev: lambda read from device memory (the captured trial graph's launches keep one argument set)
    const double lambda = lam_dev ? lam_dev[blockIdx.y] : lo.lam[blockIdx.y];
    arena += blockIdx.y * lo.arena;
    int R = brows[b], Cc = bcols[b], ld = bld[b];
    const double *h = hval + val_off[b];
    double *a = arena + barena[b];
    bool dg = bdiag[b] != 0;
    for (int i = 0; i < R; i++)
        for (int j = 0; j < Cc; j++) a[(int64_t)j * ld + i] = h[i * Cc + j] + ((dg && i == j) ? lambda : 0.0);
}

// ------------------------------------------------------------------------------------------
// multifrontal LDL^T
// ------------------------------------------------------------------------------------------
// extend-add of one child contribution block into its parent: task (child, j0, i0) covers CB columns
// j0..j0+15 and rows i0..i0+255 (lower triangle).  Each thread owns one CB row: its parent row index
// and the 16 child/parent values are loaded up front (one latency round); each parent entry is
// written by exactly one thread of the launch (slot-0 and slot-1 children run in separate launches,
// so the summation order is fixed).
__global__ void __launch_bounds__(256) k_ea(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                            double *__restrict__ arena, const LaneOff lo) {
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena;
    int c = tasks[3 * t], j0 = tasks[3 * t + 1], i0 = tasks[3 * t + 2];
    int p = fd.parent[c];
    int mc = fd.m[c], sc = fd.s[c], mp = fd.m[p];
    int u = mc - sc;
    const int32_t *bm = fd.bmap + fd.bmap_off[c];
    const double *Fc = arena + fd.arena_off[c] + (int64_t)sc * mc + sc;
    double *Fp = arena + fd.arena_off[p];
    const int i = i0 + (int)threadIdx.x;
    if (i >= u) return;
    const int bi = bm[i];
    const int nj = min(16, min(u - j0, i - j0 + 1));       // columns j0..j0+nj-1 with j <= i
    double cv[16], pv[16];
    int64_t pj[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        pj[q] = (q < nj) ? (int64_t)bm[j0 + q] * mp + bi : 0;
        cv[q] = (q < nj) ? Fc[(int64_t)(j0 + q) * mc + i] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) pv[q] = (q < nj) ? Fp[pj[q]] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++)
        if (q < nj) Fp[pj[q]] = pv[q] + cv[q];
}


// standalone panel factorization (first panel of every front of a level; later panels are
// factored by the update launch of the previous panel, see k_update)
// ---- fused TRSM: the row tiles of a panel are solved by the launch that factors its diagonal tile.
// Cross-workgroup hand-off inside one launch, across XCDs (each has its own L2): the factoring
// workgroup writes W = Linv^T D^{-1} (the TRSM operand, 64 x 64) to the panel's slot of `wbuf` with
// agent-coherent stores (relaxed agent-scope atomics: sc1 stores, no L2 write-back), waits for them
// to complete, then stores the factorization epoch into the panel's flag the same way.  A row-tile
// workgroup — placed after every diagonal task of its launch, so dispatched after it (in-order
// dispatch: it never holds a slot the diagonal task needs) — polls the flag with coherent loads and
// reads W coherently.  No release/acquire fences: at agent scope those write back / invalidate the
// whole L2.  A poll that outlives kSpinLimit sets kStatusWaitTimeout (a device error) instead of
// hanging.
constexpr int kSpinLimit = 1 << 22;
__device__ __forceinline__ void st_coherent(double *p, double v) {
    st_sc1((unsigned long long *)p, __builtin_bit_cast(unsigned long long, v));
}
__device__ __forceinline__ double ld_coherent(const double *p) {
    return __builtin_bit_cast(double, ld_sc1((unsigned long long *)p));
}
// W[k][c] = Linv[c][k] / d_c from the factored block in LDS (X[c][k] at S[k][c], D at S[c][c]) —
// the products k_trsm forms from the stored inverse and the front's diagonal
__device__ __forceinline__ void publish_panel(const double (*S)[DP], int kb, double *W, int *pf, int epoch) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int idx = threadIdx.x + 256 * q, kk = idx >> 6, c = idx & 63;
        double v = 0.0;
        if (kk < kb && c < kb) v = (c > kk ? S[kk][c] : (c == kk ? 1.0 : 0.0)) * (1.0 / S[c][c]);
        st_coherent(W + idx, v);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0): this thread's W stores are complete
    __syncthreads();
    if (threadIdx.x == 0) st_sc1(pf, epoch);
}
__device__ __forceinline__ void wait_panel(const int *pf, int epoch, int *flag) {
    if (threadIdx.x == 0) {
        int it = 0;
        while (ld_sc1(pf) != epoch) {
            if (++it > kSpinLimit) { atomicOr(flag, kStatusWaitTimeout); break; }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}
// rows r0..r0+63 of panel k1 (kb columns), pre-solve values in T[c][r] (LDS): L = T W, stored to the
// front — k_trsm's arithmetic (same products, same MFMA order).  One 4-k-step group at a time with
// scheduling barriers: unconstrained, the scheduler hoists every load and k_update spills.
__device__ __forceinline__ void tile_trsm(const double (*T)[DP], double *F, int m, int k1, int kb, int r0,
                                          const double *W) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rb = (w & 1) * 32, cb = (w >> 1) * 32;
    const int kl = lane >> 4, il = lane & 15;
    const int kb4 = (kb + 3) & ~3;
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int grp = 0; grp < 4; grp++) {
        if (16 * grp >= kb4) break;
        double p0[4], p1[4], q0[4], q1[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int kk = 16 * grp + 4 * u + kl;
            p0[u] = ld_coherent(W + kk * 64 + cb + il);
            p1[u] = ld_coherent(W + kk * 64 + cb + 16 + il);
            q0[u] = T[kk][rb + il];
            q1[u] = T[kk][rb + 16 + il];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (16 * grp + 4 * u < kb4) {
                acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0[u], q0[u], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0[u], q1[u], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1[u], q0[u], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1[u], q1[u], acc[1][1], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int c = cb + 16 * a + kl + 4 * g, r = rb + 16 * b + il;
                if (c < kb && r0 + r < m) F[(int64_t)(k1 + c) * m + r0 + r] = acc[a][b][g];
            }
}

// the first panel of every front of a level (later panels are factored by the update launch that
// finishes their diagonal tile, see k_update); tasks past ndiag are that panel's row tiles (fused TRSM)
// TAIL: tasks past ndiag are fused-TRSM tiles (separate instantiation, as k_update's)
template <bool TAIL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TAIL ? 1 : 4))) k_diag(int ntask, int ndiag, const int32_t *__restrict__ tasks, const FrontDev fd,
                                              double *__restrict__ arena, double *__restrict__ inv,
                                              int *__restrict__ flag, int *__restrict__ pflag, double *__restrict__ wbuf,
                                              int epoch, const LaneOff lo) {
    __shared__ double S[64][DP];
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; flag += blockIdx.y; pflag += blockIdx.y * lo.pflag;
    if (wbuf) wbuf += blockIdx.y * lo.pflag * 4096;
    const int f = tasks[3 * t], k0 = tasks[3 * t + 1], r0 = tasks[3 * t + 2];
    const int m = fd.m[f], s = fd.s[f];
    double *F = arena + fd.arena_off[f];
    const int pid = fd.panel_off[f] + k0 / 64;
    if (t < ndiag) {
        diag_panel_v2(F, m, s, k0, inv + fd.inv_off[f] + (int64_t)(k0 / 64) * 4096, S, flag, TAIL);
        if (TAIL) publish_panel(S, min(64, s - k0), wbuf + (int64_t)pid * 4096, pflag + pid, epoch);
        return;
    }
    if (!TAIL) return;
    const int kb = min(64, s - k0);
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        v[q] = (c < kb && r0 + r < m) ? F[(int64_t)(k0 + c) * m + r0 + r] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        S[c][r] = v[q];
    }
    wait_panel(pflag + pid, epoch, flag);
    tile_trsm(S, F, m, k0, kb, r0, wbuf + (int64_t)pid * 4096);
}

// f64 MFMA tile: C(64x64) = sum_k P[k][c] Q[k][r], P/Q k-major in LDS ([k][index]); wave w owns the
// 32x32 quadrant (rows (w&1)*32, cols (w>>1)*32) as 2x2 v_mfma_f64_16x16x4 tiles.  The MFMA A operand
// is indexed by the column c and B by the row r, so the accumulator's lane&15 runs along rows r:
// 16 consecutive doubles per store of the column-major front.  acc[a][b][reg]: column
// cb + 16a + (lane>>4) + 4 reg, row rb + 16b + (lane&15).
constexpr int LDP = 66;

__device__ __forceinline__ void mfma_tile(const double (*P)[LDP], const double (*Q)[LDP], int kb4, dbl4 acc[2][2]) {
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int rb = (w & 1) * 32, cb = (w >> 1) * 32;
    int kl = lane >> 4, il = lane & 15;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < kb4; k += 4) {
        double p0 = P[k + kl][cb + il], p1 = P[k + kl][cb + 16 + il];
        double q0 = Q[k + kl][rb + il], q1 = Q[k + kl][rb + 16 + il];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q1, acc[1][1], 0, 0, 0);
    }
}

// rows r0..r0+63 below the panel: L_r = F_r L11^{-T} D^{-1}  (GEMM with the panel inverse).
// The inverse (scaled by 1/d_c) is staged once in LDS (shared by the 4 waves); each wave's row
// operands come straight from the front, all issued before the MFMA chain.
__global__ void __launch_bounds__(256) k_trsm(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                              double *__restrict__ arena, const double *__restrict__ inv,
                                              const LaneOff lo) {
    __shared__ double Ps[64][LDP];   // Ps[k][c] = Linv[c][k] / d_c
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv;
    int f = tasks[3 * t], k0 = tasks[3 * t + 1], r0 = tasks[3 * t + 2];
    int m = fd.m[f], s = fd.s[f];
    int kb = min(64, s - k0), kb4 = (kb + 3) & ~3;
    double *F = arena + fd.arena_off[f];
    const double *Li = inv + fd.inv_off[f] + (int64_t)(k0 / 64) * 4096;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rb = (w & 1) * 32, cb = (w >> 1) * 32;
    const int kl = lane >> 4, il = lane & 15;
    // row operands of this wave: rows r0 + rb + il (+16), columns k0 + 4j + kl
    const bool q0ok = r0 + rb + il < m, q1ok = r0 + rb + 16 + il < m;
    double q0v[16], q1v[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int k = 4 * j + kl;
        const double *col = F + (int64_t)(k0 + k) * m + r0 + rb + il;
        q0v[j] = (k < kb && q0ok) ? col[0] : 0.0;
        q1v[j] = (k < kb && q1ok) ? col[16] : 0.0;
    }
    {
        const int c = threadIdx.x & 63, kq = threadIdx.x >> 6;
        const double rdc = (c < kb) ? 1.0 / F[(int64_t)(k0 + c) * m + k0 + c] : 0.0;
        double pv[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            int k = kq + 4 * q;
            pv[q] = (k < kb && c < kb) ? Li[(int64_t)k * kb + c] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 16; q++) Ps[kq + 4 * q][c] = pv[q] * rdc;
    }
    __syncthreads();
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if (4 * j < kb4) {
            const double p0 = Ps[4 * j + kl][cb + il], p1 = Ps[4 * j + kl][cb + 16 + il];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q0v[j], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q1v[j], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q0v[j], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q1v[j], acc[1][1], 0, 0, 0);
        }
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                int c = cb + 16 * a + kl + 4 * g, r = rb + 16 * b + il;
                if (c < kb && r0 + r < m) F[(int64_t)(k0 + c) * m + r0 + r] = acc[a][b][g];
            }
}

// XCD-aware task order: the 8 XCDs receive blockIdx round-robin, so block b runs task
// (b % 8) * ceil(n/8) + b / 8 — each XCD works through one contiguous slice of the task list (nearby
// tiles share panel rows in that XCD's L2).  The grid is rounded up to a multiple of 8.
__device__ __forceinline__ int xcd_task(int ntask) {
    int per = (ntask + 7) >> 3;
    return (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
}

// trailing update of tile (ti, tj): C -= L_i D L_j^T over L columns [kA, kA + K),
// K = min(kmax, s - kA) (one 64-panel for the inner updates, a whole outer block otherwise).
// Operands are staged through LDS one k-chunk (16 columns) at a time: thread t loads column
// t / 16 of the chunk, rows 4 (t % 16) .. +3 of both 64-row panels (L_j scaled by d_k once, at
// staging) with 16-byte loads — one d load + four 16-byte loads per thread per 16 k instead of 20
// scalar loads per lane — double-buffered (chunk c+1's loads in flight during chunk c's MFMAs), one
// barrier per chunk; each wave reads its 32x32 quadrant's fragments from LDS.  Same products and
// summation order as the register-streaming kernel it replaced (bit-identical), 1.3-1.5x faster
// (tools/micro/upd_bench.hip: 30 -> 42 TF/s on 2000-row fronts, K = 256).  The staging buffers
// alias the fused panel factorization's LDS.
constexpr int kUpdKC = 16;                 // k columns per staged chunk
// two consecutive column entries p[0..1] of which nvalid remain in the column (16-byte load when
// aligned; odd m gives odd column starts)
__device__ __forceinline__ dbl2 ld2(const double *p, int nvalid) {
    if (nvalid >= 2 && ((uintptr_t)p & 15) == 0) return *(const dbl2 *)p;
    return dbl2{nvalid > 0 ? p[0] : 0.0, nvalid > 1 ? p[1] : 0.0};
}
constexpr int kUpdLQ = 64 + 4;             // padded staged column (doubles)
union UpdSmem {
    struct { double P[2][kUpdKC][kUpdLQ], Q[2][kUpdKC][kUpdLQ]; } st;
    double S[64][DP];
};
#ifndef DEFTRI_UPD_WPE
#define DEFTRI_UPD_WPE 4   // waves per EU of k_update (tuning knob)
#endif

// TAIL: the launch carries fused-TRSM tail tiles (a separate instantiation: the tail path's registers
// would otherwise spill the plain launches' main loop).  F32 (deftri_set_factor_precision, the
// fp32-vs-fp64 sweep): the products run on v_mfma_f32_16x16x4 (operands rounded to fp32 at the
// fragment read, fp32 accumulation over the launch's K columns, the result subtracted from the fp64
// C tile); its accumulator's row map differs from the f64 instruction's (row = 4 (lane >> 4) + reg).
typedef float flt4 __attribute__((ext_vector_type(4)));
template <bool TAIL, bool F32 = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEFTRI_UPD_WPE))) k_update(int ntask, int ntail, const int32_t *__restrict__ tasks, int kA, int kmax,
                                                int inner, const FrontDev fd, double *__restrict__ arena,
                                                double *__restrict__ inv, int *__restrict__ flag,
                                                int *__restrict__ pflag, double *__restrict__ wbuf, int epoch,
                                                const LaneOff lo) {
    __shared__ UpdSmem sm;
    int t = xcd_task(ntask);
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; flag += blockIdx.y; pflag += blockIdx.y * lo.pflag;
    if (wbuf) wbuf += blockIdx.y * lo.pflag * 4096;
    int f = tasks[3 * t], ti = tasks[3 * t + 1], tj = tasks[3 * t + 2];
    int m = fd.m[f], s = fd.s[f];
    int K = min(kmax, s - kA);
    // inner updates stop at the end of the outer block (own columns): a tile straddling it must not
    // touch the columns the outer update will cover
    int cend = inner == 1 ? min(s, (kA / kOuter + 1) * kOuter) : inner == 2 ? min(s, (kA / kOuter + 2) * kOuter)
             : inner == 3 ? s : m;
    double *F = arena + fd.arena_off[f];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rb = ti + (w & 1) * 32, cb = tj + (w >> 1) * 32;
    const int kl = lane >> 4, il = lane & 15;
    const int qr = (w & 1) * 32, pc = (w >> 1) * 32;     // quadrant offsets inside the staged panels
    // staging role: column sk of the chunk, rows sr..sr+3 of both panels
    const int sk = tid >> 4, sr = (tid & 15) * 4;
    const int pn = m - (tj + sr), qn = m - (ti + sr);   // rows left in the column from the staged rows
    dbl2 pv0, pv1, qv0, qv1;
    double dv;
    auto stage_load = [&](int c0) {
        const int kk = c0 + sk;
        const bool ok = kk < K;
        const double *col = F + (int64_t)(kA + kk) * m;
        dv = ok ? col[kA + kk] : 0.0;
        pv0 = ld2(col + tj + sr, ok ? pn : 0);
        pv1 = ld2(col + tj + sr + 2, ok ? pn - 2 : 0);
        qv0 = ld2(col + ti + sr, ok ? qn : 0);
        qv1 = ld2(col + ti + sr + 2, ok ? qn - 2 : 0);
    };
    auto stage_store = [&](int buf) {
        *(dbl2 *)&sm.st.P[buf][sk][sr] = pv0 * dv;
        *(dbl2 *)&sm.st.P[buf][sk][sr + 2] = pv1 * dv;
        *(dbl2 *)&sm.st.Q[buf][sk][sr] = qv0;
        *(dbl2 *)&sm.st.Q[buf][sk][sr + 2] = qv1;
    };
    stage_load(0);
    // C tile: acc layout (a, b, g) -> column cb + ccol(a, g), row rb + 16b + il.  Plain launches
    // fetch it before the K loop; TAIL launches during the last chunk (registers)
    auto ccol = [&](int a, int g) { return 16 * a + (F32 ? 4 * kl + g : kl + 4 * g); };
    double cv[2][2][4];
    auto load_c = [&]() {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    int c = cb + ccol(a, g), r = rb + 16 * b + il;
                    cv[a][b][g] = (c < m && r < m) ? F[(int64_t)c * m + r] : 0.0;
                }
    };
    if (!TAIL) load_c();
    dbl4 acc[2][2];
    flt4 accf[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) { acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0}; accf[a][b] = flt4{0.f, 0.f, 0.f, 0.f}; }
    stage_store(0);
    __syncthreads();
    auto mfma_chunk = [&](int buf) {
#pragma unroll
        for (int k4 = 0; k4 < kUpdKC; k4 += 4) {
            const double p0 = sm.st.P[buf][k4 + kl][pc + il], p1 = sm.st.P[buf][k4 + kl][pc + 16 + il];
            const double q0 = sm.st.Q[buf][k4 + kl][qr + il], q1 = sm.st.Q[buf][k4 + kl][qr + 16 + il];
            if constexpr (F32) {
                const float p0f = (float)p0, p1f = (float)p1, q0f = (float)q0, q1f = (float)q1;
                accf[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p0f, q0f, accf[0][0], 0, 0, 0);
                accf[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p0f, q1f, accf[0][1], 0, 0, 0);
                accf[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p1f, q0f, accf[1][0], 0, 0, 0);
                accf[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p1f, q1f, accf[1][1], 0, 0, 0);
            } else {
                acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q1, acc[1][1], 0, 0, 0);
            }
        }
    };
    const int nch = (K + kUpdKC - 1) / kUpdKC;
    if constexpr (TAIL) {
        for (int c = 0; c + 1 < nch; c++) {
            stage_load((c + 1) * kUpdKC);
            mfma_chunk(c & 1);
            stage_store((c + 1) & 1);
            __syncthreads();
        }
        load_c();
        mfma_chunk((nch - 1) & 1);
        __syncthreads();
    } else {
        for (int c = 0; c < nch; c++) {
            const int buf = c & 1;
            if (c + 1 < nch) stage_load((c + 1) * kUpdKC);
            mfma_chunk(buf);
            if (c + 1 < nch) stage_store(buf ^ 1);
            __syncthreads();
        }
    }
    if constexpr (F32) {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) acc[a][b][g] = (double)accf[a][b][g];
    }
    // fused TRSM tile (i > k1, k1) of the panel this launch factors: the updated tile goes to LDS
    // (columns past the panel, if any, are stored as plain update results), then, once the panel's
    // factorization is published, its rows are solved in place
    if (TAIL && t >= ntask - ntail) {
        const int k1 = kA + K, kb = min(64, s - k1);
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int cl = cb - tj + ccol(a, g), rl = rb - ti + 16 * b + il;
                    const double v = cv[a][b][g] - acc[a][b][g];
                    if (cl < kb) sm.S[cl][rl] = v;
                    else if (tj + cl < cend && ti + rl < m) F[(int64_t)(tj + cl) * m + ti + rl] = v;
                }
        const int pid = fd.panel_off[f] + k1 / 64;
        wait_panel(pflag + pid, epoch, flag);
        tile_trsm(sm.S, F, m, k1, kb, ti, wbuf + (int64_t)pid * 4096);
        return;
    }
    // the front's last trailing update produces its final contribution block: a direct front adds
    // it straight into the parent (lower triangle; bmap is monotone, each parent entry has one writer
    // in this launch) instead of leaving it for an extend-add
    if (!inner && kA + K == s && fd.direct[f]) {
        const int p = fd.parent[f], mp = fd.m[p];
        const int32_t *bm = fd.bmap + fd.bmap_off[f] - s;
        double *Fp = arena + fd.arena_off[p];
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    int c = cb + ccol(a, g), r = rb + 16 * b + il;
                    if (c < m && r < m && r >= c) Fp[(int64_t)bm[c] * mp + bm[r]] += cv[a][b][g] - acc[a][b][g];
                }
    } else if (!TAIL && ti == tj && ti == kA + K && s > kA + K) {
        // the tile that carries the next panel's factorization: its kb x kb diagonal block goes
        // straight into the factorization's LDS layout (lower triangle, zero upper, identity
        // padding), the rest of the tile to the front
        const int kb = min(64, s - (kA + K));
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int cl = cb - tj + ccol(a, g), rl = rb - ti + 16 * b + il;
                    const double v = cv[a][b][g] - acc[a][b][g];
                    if (cl < kb && rl < kb) {
                        sm.S[rl][cl] = (rl >= cl) ? v : 0.0;
                    } else {
                        sm.S[rl][cl] = (rl == cl) ? 1.0 : 0.0;
                        if (tj + cl < cend && ti + rl < m) F[(int64_t)(tj + cl) * m + ti + rl] = v;
                    }
                }
    } else {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    int c = cb + ccol(a, g), r = rb + 16 * b + il;
                    if (c < cend && r < m) F[(int64_t)c * m + r] = cv[a][b][g] - acc[a][b][g];
                }
    }
    // the diagonal tile of the next panel is final once this tile is: factor it here (its LDL^T
    // overlaps the rest of this launch instead of costing its own launch on the critical path;
    // these tiles are first in the task list)
    int k1 = kA + K;
    if (ti == tj && ti == k1 && s > k1) {
        __syncthreads();
        __threadfence_block();
        diag_panel_v2(F, m, s, k1, inv + fd.inv_off[f] + (int64_t)(k1 / 64) * 4096, sm.S, flag, TAIL, !TAIL);
        if (TAIL) {
            const int pid = fd.panel_off[f] + k1 / 64;
            publish_panel(sm.S, min(64, s - k1), wbuf + (int64_t)pid * 4096, pflag + pid, epoch);
        }
    }
}

// ------------------------------------------------------------------------------------------
// substitution
// ------------------------------------------------------------------------------------------
// forward gather: v = [rhs of own rows; 0 on boundary rows] + the children's update vectors (slot 0
// then slot 1: fixed order)
// (point-sharded plan: the rank's top front starts its boundary rows from the rank's partial b of
// those remote vertices, `bpart`; they travel up with the forward-update vector)
__global__ void __launch_bounds__(256) k_fwd_gather(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                    const double *__restrict__ rhs, const double *__restrict__ bpart,
                                                    double *__restrict__ vec, const LaneOff lo) {
    int t = blockIdx.x;
    if (t >= ntask) return;
    vec += blockIdx.y * lo.vec;
    int f = tasks[3 * t];
    int m = fd.m[f], s = fd.s[f];
    const int32_t *rows = fd.rows + fd.rows_off[f];
    double *v = vec + fd.vec_off[f];
    const bool inject = bpart != nullptr && fd.rhs_bnd[f] != 0;
    for (int r = threadIdx.x; r < m; r += blockDim.x) v[r] = (r < s) ? rhs[rows[r]] : (inject ? bpart[rows[r]] : 0.0);
    __syncthreads();
    for (int slot = 0; slot < fd.nchild[f]; slot++) {
        int c = (slot == 0) ? fd.child0[f] : fd.child1[f];
        int uc = fd.m[c] - fd.s[c];
        const double *vc = vec + fd.vec_off[c] + fd.s[c];
        const int32_t *bm = fd.bmap + fd.bmap_off[c];
        for (int i = threadIdx.x; i < uc; i += blockDim.x) v[bm[i]] += vc[i];
        __syncthreads();
    }
}

// forward panel step (front f, panel k0): every task forms y_p = L_pp^{-1} v_p from the stored
// panel inverse (64x64 GEMV from L2); task r0 == k0 publishes y_p, tasks r0 > k0 update the 64 rows
// r0.. below the panel: v_r -= L[r, panel] y_p.  All global loads of a task are issued up front
// (these launches are latency-bound: one load round instead of three).
__global__ void __launch_bounds__(256) k_fwd_step(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                  const double *__restrict__ arena, const double *__restrict__ inv,
                                                  double *__restrict__ vec, double *__restrict__ yvec,
                                                  const LaneOff lo) {
    __shared__ double vs[64];
    __shared__ double ys[64];
    __shared__ double red[4][64];
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; vec += blockIdx.y * lo.vec; yvec += blockIdx.y * lo.vec;
    int f = tasks[3 * t], k0 = tasks[3 * t + 1], r0 = tasks[3 * t + 2];
    int m = fd.m[f], s = fd.s[f];
    int kb = min(64, s - k0);
    const double *F = arena + fd.arena_off[f];
    const double *Li = inv + fd.inv_off[f] + (int64_t)(k0 / 64) * 4096;
    double *v = vec + fd.vec_off[f];
    const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int r = r0 + lane;
    const bool below = r0 != k0 && r < m;
    double vk = (threadIdx.x < kb) ? v[k0 + threadIdx.x] : 0.0;
    double li[16], fv[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int j = part + 4 * q;
        li[q] = (j <= lane && lane < kb) ? Li[(int64_t)j * kb + lane] : 0.0;
        fv[q] = (below && j < kb) ? F[(int64_t)(k0 + j) * m + r] : 0.0;
    }
    if (threadIdx.x < 64) vs[threadIdx.x] = vk;
    __syncthreads();
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += li[q] * vs[part + 4 * q];
    red[part][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64) ys[lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
    if (r0 == k0) {
        if (threadIdx.x < kb) yvec[fd.vec_off[f] + k0 + threadIdx.x] = ys[threadIdx.x];
        return;
    }
    acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += fv[q] * ys[part + 4 * q];
    red[part][lane] = acc;
    __syncthreads();
    if (part == 0 && r < m) v[r] -= (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// backward init (front f, own columns c0..c0+15): w_c = y_c / d_c - sum_{i >= s} L[i][c] x[rows[i]].
// The boundary solution x_B (gathered through rows[]) is staged once in LDS for the task's 16
// columns; wave w accumulates its 4 columns together (4 independent coalesced column streams).
// Per column the lane-strided order and the shuffle tree are the single-column ones.
constexpr int kBwdStage = 4096;
__global__ void __launch_bounds__(256) k_bwd_init(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                  const double *__restrict__ arena, const double *__restrict__ x,
                                                  const double *__restrict__ yvec, double *__restrict__ vec,
                                                  const LaneOff lo) {
    __shared__ double xb[kBwdStage];
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; x += blockIdx.y * lo.x; yvec += blockIdx.y * lo.vec; vec += blockIdx.y * lo.vec;
    int f = tasks[3 * t], c0 = tasks[3 * t + 1];
    int m = fd.m[f], s = fd.s[f];
    const double *F = arena + fd.arena_off[f];
    const int32_t *rows = fd.rows + fd.rows_off[f];
    int64_t vo = fd.vec_off[f];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c1 = min(c0 + kBwdCols, s);
    const int u = m - s;
    const bool staged = u <= kBwdStage;
    if (staged) {
        for (int i = threadIdx.x; i < u; i += 256) xb[i] = x[rows[s + i]];
        __syncthreads();
    }
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const double *col[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = c0 + wv + 4 * k;
        ok[k] = c < c1;
        col[k] = F + (int64_t)(ok[k] ? c : c0) * m + s;
    }
    // 4 row strides per round: 16 column loads in flight per lane, accumulated in row order
    for (int i0 = lane; i0 < u; i0 += 256) {
        double xv[4], lv[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = i0 + 64 * j;
            const bool in = i < u;
            xv[j] = in ? (staged ? xb[i] : x[rows[s + i]]) : 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) lv[k][j] = (in && ok[k]) ? col[k][i] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (i0 + 64 * j < u && ok[k]) acc[k] += lv[k][j] * xv[j];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_down(acc[k], off);
        const int c = c0 + wv + 4 * k;
        if (lane == 0 && ok[k]) vec[vo + c] = yvec[vo + c] / F[(int64_t)c * m + c] - acc[k];
    }
}

// backward panel step (front f, panel k0; panels run in descending order): every task forms
// x_p = L_pp^{-T} w_p from the panel inverse; task q0 == k0 scatters x_p to the global solution,
// tasks q0 < k0 update w[q0..q0+63] -= L[panel rows, q]^T x_p.  Thread (lane, part) owns output
// lane and every 4th term; loads issued up front, partial sums reduced through LDS in fixed order.
__global__ void __launch_bounds__(256) k_bwd_step(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                  const double *__restrict__ arena, const double *__restrict__ inv,
                                                  double *__restrict__ vec, double *__restrict__ x,
                                                  const LaneOff lo) {
    __shared__ double ws[64];
    __shared__ double xs[64];
    __shared__ double red[4][64];
    int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; vec += blockIdx.y * lo.vec; x += blockIdx.y * lo.x;
    int f = tasks[3 * t], k0 = tasks[3 * t + 1], q0 = tasks[3 * t + 2];
    int m = fd.m[f], s = fd.s[f];
    int kb = min(64, s - k0);
    const double *F = arena + fd.arena_off[f];
    const double *Li = inv + fd.inv_off[f] + (int64_t)(k0 / 64) * 4096;
    double *w = vec + fd.vec_off[f];
    const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
    const bool own = q0 == k0;
    double wk = (threadIdx.x < kb) ? w[k0 + threadIdx.x] : 0.0;
    double lv[16], fv[16];
    const double *Fq = F + (int64_t)(q0 + lane) * m + k0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int j = part + 4 * q;
        lv[q] = (lane < kb && j < kb && j >= lane) ? Li[(int64_t)lane * kb + j] : 0.0;   // Linv[j][lane]
        fv[q] = (!own && j < kb) ? Fq[j] : 0.0;                                         // L[k0+j][q0+lane]
    }
    if (threadIdx.x < 64) ws[threadIdx.x] = wk;
    __syncthreads();
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += lv[q] * ws[part + 4 * q];
    red[part][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64) xs[lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
    if (own) {
        const int32_t *rows = fd.rows + fd.rows_off[f];
        if (threadIdx.x < kb) x[rows[k0 + threadIdx.x]] = xs[threadIdx.x];
        return;
    }
    acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += fv[q] * xs[part + 4 * q];
    red[part][lane] = acc;
    __syncthreads();
    if (part == 0) w[q0 + lane] -= (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// ---- chained substitution: one launch per level and direction.  The per-panel launches above
// become cross-workgroup hand-offs inside one launch (the protocol of the fused TRSM: agent-coherent
// stores of the panel's 64-entry result, an epoch flag, bounded polls).  A workgroup only waits on
// workgroups with smaller indices (forward: row tiles in ascending order, backward: column tiles in
// descending order), so in-order dispatch guarantees progress.  Per row / column the arithmetic is
// k_fwd_step's / k_bwd_step's (same products, same reduction order): bit-identical results.
__device__ __forceinline__ void poll_flag(const int *pf, int epoch, int *flag) {
    if (threadIdx.x == 0) {
        int it = 0;
        while (ld_sc1(pf) != epoch) {
            if (++it > kSpinLimit) { atomicOr(flag, kStatusWaitTimeout); break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}
__device__ __forceinline__ void raise_flag(int *pf, int epoch) {
    __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0): this thread's coherent stores are complete
    __syncthreads();
    if (threadIdx.x == 0) st_sc1(pf, epoch);
}

// forward: task (front f, rows r0..r0+63).  Panels k0 < min(r0, s): wait for y_k0, v_rows -= L y;
// then, if r0 < s, the tile's own panel: y = L_pp^{-1} v_p, published (coherent) in yvec, and the
// tile's rows below the panel (r >= s when the panel is partial) take its update too.
__global__ void __launch_bounds__(256) k_fwd_chain(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                   const double *__restrict__ arena, const double *__restrict__ inv,
                                                   double *__restrict__ vec, double *__restrict__ yvec,
                                                   int *__restrict__ pflag, int epoch, int *__restrict__ flag,
                                                   const LaneOff lo) {
    __shared__ double vs[64];
    __shared__ double ys[64];
    __shared__ double red[4][64];
    const int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; vec += blockIdx.y * lo.vec; yvec += blockIdx.y * lo.vec;
    pflag += blockIdx.y * lo.pflag; flag += blockIdx.y;
    const int f = tasks[3 * t], r0 = tasks[3 * t + 1];
    const int m = fd.m[f], s = fd.s[f];
    const double *F = arena + fd.arena_off[f];
    double *v = vec + fd.vec_off[f];
    double *yv = yvec + fd.vec_off[f];
    const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int r = r0 + lane;
    double vr = (part == 0 && r < m) ? v[r] : 0.0;
    const int kend = min(r0, s);
    for (int k0 = 0; k0 < kend; k0 += 64) {
        const int kb = min(64, s - k0);
        double fv[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = part + 4 * q;
            fv[q] = (r < m && j < kb) ? F[(int64_t)(k0 + j) * m + r] : 0.0;    // issued before the wait
        }
        poll_flag(pflag + fd.panel_off[f] + k0 / 64, epoch, flag);
        if (threadIdx.x < 64) ys[threadIdx.x] = threadIdx.x < kb ? ld_coherent(yv + k0 + threadIdx.x) : 0.0;
        __syncthreads();
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) acc += fv[q] * ys[part + 4 * q];
        red[part][lane] = acc;
        __syncthreads();
        if (part == 0) vr -= (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        __syncthreads();
    }
    if (r0 < s) {
        const int kb = min(64, s - r0);
        const double *Li = inv + fd.inv_off[f] + (int64_t)(r0 / 64) * 4096;
        double li[16], fv[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = part + 4 * q;
            li[q] = (j <= lane && lane < kb) ? Li[(int64_t)j * kb + lane] : 0.0;
            fv[q] = (lane >= kb && r < m && j < kb) ? F[(int64_t)(r0 + j) * m + r] : 0.0;
        }
        if (part == 0) vs[lane] = lane < kb ? vr : 0.0;
        __syncthreads();
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) acc += li[q] * vs[part + 4 * q];
        red[part][lane] = acc;
        __syncthreads();
        if (threadIdx.x < 64) ys[lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        __syncthreads();
        if (threadIdx.x < kb) st_coherent(yv + r0 + threadIdx.x, ys[threadIdx.x]);
        raise_flag(pflag + fd.panel_off[f] + r0 / 64, epoch);
        if (kb < 64) {                                     // rows s.. of this tile: this panel's update
            acc = 0.0;
#pragma unroll
            for (int q = 0; q < 16; q++) acc += fv[q] * ys[part + 4 * q];
            red[part][lane] = acc;
            __syncthreads();
            if (part == 0 && lane >= kb) vr -= (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        }
    }
    if (part == 0 && r < m && r >= s) v[r] = vr;           // the contribution rows the parent gathers
}

// backward: task (front f, own columns c0..c0+63), after k_bwd_init.  Panels k0 > c0, descending:
// wait for x_k0, w_cols -= L[panel rows, cols]^T x; then the tile's own panel: x = L_pp^{-T} w_p,
// published (coherent) in yvec (whose y this level's k_bwd_init has consumed) and scattered to x.
__global__ void __launch_bounds__(256) k_bwd_chain(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                   const double *__restrict__ arena, const double *__restrict__ inv,
                                                   double *__restrict__ vec, double *__restrict__ yvec,
                                                   double *__restrict__ x, int *__restrict__ pflag, int epoch,
                                                   int *__restrict__ flag, const LaneOff lo) {
    __shared__ double ws[64];
    __shared__ double xs[64];
    __shared__ double red[4][64];
    const int t = blockIdx.x;
    if (t >= ntask) return;
    arena += blockIdx.y * lo.arena; inv += blockIdx.y * lo.inv; vec += blockIdx.y * lo.vec; yvec += blockIdx.y * lo.vec;
    x += blockIdx.y * lo.x; pflag += blockIdx.y * lo.pflag; flag += blockIdx.y;
    const int f = tasks[3 * t], c0 = tasks[3 * t + 1];
    const int m = fd.m[f], s = fd.s[f];
    const double *F = arena + fd.arena_off[f];
    const double *w = vec + fd.vec_off[f];
    double *yv = yvec + fd.vec_off[f];
    const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int kbq = min(64, s - c0);
    double wq = (part == 0 && lane < kbq) ? w[c0 + lane] : 0.0;
    const double *Fq = F + (int64_t)(c0 + lane) * m;
    for (int k0 = ((s - 1) / 64) * 64; k0 > c0; k0 -= 64) {
        const int kb = min(64, s - k0);
        double fv[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = part + 4 * q;
            fv[q] = (j < kb) ? Fq[k0 + j] : 0.0;                            // L[k0+j][c0+lane]
        }
        poll_flag(pflag + fd.panel_off[f] + k0 / 64, epoch, flag);
        if (threadIdx.x < 64) xs[threadIdx.x] = threadIdx.x < kb ? ld_coherent(yv + k0 + threadIdx.x) : 0.0;
        __syncthreads();
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) acc += fv[q] * xs[part + 4 * q];
        red[part][lane] = acc;
        __syncthreads();
        if (part == 0) wq -= (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        __syncthreads();
    }
    const double *Li = inv + fd.inv_off[f] + (int64_t)(c0 / 64) * 4096;
    double lv[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int j = part + 4 * q;
        lv[q] = (lane < kbq && j < kbq && j >= lane) ? Li[(int64_t)lane * kbq + j] : 0.0;   // Linv[j][lane]
    }
    if (part == 0) ws[lane] = wq;
    __syncthreads();
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += lv[q] * ws[part + 4 * q];
    red[part][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64) xs[lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
    if (threadIdx.x < kbq) {
        st_coherent(yv + c0 + threadIdx.x, xs[threadIdx.x]);
        x[fd.rows[fd.rows_off[f] + c0 + threadIdx.x]] = xs[threadIdx.x];
    }
    raise_flag(pflag + fd.panel_off[f] + c0 / 64, epoch);
}

// ------------------------------------------------------------------------------------------
// state update, reductions
// ------------------------------------------------------------------------------------------
// skipped when the factorization flagged a zero pivot (the trial is rejected and the state restored)
__global__ void k_update_state(int P, int S, int Q, const double *__restrict__ dx, double *__restrict__ points,
                               double *__restrict__ scales, double *__restrict__ tg, const int *__restrict__ flag,
                               const int *gate) {
#pragma clang fp contract(off)
    int i = TID;
    if (flag && *flag) return;
    if (gate && !*gate) return;
    int64_t pbase = 6 * (int64_t)Q + S;
    if (i < P) {
        points[3 * (int64_t)i] += dx[pbase + 3 * (int64_t)i];
        points[3 * (int64_t)i + 1] += dx[pbase + 3 * (int64_t)i + 1];
        points[3 * (int64_t)i + 2] += dx[pbase + 3 * (int64_t)i + 2];
    }
    if (i < S) scales[i] += dx[6 * (int64_t)Q + i];
    if (i < Q) {
        double u[6];
        for (int k = 0; k < 6; k++) u[k] = dx[6 * (int64_t)i + k];
        SE3 T = se3_load(tg + 7 * i);
        SE3 Ex = se3_exp(u);
        SE3 Tn = se3_mul(Ex, T);
        se3_store(Tn, tg + 7 * i);
    }
}

__global__ void k_update_state_bak(int P, int S, int Q, const double *__restrict__ dx, double *__restrict__ points,
                                   double *__restrict__ scales, double *__restrict__ tg, double *__restrict__ pb,
                                   double *__restrict__ sb, double *__restrict__ tb, int restore) {
#pragma clang fp contract(off)
    const int i = TID;
    const int64_t pbase = 6 * (int64_t)Q + S;
    if (i < P) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const int64_t k = 3 * (int64_t)i + c;
            const double base = restore ? pb[k] : points[k];
            if (!restore) pb[k] = base;
            points[k] = base + dx[pbase + k];
        }
    }
    if (i < S) {
        const double base = restore ? sb[i] : scales[i];
        if (!restore) sb[i] = base;
        scales[i] = base + dx[6 * (int64_t)Q + i];
    }
    if (i < Q) {
        double u[6];
        for (int k = 0; k < 6; k++) u[k] = dx[6 * (int64_t)i + k];
        double *src = restore ? tb + 7 * i : tg + 7 * i;
        SE3 T = se3_load(src);
        if (!restore)
            for (int k = 0; k < 7; k++) tb[7 * i + k] = tg[7 * i + k];
        SE3 Ex = se3_exp(u);
        SE3 Tn = se3_mul(Ex, T);
        se3_store(Tn, tg + 7 * i);
    }
}

// a trial's prologue in one launch: the state backup (push_state's three copies) — or, after a
// rejected trial, its restore from the backup (pop_state's) — the zero-pivot flag and the PCG records
// cleared (two fills); grid-stride over the longest of them
__global__ void __launch_bounds__(256) k_trial_begin(int P, int S, int Q, const double *__restrict__ src_points,
                                                     const double *__restrict__ src_scales, const double *__restrict__ src_tg,
                                                     double *__restrict__ dst_points, double *__restrict__ dst_scales,
                                                     double *__restrict__ dst_tg, int *__restrict__ flag,
                                                     double *__restrict__ zero, int64_t nzero, int64_t n) {
    for (int64_t i = TID; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < 3 * (int64_t)P) dst_points[i] = src_points[i];
        if (i < S) dst_scales[i] = src_scales[i];
        if (i < 7 * (int64_t)Q) dst_tg[i] = src_tg[i];
        if (i < nzero) zero[i] = 0.0;
        if (i == 0) *flag = 0;
    }
}

// the device-driven LM's prologue (kernels.h LmState): k_trial_begin's work in the direction the last
// decision chose, gated; thread 0 folds the linearization that ran before it into the state
__global__ void __launch_bounds__(256) k_trial_begin_dev(int P, int S, int Q, double *__restrict__ points,
                                                         double *__restrict__ scales, double *__restrict__ tg,
                                                         double *__restrict__ points_bak, double *__restrict__ scales_bak,
                                                         double *__restrict__ tg_bak, int *__restrict__ flag,
                                                         double *__restrict__ zero, int64_t nzero, int64_t n, LmState *lm,
                                                         const double *__restrict__ scal, double tau, double user_lambda) {
    if (!lm->gate_trial) return;
    const bool restore = lm->restore != 0;
    if (TID == 0 && lm->gate_lin) {
        lm->cur = scal[0];                       // currentChi of the new linearization point
        if (lm->it == 0) {                       // g2o: lambda = tau * max diag H at iteration 0
            lm->lam = user_lambda > 0 ? user_lambda : tau * scal[2];
            lm->ni = 2.0;
        }
    }
    const double *sp = restore ? points_bak : points, *ss = restore ? scales_bak : scales, *stg = restore ? tg_bak : tg;
    double *dp = restore ? points : points_bak, *ds = restore ? scales : scales_bak, *dtg = restore ? tg : tg_bak;
    for (int64_t i = TID; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < 3 * (int64_t)P) dp[i] = sp[i];
        if (i < S) ds[i] = ss[i];
        if (i < 7 * (int64_t)Q) dtg[i] = stg[i];
        if (i < nzero) zero[i] = 0.0;
        if (i == 0) *flag = 0;
    }
}

// the device-driven LM's decision (one thread; spcg_solver.cpp solve_lm_dev's host loop restated)
__global__ void k_lm_decide(LmState *lm, const double *__restrict__ scal, const double *__restrict__ rec,
                            double *__restrict__ chi_it, int32_t *__restrict__ trials_it, int max_report, LmState *snap,
                            int slot) {
    if (threadIdx.x != 0 || !lm->gate_trial) return;
    LmState L = *lm;
    const int st = (int)rec[0];
    if (st == 0) {                               // the step needs more CG iterations than queued: the host's
        L.stop = 3;
        L.stop_slot = slot;
        L.gate_trial = L.gate_lin = 0;
        *lm = L;
        *snap = L;
        return;
    }
    if (st == 5) {                               // kSpTimeout (spcg.h): the merged chain's alpha hand-off timed
        L.stop = 4;                              // out — a scheduling fault, never a rejected trial: no lambda
        L.stop_slot = slot;                      // change, every later slot gated off; the host raises it
        L.gate_trial = L.gate_lin = 0;
        *lm = L;
        *snap = L;
        return;
    }
    const bool solved = st == 1;                 // kSpConverged (spcg.h)
    L.pcg_iterations += (int64_t)rec[1];
    if (solved) { L.pcg_trials++; L.last_its = (int)rec[1]; }
    else L.pcg_fail++;
    const double tempChi = solved ? scal[0] : 1.7976931348623157e308;
    double rho = L.cur - tempChi;
    const double scale = (solved ? scal[1] : 0.0) + 1e-3;
    rho /= scale;
    L.trials_total++;
    bool broke = false;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        const double scaleFactor = fmax(1. / 3., alpha);
        L.lam *= scaleFactor;
        L.ni = 2;
        L.cur = tempChi;
        L.restore = 0;
    } else {
        L.lam *= L.ni;
        L.ni *= 2;
        L.restore = 1;
        L.trials_rejected++;
        broke = !isfinite(L.lam);
    }
    L.q++;
    L.rho = rho;
    L.need_lin = 0;
    if (broke || !(rho < 0 && L.q < L.max_trials)) {     // the iteration's trial loop ends
        if (L.it < max_report) { chi_it[L.it] = L.cur; trials_it[L.it] = L.q; }
        const bool term = L.q == L.max_trials || rho == 0 || !isfinite(L.lam);
        L.it++;
        L.q = 0;
        L.need_lin = 1;
        if (term) { L.stop = 2; L.stop_slot = slot; }
        else if (L.it >= L.n_it) { L.stop = 1; L.stop_slot = slot; }
    }
    L.slot = slot;
    L.gate_trial = L.stop == 0 ? 1 : 0;
    L.gate_lin = (L.gate_trial && L.need_lin) ? 1 : 0;
    *lm = L;
    *snap = L;
}

// a trial's read-back in one launch (in place of two or three copies): the scalars, the zero-pivot
// flag and a PCG record stored straight into pinned host memory, visible to the host once the stream
// is synchronized
// is synchronized (a host spin on a sequence value stored last measured the same as the
// synchronization: 0.846 vs 0.844 ms per C2 trial)
__global__ void k_trial_readback(const double *__restrict__ scal, int ns, const int *__restrict__ flag,
                                 const double *__restrict__ rec, int nrec, double *h_scal, int *h_flag,
                                 double *h_rec) {
    const int t = threadIdx.x;
    if (t < ns) h_scal[t] = scal[t];
    if (t == 0) *h_flag = *flag;
    if (rec && t < nrec) h_rec[t] = rec[t];
}

__global__ void __launch_bounds__(256) k_sum_partial(int64_t n, const double *__restrict__ a,
                                                     const double *__restrict__ b, double lambda, int mode,
                                                     const double *__restrict__ w, double *__restrict__ part) {
    // mode 0: sum a ; 1: sum a*(lambda*a + b) ; 3: sum a*(lambda*w*a + b) (point-sharded: w = 1 on
    // this rank's dofs, so the lambda term counts every dof once over the ranks while b is partial)
    __shared__ double red[256];
    int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    int64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    double acc = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        double v = a[i];
        acc += (mode == 0) ? v : (mode == 1) ? v * (lambda * v + b[i]) : v * (lambda * w[i] * v + b[i]);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// one wave: lane l sums partials l, l+64, ... in order, then a fixed butterfly (deterministic)
__global__ void __launch_bounds__(256) k_sum_multi_partial(const SumJobs J, double *__restrict__ part) {
    const SumJob &jb = J.j[blockIdx.y];
    __shared__ double red[256];
    const int64_t n = jb.n;
    int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    int64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    double acc = 0.0;
    const int mode = jb.mode;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        double v = jb.a[i];
        acc += (mode == 0) ? v : (mode == 1) ? v * (jb.lambda * v + jb.b[i]) : v * (jb.lambda * jb.w[i] * v + jb.b[i]);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

// one wave per job: its parts strided over the lanes, then the butterfly (k_sum_final's order)
// k_sum_multi_partial + k_sum_multi_final in one launch (the same sums in the same order): every
// workgroup publishes its partial with an agent-scope atomic store and takes a ticket; the last one
// forms the totals from the partials (agent-scope loads) and, when rb.h_scal is set, also does
// k_trial_readback's copies into pinned host memory.  *cnt is 0 between launches.
__global__ void __launch_bounds__(256) k_sum_multi_fused(const SumJobs J, double *__restrict__ part, int *cnt,
                                                         const ReadBack rb) {
    if (J.gate && !*J.gate) return;
    const SumJob &jb = J.j[blockIdx.y];
    __shared__ double red[256];
    __shared__ int last;
    const int64_t n = jb.n;
    int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    int64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    double acc = 0.0;
    const int mode = jb.mode;
    const double lam = jb.lambda_dev ? *jb.lambda_dev : jb.lambda;
    // k_sum_multi_partial's strided order (blockDim 256), eight (mode 0) / four elements' loads in
    // flight per step, added in order
    int64_t i = lo + threadIdx.x;
    if (mode == 0) {
        for (; i + 7 * 256 < hi; i += 8 * 256) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = jb.a[i + 256 * u];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
        }
    } else {
        for (; i + 3 * 256 < hi; i += 4 * 256) {
            double v[4], bb[4], ww[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                v[u] = jb.a[i + 256 * u];
                bb[u] = jb.b[i + 256 * u];
                ww[u] = mode == 1 ? 1.0 : jb.w[i + 256 * u];
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                acc += (mode == 1) ? v[u] * (lam * v[u] + bb[u]) : v[u] * (lam * ww[u] * v[u] + bb[u]);
        }
    }
    for (; i < hi; i += 256) {
        double v = jb.a[i];
        acc += (mode == 0) ? v : (mode == 1) ? v * (lam * v + jb.b[i]) : v * (lam * jb.w[i] * v + jb.b[i]);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    const int nparts = gridDim.x, nblk = gridDim.x * gridDim.y;
    if (threadIdx.x == 0) {
        st_sc1(part + (int64_t)blockIdx.y * gridDim.x + blockIdx.x, red[0]);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        last = ticket_last(cnt, nblk, (int)(blockIdx.y * gridDim.x + blockIdx.x));
    }
    __syncthreads();
    if (!last) return;
    __shared__ double s[kMaxSumJobs];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < J.nj) {
        double a = 0.0;
        int i = lane;
        for (; i + 7 * 64 < nparts; i += 8 * 64) {        // eight loads in flight, added in order
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                v[u] = ld_sc1(part + (int64_t)w * nparts + i + 64 * u);
#pragma unroll
            for (int u = 0; u < 8; u++) a += v[u];
        }
        for (; i < nparts; i += 64)
            a += ld_sc1(part + (int64_t)w * nparts + i);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
        if (lane == 0) {
            const double v = J.j[w].n > 0 ? a : 0.0;
            *J.j[w].out = v;
            s[w] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && J.total) *J.total = (s[0] + s[2]) + s[1];
    __syncthreads();
    if (rb.h_scal) {
        const int t = threadIdx.x;
        if (t < rb.ns) rb.h_scal[t] = rb.scal[t];
        if (t == 0) *rb.h_flag = *rb.flag;
        if (rb.rec && t < rb.nrec) rb.h_rec[t] = rb.rec[t];
    }
}

__global__ void k_sum_multi_final(const SumJobs J, int nparts, const double *__restrict__ part) {
    __shared__ double s[kMaxSumJobs];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double acc = 0.0;
    for (int i = lane; i < nparts; i += 64) acc += part[(int64_t)w * nparts + i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        const double v = J.j[w].n > 0 ? acc : 0.0;
        *J.j[w].out = v;
        s[w] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0 && J.total) *J.total = (s[0] + s[2]) + s[1];
}

__global__ void k_sum_final(int n, const double *__restrict__ part, double *__restrict__ out) {
    const int lane = threadIdx.x;
    double acc = 0.0;
    for (int i = lane; i < n; i += 64) acc += part[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) *out = acc;
}

__global__ void __launch_bounds__(256) k_maxdiag(int64_t nblocks, const int64_t *__restrict__ val_off,
                                                 const int32_t *__restrict__ bcols, const int32_t *__restrict__ bdiag,
                                                 const double *__restrict__ hval, double *__restrict__ part) {
    __shared__ double red[256];
    int64_t chunk = (nblocks + gridDim.x - 1) / gridDim.x;
    int64_t lo = blockIdx.x * chunk, hi = min(nblocks, lo + chunk);
    double mx = 0.0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += blockDim.x) {
        if (!bdiag[b]) continue;
        int c = bcols[b];
        const double *h = hval + val_off[b];
        for (int k = 0; k < c; k++) mx = fmax(mx, fabs(h[k * c + k]));
    }
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_max_final(int n, const double *__restrict__ part, double *__restrict__ out) {
    const int lane = threadIdx.x;
    double mx = 0.0;
    for (int i = lane; i < n; i += 64) mx = fmax(mx, part[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
    if (lane == 0) *out = mx;
}

// y = H x from the stored blocks (diagnostics; H symmetric, blocks hold the lower triangle)
__global__ void k_hmul(int64_t nblocks, const int64_t *__restrict__ val_off, const int32_t *__restrict__ brows,
                       const int32_t *__restrict__ bcols, const int64_t *__restrict__ brow_dof,
                       const int64_t *__restrict__ bcol_dof, const int32_t *__restrict__ bdiag,
                       const double *__restrict__ hval, const double *__restrict__ x, double *__restrict__ y) {
    int64_t b = TID;
    if (b >= nblocks) return;
    int R = brows[b], Cc = bcols[b];
    const double *h = hval + val_off[b];
    int64_t r0 = brow_dof[b], c0 = bcol_dof[b];
    for (int i = 0; i < R; i++)
        for (int j = 0; j < Cc; j++) {
            double hv = h[i * Cc + j];
            atomicAdd(&y[r0 + i], hv * x[c0 + j]);          // diagnostics only (not on the LM path)
            if (!bdiag[b]) atomicAdd(&y[c0 + j], hv * x[r0 + i]);
        }
}

// ------------------------------------------------------------------------------------------
// point-sharded plan: cross-rank transfers (DistPlan in symbolic.h)
// ------------------------------------------------------------------------------------------
// lower triangle of a contribution block (u x u at (s, s) of a column-major m x m front) packed
// column by column: column j holds rows j..u-1 at j*u - j(j-1)/2 (contiguous in the arena too)
__global__ void __launch_bounds__(256) k_pack_cb(const double *__restrict__ cb, int m, int u, double *__restrict__ buf) {
    const int j = blockIdx.x;
    if (j >= u) return;
    const int64_t off = (int64_t)j * u - (int64_t)j * (j - 1) / 2;
    const double *src = cb + (int64_t)j * m;
    for (int i = j + (int)threadIdx.x; i < u; i += blockDim.x) buf[off + (i - j)] = src[i];
}

// extend-add of a packed contribution block received from another rank into the parent front
// (task shape and fixed per-entry order as k_ea)
__global__ void __launch_bounds__(256) k_ea_packed(int ntask, const int32_t *__restrict__ tasks, const FrontDev fd,
                                                   const double *__restrict__ buf, double *__restrict__ arena) {
    int t = blockIdx.x;
    if (t >= ntask) return;
    int c = tasks[3 * t], j0 = tasks[3 * t + 1], i0 = tasks[3 * t + 2];
    int p = fd.parent[c];
    int u = fd.m[c] - fd.s[c], mp = fd.m[p];
    const int32_t *bm = fd.bmap + fd.bmap_off[c];
    double *Fp = arena + fd.arena_off[p];
    const int i = i0 + (int)threadIdx.x;
    if (i >= u) return;
    const int bi = bm[i];
    const int nj = min(16, min(u - j0, i - j0 + 1));
    double cv[16], pv[16];
    int64_t pj[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int j = j0 + q;
        pj[q] = (q < nj) ? (int64_t)bm[j] * mp + bi : 0;
        cv[q] = (q < nj) ? buf[(int64_t)j * u - (int64_t)j * (j - 1) / 2 + (i - j)] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) pv[q] = (q < nj) ? Fp[pj[q]] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++)
        if (q < nj) Fp[pj[q]] = pv[q] + cv[q];
}

__global__ void k_gather_idx(int n, const int32_t *__restrict__ idx, const double *__restrict__ src,
                             double *__restrict__ dst) {
    int i = TID;
    if (i < n) dst[i] = src[idx[i]];
}

__global__ void k_scatter_idx(int n, const int32_t *__restrict__ idx, const double *__restrict__ src,
                              double *__restrict__ dst) {
    int i = TID;
    if (i < n) dst[idx[i]] = src[i];
}

// diagonal entries of this rank's diagonal blocks (its own and the partial ones of remote vertices)
// into a dof vector; summed over the ranks it is diag(H) (lambda init, g2o computeLambdaInit)
__global__ void k_diag_entries(int64_t nblocks, const int64_t *__restrict__ val_off, const int32_t *__restrict__ bcols,
                               const int64_t *__restrict__ brow_dof, const int64_t *__restrict__ bcol_dof,
                               const double *__restrict__ hval, double *__restrict__ diagv) {
    int64_t b = TID;
    if (b >= nblocks || brow_dof[b] != bcol_dof[b]) return;
    const int c = bcols[b];
    const double *h = hval + val_off[b];
    for (int k = 0; k < c; k++) diagv[bcol_dof[b] + k] = h[k * c + k];
}

__global__ void __launch_bounds__(256) k_absmax_partial(int64_t n, const double *__restrict__ a, double *__restrict__ part) {
    __shared__ double red[256];
    int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    int64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    double mx = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mx = fmax(mx, fabs(a[i]));
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_int_to_double(int n, const int *__restrict__ a, double *__restrict__ out) {
    int i = TID;
    if (i < n) out[i] = (double)a[i];
}

}  // namespace dev

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static inline unsigned nb(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// optional per-launch device timing (deftri_profile_trial); off on the solve path
thread_local KProf *g_prof = nullptr;
thread_local double g_work = 0;   // algorithmic work of the next launch (profiling only)
thread_local int g_level = -1;    // elimination-tree level of the launches being issued (profiling only)
void set_profiler(KProf *p) { g_prof = p; }
bool profiling() { return g_prof != nullptr; }
static hipEvent_t prof_event() {
    KProf &P = *g_prof;
    if (P.next == P.pool.size()) { hipEvent_t e; hipEventCreate(&e); P.pool.push_back(e); }
    return P.pool[P.next++];
}
// the same timing for launches issued from other translation units (pcg.hip)
hipEvent_t prof_begin(hipStream_t st) {
    if (!g_prof) return nullptr;
    hipEvent_t e = prof_event();
    hipEventRecord(e, st);
    return e;
}
void prof_end(const char *name, hipEvent_t e0, unsigned grid, double work, hipStream_t st) {
    if (!g_prof || !e0) return;
    hipEvent_t e1 = prof_event();
    hipEventRecord(e1, st);
    g_prof->recs.push_back({name, e0, e1, grid, work, g_level});
}
// (an empty grid — nothing to do, n = 0 — is not launched: HIP would refuse it and leave the error
// pending for the next hipGetLastError of the thread)
#define LAUNCH(NAME, KER, GRID, BLOCK, ST, ...)                                     \
    do {                                                                             \
        if (dim3(GRID).x == 0) break;                                                \
        hipEvent_t e0_ = nullptr;                                                    \
        if (g_prof) { e0_ = prof_event(); hipEventRecord(e0_, ST); }                 \
        hipLaunchKernelGGL(KER, GRID, BLOCK, 0, ST, __VA_ARGS__);                    \
        if (g_prof) {                                                                \
            hipEvent_t e1_ = prof_event();                                           \
            hipEventRecord(e1_, ST);                                                 \
            g_prof->recs.push_back({NAME, e0_, e1_, dim3(GRID).x, g_work, g_level}); \
            g_work = 0;                                                              \
        }                                                                            \
    } while (0)

// DEFTRI_ARAP_J_FULL=1: the numeric ARAP Jacobian with every evaluation in full (k_lin_arap<3>,
// the A/B and bit-identity reference of the piece-reusing k_lin_arap<2>)
static bool arap_j_full() {
    static const bool v = std::getenv("DEFTRI_ARAP_J_FULL") != nullptr;
    return v;
}

void launch_linearize(const DevProblem &P, hipStream_t st, bool want_jac, bool analytic) {
    const bool pre = want_jac && !analytic && P.E > 0;   // the numeric Jacobians read the pair table
    const int nbr = P.R > 0 ? (int)nb(P.R, 128) : 0, nbd = P.D > 0 ? (int)nb(P.D, 128) : 0;
    const int nbp = pre ? (int)nb((int64_t)P.Q * dev::kArapPre, 128) : 0;
    LAUNCH("lin_pts", dev::k_lin_pts, dim3(nbr + nbd + nbp), dim3(128), st, P, nbr, nbd, want_jac ? 1 : 0,
           analytic ? 1 : 0);
    if (P.E > 0)
        LAUNCH("lin_arap", (!want_jac ? dev::k_lin_arap<0> : analytic ? dev::k_lin_arap<1> : arap_j_full() ? dev::k_lin_arap<3> : dev::k_lin_arap<2>),
                           dim3(nb(P.E, 128)), dim3(128), st, P.E, P.arap_pts, P.arap_pair,
                           P.arap_rot, P.arap_w, P.rot, P.pair_area, P.pair_info, P.points, P.tg,
                           pre ? P.tg_pre : nullptr, P.Jarap, P.Warap, P.Earap, P.chi_arap, want_jac ? 1 : 0,
                           analytic ? 1 : 0, P.jarap_ld, P.gate_lin, P.lin_part ? P.lin_part + nbr + nbd : nullptr,
                           P.n_arap_sum);
}

void launch_assemble(const DevProblem &P, const DevPlan &L, hipStream_t st) {
    dev::EdgeJ ej{P.Jrep, P.Wrep, P.Erep, P.Jdep, P.Wdep, P.Edep, P.Jarap, P.Warap, P.Earap};
    if (L.nhchunks > 0)
        LAUNCH("hchunk", dev::k_hchunk, dim3(nb(L.nhchunks, 64)), dim3(64), st, L.nhchunks, L.hcontrib,
                           L.hchunk_begin, L.hchunk_len, ej, L.hpart);
    if (L.nblocks > 0)
        LAUNCH("hfinal", dev::k_hfinal, dim3(nb(L.nblocks, 128)), dim3(128), st, L.nblocks,
                           L.hblk_chunk_begin, L.blk_val_off, L.blk_rows, L.blk_cols, L.hpart, L.hval);
    if (L.nheavy_h > 0) {
        LAUNCH("hfinal_heavy", dev::k_heavy_split<36>, dim3((unsigned)(L.nheavy_h * dev::kHeavySplit)), dim3(256), st,
               L.heavy_h, L.hblk_chunk_begin, L.hpart, L.heavy_scratch);
        LAUNCH("hfinal_heavy", dev::k_heavy_final<36>, dim3((unsigned)L.nheavy_h), dim3(64), st, L.heavy_h,
               L.blk_val_off, L.blk_rows, L.blk_cols, L.heavy_scratch, L.hval);
    }
    if (L.nbchunks > 0)
        LAUNCH("bchunk", dev::k_bchunk, dim3(nb(L.nbchunks, 128)), dim3(128), st, L.nbchunks, L.bcontrib,
                           L.bchunk_begin, L.bchunk_len, ej, L.bpart);
    if (L.nv > 0)
        LAUNCH("bfinal", dev::k_bfinal, dim3(nb(L.nv, 128)), dim3(128), st, L.nv, L.bv_chunk_begin, L.voff,
                           L.vdim, L.bpart, L.b);
    if (L.nheavy_b > 0) {
        LAUNCH("bfinal_heavy", dev::k_heavy_split<6>, dim3((unsigned)(L.nheavy_b * dev::kHeavySplit)), dim3(256), st,
               L.heavy_b, L.bv_chunk_begin, L.bpart, L.heavy_scratch);
        LAUNCH("bfinal_heavy", dev::k_heavy_final<6>, dim3((unsigned)L.nheavy_b), dim3(64), st, L.heavy_b, L.voff,
               L.vdim, (const int32_t *)nullptr, L.heavy_scratch, L.b);
    }
}

void launch_scatter_lanes(const DevPlan &L, hipStream_t st, const double *lam_dev) {
    // lanes' arenas are contiguous (stride lo.arena >= arena_size): one fill covers them all
    const int64_t span = L.nlanes > 1 ? (int64_t)(L.nlanes - 1) * L.lo.arena + L.arena_size : L.arena_size;
    hipMemsetAsync(L.arena, 0, sizeof(double) * (size_t)span, st);
    if (L.nblocks > 0)
        LAUNCH("scatter", dev::k_scatter, dim3(nb(L.nblocks, 128), L.nlanes), dim3(128), st, L.nblocks,
               L.blk_val_off, L.blk_rows, L.blk_cols, L.blk_arena, L.blk_ld, L.blk_diag, L.hval, L.lo, lam_dev,
               L.arena);
}

void launch_scatter(const DevPlan &L, double lambda, hipStream_t st, const double *lam_dev) {
    DevPlan one = L;
    one.nlanes = 1;
    one.lo.lam[0] = lambda;
    launch_scatter_lanes(one, st, lam_dev);
}

// a fresh epoch per factorization / substitution: the panel flags never need clearing
static std::atomic<int> g_epoch{16};      // factorization epochs start past the substitution's fixed 1 / 2
static int next_epoch() {
    int e = ++g_epoch;
    if (e <= 16) { g_epoch = 17; e = 17; }
    return e;
}

void launch_factor(const DevPlan &L, hipStream_t st, hipStream_t side, hipEvent_t *ev, int nev, LevelHook hook,
                   void *hook_user) {
    const int epoch = next_epoch();
    int evi = 0;
    hipEvent_t prev_side = nullptr, cur_side = nullptr;   // events of the last two side-stream updates
    for (size_t h = 0; h < L.levels.size(); h++) {
        const auto &lv = L.levels[h];
        g_level = (int)h;
        if (hook) hook(hook_user, kHookFactor, (int)h);      // cross-rank contribution blocks into this level
        for (int slot = 0; slot < 2; slot++)
            if (lv.nea[slot] > 0)
                LAUNCH("ea", dev::k_ea, dim3(lv.nea[slot], L.nlanes), dim3(256), st, lv.nea[slot],
                                   L.tasks + 3 * lv.ea_off[slot], L.fd, L.arena, L.lo);
        for (const auto &stp : lv.steps) {
            if (stp.ndiag > 0)
                LAUNCH("diag", stp.ndiag_tail ? dev::k_diag<true> : dev::k_diag<false>, dim3(stp.ndiag + stp.ndiag_tail, L.nlanes), dim3(256), st,
                       stp.ndiag + stp.ndiag_tail, stp.ndiag, L.tasks + 3 * stp.diag_off, L.fd, L.arena, L.inv, L.flag,
                       L.pflag, L.wbuf, epoch, L.lo);
            if (stp.ntrsm > 0)
                LAUNCH("trsm", dev::k_trsm, dim3(stp.ntrsm, L.nlanes), dim3(256), st, stp.ntrsm,
                                   L.tasks + 3 * stp.trsm_off, L.fd, L.arena, L.inv, L.lo);
            if (stp.stream == 1) {
                // "rest" update of an outer block: after the block's panel chain on the main stream,
                // concurrent with the next block's lookahead + panel chain there
                prev_side = cur_side;
                cur_side = nullptr;
                if (stp.nupd > 0) {
                    hipEvent_t e = ev[evi++ % nev];
                    hipEventRecord(e, st);
                    hipStreamWaitEvent(side, e, 0);
                    g_work = stp.upd_flops;
                    LAUNCH("update", (stp.ntail ? dev::k_update<true> : L.f32_update ? dev::k_update<false, true> : dev::k_update<false>), dim3(8 * nb(stp.nupd, 8), L.nlanes), dim3(256), side, stp.nupd,
                           stp.ntail, L.tasks + 3 * stp.upd_off, stp.kA, stp.kmax, stp.inner, L.fd, L.arena, L.inv,
                           L.flag, L.pflag, L.wbuf, epoch, L.lo);
                    cur_side = ev[evi++ % nev];
                    hipEventRecord(cur_side, side);
                }
                continue;
            }
            if (stp.wait_side >= 1 && prev_side) hipStreamWaitEvent(st, prev_side, 0);
            if (stp.wait_side == 2 && cur_side) hipStreamWaitEvent(st, cur_side, 0);
            if (stp.nupd > 0) {
                g_work = stp.upd_flops;
                LAUNCH("update", (stp.ntail ? dev::k_update<true> : L.f32_update ? dev::k_update<false, true> : dev::k_update<false>), dim3(8 * nb(stp.nupd, 8), L.nlanes), dim3(256), st, stp.nupd,
                       stp.ntail, L.tasks + 3 * stp.upd_off, stp.kA, stp.kmax, stp.inner, L.fd,
                       L.arena, L.inv, L.flag, L.pflag, L.wbuf, epoch, L.lo);
            }
        }
        // the level's side-stream work must be complete before the next level (or the solve) reads it
        if (cur_side) hipStreamWaitEvent(st, cur_side, 0);
        if (prev_side) hipStreamWaitEvent(st, prev_side, 0);
        prev_side = cur_side = nullptr;
    }
}

void launch_solve(const DevPlan &L, const double *rhs, double *x, hipStream_t st, const double *bpart,
                  LevelHook hook, void *hook_user) {
    // chained substitution (one launch per level and direction) unless DEFTRI_SOLVE_CHAIN=0
    static const bool chain = [] { const char *e = std::getenv("DEFTRI_SOLVE_CHAIN"); return !(e && std::atoi(e) == 0); }();
    const bool ch = chain && L.pflag != nullptr;
    // the flags are cleared per substitution and the epochs fixed (1 forward, 2 backward), so a
    // captured trial graph replays correctly
    const int fe = 1, be = 2;
    if (ch) {
        const int64_t span = (L.nlanes > 1 ? (int64_t)(L.nlanes - 1) * L.lo.pflag : 0) + std::max<int64_t>(L.npanels, 1);
        hipMemsetAsync(L.pflag, 0, sizeof(int) * (size_t)span, st);
    }
    for (size_t h = 0; h < L.levels.size(); h++) {
        const auto &lv = L.levels[h];
        g_level = (int)h;
        if (hook) hook(hook_user, kHookForward, (int)h);     // cross-rank forward-update vectors
        if (lv.nfwd > 0)
            LAUNCH("fwd_gather", dev::k_fwd_gather, dim3(lv.nfwd, L.nlanes), dim3(256), st, lv.nfwd,
                   L.tasks + 3 * lv.fwd_off, L.fd, rhs, bpart, L.vec, L.lo);
        if (ch) {
            if (lv.nfchain > 0)
                LAUNCH("fwd_chain", dev::k_fwd_chain, dim3(lv.nfchain, L.nlanes), dim3(256), st, lv.nfchain,
                       L.tasks + 3 * lv.fchain_off, L.fd, L.arena, L.inv, L.vec, L.yvec, L.pflag, fe, L.flag, L.lo);
            continue;
        }
        for (const auto &sp : lv.fsteps)
            if (sp.n > 0)
                LAUNCH("fwd_step", dev::k_fwd_step, dim3(sp.n, L.nlanes), dim3(256), st, sp.n, L.tasks + 3 * sp.off,
                       L.fd, L.arena, L.inv, L.vec, L.yvec, L.lo);
    }
    for (size_t hh = L.levels.size(); hh-- > 0;) {
        const auto &lv = L.levels[hh];
        g_level = (int)hh;
        if (lv.nbgemv > 0)
            LAUNCH("bwd_init", dev::k_bwd_init, dim3(lv.nbgemv, L.nlanes), dim3(256), st, lv.nbgemv,
                   L.tasks + 3 * lv.bgemv_off, L.fd, L.arena, x, L.yvec, L.vec, L.lo);
        if (ch) {
            if (lv.nbchain > 0)
                LAUNCH("bwd_chain", dev::k_bwd_chain, dim3(lv.nbchain, L.nlanes), dim3(256), st, lv.nbchain,
                       L.tasks + 3 * lv.bchain_off, L.fd, L.arena, L.inv, L.vec, L.yvec, x, L.pflag, be, L.flag, L.lo);
        } else {
            for (const auto &sp : lv.bsteps)
                if (sp.n > 0)
                    LAUNCH("bwd_step", dev::k_bwd_step, dim3(sp.n, L.nlanes), dim3(256), st, sp.n, L.tasks + 3 * sp.off,
                           L.fd, L.arena, L.inv, L.vec, x, L.lo);
        }
        if (hook) hook(hook_user, kHookBackward, (int)hh);   // boundary solutions down to other ranks
    }
}

void launch_pack_cb(const DevPlan &L, int64_t arena_off, int m, int s, double *buf, hipStream_t st) {
    const int u = m - s;
    if (u > 0)
        LAUNCH("pack_cb", dev::k_pack_cb, dim3(u), dim3(256), st, L.arena + arena_off + (int64_t)s * m + s, m, u, buf);
}

void launch_ea_packed(const DevPlan &L, int64_t ea_off, int nea, const double *buf, hipStream_t st) {
    if (nea > 0)
        LAUNCH("ea_packed", dev::k_ea_packed, dim3(nea), dim3(256), st, nea, L.tasks + 3 * ea_off, L.fd, buf, L.arena);
}

void launch_gather_idx(int n, const int32_t *idx, const double *src, double *dst, hipStream_t st) {
    if (n > 0) LAUNCH("gather_idx", dev::k_gather_idx, dim3(nb(n, 256)), dim3(256), st, n, idx, src, dst);
}

void launch_scatter_idx(int n, const int32_t *idx, const double *src, double *dst, hipStream_t st) {
    if (n > 0) LAUNCH("scatter_idx", dev::k_scatter_idx, dim3(nb(n, 256)), dim3(256), st, n, idx, src, dst);
}

void launch_diag_entries(const DevPlan &L, double *diagv, hipStream_t st) {
    hipMemsetAsync(diagv, 0, sizeof(double) * (size_t)L.ndof, st);
    if (L.nblocks > 0)
        LAUNCH("diag_entries", dev::k_diag_entries, dim3(nb(L.nblocks, 128)), dim3(128), st, L.nblocks, L.blk_val_off,
               L.blk_cols, L.blk_row_dof, L.blk_col_dof, L.hval, diagv);
}

void launch_absmax(int64_t n, const double *a, double *part, int nparts, double *out, hipStream_t st) {
    if (n <= 0) { hipMemsetAsync(out, 0, sizeof(double), st); return; }
    LAUNCH("absmax_partial", dev::k_absmax_partial, dim3(nparts), dim3(256), st, n, a, part);
    LAUNCH("max_final", dev::k_max_final, dim3(1), dim3(64), st, nparts, part, out);
}

void launch_int_to_double(int n, const int *a, double *out, hipStream_t st) {
    if (n > 0) LAUNCH("int_to_double", dev::k_int_to_double, dim3(nb(n, 64)), dim3(64), st, n, a, out);
}

void launch_update_state(const DevProblem &P, const double *dx, hipStream_t st, const int *flag) {
    int n = P.P > P.S ? P.P : P.S;
    if (P.Q > n) n = P.Q;
    if (n > 0)
        LAUNCH("update_state", dev::k_update_state, dim3(nb(n, 128)), dim3(128), st, P.P, P.S, P.Q, dx, P.points,
                           P.scales, P.tg, flag, P.gate_trial);
}

void launch_update_state_bak(const DevProblem &P, const double *dx, bool restore, hipStream_t st) {
    int n = P.P > P.S ? P.P : P.S;
    if (P.Q > n) n = P.Q;
    if (n > 0)
        LAUNCH("update_state", dev::k_update_state_bak, dim3(nb(n, 128)), dim3(128), st, P.P, P.S, P.Q, dx, P.points,
               P.scales, P.tg, P.points_bak, P.scales_bak, P.tg_bak, restore ? 1 : 0);
}

void launch_trial_begin(const DevProblem &P, int *flag, double *zero, int64_t nzero, hipStream_t st, bool restore) {
    int64_t n = std::max<int64_t>(std::max<int64_t>(3 * (int64_t)P.P, 7 * (int64_t)P.Q), std::max<int64_t>(P.S, nzero));
    n = std::max<int64_t>(n, 1);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    if (restore)
        LAUNCH("trial_begin", dev::k_trial_begin, dim3(grid), dim3(256), st, P.P, P.S, P.Q, P.points_bak, P.scales_bak,
               P.tg_bak, P.points, P.scales, P.tg, flag, zero, nzero, n);
    else
        LAUNCH("trial_begin", dev::k_trial_begin, dim3(grid), dim3(256), st, P.P, P.S, P.Q, P.points, P.scales, P.tg,
               P.points_bak, P.scales_bak, P.tg_bak, flag, zero, nzero, n);
}

void launch_trial_begin_dev(const DevProblem &P, int *flag, double *zero, int64_t nzero, LmState *lm, const double *scal,
                            double tau, double user_lambda, hipStream_t st) {
    int64_t n = std::max<int64_t>(std::max<int64_t>(3 * (int64_t)P.P, 7 * (int64_t)P.Q), std::max<int64_t>(P.S, nzero));
    n = std::max<int64_t>(n, 1);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    LAUNCH("trial_begin", dev::k_trial_begin_dev, dim3(grid), dim3(256), st, P.P, P.S, P.Q, P.points, P.scales, P.tg,
           P.points_bak, P.scales_bak, P.tg_bak, flag, zero, nzero, n, lm, scal, tau, user_lambda);
}

void launch_lm_decide(LmState *lm, const double *scal, const double *rec, double *chi_it, int32_t *trials_it, int max_report,
                      LmState *snap, int slot, hipStream_t st) {
    LAUNCH("lm_decide", dev::k_lm_decide, dim3(1), dim3(64), st, lm, scal, rec, chi_it, trials_it, max_report, snap, slot);
}

void launch_trial_readback(const double *scal, int ns, const int *flag, const double *rec, int nrec, double *h_scal,
                           int *h_flag, double *h_rec, hipStream_t st) {
    LAUNCH("trial_readback", dev::k_trial_readback, dim3(1), dim3(64), st, scal, ns, flag, rec, nrec, h_scal, h_flag,
           h_rec);
}

void launch_sum(int64_t n, const double *a, const double *b, double lambda, int mode, double *part, int nparts,
                double *out, hipStream_t st, const double *w) {
    if (n <= 0) { hipMemsetAsync(out, 0, sizeof(double), st); return; }
    LAUNCH("sum_partial", dev::k_sum_partial, dim3(nparts), dim3(256), st, n, a, b, lambda, mode, w, part);
    LAUNCH("sum_final", dev::k_sum_final, dim3(1), dim3(64), st, nparts, part, out);
}

void launch_lin_chi(const DevProblem &P, hipStream_t st) {
    const int nbr = P.R > 0 ? (int)nb(P.R, 128) : 0, nbd = P.D > 0 ? (int)nb(P.D, 128) : 0;
    const int nba = P.E > 0 ? (int)nb(P.E, 128) : 0;
    if (nbr + nbd + nba > 0) LAUNCH("lin_chi", dev::k_lin_chi, dim3(nbr + nbd + nba), dim3(128), st, P, nbr, nbd);
}

void lin_chi_blocks(const DevProblem &P, int nbk[4]) {
    nbk[0] = P.R > 0 ? (int)nb(P.R, 128) : 0;
    nbk[1] = P.D > 0 ? (int)nb(P.D, 128) : 0;
    nbk[2] = P.n_arap_sum > 0 ? (int)nb(P.n_arap_sum, 128) : 0;
    nbk[3] = 0;
}

void launch_part_sums(const double *part, const int nbk[4], double *out, double *den_out, double *total, const int *gate,
                      hipStream_t st) {
    LAUNCH("part_sums", dev::k_part_sums, dim3(1), dim3(256), st, part, nbk[0], nbk[1], nbk[2], nbk[3], out, den_out, total,
           gate);
}

// edges per thread of the trial evaluation: C2 on HIP events (profiles/r05ex_trial_eval_ab.log) 1: 26.0
// us, 2: 23.2, 4: 23.2, 8: 26.8
int eval_edges_per_thread() { return 2; }

static void eval_blocks(const DevProblem &P, const EvalJob &J, int &nbr, int &nbd, int &nba, int &nbx) {
    const int64_t run = 256 * (int64_t)eval_edges_per_thread();
    nbr = P.R > 0 ? (int)((P.R + run - 1) / run) : 0;
    nbd = P.D > 0 ? (int)((P.D + run - 1) / run) : 0;
    nba = J.n_arap > 0 ? (int)((J.n_arap + run - 1) / run) : 0;
    nbx = J.n_den > 0 ? (int)((J.n_den + run - 1) / run) : 0;
}

void trial_eval_blocks(const DevProblem &P, const EvalJob &J, int nb[4]) { eval_blocks(P, J, nb[0], nb[1], nb[2], nb[3]); }

void trial_eval_host_sums(const double *h_part, const int nb[4], double out[4]) {
    int lo = 0;
    for (int k = 0; k < 4; k++) {
        const int hi = lo + nb[k];
        double v[64];
        for (int l = 0; l < 64; l++) {
            double a = 0.0;
            for (int i = lo + l; i < hi; i += 64) a += h_part[i];
            v[l] = a;
        }
        for (int off = 32; off > 0; off >>= 1) {
            double u[64];
            for (int l = 0; l < 64; l++) u[l] = v[l] + v[l ^ off];
            for (int l = 0; l < 64; l++) v[l] = u[l];
        }
        out[k] = v[0];
        lo = hi;
    }
}

int64_t trial_eval_parts(const DevProblem &P, const EvalJob &J) {
    int nbr, nbd, nba, nbx;
    eval_blocks(P, J, nbr, nbd, nba, nbx);
    return std::max<int64_t>(1, (int64_t)nbr + nbd + nba + nbx);
}

void launch_trial_eval(const DevProblem &P, const EvalJob &J, double *part, int *cnt, const ReadBack &rb, hipStream_t st) {
    int nbr, nbd, nba, nbx;
    eval_blocks(P, J, nbr, nbd, nba, nbx);
    // an empty problem still runs one workgroup: the sums are written (0) and the read-back done
    const int grid = std::max(1, nbr + nbd + nba + nbx);
    LAUNCH("trial_eval", dev::k_trial_eval, dim3(grid), dim3(256), st, P, J, eval_edges_per_thread(), nbr, nbd, nba, part,
           cnt, rb);
}

void launch_sum_multi_fused(const SumJobs &J, double *part, int nparts, int *cnt, const ReadBack &rb, hipStream_t st) {
    if (J.nj <= 0) return;
    LAUNCH("sum_fused", dev::k_sum_multi_fused, dim3(nparts, J.nj), dim3(256), st, J, part, cnt,
           rb);
}

void launch_sum_multi(const SumJobs &J, double *part, int nparts, hipStream_t st) {
    if (J.nj <= 0) return;
    LAUNCH("sum_partial", dev::k_sum_multi_partial, dim3(nparts, J.nj), dim3(256), st, J, part);
    LAUNCH("sum_final", dev::k_sum_multi_final, dim3(1), dim3(64 * J.nj), st, J, nparts, part);
}

void launch_maxdiag(const DevPlan &L, double *part, int nparts, double *out, hipStream_t st) {
    LAUNCH("maxdiag", dev::k_maxdiag, dim3(nparts), dim3(256), st, L.nblocks, L.blk_val_off, L.blk_cols,
                       L.blk_diag, L.hval, part);
    LAUNCH("max_final", dev::k_max_final, dim3(1), dim3(64), st, nparts, part, out);
}

void launch_hmul(const DevPlan &L, const int64_t *brow_dof, const int64_t *bcol_dof, const double *x, double *y,
                 int64_t n, hipStream_t st) {
    hipMemsetAsync(y, 0, sizeof(double) * (size_t)n, st);
    if (L.nblocks > 0)
        LAUNCH("hmul", dev::k_hmul, dim3(nb(L.nblocks, 128)), dim3(128), st, L.nblocks, L.blk_val_off,
                           L.blk_rows, L.blk_cols, brow_dof, bcol_dof, L.blk_diag, L.hval, x, y);
}

}  // namespace deftri
