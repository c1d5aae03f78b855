// ba.h — device view and launchers of the bundle-adjustment (BlockSolver_6_3 Schur) LM path.
//
// Replaces, for the reference's BA entry points (g2oBundleAdjustment.cc:38-444), g2o's
//   computeActiveErrors / EdgeSE3ProjectXYZ::linearizeOplus (g2oTypes.cc:121-142)   -> k_ba_edges
//   BlockSolver::buildSystem (Hll, Hpp, Hpl blocks, b)                                -> k_ba_points, k_ba_pose_chunk/_final
//   BlockSolver::solve: Dinv = Hll^-1, Hschur = Hpp - Hpl Dinv Hpl^T, bschur          -> k_ba_schur_points, k_ba_schur_gemm,
//                                                                                        k_ba_schur_reduce
//   LinearSolverEigen on Hschur (SimplicialLDLT)                                      -> k_ba_dense_ldlt (one workgroup)
//   xl = Dinv (bl - Hpl^T xp), OptimizableGraph::update                              -> k_ba_backsub, k_ba_update
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace deftri {

constexpr int kBaPoseChunk = 256;      // edges per pose-assembly chunk
constexpr int kBaStageEdges = 128;     // edges staged in LDS per Schur-GEMM step
constexpr int kBaLdsMaxN = 112;        // dense LDL^T kept in LDS up to this order (112^2 doubles = 98 KB)

struct BADev {
    int32_t K = 0, P = 0, E = 0;          // poses, points, edges (edges sorted by point)
    int32_t nfree = 0, ns = 0;            // free active poses, 6 * nfree
    int32_t dense_positive = 0;           // 1: reject non-positive pivots (no free points)
    double huber = 0;
    // state
    double *poses = nullptr, *poses_bak = nullptr, *points = nullptr, *points_bak = nullptr;
    float *kb8 = nullptr;                  // [K*8]
    // edges (point-sorted)
    int32_t *e_point = nullptr, *e_pose = nullptr;
    double *obs = nullptr, *info = nullptr;
    uint8_t *robust = nullptr, *active = nullptr;
    int32_t *pt_ptr = nullptr;             // [P+1] CSR: point -> edge range
    uint8_t *pt_free = nullptr;            // [P] hessian point (active, not fixed)
    int32_t *pose_sidx = nullptr;          // [K] Schur block of a free active pose, -1 otherwise
    // pose -> edges (CSR of edge ids) and its chunks
    int32_t *pose_edges = nullptr;         // [E]
    int32_t nchunk = 0;
    int32_t *chunk_pose = nullptr, *chunk_beg = nullptr, *chunk_len = nullptr;   // [nchunk]
    int32_t *pose_chunk_ptr = nullptr;     // [K+1]
    // Schur GEMM stages: contiguous point ranges with <= kBaStageEdges edges each
    int32_t nstage = 0, ngroup = 0;
    int32_t *stage_pt = nullptr;           // [nstage+1] first point of each stage (VALU path, ns >= 128)
    int32_t mgroup = 0, mstages_per_group = 0;   // MFMA path: 16-point stages, consecutive per workgroup
    int32_t *group_stage = nullptr;        // [ngroup+1] stages per workgroup
    int32_t *pslot = nullptr;              // [E] Schur block of the edge's pose (-1: not in S); set on the
                                           //     lead edge of each (point, pose) pair only
    int32_t *lead = nullptr;               // [E] first edge of the same (point, pose) pair
    // initializeOptimization(level) inputs / scratch (device-side active set)
    uint8_t *e_level = nullptr;            // [E] edge level (point order)
    uint8_t *pt_fixed = nullptr, *pose_fixed = nullptr;   // [P], [K]
    int32_t *pose_flag = nullptr;          // [K] pose has an active edge on this rank
    uint8_t *pt_act = nullptr;             // [P] point has an active edge
    int32_t *icount = nullptr;             // [1] free points
    // linearization (per edge)
    double *err = nullptr, *wgt = nullptr, *chi = nullptr, *chi2raw = nullptr;
    double *wr = nullptr;                  // [E*2] omega_r = -rho' Omega e
    double *Jp = nullptr, *JT = nullptr;   // [E*6] (2x3), [E*12] (2x6)
    double *Wb = nullptr, *Y = nullptr;    // [E*18] Hpl block (6x3 row-major) and Hpl Dinv
    double *v = nullptr;                   // [E*6]  Hpl (Dinv bl)
    // per point
    double *Hll = nullptr, *bl = nullptr, *Dinv = nullptr, *dxl = nullptr;
    double *dbl = nullptr;                 // [P*3] Dinv bl
    // per pose
    double *pchunk = nullptr;              // [nchunk*27]: lower-triangle Hpp (21) + bp (6)
    double *Hpp = nullptr, *bp = nullptr;  // [K*36], [K*6]
    // reduced system
    double *Spart = nullptr;               // [ngroup * NE], NE = ns(ns+1)/2 + ns
    double *Sred = nullptr;                // [NE]: -sum Hpl Dinv Hlp (lower triangle), -sum Hpl Dinv bl (this rank)
    double *S = nullptr;                   // [ns*ns] factor workspace
    double *xp = nullptr;                  // [ns]
    double *dxp = nullptr;                 // [K*6] pose steps in pose order
    int *flag = nullptr;
    // scalars
    double *part = nullptr;                // reduction partials
    double *scal = nullptr;                // [8]
};

void ba_set_profiler(KProf *p);
// errors of active edges (and Jacobians when want_jac; chi[] = robust chi2), or with all_edges
// the errors of every edge selected by sel (NULL = all; point order) — e->computeError()
void ba_launch_edges(const BADev &B, hipStream_t st, bool want_jac, bool all_edges, const uint8_t *sel = nullptr);
void ba_launch_chi2_sum(const BADev &B, double *out, hipStream_t st);
void ba_launch_points(const BADev &B, hipStream_t st);
void ba_launch_poses(const BADev &B, hipStream_t st);
void ba_launch_maxdiag(const BADev &B, double *out, hipStream_t st);
void ba_launch_schur(const BADev &B, double lambda, hipStream_t st);
void ba_launch_dense_solve(const BADev &B, double lambda, hipStream_t st);
void ba_launch_backsub_update(const BADev &B, hipStream_t st);
void ba_launch_scale(const BADev &B, double lambda, double *out_pts, double *out_pose, hipStream_t st);
// initializeOptimization(level) on the device: active edges, per-pose / per-point activity
void ba_launch_active(const BADev &B, int level, hipStream_t st);
// free points (count into icount) and the Schur slot of each pair's lead edge, given pose_sidx
void ba_launch_free_slots(const BADev &B, hipStream_t st);
void ba_launch_edge_chi2(const BADev &B, const int32_t *perm, double *chi2_out, uint8_t *dpos_out, hipStream_t st);

}  // namespace deftri
