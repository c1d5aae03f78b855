// pcg.h — the LM step (H + lambda I) dx = b by block-Jacobi preconditioned conjugate gradients
// (pcg.hip), the north star's "LM damping + PCG step", with the multifrontal LDL^T as the fallback.
//
// H stays in the assembled vertex-pair blocks (DevPlan::hval: one block per coupled vertex pair,
// lower triangle in elimination order).  The plan adds a row view of them: per vertex v, the entries
// (block, other vertex's first dof and dimension, transposed?) that make row v of H, so the product
// is a gather (one thread per vertex, fixed entry order, no atomics).  Rows with more than
// kPcgHeavy entries (the global T_g and scale vertices, coupled to every point) are split over
// workgroups of kPcgChunk entries whose partial rows are summed in chunk order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace deftri {

constexpr int kPcgHeavy = 128;      // entries above which a row is reduced by workgroups
constexpr int kPcgChunk = 2048;     // entries per workgroup of a heavy row
constexpr int kPcgRec = 8;          // doubles per iteration record
constexpr int kPcgMaxHeavyDofs = 2048;
// iteration record fields (record 0: setup; record k + 1: iteration k)
enum { PR_RZ = 0, PR_RR = 1, PR_PQ = 2, PR_ALPHA = 3, PR_STATUS = 4, PR_ITS = 5 };
// PR_STATUS: 0 running, 1 converged, 2 breakdown (p.Ap <= 0 / non-finite), 3 preconditioner block
// not positive definite
enum { kPcgRunning = 0, kPcgConverged = 1, kPcgBreakdown = 2, kPcgBadBlock = 3 };

struct PcgEnt {             // 16 bytes: one load
    int64_t val_off;        // block values (row-major R x C in hval)
    int32_t odof;           // first dof of the other vertex
    int16_t odim;           // its dimension
    int16_t tr;             // 1: the block is stored as (other row, this column): use its transpose
};

// host-built row view of the block structure (single-rank plans)
struct PcgHost {
    std::vector<int64_t> ent_begin;      // per vertex (nv + 1)
    std::vector<PcgEnt> ent;
    std::vector<int32_t> light_v;        // vertices handled one per thread, in vertex order
    std::vector<int32_t> heavy_v;        // heavy vertices
    std::vector<int32_t> hc_vertex;      // per heavy chunk: heavy index
    std::vector<int64_t> hc_beg, hc_end; // entry range of the chunk
    std::vector<int32_t> h_first;        // per heavy vertex: first chunk (nheavy + 1)
    std::vector<int32_t> h_dofbase;      // per heavy vertex: first heavy dof (nheavy + 1)
    std::vector<int32_t> v_heavy;        // per vertex: heavy index or -1
    std::vector<int64_t> diag_off;       // per vertex: val_off of its diagonal block
    std::vector<int64_t> moff;           // per vertex: offset of its preconditioner block (dim^2)
    int64_t msize = 0;
};
bool build_pcg_host(int64_t nv, const std::vector<int64_t> &voff, const std::vector<int32_t> &vdim,
                    const std::vector<int64_t> &blk_val_off, const std::vector<int32_t> &blk_rows,
                    const std::vector<int32_t> &blk_cols, const std::vector<int64_t> &blk_row_dof,
                    const std::vector<int64_t> &blk_col_dof, PcgHost &out, std::string &err);

struct PcgDev {
    int64_t nv = 0, ndof = 0;
    int32_t nlight = 0, nheavy = 0, nhchunks = 0, nheavy_dofs = 0;
    int32_t nA_light = 0;                // workgroups of the light part of the product launch
    int32_t nB = 0;                      // workgroups of the vertex launches (setup / update)
    const int64_t *ent_begin = nullptr;
    const PcgEnt *ent = nullptr;
    const int32_t *light_v = nullptr, *heavy_v = nullptr, *hc_vertex = nullptr, *h_first = nullptr;
    const int32_t *h_dofbase = nullptr, *v_heavy = nullptr;
    const int64_t *hc_beg = nullptr, *hc_end = nullptr, *diag_off = nullptr, *moff = nullptr;
    const int64_t *voff = nullptr;
    const int32_t *vdim = nullptr;
    double *minv = nullptr;              // (H_vv + lambda I)^-1 per vertex
    double *r = nullptr, *z = nullptr, *p[2] = {nullptr, nullptr}, *q = nullptr;
    double *hq = nullptr;                // per heavy chunk: 6 partial row sums
    double *partA = nullptr;             // per light workgroup of the product: p.q
    double *partB = nullptr;             // per vertex workgroup: (r.z, r.r)
    double *rec = nullptr;               // (max_it + 2) x kPcgRec
    int32_t max_it = 0;
    double tol2 = 0;                     // squared relative residual tolerance
};

// one solve's launches (x = dx).  setup: preconditioner blocks at lambda, r = b, z = M r, x = 0.
void launch_pcg_setup(const PcgDev &G, const double *hval, const double *b, double lambda, double *x,
                      hipStream_t st);
// iteration it: product q = (H + lambda I) p (p = z + beta p_prev formed on the fly) after the
// convergence test of the residual the previous update left
void launch_pcg_product(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st);
// iteration it: alpha, x += alpha p, r -= alpha q, z = M r, partial (r.z, r.r)
void launch_pcg_update(const PcgDev &G, int it, double lambda, double *x, hipStream_t st);

}  // namespace deftri
