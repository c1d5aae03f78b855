// pcg.h — the LM step (H + lambda I) dx = b by block-Jacobi preconditioned conjugate gradients
// (pcg.hip), the north star's "LM damping + PCG step", with the multifrontal LDL^T as the fallback.
//
// H stays in the assembled vertex-pair blocks (DevPlan::hval: one block per coupled vertex pair,
// lower triangle in elimination order).  The plan adds a row view of them: per vertex v, the entries
// (block, other vertex's first dof and dimension, transposed?) that make row v of H, so the product
// is a gather (fixed entry order, no atomics).  Three row classes:
//   * sliced rows (3-dof points, the bulk): 64 rows per slice (one wave), taken in the plan's
//     nested-dissection order (a slice's rows are mesh neighbours, so the lanes' gathers share
//     cache lines) and sorted by their count of 3x3 point-point blocks inside windows of
//     kPcgSortWindow rows so a slice pads little; those blocks are repacked once per LM iteration
//     (after the assembly) into slot-major, lane-interleaved copies in the rows' orientation —
//     every load of the product is coalesced; the row's other couplings (T_g, scale) follow as
//     per-lane entries;
//   * other light rows: one thread per row over its entries;
//   * heavy rows (> kPcgHeavy entries: the global T_g and scale vertices, coupled to every point):
//     workgroups of kPcgChunk entries whose partial rows are summed in chunk order.
// The vectors the product gathers are interleaved per dof: zp = (z, p_prev) and pq = (p, q).
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
constexpr int kPcgSortWindow = 512;
// iteration record fields (record 0: setup; record k + 1: iteration k)
enum { PR_RZ = 0, PR_RR = 1, PR_PQ = 2, PR_ALPHA = 3, PR_STATUS = 4, PR_ITS = 5, PR_PQA = 6 };
// PR_PQA (matrix-free plans): the sliced rows' p.q, summed once by k_pcg_heavy's last workgroup
// instead of by every update workgroup; likewise k_pcg_dots sums the (r.z, r.r) partials once per
// iteration for the product
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
    std::vector<int32_t> hc_vertex;      // per heavy chunk (kPcgChunk entries of hres): heavy index
    std::vector<int64_t> hc_beg, hc_end; // entry range of the chunk (in hres; a heavy vertex's chunks are contiguous)
    std::vector<int32_t> h_first;        // per heavy vertex: first chunk (nheavy + 1)
    std::vector<int32_t> h_dofbase;      // per heavy vertex: first heavy dof (nheavy + 1)
    std::vector<int32_t> v_heavy;        // per vertex: heavy index or -1
    std::vector<int64_t> diag_off;       // per vertex: val_off of its diagonal block
    std::vector<int64_t> moff;           // per vertex: offset of its preconditioner block (dim^2)
    int64_t msize = 0;
    // sliced rows: slice s covers rows sl_v[64 s .. 64 s + 63] (-1: padding), 3x3 slots
    // sl_off[s] .. sl_off[s] + sl_n[s] - 1 (global slot g: values [g][9][64], dof of the other
    // point [g][64], source block [g][64] = val_off | transposed << 62, -1 padding), extra entries
    // slots sl_xoff[s] .. + sl_nx[s] - 1 ([g][64], odim 0 = padding)
    std::vector<int32_t> sl_v, sl_n, sl_nx;
    std::vector<int64_t> sl_off, sl_xoff;
    std::vector<int32_t> sl_col;
    std::vector<int64_t> sl_map;
    std::vector<PcgEnt> sl_x;
    // heavy slots: slice s couples to heavy vertices through slots sl_hoff[s] .. + sl_hn[s] - 1;
    // slot g: heavy index hs_hk[g], source block per lane hs_map[g][64] (3 x od in the row's
    // orientation, od = the heavy vertex's dimension); per heavy vertex its slots in ascending order
    // (hv_slot_begin; slot g's partial at position hs_pos[g]); heavy rows keep as entries (hres, chunked) only their couplings
    // to vertices outside the slices
    std::vector<int32_t> sl_hn, hs_hk;
    std::vector<int64_t> hs_voff;        // per heavy slot: first double2 of its values (ceil(3 od / 2) x 64)
    int64_t hs_size = 0;                 // doubles of all heavy slots' values
    std::vector<int64_t> sl_hoff, hs_map, hv_slot_begin, hs_pos;
    std::vector<PcgEnt> hres;
    double product_bytes = 0, product_flops = 0;   // per product launch (roofline)
};
bool build_pcg_host(int64_t nv, const std::vector<int64_t> &voff, const std::vector<int32_t> &vdim,
                    const std::vector<int64_t> &blk_val_off, const std::vector<int32_t> &blk_rows,
                    const std::vector<int32_t> &blk_cols, const std::vector<int64_t> &blk_row_dof,
                    const std::vector<int64_t> &blk_col_dof, const std::vector<int64_t> &elim_pos, PcgHost &out,
                    std::string &err);

// Matrix-free product (round 2, default where the plan fits): H is never assembled for a PCG step.
// Every 3-dof point is a sliced row (64 per slice, nested-dissection order dealt to XCDs); a slice's
// workgroup loads the linearized ARAP edges touching its points ("local edges"; an edge touching
// several slices is loaded by each), forms
// s_e = W_e (J_e p) once per edge and stores J_{e,v}^T s_e per point role in LDS; each lane then
// sums its row's incidences and its own single-point edges (reprojection, depth).  The global rows
// (T_g, depth scales) are summed from per-slice
// partials of the edges a slice owns (an edge is owned by the first slice holding one of its
// points).  The block-Jacobi preconditioner's diagonal blocks and b come from the same structure
// once per LM iteration (k_mf_lin).  H + b are assembled only if a step falls back to the LDL^T.
constexpr int kMfMaxT = 2;          // T_g vertices one slice's owned ARAP edges may touch (record field: < 8)
constexpr int kMfMaxS = 4;          // depth scales one slice's depth edges may touch
constexpr int kMfMaxH = kMfMaxT + kMfMaxS;
constexpr int kMfMaxLds = 5120;     // doubles of per-slice contributions in LDS (40 KB)
constexpr int kMfLin = 27;          // per heavy slot of k_mf_lin: 21 (lower 6x6) + 6 (b)
enum { MF_ARAP = 0, MF_REP = 1, MF_DEP = 2 };

struct PcgMfHost {
    std::vector<int32_t> heavy_v, h_dofbase, v_heavy, h_first;
    std::vector<int32_t> sl_v;                     // nsl * 64 rows (-1 padding)
    std::vector<int64_t> le_off;                   // per slice: first local edge
    std::vector<int32_t> le_n, le_na;              // per slice: local edges, of which ARAP
    // local edge record: kind << 62 | role mask << 58 | (heavy slot + 1, 0 = not owned) << 55 |
    // LDS base << 40 | edge; the roles whose point is in the slice get consecutive 3-vectors at base
    std::vector<int64_t> le;
    std::vector<int64_t> in_off;                   // per slice: first incidence slot
    std::vector<int32_t> in_n;                     // per slice: incidence slots
    std::vector<int32_t> inc;                      // [slot][64]: LDS offset of the row's 3-vector (-1 padding)
    std::vector<int32_t> inc2;                     // [slot][64]: local edge << 2 | role (-1 padding)
    // per slice its heavy slots: the T_g vertices of its owned ARAP edges (sl_nt of them, first),
    // then the scales of its points' depth edges
    std::vector<int32_t> sl_hn, sl_nt, hs_hk;
    std::vector<int64_t> sl_hoff, hv_slot_begin, hs_pos;
    // the rows' single-point edges (reprojection, depth), summed by their own lane:
    // [slot][64] = depth << 30 | (scale slot + 1) << 27 | edge, -1 padding
    std::vector<int64_t> sl_meta;                  // per slice: le_off, in_off, own_off, counts (ne | ni << 16 | no << 24 | nt << 32 | nh << 36)
    std::vector<int32_t> sl_hpos;                  // per slice, kMfMaxH: its heavy slots' partial positions
    std::vector<int64_t> own_off;
    std::vector<int32_t> own_n, own;
    std::vector<int32_t> adof, atdof, rdof, ddof;  // dofs of the edges' vertices
    std::vector<int64_t> moff;
    int64_t msize = 0;
    int32_t max_lds = 0;
    double product_bytes = 0, product_flops = 0;
};
// edges: rep_point[R], dep_point/dep_scale[D], arap_pts[4E], arap_pair[E]; vertex ids T_g q -> q,
// scale k -> Q + k, point p -> Q + S + p.  False (with err) when the plan does not fit the kernels.
bool build_pcg_mf(int64_t nv, const std::vector<int64_t> &voff, const std::vector<int32_t> &vdim,
                  const std::vector<int64_t> &elim_pos, int Q, int S, int R, int D, int E,
                  const int32_t *rep_point, const int32_t *dep_point, const int32_t *dep_scale,
                  const int32_t *arap_pts, const int32_t *arap_pair, PcgMfHost &out, std::string &err);

struct PcgDev {
    int64_t nv = 0, ndof = 0;
    int32_t mf = 0, mf_lds = 0;          // matrix-free product; its dynamic LDS (doubles)
    const int64_t *mf_le_off = nullptr, *mf_le = nullptr, *mf_in_off = nullptr;
    const int32_t *mf_le_n = nullptr, *mf_le_na = nullptr, *mf_in_n = nullptr, *mf_inc = nullptr, *mf_inc2 = nullptr;
    const int32_t *mf_adof = nullptr, *mf_atdof = nullptr, *mf_rdof = nullptr, *mf_ddof = nullptr;
    const int32_t *mf_sl_nt = nullptr, *mf_own_n = nullptr, *mf_own = nullptr;
    const int64_t *mf_own_off = nullptr, *mf_sl_meta = nullptr;
    const int32_t *mf_sl_hpos = nullptr;
    const double *Jarap = nullptr, *Warap = nullptr, *Earap = nullptr;
    const double *Jrep = nullptr, *Wrep = nullptr, *Erep = nullptr;
    const double *Jdep = nullptr, *Wdep = nullptr, *Edep = nullptr;
    double *mf_diag = nullptr;           // per vertex (moff): its diagonal block of H
    double *mf_hlin = nullptr;           // per heavy slot position: kMfLin partials
    double *mf_dvec = nullptr;           // diagonal of H per dof (max diag)
    double *b = nullptr;                 // the plan's b (k_mf_lin writes it)
    int32_t nlight = 0, nheavy = 0, nhchunks = 0, nheavy_dofs = 0;
    int32_t nA_light = 0;                // workgroups of the light part of the product launch
    int32_t nsl = 0, nA_sl = 0;          // slices; their workgroups (one per slice) lead the launch
    int64_t nslots = 0;                  // 3x3 slots of all slices
    const int32_t *sl_v = nullptr, *sl_n = nullptr, *sl_nx = nullptr, *sl_col = nullptr;
    const int64_t *sl_off = nullptr, *sl_xoff = nullptr, *sl_map = nullptr;
    const PcgEnt *sl_x = nullptr;
    double *sl_val = nullptr;            // repacked 3x3 blocks: nslots x 5 x 64 double2 (9 values + column dof)
    int64_t nhslots = 0;
    const int32_t *sl_hn = nullptr, *hs_hk = nullptr;
    const int64_t *sl_hoff = nullptr, *hs_map = nullptr, *hv_slot_begin = nullptr, *hs_pos = nullptr;
    const int64_t *hs_voff = nullptr;
    const PcgEnt *hres = nullptr;        // heavy rows' remaining entries (hc_beg / hc_end index these)
    double *hs_val = nullptr;            // repacked heavy-slot blocks: per slot ceil(3 od / 2) x 64 double2
    double *hs_part = nullptr;           // per heavy slot: 6 partial sums of the heavy row
    double *hqf = nullptr;               // per heavy dof: q = (H + lambda I) p of the heavy rows
    int32_t nB = 0;                      // workgroups of the vertex launches (setup / update)
    const int64_t *ent_begin = nullptr;
    const PcgEnt *ent = nullptr;
    const int32_t *light_v = nullptr, *heavy_v = nullptr, *hc_vertex = nullptr, *h_first = nullptr;
    const int32_t *h_dofbase = nullptr, *v_heavy = nullptr;
    const int64_t *hc_beg = nullptr, *hc_end = nullptr, *diag_off = nullptr, *moff = nullptr;
    const int64_t *voff = nullptr;
    const int32_t *vdim = nullptr;
    double *minv = nullptr;              // (H_vv + lambda I)^-1 per vertex
    double *r = nullptr;
    double *zp = nullptr;                // (z, p_prev) per dof
    double *pq = nullptr;                // (p, q) per dof
    double *partA = nullptr;             // per sliced / light workgroup of the product: p.q
    double *partB = nullptr;             // per vertex workgroup: (r.z, r.r)
    double *rec = nullptr;               // (max_it + 2) x kPcgRec
    int32_t max_it = 0;
    double tol2 = 0;                     // squared relative residual tolerance
};

// after an assembly: the sliced rows' 3x3 blocks from hval into sl_val
void launch_pcg_repack(const PcgDev &G, const double *hval, hipStream_t st);
// matrix-free: per LM iteration (after the linearization) the diagonal blocks and b; with
// want_dvec the diagonal of H per dof too (max diag for the initial lambda)
void launch_mf_lin(const PcgDev &G, bool want_dvec, hipStream_t st);
// one solve's launches (x = dx).  setup: preconditioner blocks at lambda, r = b, z = M r, x = 0.
// rec_cleared: the records were cleared by the trial's prologue (launch_trial_begin)
void launch_pcg_setup(const PcgDev &G, const double *hval, const double *b, double lambda, double *x,
                      hipStream_t st, bool rec_cleared = false);
// iteration it: product q = (H + lambda I) p (p = z + beta p_prev formed on the fly) after the
// convergence test of the residual the previous update left
void launch_pcg_product(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st);
// iteration it, after the product: the heavy rows' q (one workgroup per dof: slot partials +
// remaining entries) and the generic light rows
void launch_pcg_heavy(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st);
// iteration it: alpha, x += alpha p, r -= alpha q, z = M r, partial (r.z, r.r)
void launch_pcg_update(const PcgDev &G, int it, double lambda, double *x, hipStream_t st);

}  // namespace deftri
