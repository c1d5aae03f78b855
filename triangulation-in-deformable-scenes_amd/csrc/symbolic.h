// symbolic.h — host-side analysis of the LM normal equations for the device LDL^T.
//
// Replaces g2o's BlockSolverX + LinearSolverEigen structure analysis
// (reference g2oBundleAdjustment.cc:619-628 builds the solver; the LM calls buildStructure()
// on iteration 0).  Instead of Eigen's AMD + SimplicialLDLT we build a multifrontal plan:
//   * fill-reducing order: geometric nested dissection of the point vertices on their mesh-plane
//     coordinates (the same 2-D plane the reference triangulates, Geometry.cc:317-368), global
//     vertices (T_g, depth scales) last;
//   * one dense front per dissection node (leaf subdomain or separator), column-major fp64 in one
//     HBM arena; boundary rows = later-eliminated coupled vertices;
//   * assembly lists: every entry of H (vertex-pair blocks) and of b is produced by a fixed-order
//     gather over per-edge contributions (deterministic, no atomics);
//   * per-level task lists for the batched dense kernels (diag LDL^T, TRSM, trailing update,
//     extend-add, forward/backward substitution).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/deftri.h"

namespace deftri {

// edge kinds in contribution records
enum : int { EK_REP = 0, EK_DEP = 1, EK_ARAP = 2 };

// contribution record: (edge kind, edge index, role of the column vertex, role of the row vertex)
static inline uint64_t contrib_pack(int kind, int64_t edge, int role_col, int role_row) {
    return (uint64_t)edge | ((uint64_t)kind << 40) | ((uint64_t)role_col << 44) | ((uint64_t)role_row << 48);
}

constexpr int kPanel = 64;          // panel width of the blocked dense kernels
#ifndef DEFTRI_OUTER
#define DEFTRI_OUTER 256
#endif
constexpr int kOuter = DEFTRI_OUTER; // outer block: trailing updates beyond it use K = kOuter (tuning knob)
#ifndef DEFTRI_CHUNK
#define DEFTRI_CHUNK 64
#endif
constexpr int kChunk = DEFTRI_CHUNK; // contributions per gather chunk (A/B 32/64/128: 64 best, tuning knob)
constexpr int kBwdCols = 16;        // own columns per backward-init task

struct Front {
    int64_t arena_off;   // m*m doubles, column-major, ld = m
    int64_t vec_off;     // m doubles of solve workspace
    int64_t rows_off;    // m entries of `rows` (problem dof of each local row)
    int64_t bmap_off;    // (m - s) entries of `bmap` (local row in the parent front)
    int64_t inv_off;     // inverses of the unit-lower panel triangles: panel p at inv_off + p*64*64
                         // (kb x kb, column-major, ld = kb)
    int32_t m, s;
    int32_t parent;
    int32_t height;
    int32_t direct;      // 1: the final trailing update adds this front's contribution block straight
                         //    into the parent (no extend-add); 0: extend-add (a same-level slot-1 sibling)
    int32_t nchild;
    int32_t child[2];
    int32_t owner;       // rank that assembles and factors this front (0 on one rank)
    int32_t rhs_bnd;     // 1: this rank's top front under a remote parent — its boundary rows start the
                         //    forward solve from the rank's partial b of those (remote) vertices
    int32_t panel_off;   // index of this front's first panel in the plan's per-panel "factored" flags
};

// Point-sharded plan (subtree-to-rank mapping of the nested-dissection tree).  Every rank runs the
// same analysis; the top of the tree is split by rank ranges (a front with ranks [lo, hi) is owned by
// lo, its children get [lo, mid) and [mid, hi), mid by subtree flops) until a range holds one rank,
// whose whole subtree it then owns.  An edge is owned (linearized, chi2-summed) by the owner of the
// front of its first-eliminated vertex.  Its contributions to blocks of a remote front (an ancestor)
// are assembled into the contribution-block region of the rank's top front instead — those rows are
// boundary rows there — so they reach the owner through the one cross-rank transfer per rank: the
// packed lower triangle of that top front's contribution block (factorization), its forward-update
// vector (forward solve) and, back down, the solution of its boundary rows (backward solve).
struct DistPlan {
    int32_t rank = 0, nranks = 1;
    int32_t top = -1;                  // this rank's top front when its parent is remote, else -1
    struct Xfer {
        int32_t child = 0, parent = 0, src = 0, dst = 0, level = 0;   // level = height of the parent
        int32_t u = 0;                 // contribution-block order of the child
        int64_t buf_off = 0;           // this rank's staging buffer (packed u(u+1)/2 doubles), if a party
        int64_t ea_off = 0; int32_t nea = 0;   // receiver: packed extend-add tasks (child, j0, i0)
    };
    std::vector<Xfer> xfers;           // global list (identical on every rank), by level then child
    int64_t xbuf_size = 0;
    std::vector<int32_t> own_rep, own_dep, own_arap;   // global ids of the edges this rank owns
    std::vector<int32_t> vertex_owner;                 // per vertex (problem order)
    std::vector<uint8_t> dof_local;                    // per dof: its front is factored on this rank
    double factor_flops_total = 0;                     // all ranks
    int64_t nnz_factor_total = 0;
};

struct Symbolic {
    // vertices in problem order: [T_g per pair][scales][points]
    int64_t nv = 0, ndof = 0;
    std::vector<int32_t> vdim;
    std::vector<int64_t> voff;
    std::vector<int64_t> elim_pos;      // vertex -> elimination position
    // fronts
    std::vector<Front> fronts;
    std::vector<int32_t> rows;
    std::vector<int32_t> bmap;
    int64_t arena_size = 0, vec_size = 0, inv_size = 0;
    int64_t npanels = 0;                         // panels of this rank's fronts (flag slots)
    bool trsm_fused = false;                     // task lists carry fused-TRSM tail tiles (DEFTRI_TRSM_FUSE=1)
    int32_t nlevels = 0;
    std::vector<std::vector<int32_t>> level_fronts;   // this rank's fronts by height, ascending
    double factor_flops = 0;          // this rank's fronts
    double update_flops = 0, diag_flops = 0, trsm_flops = 0;   // per factorization, by kernel
    int64_t nnz_factor = 0;

    // H blocks: column vertex c (eliminated no later than the row vertex r)
    int64_t nblocks = 0, hval_size = 0;
    std::vector<int64_t> blk_val_off;    // offset into Hval (rows x cols, row-major)
    std::vector<int32_t> blk_rows, blk_cols;
    std::vector<int64_t> blk_arena;      // arena index of entry (0,0)
    std::vector<int32_t> blk_ld;
    std::vector<int32_t> blk_diag;       // 1 if diagonal block (row vertex == column vertex)
    std::vector<int64_t> blk_row_dof, blk_col_dof;   // first dof of the block's row / column vertex
    // contributions to H blocks, chunked
    std::vector<uint64_t> hcontrib;
    std::vector<int64_t> hchunk_begin;   // per chunk: first contribution
    std::vector<int32_t> hchunk_len;
    std::vector<int32_t> hchunk_block;
    std::vector<int64_t> hblk_chunk_begin; // per block: first chunk (CSR, nblocks+1)
    // contributions to b (per vertex), chunked the same way; role_row unused
    std::vector<uint64_t> bcontrib;
    std::vector<int64_t> bchunk_begin;
    std::vector<int32_t> bchunk_len;
    std::vector<int32_t> bchunk_vertex;
    std::vector<int64_t> bv_chunk_begin;   // per vertex (nv+1)

    // per-level task lists (device copies are flat arrays with offsets)
    struct StepTasks {
        int64_t diag_off = 0; int32_t ndiag = 0;      // fronts with own cols at this panel
        int64_t trsm_off = 0; int32_t ntrsm = 0;      // (front, row-tile) pairs
        int64_t upd_off = 0; int32_t nupd = 0;        // (front, tile-i, tile-j) triples
        // fused TRSM: the last ntail update tasks are the column tiles (i > k1, k1) of a panel whose
        // diagonal tile this launch factors — after their update they wait for that panel's flag and
        // solve their rows in place; the diag launch likewise carries ndiag_tail (front, k0, r0) tiles
        // right after its ndiag tasks
        int32_t ntail = 0, ndiag_tail = 0;
        int32_t k0 = 0;                               // panel of diag / trsm
        int32_t kA = 0, kmax = 0;                     // update: L columns [kA, kA + min(kmax, s - kA))
        int32_t inner = 0;                            // column clip: 0 none, 1 end of this outer block
                                                      // (inner update), 2 end of the next block (lookahead)
        int32_t stream = 0;                           // 0: main stream; 1: side stream (trailing "rest"
                                                      // update, overlaps the next block's panel chain)
        int32_t wait_side = 0;                        // main stream waits for side launches first:
                                                      // 1 the one before the latest, 2 all of them
        double upd_flops = 0;                         // algorithmic flops of this update launch
    };
    struct LevelTasks {
        int64_t ea_off[2] = {0, 0}; int32_t nea[2] = {0, 0};   // extend-add (child slot 0/1): (parent, child col)
        std::vector<StepTasks> steps;
        // substitution: forward = gather (one task per front) then one launch per panel step with
        // (front, k0, r0) tasks — r0 == k0: solve the panel triangle and publish y; r0 > k0: rows
        // r0..r0+63 below the panel -= L[r, panel] y.  Backward = init (front, c0: 16 own columns,
        // w = y/d - L21^T x_B) then panel steps in descending order with (front, k0, q0) tasks —
        // q0 == k0: solve L_pp^T x = w_p and scatter x; q0 < k0: w[q0..q0+63] -= L[panel, q]^T x_p.
        int64_t fwd_off = 0; int32_t nfwd = 0;                 // fronts (gather)
        struct SolveStep { int64_t off = 0; int32_t n = 0; };
        std::vector<SolveStep> fsteps, bsteps;                 // bsteps: already in execution order
        int64_t bgemv_off = 0; int32_t nbgemv = 0;             // (front, c0) backward init, 16 columns each
        // chained substitution (one launch per level and direction, k_fwd_chain / k_bwd_chain):
        // forward (front, r0) row tiles of 64 in ascending r0 per front — each waits for the panels
        // above it, applies them, and publishes its own panel's y; backward (front, c0) own-column
        // tiles in descending c0 per front — each waits for the panels after it and publishes x
        int64_t fchain_off = 0; int32_t nfchain = 0;
        int64_t bchain_off = 0; int32_t nbchain = 0;
    };
    std::vector<LevelTasks> levels;
    std::vector<int32_t> task_i32;     // flat task storage (3 ints per task record)

    DistPlan dist;
    std::string error;
};

// Build the plan of rank `rank` of `nranks` for a validated problem (nranks = 1: the whole plan).
// Returns false (and sets error) on failure.
bool analyse(const deftri_problem_desc &d, Symbolic &S, int leaf_points = 32, int rank = 0,
             int nranks = 1);   // leaf 32: best of 8..64 at C2

}  // namespace deftri
