// spcg.h — the point-sharded matrix-free PCG plan ("iterative plan"): the LM step
// (H + lambda I) dx = b of arapOptimization's g2o solve (reference Modules/Optimization/
// g2oBundleAdjustment.cc:608-1008, optimizer call :959-962) for graphs of any keyframe count,
// sharded over ranks (one GPU each) without the multifrontal analysis.
//
// Rows.  Every point is a row; the keyframe copies of a mesh vertex (the points an ARAP edge pairs
// at roles (0, 1) and (2, 3), g2oBundleAdjustment.cc:871-953) form one group, groups are ordered
// by the Morton code of their mesh-plane position (deftri_problem_desc.order_xy) and dealt to the
// ranks in contiguous, work-balanced ranges.  The device state keeps the points in this row order;
// dof layout [T_g 6 per pair][scales][rows 3 each].  The global vertices (T_g, depth scales) are
// "heavy": replicated on every rank.
//
// Edges of a rank.  Reprojection and depth edges of its rows; ARAP edges with at least one point
// in its rows ("local"), owned (chi2, heavy sums) by the rank of their point 0.  The points of
// local edges on other ranks are the rank's halo.
//
// One product q = (H + lambda I) p, H = sum_e J_e^T W_e J_e, never assembled:
//   phase 1 (per local ARAP edge, edge-parallel): s_e = W_e (J_e p) over the edge's 4 points and
//            its pair's T_g; s_e stored; owned edges add J_T^T s_e into a per-block partial of
//            their T_g; per depth edge (blocks by scale) c_e . p_row + W J_s^2 p_s into the
//            scale's partial;
//   phase 2 (per own row, row-parallel): q_v = lambda p_v + D_v p_v + sum_dep c_e p_s(e)
//            + sum over its ARAP incidences J_{e,role}^T s_e, where D_v folds the row's
//            reprojection and depth point blocks (single-point edges: camera fixed) and c_e = W J_p J_s;
//   heavy  : q_h = (sum of its blocks' partials, all ranks) + lambda p_h.
// No atomics; every sum has a fixed order, so a solve on a given rank count is bit-reproducible.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/deftri.h"
#include "kernels.h"

namespace deftri {

constexpr int kSpBlock = 256;          // edges per phase-1 block / rows per row block
constexpr int kSpRed = 16;             // doubles per iteration in the reduction record
constexpr int kSpPart = 8;             // doubles per phase-1 block partial
constexpr int kSpLin = 27;             // doubles per block partial of the per-iteration heavy lin (21 H + 6 b)
constexpr int kSpSortWindow = 512;     // rows sorted by entry count inside windows of this many
constexpr int kSpWaveSplit = 16;       // phase-2 waves with rows of more slots take 32 rows on lane pairs
constexpr int kSpRowSplit = 1;         // phase 2: waves per row-wave's slot list (DEFTRI_SP_ROW_SPLIT)
constexpr int kSpP2Step = 8;           // phase 2: slots per step (DEFTRI_SP_P2_STEP = 4 or 8)
constexpr int kSpGlinGroup = 8;        // k_sp_glin_blocks: owned ARAP blocks per workgroup at most
constexpr int kSpGlinStep = 8;         // k_sp_glin_rows: slots per step (DEFTRI_SP_GLIN_STEP = 4 or 8)
constexpr int kSpGuessMargin = 1;      // CG iterations queued per trial: last converged count + this
constexpr int kSpHeavySplit = 512;         // heavy sums by one workgroup per heavy vertex above this many blocks
constexpr int kSpUpdRows = 256;           // rows per k_sp_update workgroup (one thread per dof)
constexpr int kSpHeavyChunk = 128;        // block partials per k_sp_glin_heavy workgroup
constexpr int kSpFuseHeavyMax = 8192;      // one rank: heavy block partials one workgroup reduces after phase 2
constexpr int64_t kSpMergeMinDof = 50000;  // one rank: the merged (two-launch) CG chain from this many unknowns
// tile mode (spcg_tile.cpp): the fused product, every ARAP edge read once — one pair (one rank or
// sharded), or on one rank several pairs (tiles per pair, tile_multi)
constexpr int kSpTileUnits = 128;          // mesh vertices (keyframe-copy groups) per tile at most
constexpr int kSpTileLds = 39 * 1024;      // dynamic LDS bytes per tile at most (with ~0.6 KB static: 4 workgroups per CU)
constexpr int kSpTilePartsMax = 2048;      // tile grids above this: ticketed CG sums (spcg_solver.cpp)
constexpr int kSpTileLdsFixed = 2048;      // the tile kernel's fixed dynamic LDS (heavy p; the heavy workgroup's sums)
// tile entry meta word 0: LDS rows of p1_j (bits 0-11), p2_j (12-23), flags; word 1: LDS slots of
// p1_j (0-11), p2_j (12-23), the unit's first tile row (24-31)
constexpr uint32_t kTmHead = 1u << 24, kTmLast = 1u << 25, kTmSwap = 1u << 26, kTmValid = 1u << 27, kTmCut = 1u << 28;
// sharded tile plans: kTmDrop — an owned edge whose j vertex is another rank's (its j rows' share is
// that rank's); kTmForeign — a halo-only edge (another rank's i vertex, this tile's j vertex): its i
// rows in the j fields, its j rows at ub / swap, only the j rows' slots written, no owned sums
constexpr uint32_t kTmDrop = 1u << 29, kTmForeign = 1u << 30;
enum { SP_ARAP = 0, SP_DEP = 1 };
// solve status (record word 0).  kSpTimeout: the merged chain's alpha hand-off was not seen within
// its poll bound (phase 2's workgroup 0 not resident while the others waited): an error, never a
// rejected trial (SpSolver raises it and switches the context to the separate alpha launch)
enum { kSpRunning = 0, kSpConverged = 1, kSpBreakdown = 2, kSpBadBlock = 3, kSpBudget = 4, kSpTimeout = 5 };

// the transport of a sharded solve (solver.cpp: RCCL on the solver stream, or the caller's host
// callback); every rank issues the same calls in the same order
struct SpTransport {
    virtual ~SpTransport() {}
    virtual int allreduce(double *dev, int64_t n, int op, hipStream_t st) = 0;   // op 0 sum, 1 max
    struct Op { int peer; bool send; double *buf; int64_t n; };
    virtual int p2p(const std::vector<Op> &ops, hipStream_t st) = 0;             // one global order
};

// host plan of one rank
struct SpPlanHost {
    int rank = 0, nranks = 1;
    int32_t P = 0, Q = 0, S = 0;
    int64_t hd = 0;                                    // heavy dofs 6Q + S
    std::vector<int32_t> row_of_point, point_of_row;   // global row order
    std::vector<int32_t> rank_row_begin;               // nranks + 1
    int32_t lo = 0, hi = 0;                            // own rows
    // local edges (global ids) in device order
    std::vector<int32_t> arap_ids;                     // [owned (pair, row0) | halo-only (pair, row0)]
    int32_t n_arap_owned = 0;
    std::vector<int32_t> rep_ids, dep_ids;             // the own rows' edges, sorted by row (stable)
    std::vector<int32_t> rot_ids;                      // rotation-table rows used, local index order
    std::vector<int32_t> arap_rot_local;               // [2 * local arap]
    // phase-1 blocks: (kind | owned << 8, heavy vertex (pair or scale), begin, end)
    std::vector<int32_t> blk;                          // 4 per block
    std::vector<int32_t> hv_blk;                       // per heavy vertex (Q + S): its partial blocks, CSR
    std::vector<int64_t> hv_blk_off;                   // Q + S + 1
    std::vector<int32_t> dperm;                        // local depth edges sorted by (scale, row)
    // row CSR (own rows, local index)
    std::vector<int64_t> inc_off;                      // nown + 1
    std::vector<int32_t> inc;                          // local arap edge << 2 | role
    std::vector<int32_t> rep_off, dep_off;             // nown + 1, into the local rep / dep arrays
    // phase-2 wave layout: rows dealt to 64-lane waves (sorted by entry count inside windows of
    // kSpSortWindow rows so a wave pads little); wave w's entries are slots woff[w] .. woff[w + 1] - 1,
    // slot k of lane j at [k][64] + j.  pmap: ARAP incidence le << 2 | role, depth coupling -(2 + j)
    // (local depth edge j), -1 padding; pidx (what phase 2 multiplies the slot's J by): s[le] for
    // ARAP, -(2 + scale) for a depth coupling (p of the scale), -1 padding
    std::vector<int32_t> rowmap;                       // [nwaves * 64]: local row per lane (-1 padding)
    std::vector<int64_t> woff;                         // nwaves + 1, in slots
    std::vector<uint8_t> wsplit;                       // per wave: 1 = 32 rows on lane pairs (j, j + 32)
    std::vector<int32_t> pmap, pidx;                   // [slots * 64]
    int32_t max_heavy_blocks = 0;                      // most phase-1 blocks of one heavy vertex
    // halo exchange: rows (global) sent to / received from each peer, ascending
    std::vector<std::vector<int32_t>> send_rows, recv_rows;
    int64_t halo_rows = 0;
    double product_bytes = 0;                          // algorithmic bytes of phase 1 + 2 (one CG iteration)
    double phase1_bytes = 0, phase2_bytes = 0;
    // tile mode (spcg_tile.cpp; the local ARAP edges are then in tile-entry order)
    bool tile = false;
    std::string tile_why;                              // why a requested tile layout was not built
    int32_t ntile = 0, tile_segmax = 1, tile_lds = 0;
    int64_t tile_entries = 0, tile_cross = 0, tile_halo_rows = 0;
    std::vector<int32_t> tile_tab;                     // 8 per tile: r0, nr, nh, e0, ne, h0, ns, pair
    // several pairs (tile_multi): a tile's own rows are listed (tile_trow from r0: row | home << 31,
    // home = the first tile holding the row, which adds its diagonal terms and stores q; the others
    // store their share in share plane tile_tdst - 1); tiles of pair q are tile_poff[q] .. [q + 1] - 1
    bool tile_multi = false;
    std::vector<int32_t> tile_trow, tile_tdst, tile_poff;   // tile_tdst: the entry's share (0 = home)
    std::vector<int32_t> tile_nshare;                  // per row: its shares (tiles); planes = max - 1
    int32_t tile_planes = 0;
    std::vector<uint32_t> tile_m0, tile_m1;            // per entry (padded to 64 per chunk)
    std::vector<int32_t> tile_chunk;                   // 2 per chunk: first le, first cross slot
    std::vector<int32_t> tile_rs;                      // per own row (entry): LDS slot begin | count << 16
    std::vector<int32_t> tile_halo;                    // the tiles' halo rows (global row ids)
    std::vector<int32_t> tile_xoff;                    // per own row its cross slots (destination order)
    std::vector<int32_t> tile_xdst;                    // per cut entry (source order): its 2 cross slots
    double tile_bytes[2] = {0, 0};                     // algorithmic bytes per CG iteration: product, update
};
// the groups and rows build_tiles needs (spcg_plan.cpp step 5)
// the Z-order (Morton) key of a point from its (x, y) in a bounding box, 21 bits per coordinate — the
// plans' point orders (a Hilbert curve measured no better: C2 and C5 slower, 500k and C3 1-3 % faster)
inline uint64_t curve_key(double x, double y, const double lo[2], const double hi[2]) {
    uint32_t k[2];
    const double v[2] = {x, y};
    for (int c = 0; c < 2; c++) {
        const double span = hi[c] > lo[c] ? hi[c] - lo[c] : 1.0;
        double t = std::isfinite(v[c]) ? (v[c] - lo[c]) / span : 0.0;
        t = t < 0.0 ? 0.0 : t > 1.0 ? 1.0 : t;
        k[c] = (uint32_t)(t * 2097151.0);
    }
    uint64_t m = 0;
    for (int b = 0; b < 21; b++) m |= (uint64_t)((k[0] >> b) & 1u) << (2 * b) | (uint64_t)((k[1] >> b) & 1u) << (2 * b + 1);
    return m;
}

struct TileInput {
    int32_t P = 0, ng = 0;
    int64_t E = 0;
    const int32_t *ap = nullptr;                       // arap_pts [E][4]
    const int32_t *gpos = nullptr;                     // per point: its group's Morton position
    const int32_t *row_of_point = nullptr;
    // several pairs (build_tiles_multi)
    int32_t Q = 1, S = 0;
    const int32_t *pair = nullptr;                     // arap_pair [E]
    int64_t D = 0;
    const int32_t *dep_point = nullptr, *dep_scale = nullptr;
    const double *points = nullptr;                    // [P][3]: a pair's units ordered by their mesh positions
};
// tile layout of a one-rank, one-pair plan: false (why) when the graph does not fit tile mode; order:
// the ARAP edges in tile-entry order (the plan's local edge order)
// order: the owned ARAP edges in tile-entry order (the plan's first local edges), order_foreign: the
// halo-only ones (sharded plans; after them); H.lo / H.hi the rank's rows
bool build_tiles(const TileInput &in, SpPlanHost &H, std::vector<int32_t> &order, std::vector<int32_t> &order_foreign,
                 std::string &why);
// the same on one rank for a graph of several keyframe pairs (the all-pairs graph of
// g2oBundleAdjustment.cc:640-645 or its window): tiles per pair over (pair, group) units
bool build_tiles_multi(const TileInput &in, SpPlanHost &H, std::vector<int32_t> &order, std::string &why);
// host emulation of one tile-mode product with its layout checks (tests; spcg_tile.cpp)
int sp_emulate_tile_product(const deftri_problem_desc &d, const SpPlanHost &H, const double *Ja, const double *Wa,
                            const double *Jr, const double *Wr, const double *Jd, const double *Wd, double lambda,
                            const double *p, double *q, std::string &why);
// rank's plan of a validated problem; false (err) when the problem cannot be planned
// tile: try the tile layout (one rank, one pair; spcg_tile.cpp) — out.tile says whether it was built
bool build_sp_plan(const deftri_problem_desc &d, int rank, int nranks, bool fp32_jac, SpPlanHost &out,
                   std::string &err, bool tile = false);
// host emulation of one sharded product on the plan (tests; spcg_plan.cpp)
int sp_emulate_product(const deftri_problem_desc &d, const SpPlanHost &H, const double *Ja, const double *Wa,
                       const double *Jr, const double *Wr, const double *Jd, const double *Wd, double lambda,
                       const double *p, double *q, const std::function<int(int, int, double *, int64_t)> &xfer);

// device view (kernels)
struct SpDev {
    int32_t P = 0, Q = 0, S = 0;
    int64_t hd = 0, ndof = 0;
    int32_t row0 = 0, nown = 0;
    int32_t nblk = 0, nrb = 0;                         // phase-1 blocks, row blocks
    int32_t include_heavy = 1;                         // this rank counts the replicated heavy dofs in sums
    const int4 *blk = nullptr;
    const int2 *glb = nullptr;                            // k_sp_glin_blocks' groups: (first block, count)
    int32_t nglb = 0;
    const int32_t *hv_blk = nullptr;
    const int64_t *hv_blk_off = nullptr;
    const int32_t *apts = nullptr, *apair = nullptr;   // local ARAP edges: rows, pair
    const double *Ja = nullptr, *Wa = nullptr, *Ea = nullptr;
    const float *Ja32 = nullptr;                       // fp32 copy of Ja (deftri_set_jacobian_storage 1)
    const double *Jr = nullptr, *Wr = nullptr, *Er = nullptr;
    const double *Jd = nullptr, *Wd = nullptr, *Ed = nullptr;
    const int32_t *dsc = nullptr, *drow = nullptr, *dperm = nullptr;
    const int64_t *inc_off = nullptr;
    const int32_t *inc = nullptr, *rep_off = nullptr, *dep_off = nullptr;
    int64_t jld = 0;                                   // column stride of Ja / Ja32 ([18][jld])
    int32_t nwaves = 0, heavy_split = 0;
    // phase 2: each row-wave's slot steps split over rs waves (1, 2, 4); its workgroups hold 4 / rs
    // row-waves, nrb2 = ceil(nwaves rs / 4) of them (p.q partials rpart [nrb2])
    int32_t rs = 1, nrb2 = 0;
    int32_t p2u = 8;                                   // phase 2's slots per step (8 or 4)
    int32_t glu = 8;                                   // k_sp_glin_rows' slots per step (8 or 4)
    int64_t nslots = 0;                                // wave-layout slots (x 64 lanes)
    const int32_t *rowmap = nullptr, *pmap = nullptr, *pidx = nullptr;
    const int64_t *woff = nullptr;
    const uint8_t *wsplit = nullptr;                   // per wave: rows on lane pairs (spcg_plan.cpp 8b)
    double *pj = nullptr;                              // packed J slices: [3][nslots * 64] (fp64)
    float *pj32 = nullptr;                             // the same in fp32 (fp32 Jacobian storage)
    // per-LM-iteration
    double *Hv = nullptr, *Dv = nullptr, *Mv = nullptr;   // own rows: 6 each (lower 3x3: 00 10 11 20 21 22)
    double *cdep = nullptr, *wss = nullptr;               // per local depth edge: W J_p J_s (3), W J_s^2
    double *hl = nullptr;                                 // [H_T lower 21 per pair | H_s per scale | b (ndof)]
    double *b = nullptr;                                  // = hl + 21 Q + S
    double *Mh = nullptr;                                 // heavy preconditioner: 36 per pair, 1 per scale
    double *lpart = nullptr;                              // glin block partials [nblk][27]
    double *mpart = nullptr;                              // row-block max diag
    // CG
    double *r = nullptr, *q = nullptr, *x = nullptr;
    double2 *zp = nullptr;                                // (z, p) per dof
    double *s = nullptr;                                  // phase-1 s_e per local ARAP edge
    double *part = nullptr;                               // phase-1 block partials [nblk][8]
    double *rpart = nullptr;                              // phase-2 row-block partials p.q [nrb2]
    double *upart = nullptr;
    double *hbuf = nullptr;                               // [pq_rows, heavy sums (hd)]
    // [max_it + 2][kSpRed]: rz, rr, stop, alpha.  stop (word 2 of iteration it + 1): a breakdown /
    // hand-off timeout found inside iteration it's phase 2 (merged chain).  It is read from the next
    // launch on, so every workgroup of one launch sees the same state: a status written into rec[0]
    // during phase 2 would send the workgroups dispatched after it home before their tickets
    double *red = nullptr;
    double *rec = nullptr;                                // [8]: status, its
    int *cnt = nullptr;                                   // [48] last-workgroup tickets, 16 per site (0 between launches)
    // k_sp_glin_heavy chunks: chunk j sums hv_blk[ch_lo[j] .. ch_lo[j + 1]) of heavy ch_h[j]; heavy h
    // owns chunks hch_off[h] .. hch_off[h + 1] (at least one); chpart [nch][27]; hcnt per heavy
    int32_t nch = 0;
    const int32_t *ch_h = nullptr, *hch_off = nullptr;
    const int64_t *ch_lo = nullptr;
    double *chpart = nullptr;
    int *hcnt = nullptr;
    int32_t fuse = 0;                                     // one rank: dots in the update's / setup's last workgroup
    int32_t fuse_heavy = 0;                               // ... and k_sp_heavy in k_sp_phase2's last workgroup
    // one rank, two launches per CG iteration (merged chain): phase 1 also forms p.Ap (alpha in its
    // last workgroup), phase 2 also updates x, r, z and forms (r.z, r.r) of the next iteration
    int32_t merged = 0;
    int32_t m_nx = 0;                                     // phase 1's extra workgroups (heavy p + row terms), 8k
    int32_t m_nh = 0;                                     // phase 2's heavy workgroups, 8k
    double *ph = nullptr;                                 // p of the heavy dofs this iteration (phase 1 -> 2)
    double *m1part = nullptr;                             // phase-1 p.Ap per workgroup [m1n = m_nx + nblk]
    int32_t m1n = 0;
    int32_t alpha_kernel = 0;                             // alpha by k_sp_alpha between the phases (no hand-off)
    int32_t inj_timeout_it = -1;                          // tests: the hand-off of this CG iteration times out
    // sharded single-reduction chain (sd, any rank count with a transport): per CG iteration phase 1
    // and phase 2 form w = A z and this rank's part of xb, the host all-reduces xb, k_sp_update_sd
    // updates and fills the send buffer; the boundary rows' (z, p) land in the receive region of zp
    // (rows P .. P + halo: apts_p maps the local edges' halo rows there)
    int32_t sd = 0;
    double *sv = nullptr;                                 // s = A p by recurrence (ndof)
    double *xb = nullptr;                                 // [3 + hd]: r.z, r.r, z.Az, heavy sums of A z
    const int32_t *apts_p = nullptr;                      // local ARAP edges' rows, halo rows -> P + k
    const int32_t *snd_off = nullptr, *snd_slot = nullptr;   // own row l: send slots (rows of sbuf)
    double *sbuf = nullptr;                               // [send rows][6]: (z, p) of 3 dofs
    double *m2part = nullptr;                             // phase-2 (r.z, r.r) per workgroup [m_nh + row grid][2]
    double *gsum = nullptr;                               // per XCD group sums [2 sites][8][2]
    int32_t max_it = 0;
    double tol2 = 0;
    // tile mode (G.tile): k_sp_tile (the fused product + p.Ap) and k_sp_tupd (cross slots, alpha, update)
    int32_t tile = 0, ntile = 0, tile_lds = 0, tile_segmax = 1;
    const int32_t *ttab = nullptr;                        // [ntile][8]
    const uint2 *tmeta = nullptr;                         // per entry (word 0, word 1)
    const int2 *tchunk = nullptr;                         // per chunk (first le, first cross slot)
    const int32_t *trs = nullptr, *thalo = nullptr, *txoff = nullptr;
    const int2 *txdst = nullptr;                          // per cut entry: its two cross slots (destination order)
    double *xc = nullptr;                                 // cross slots [n][3], by target row
    const double *pinfo = nullptr;                        // per pair: Omega (= W of its ARAP edges)
    int32_t t_grid = 0;                                   // k_sp_tile's workgroups (tiles XCD-dealt + heavy)
    int32_t tmulti = 0;                                   // several pairs (SpPlanHost::tile_multi)
    const int32_t *trow = nullptr, *tdst = nullptr, *tpoff = nullptr, *tnshare = nullptr;
    const int32_t *tdep = nullptr;             // per tile row: 2 j + (scale & 1) of its depth edge j in the tile's pair, or -1
    double *qs = nullptr;                                 // share planes [planes][nown][3]
    int32_t ovl = 0;                                      // sharded: halo exchange beside the interior product
    const int32_t *p1list = nullptr;                      // sharded phase 1: the launch's workgroups -> logical ones
    int32_t tparts = 0;                                   // tile mode: each k_sp_tile workgroup sums the update's
                                                          // (r.z, r.r) partials itself (no ticket chain in k_sp_tupd)
    // device-driven LM (SpSolver::solve_lm_dev): a trial's kernels return at once when *gate == 0, the
    // per-iteration ones when *lgate == 0; lambda from *lam_dev instead of the launch argument
    const int *gate = nullptr, *lgate = nullptr;
    const double *lam_dev = nullptr;
};

// launchers (spcg.hip); `heavy_stage` of k_sp_heavy: 0 both halves (one rank), 1 sums, 2 finish
void sp_launch_glin(const SpDev &G, bool fp32, hipStream_t st);   // rows + blocks + heavy sums (rank partial)
void sp_launch_maxdiag(const SpDev &G, double *out, hipStream_t st);   // rank max of the rows' diagonal
void sp_launch_maxdiag_heavy(const SpDev &G, double *out, hipStream_t st);   // out = max(out, heavy diagonal)
void sp_launch_cvt_j(const double *J, float *J32, int64_t n, hipStream_t st, const int *gate = nullptr);
void sp_launch_setup(const SpDev &G, const double *rhs, double lambda, hipStream_t st);
void sp_launch_dots(const SpDev &G, int it, hipStream_t st);
// last: the chain's last queued iteration (tile mode with G.tparts: its update records the state of
// iteration it + 1 — the only k_sp_tupd that takes the ticketed sum)
void sp_launch_product(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, bool last = true);
void sp_launch_heavy(const SpDev &G, int it, double lambda, int stage, hipStream_t st);
int sp_merged_grid1(const SpDev &G);    // merged chain: phase-1 / phase-2 grid sizes
int sp_merged_grid2(const SpDev &G);
void sp_launch_update(const SpDev &G, int it, hipStream_t st);
void sp_launch_tile_product(const SpDev &G, double lambda, bool fp32, hipStream_t st);   // q = (H + lambda I) p
// sharded tile chain: w = A z by tiles (k_sp_tile, beta 0) and the rank's record xb (k_sp_txb)
// (list: the launch's logical workgroups, n of them — nullptr / t_grid: all; txb: then k_sp_txb)
void sp_launch_tile_sd(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, const int32_t *list, int n,
                       bool txb);
void sp_launch_update_sd(const SpDev &G, int it, double lambda, int tail, hipStream_t st);
// sharded chain, phase 1 over `n` of its logical workgroups (list: their indices; nullptr: all, n =
// sp_merged_grid1) and phase 2
void sp_launch_sd_phase1(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, const int32_t *list, int n);
void sp_launch_sd_phase2(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st);
void sp_launch_halo_pack(int n, const int32_t *rows, int width, int64_t base, const double *src, double *buf,
                         hipStream_t st);
void sp_launch_halo_unpack(int n, const int32_t *rows, int width, int64_t base, const double *buf, double *dst, hipStream_t st);
void sp_launch_load_p(int64_t n, const double *v, double2 *zp, hipStream_t st);
void sp_launch_permute_in(int32_t P, int64_t hd, const int32_t *row_of_point, const double *src, double *dst,
                          hipStream_t st);
void sp_launch_permute_out(int32_t P, int64_t hd, const int32_t *row_of_point, const double *src, double *dst,
                           hipStream_t st);

// The LM solve on the iterative plan (one rank).  Owned by the C-ABI context (solver.cpp).
// the value arrays of a problem in a plan's layout (SpSolver::gather_values)
struct SpValues {
    std::vector<double> pts, tg, sc, cpose, camR, ro, ri, dm, di, aw, rot, parea, pinfo;
    std::vector<float> kb8;
};

class SpSolver {
 public:
    // force_sharded: the sharded chain and the transport's collectives even on one rank (a context
    // with an RCCL communicator of one rank: the production transport exercised on one GPU)
    SpSolver(int device, hipStream_t st, int rank, int nranks, SpTransport *tr, bool force_sharded = false);
    ~SpSolver();
    int upload(const deftri_problem_desc &d);
    std::function<void()> before_alloc;            // upload: called once after the host plan build
    int refresh(const deftri_problem_desc &d);     // same structure: values only, plan kept
    int solve_lm(const deftri_lm_params &prm, deftri_report &R);
    int download(double *points, double *scales, double *tg);
    int reset_state();
    int chi2(double *out);
    int gradient(double *b, double *hdiag, int64_t n, bool analytic);
    int damped_solve(double lambda, const double *rhs, double *x, int64_t n);
    int hessian_product(double lambda, const double *x, double *y, int64_t n);   // y = (H + lambda I) x
    int profile_trial(double lambda, KProf &prof, bool analytic);
    int vertex_owner(int32_t *owner, int64_t nv) const;
    int64_t ndof() const { return G.ndof; }
    // algorithmic bytes per CG iteration of phase 1 / 2; the merged chain adds its own work: phase 1
    // the rows' p.(D + lambda)p terms ((z, p) and D in) and the heavy p (in, out), phase 2 the update
    // (x, r in / out and M in per row, q no longer stored)
    double product_bytes_phase(int k) const {
        if (G.tile) return H.tile_bytes[k == 1 ? 0 : 1];
        if (k == 1) return H.phase1_bytes + (G.merged ? (double)G.nown * (48 + 48) + (double)G.hd * (16 + 8) : 0.0);
        return H.phase2_bytes + (G.merged ? (double)G.nown * (24 + 24 + 24 + 24 + 48 - 24) : 0.0);
    }
    double product_bytes() const { return product_bytes_phase(1) + product_bytes_phase(2); }
    // SURVEY.md §8(d) B_pcg = 176 E + 48 R + 40 D + 156 P on this rank's share (owned ARAP edges, own
    // rows' edges, own rows): the minimal-traffic count the bench line's frac_survey is priced on
    double survey_bytes() const {
        return 176.0 * H.n_arap_owned + 48.0 * (double)H.rep_ids.size() + 40.0 * (double)H.dep_ids.size() +
               156.0 * (double)(H.hi - H.lo);
    }
    int64_t halo_rows() const { return H.halo_rows; }
    bool sharded() const { return shard_; }
    int32_t cg_collectives() const { return !shard_ ? 0 : G.sd ? 1 : 2; }   // all-reduces per CG iteration
    int32_t own_rows() const { return H.hi - H.lo; }
    int32_t n_blocks() const { return G.nblk; }
    int32_t n_row_blocks() const { return G.nrb; }
    int32_t n_arap_local() const { return (int32_t)H.arap_ids.size(); }
    int32_t n_tiles() const { return G.tile ? G.ntile : 0; }
    bool halo_overlap() const { return G.sd && G.ovl; }
    int32_t cg_launches() const {     // per CG iteration: [dots], phase 1, phase 2, [heavy x 1-2], update
        if (G.sd) return 3;                      // + one all-reduce and one grouped send / receive
        if (G.merged) return G.alpha_kernel ? 3 : 2;
        const int heavy = G.fuse_heavy ? 0 : (nranks_ > 1 || G.heavy_split) ? 2 : 1;
        return (G.fuse ? 0 : 1) + (G.nblk > 0 ? 1 : 0) + 1 + heavy + 1;
    }
    // settings
    double tol = 1e-12;
    int max_it = 0;                  // 0: the default budget
    int fp32_jac = 0;                // ARAP Jacobians stored in fp32 for the product
    int last_its = 8;
    int step_its = 0, step_solved = 0;
    std::string err;

 private:
    int dev_ = 0;
    hipStream_t st_ = nullptr;
    int rank_ = 0, nranks_ = 1;
    SpTransport *tr_ = nullptr;
    bool shard_ = false;                  // the sharded control flow (nranks > 1, or forced with a transport)
    SpPlanHost H;
    SpDev G;
    DevProblem P;
    std::vector<void *> allocs_;
    std::vector<double *> init_;      // initial state (points plan order, scales, tg)
    double *d_entry[3] = {nullptr, nullptr, nullptr};   // the state at solve_lm's entry (restored on an error)
    bool in_lm_ = false;                                // inside solve_lm (d_entry holds its entry state)
    int save_entry();
    double *d_scal = nullptr, *d_part = nullptr, *d_dx0 = nullptr, *d_tmp = nullptr;
    int *d_flag = nullptr;
    int *d_sumcnt = nullptr;           // launch_sum_multi_fused's / launch_trial_eval's ticket
    double *d_epart = nullptr;         // launch_trial_eval's partials
    int64_t n_epart_ = 0;
    double *h_epart_ = nullptr;        // pinned: the partials of a host-finished trial evaluation
    int eval_nb_[4] = {0, 0, 0, 0};    // its workgroups per kind (trial_eval_blocks)
    // the linearization's chi2 partials (one rank: DevProblem::lin_part): in HBM for launch_part_sums,
    // pinned for the host loop, which adds them after its synchronization (lin_host_pending_)
    double *d_lpart_ = nullptr, *h_lpart_ = nullptr;
    int lin_nb_[4] = {0, 0, 0, 0};
    bool lin_host_pending_ = false;
    double lin_chi_host() const;       // the pending partials' total ((rep + arap) + dep)
    double *hpin = nullptr;
    int *ipin = nullptr;
    int32_t *d_send_rows = nullptr, *d_recv_rows = nullptr;
    double *d_xbuf = nullptr;
    std::vector<int64_t> send_off_, recv_off_;   // per peer, into the row lists (and x 6 per row)
    int32_t *d_row_of_point = nullptr;
    LmState *d_lm = nullptr, *h_snap = nullptr;   // device-driven LM state; its pinned copy
    double *d_chi_it = nullptr;
    int32_t *d_trials_it = nullptr;
    bool have_ = false;
    template <class T> int alloc(T **p, int64_t n);
    template <class T> int put(T **p, const std::vector<T> &v);
    int fail(int code, const std::string &m) { err = m; return code; }
    int hand_off_timeout();
    int budget() const;
    int lin_iteration(bool analytic, bool want_max, bool &ok, bool host_chi = false);
    int eval_chi2(bool analytic, int slot, const SumJob *extra, const ReadBack *rb = nullptr, double *h_part = nullptr,
                  double *rec_clear = nullptr, int64_t nclear = 0);
    int cg_setup(double lambda, const double *rhs);
    int cg_chain(double lambda, int from, int to);
    int cg_tail(int n, double lambda);
    int halo(int width, double *vec, bool zp);
    int halo_sd();
    // sharded chain with the halo exchange overlapped (G.ovl): phase 1's workgroups that read no halo
    // row (d_p1int) run while the boundary rows' (z, p) travel on cs_; the rest (d_p1bnd) wait for
    // ev_halo_.  int_pending_: the iteration whose interior phase 1 is already queued
    hipStream_t cs_ = nullptr;
    hipEvent_t ev_upd_ = nullptr, ev_halo_ = nullptr;
    int32_t *d_p1int = nullptr, *d_p1bnd = nullptr;
    int n_p1int = 0, n_p1bnd = 0, int_pending_ = -1;
    int sd_product(int it, double lambda);
    int sd_exchange(int next_it, double lambda);
    int pcg_solve(double lambda, const double *rhs, bool &solved, int &its);
    int solve_lm_dev(const deftri_lm_params &prm, deftri_report &R);
    void gather_values(const deftri_problem_desc &d, SpValues &v) const;
};

}  // namespace deftri
