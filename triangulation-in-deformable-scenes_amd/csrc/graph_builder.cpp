// graph_builder.cpp — host construction of the non-rigid BA graph, following the reference's
// arapOptimization graph build (Modules/Optimization/g2oBundleAdjustment.cc:640-953) and helpers
// in Modules/Utils/Geometry.cc:
//   extractPositions        :258-270  (drops null slots -> compacted "positions")
//   ComputeEdgeWeightsCot   :272-298  (mean of a.b/|a x b| over opposite vertices, clamped >= 0)
//   createVectorMap         :300-315  (vertex -> first position with isApprox(1e-6))
//   ComputeDelaunay...3D    :317-368  (lower-Delaunay triangles of (x, y); T = facets.count())
//   computeR                :549-604  (per-vertex Procrustes R_i = V U^T with det fix)
// and Open3D's TriangleMesh ComputeAdjacencyList / GetEdgeToVerticesMap / GetSurfaceArea.
// O(n log n) replacements for the reference's O(n^2) createVectorMap / getInvUncertainty loops;
// the getInvUncertainty result is unused by the reference (:887) and is not computed.
// Index semantics kept bit-for-bit, including the slot-vs-position quirk:
//   i = invertedPosIndexes[mpIndex]  (slot used as a position index)
//   neighbour slot = posIndexes[j]   (position index used as a slot index)
#include "graph_builder.h"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <numeric>
#include <thread>

#include "delaunay.h"
#include "procrustes.h"

namespace deftri {

namespace {

// createVectorMap(vertices = pos, positions = pos, 1e-6): vertex k -> first position p with
// (v_k - p).squaredNorm() <= 1e-12 * min(|v_k|^2, |p|^2)   (Eigen isApprox)
std::vector<int32_t> vector_map(const std::vector<double> &pos, int n) {
    std::vector<int32_t> out(n);
    std::iota(out.begin(), out.end(), 0);
    std::vector<int32_t> byx(n);
    std::iota(byx.begin(), byx.end(), 0);
    std::sort(byx.begin(), byx.end(), [&](int a, int b) { return pos[3 * a] < pos[3 * b] || (pos[3 * a] == pos[3 * b] && a < b); });
    std::vector<int32_t> rank(n);
    for (int i = 0; i < n; i++) rank[byx[i]] = i;
    const double prec2 = 1e-12;
    for (int k = 0; k < n; k++) {
        const double *v = &pos[3 * k];
        double nk = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        double rad = std::sqrt(prec2 * nk);
        int best = k;
        for (int dir = -1; dir <= 1; dir += 2) {
            for (int r = rank[k] + dir; r >= 0 && r < n; r += dir) {
                int p = byx[r];
                if (std::fabs(pos[3 * p] - v[0]) > rad) break;
                if (p >= best) continue;
                const double *w = &pos[3 * p];
                double dx = v[0] - w[0], dy = v[1] - w[1], dz = v[2] - w[2];
                double np = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
                if (dx * dx + dy * dy + dz * dz <= prec2 * std::min(nk, np)) best = p;
            }
        }
        out[k] = best;
    }
    return out;
}

// Delaunay mesh with CSR adjacency (ComputeAdjacencyList: sorted, unique neighbour lists) and the
// cotangent weight of every CSR entry (i, adj[k]) (ComputeEdgeWeightsCot, Geometry.cc:272-298):
// no hash maps — an edge's weight lives next to its neighbour index, found by a binary search in
// the lower endpoint's row.
struct Mesh {
    std::vector<int32_t> tris;
    std::vector<int32_t> off, adj;    // CSR, rows sorted
    std::vector<double> w;            // per CSR entry
    double area = 0, ms_delaunay = 0;
    int T = 0, hull = 0, skipped = 0;
    int flips = -1;                   // >= 0: repaired from the previous round's mesh by that many flips
    int deg(int i) const { return off[i + 1] - off[i]; }
    int64_t find(int i, int j) const {
        const int32_t *b = adj.data() + off[i], *e = adj.data() + off[i + 1];
        const int32_t *p = std::lower_bound(b, e, j);
        return (p != e && *p == j) ? (int64_t)(p - adj.data()) : -1;
    }
};

void mesh_cot_weights(const std::vector<double> &pos, Mesh &M);

// prev (optional): the previous round's triangulation of the same vertices — repaired by flips when
// that gives THE Delaunay triangulation (delaunay_repair: then identical to a new one), else unused
bool build_mesh(const std::vector<double> &pos, int n, Mesh &M, std::string &err, bool host_weights = true,
                const std::vector<int32_t> *prev = nullptr) {
    if (n < 3) { err = "Not enough points to create a triangular mesh."; return false; }
    std::vector<double> xy(2 * (size_t)n);
    for (int i = 0; i < n; i++) { xy[2 * i] = pos[3 * i]; xy[2 * i + 1] = pos[3 * i + 1]; }
    int skipped = 0;
    auto td = std::chrono::steady_clock::now();
    // opt-in (DEFTRI_DELAUNAY_REPAIR=1, read per build): measured at 100k points the repair is no
    // faster than a new triangulation — ~100 ns per exact in-circle test on the points' scattered
    // vertex order — and a smooth motion already folds a few slivers, which it cannot untangle
    const char *rep_env = std::getenv("DEFTRI_DELAUNAY_REPAIR");
    int flips = 0;
    if (prev && rep_env && std::atoi(rep_env) != 0 && delaunay_repair(xy.data(), n, *prev, M.tris, M.hull, flips)) {
        M.flips = flips;
    } else if (!delaunay2d(xy.data(), n, M.tris, M.hull, skipped)) {
        err = "Delaunay triangulation failed (collinear input)";
        return false;
    }
    M.ms_delaunay = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count();
    M.skipped = skipped;
    const int ntri = (int)M.tris.size() / 3;
    M.T = ntri + std::max(0, M.hull - 2);       // qhull facets.count(): lower + upper Delaunay facets
    // adjacency: 2 candidate entries per triangle corner, then per-row sort + unique + compaction
    std::vector<int32_t> cnt(n + 1, 0);
    for (int k = 0; k < 3 * ntri; k++) cnt[M.tris[k] + 1] += 2;
    for (int i = 0; i < n; i++) cnt[i + 1] += cnt[i];
    std::vector<int32_t> tmp(cnt[n]), fill(cnt.begin(), cnt.end() - 1);
    for (int t = 0; t < ntri; t++) {
        const int a = M.tris[3 * t], b = M.tris[3 * t + 1], c = M.tris[3 * t + 2];
        tmp[fill[a]++] = b; tmp[fill[a]++] = c;
        tmp[fill[b]++] = a; tmp[fill[b]++] = c;
        tmp[fill[c]++] = a; tmp[fill[c]++] = b;
        const double *p0 = &pos[3 * a], *p1 = &pos[3 * b], *p2 = &pos[3 * c];
        double x[3] = {p0[0] - p1[0], p0[1] - p1[1], p0[2] - p1[2]};
        double y[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};
        double cr[3] = {x[1] * y[2] - x[2] * y[1], x[2] * y[0] - x[0] * y[2], x[0] * y[1] - x[1] * y[0]};
        M.area += 0.5 * std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    }
    M.off.assign(n + 1, 0);
    M.adj.resize(tmp.size());
    for (int i = 0; i < n; i++) {
        int32_t *b = tmp.data() + cnt[i], *e = tmp.data() + cnt[i + 1];
        std::sort(b, e);
        e = std::unique(b, e);
        std::copy(b, e, M.adj.data() + M.off[i]);
        M.off[i + 1] = M.off[i] + (int32_t)(e - b);
    }
    M.adj.resize(M.off[n]);
    if (host_weights) mesh_cot_weights(pos, M);
    return true;
}

// cot weights (ComputeEdgeWeightsCot, Geometry.cc:272-298): per undirected edge (lo, hi), the mean of
// cot_term over its opposite vertices (at most 2 in a planar triangulation, so the sum does not
// depend on their order), clamped at 0; stored on both CSR entries
void mesh_cot_weights(const std::vector<double> &pos, Mesh &M) {
    const int n = (int)M.off.size() - 1, ntri = (int)M.tris.size() / 3;
    std::vector<double> sum(M.adj.size(), 0.0);
    std::vector<int32_t> num(M.adj.size(), 0);
    for (int t = 0; t < ntri; t++) {
        const int v3[3] = {M.tris[3 * t], M.tris[3 * t + 1], M.tris[3 * t + 2]};
        for (int k = 0; k < 3; k++) {
            const int e0 = std::min(v3[k], v3[(k + 1) % 3]), e1 = std::max(v3[k], v3[(k + 1) % 3]), v2 = v3[(k + 2) % 3];
            const int64_t at = M.find(e0, e1);
            sum[at] += cot_term(&pos[3 * e0], &pos[3 * e1], &pos[3 * v2]);
            num[at]++;
        }
    }
    M.w.assign(M.adj.size(), 0.0);
    for (int i = 0; i < n; i++)
        for (int32_t k = M.off[i]; k < M.off[i + 1]; k++) {
            const int j = M.adj[k];
            if (j < i) continue;
            M.w[k] = M.w[M.find(j, i)] = cot_weight(sum[k], num[k]);
        }
}

// MapPoint id -> graph point index (ids are >= 0): a direct table when the ids fall in a range
// at most a few times the number of points (the usual case: ORB-SLAM hands out ids from a counter),
// open addressing otherwise
struct IdIndex {
    std::vector<int64_t> key;
    std::vector<int32_t> val;
    uint64_t mask = 0;
    int64_t size = 0;
    int64_t lo = 0, span = -1;                 // span >= 0: direct table over ids [lo, lo + span)
    // ids in [id_lo, id_hi] (id_hi < id_lo: none); expect = the number of distinct ids
    void init_range(int64_t id_lo, int64_t id_hi, int64_t expect) {
        const int64_t n = id_hi >= id_lo ? id_hi - id_lo + 1 : 0;
        if (n <= std::max<int64_t>(4 * expect, 1 << 16) && n < ((int64_t)1 << 31)) {
            lo = id_lo;
            span = n;
            val.assign((size_t)n, -1);
            key.clear();
            return;
        }
        init(expect);
    }
    void init(int64_t expect) {
        span = -1;
        uint64_t cap = 16;
        while (cap < (uint64_t)std::max<int64_t>(expect, 8) * 2) cap <<= 1;
        key.assign(cap, -1);
        val.assign(cap, -1);
        mask = cap - 1;
        size = 0;
    }
    static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; return x; }
    int32_t *slot(int64_t id) {
        if (span >= 0) return &val[(size_t)(id - lo)];   // init_range saw every id
        if ((uint64_t)(size + 1) * 2 > mask + 1) grow();
        uint64_t h = mix((uint64_t)id) & mask;
        while (key[h] != -1 && key[h] != id) h = (h + 1) & mask;
        if (key[h] == -1) { key[h] = id; size++; }
        return &val[h];
    }
    int32_t get(int64_t id) const {
        if (span >= 0) return id >= lo && id - lo < span ? val[(size_t)(id - lo)] : -1;
        uint64_t h = mix((uint64_t)id) & mask;
        while (key[h] != -1) {
            if (key[h] == id) return val[h];
            h = (h + 1) & mask;
        }
        return -1;
    }
    void grow() {
        std::vector<int64_t> k0 = std::move(key);
        std::vector<int32_t> v0 = std::move(val);
        const uint64_t cap = 2 * (mask + 1);
        key.assign(cap, -1);
        val.assign(cap, -1);
        mask = cap - 1;
        for (size_t i = 0; i < k0.size(); i++)
            if (k0[i] != -1) {
                uint64_t h = mix((uint64_t)k0[i]) & mask;
                while (key[h] != -1) h = (h + 1) & mask;
                key[h] = k0[i];
                val[h] = v0[i];
            }
    }
};

// computeR over vertex ranges on a few host threads: every vertex is independent, so the result
// does not depend on the split
template <class F>
void parallel_for(int n, int min_chunk, F f) {
    static const int env_t = std::getenv("DEFTRI_HOST_THREADS") ? std::atoi(std::getenv("DEFTRI_HOST_THREADS")) : 0;
    const int hw = env_t > 0 ? env_t : (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = std::max(1, std::min({hw, 16, n / std::max(min_chunk, 1)}));
    if (nt <= 1) { f(0, n); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) {
        const int b = (int)((int64_t)n * t / nt), e = (int)((int64_t)n * (t + 1) / nt);
        th.emplace_back([=, &f] { f(b, e); });
    }
    for (auto &x : th) x.join();
}

}  // namespace

bool mesh_adjacency(const std::vector<double> &pos, int n, std::vector<std::vector<int32_t>> &adj,
                    std::vector<int32_t> &pos_index, double &area, std::string &err) {
    Mesh M;
    if (!build_mesh(pos, n, M, err)) return false;
    adj.assign(n, {});
    for (int i = 0; i < n; i++) adj[i].assign(M.adj.begin() + M.off[i], M.adj.begin() + M.off[i + 1]);
    area = M.area;
    pos_index = vector_map(pos, n);
    return true;
}

void procrustes_rotation(const double S[9], double R[9]) { procrustes_rotation_hd(S, R); }

namespace {
// every input of the graph build except the three weights, serialized: equal keys give an identical
// graph (the NLopt objective's clones of one map, repeated calls on an unchanged map)
void append(std::vector<unsigned char> &k, const void *p, size_t n) {
    const unsigned char *c = static_cast<const unsigned char *>(p);
    k.insert(k.end(), c, c + n);
}
template <class T> void append_v(std::vector<unsigned char> &k, const T &v) { append(k, &v, sizeof(T)); }
// values = false: the structure key — everything but the positions, the depth scales and the global
// transformations' values (what deformationOptimization's write-back changes between rounds)
std::vector<unsigned char> graph_key(const deftri_map &map, int pair_window, bool values = true) {
    std::vector<unsigned char> k;
    size_t sz = 64;
    for (int a = 0; a < map.n_keyframes; a++) {
        const deftri_keyframe &f = map.keyframes[a];
        sz += 160 + (size_t)std::max(f.n_slots, 0) * 24 + (size_t)std::max(f.n_obs, 0) * 16 + 4 * (size_t)std::max(f.n_scales, 0);
    }
    k.reserve(sz + (size_t)std::max(map.n_global, 0) * sizeof(deftri_global_entry));
    append_v(k, map.n_keyframes); append_v(k, pair_window); append_v(k, map.n_global);
    if (values) append(k, map.global_t, sizeof(map.global_t));
    for (int e = 0; e < map.n_global; e++) {
        append_v(k, map.globals[e].kf1); append_v(k, map.globals[e].kf2);
        if (values) append(k, map.globals[e].t, sizeof(map.globals[e].t));
    }
    for (int a = 0; a < map.n_keyframes; a++) {
        const deftri_keyframe &f = map.keyframes[a];
        append_v(k, f.id); append(k, f.pose, sizeof(f.pose)); append(k, f.kb8, sizeof(f.kb8));
        append_v(k, f.n_scales); append_v(k, f.n_slots); append_v(k, f.n_obs);
        if (values) append_v(k, f.depth_scale);
        if (f.n_scales > 0 && f.inv_sigma2) append(k, f.inv_sigma2, 4 * (size_t)f.n_scales);
        if (f.n_slots > 0) {
            append(k, f.point_id, 8 * (size_t)f.n_slots);
            if (values) append(k, f.point_pos, 12 * (size_t)f.n_slots);
            append(k, f.obs_index, 4 * (size_t)f.n_slots);
        }
        if (f.n_obs > 0) { append(k, f.kp_uv, 8 * (size_t)f.n_obs); append(k, f.kp_octave, 4 * (size_t)f.n_obs); append(k, f.depth, 4 * (size_t)f.n_obs); }
    }
    return k;
}

// T_global of pair (kf1 = b, kf2 = a): map transformation for (kf1, kf2) or identity (:664-677)
// getGlobalKeyFramesTransformation(k2->first, k1->first) = (kf1.id, kf2.id): the table entry for
// that ordered pair, a default (identity) SE3f when absent (Map.cc:332-343)
void pair_tg(const deftri_map &map, int a, int b, double Tg[7]) {
    const deftri_keyframe &kf1 = map.keyframes[b], &kf2 = map.keyframes[a];
    const double I[7] = {0, 0, 0, 1, 0, 0, 0};
    for (int i = 0; i < 7; i++) Tg[i] = I[i];
    if (map.n_global > 0) {
        for (int32_t e = 0; e < map.n_global; e++)
            if (map.globals[e].kf1 == kf1.id && map.globals[e].kf2 == kf2.id) {
                for (int i = 0; i < 7; i++) Tg[i] = map.globals[e].t[i];
                break;
            }
    } else if (a == 0 && b == 1) {
        for (int i = 0; i < 7; i++) Tg[i] = map.global_t[i];
    }
    float tn = std::sqrt((float)Tg[4] * (float)Tg[4] + (float)Tg[5] * (float)Tg[5] + (float)Tg[6] * (float)Tg[6]);
    double qn = std::sqrt(Tg[0] * Tg[0] + Tg[1] * Tg[1] + Tg[2] * Tg[2] + Tg[3] * Tg[3]);
    bool rot_id = qn > 0 && std::fabs(std::fabs(Tg[3] / qn) - 1.0) < 1e-10;
    if (tn == 0.0f && rot_id) { Tg[0] = Tg[1] = Tg[2] = 0; Tg[3] = 1; Tg[4] = Tg[5] = Tg[6] = 0; }
}

// the mesh area in the triangles' (canonical) order, GetSurfaceArea's sum (build_mesh's arithmetic)
double mesh_area(const std::vector<double> &pos, const std::vector<int32_t> &tris) {
    double area = 0;
    for (size_t t = 0; t + 2 < tris.size(); t += 3) {
        const double *p0 = &pos[3 * tris[t]], *p1 = &pos[3 * tris[t + 1]], *p2 = &pos[3 * tris[t + 2]];
        double x[3] = {p0[0] - p1[0], p0[1] - p1[1], p0[2] - p1[2]};
        double y[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};
        double cr[3] = {x[1] * y[2] - x[2] * y[1], x[2] * y[0] - x[0] * y[2], x[0] * y[1] - x[1] * y[0]};
        area += 0.5 * std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    }
    return area;
}

// The structure memo's next-round path: the same descriptor a full build of `map` would give, when
// every pair's previous mesh is still its Delaunay triangulation and its vector map the identity.
// 0 refreshed; 1 not applicable (the caller builds in full; g untouched); -1 error.
int refresh_graph(const deftri_map &map, double rep_weight, double arap_weight, double info_dep, GraphResult &g,
                  GraphDevice *gdev, std::string &err) {
    const size_t np = g.meshes.size();
    // validate every distinct mesh (pairs sharing keyframe 1 share one) on the moved positions
    std::vector<const GraphResult::MeshData *> seen;
    std::vector<std::vector<double>> P1;
    std::vector<int> mesh_of(np, -1);
    for (size_t q = 0; q < np; q++) {
        const GraphResult::MeshData *md = g.meshes[q].mesh.get();
        const auto it = std::find(seen.begin(), seen.end(), md);
        if (it != seen.end()) { mesh_of[q] = (int)(it - seen.begin()); continue; }
        if (!md->identity_map) return 1;
        const deftri_keyframe &kf1 = map.keyframes[g.meshes[q].kf1];
        std::vector<double> pos1;
        pos1.reserve(3 * (size_t)md->n1);
        for (int s = 0; s < kf1.n_slots; s++)
            if (kf1.point_id[s] >= 0)
                for (int k = 0; k < 3; k++) pos1.push_back((double)kf1.point_pos[3 * s + k]);
        if ((int)pos1.size() != 3 * md->n1) return 1;
        std::vector<double> xy(2 * (size_t)md->n1);
        for (int i = 0; i < md->n1; i++) { xy[2 * i] = pos1[3 * i]; xy[2 * i + 1] = pos1[3 * i + 1]; }
        if (!delaunay_still_valid(xy.data(), md->n1, md->tris)) return 1;
        // createVectorMap stays the identity unless two points became approximately equal
        // (isApprox 1e-6); such a pair's 2-D nearest neighbour is a Delaunay edge no longer than
        // 1e-6 |p|: no such edge, no such pair
        for (int i = 0; i < md->n1; i++) {
            const double *u = &pos1[3 * i];
            const double nu = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
            for (int32_t k = md->off[i]; k < md->off[i + 1]; k++) {
                const int j = md->adj[k];
                if (j < i) continue;
                const double *v = &pos1[3 * j];
                const double nv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
                const double dx = u[0] - v[0], dy = u[1] - v[1];
                if (dx * dx + dy * dy <= 1e-12 * std::max(nu, nv)) return 1;
            }
        }
        mesh_of[q] = (int)seen.size();
        seen.push_back(md);
        P1.push_back(std::move(pos1));
    }
    // every mesh still holds: the values
    std::vector<double> areas(seen.size());
    for (size_t m = 0; m < seen.size(); m++) areas[m] = mesh_area(P1[m], seen[m]->tris);
    size_t rbase = 0;
    for (size_t q = 0; q < np; q++) {
        const GraphResult::PairMesh &pm = g.meshes[q];
        const GraphResult::MeshData &md = *pm.mesh;
        const std::vector<double> &pos1 = P1[mesh_of[q]];
        const deftri_keyframe &kf1 = map.keyframes[pm.kf1], &kf2 = map.keyframes[pm.kf2];
        std::vector<double> pos2;
        pos2.reserve(3 * (size_t)pm.n2);
        for (int s = 0; s < kf2.n_slots; s++)
            if (kf2.point_id[s] >= 0)
                for (int k = 0; k < 3; k++) pos2.push_back((double)kf2.point_pos[3 * s + k]);
        if ((int)pos2.size() != 3 * pm.n2) { err = "graph structure memo: keyframe 2 changed"; return -1; }
        double Tg[7];
        pair_tg(map, pm.kf2, pm.kf1, Tg);
        for (int i = 0; i < 7; i++) g.tg[7 * q + i] = Tg[i];
        g.scales[2 * q] = kf1.depth_scale;
        g.scales[2 * q + 1] = kf2.depth_scale;
        g.pair_area[q] = areas[mesh_of[q]];
        g.pair_info[q] = arap_weight * std::pow((double)md.T, 2);
        double *Rs = g.rot.data() + rbase;
        double *w = g.wcat.data() + pm.w_off;
        int dev_rc = 1;
        if (gdev) {
            dev_rc = gdev->mesh_pass(md.n1, pm.n2, md.tris.data(), (int)md.tris.size() / 3, md.off.data(), md.adj.data(),
                                     (int64_t)md.adj.size(), md.pos_idx.data(), md.inv.data(), pos1.data(), pos2.data(), w, Rs,
                                     err);
            if (dev_rc < 0) return -1;
        }
        if (dev_rc != 0) {
            Mesh M;
            M.tris = md.tris; M.off = md.off; M.adj = md.adj;
            mesh_cot_weights(pos1, M);
            std::copy(M.w.begin(), M.w.end(), w);
            parallel_for(md.n1, 2048, [&](int lo, int hi) {
                for (int i = lo; i < hi; i++)
                    compute_r_vertex(i, pm.n2, md.off.data(), md.adj.data(), w, md.pos_idx.data(), md.inv.data(), pos1.data(),
                                     pos2.data(), Rs + 9 * (size_t)i);
            });
        }
        rbase += 9 * (size_t)md.n1;
    }
    // order_xy is kept: the ordering coordinates of the build that established this structure (the
    // plan's row order is a locality choice, not arithmetic of the reference), so the device keeps
    // its plan and only copies values (deftri_problem_upload's reuse test compares them)
    for (size_t i = 0; i < g.point_kf.size(); i++) {
        const float *p = map.keyframes[g.point_kf[i]].point_pos + 3 * (size_t)g.point_slot[i];
        for (int c = 0; c < 3; c++) { g.points[3 * i + c] = (double)p[c]; g.point_orig[3 * i + c] = p[c]; }
    }
    for (size_t e = 0; e < g.arap_wk.size(); e++) g.arap_w[e] = g.wcat[g.arap_wk[e]];
    for (size_t e = 0; e < g.rep_info.size(); e++) g.rep_info[e] = g.rep_base[e] * rep_weight;
    std::fill(g.dep_info.begin(), g.dep_info.end(), info_dep);
    return 0;
}

bool map_ok(const deftri_map &map, std::string &err) {
    if (map.n_keyframes < 0 || (map.n_keyframes > 0 && !map.keyframes)) { err = "bad map"; return false; }
    if (map.n_global > 0 && !map.globals) { err = "bad map: globals"; return false; }
    for (int a = 0; a < map.n_keyframes; a++) {
        const deftri_keyframe &f = map.keyframes[a];
        if (f.n_slots < 0 || f.n_obs < 0 || f.n_scales < 0 || (f.n_slots > 0 && (!f.point_id || !f.point_pos || !f.obs_index)) ||
            (f.n_obs > 0 && (!f.kp_uv || !f.kp_octave || !f.depth)) || (f.n_scales > 0 && !f.inv_sigma2)) {
            err = "bad map: keyframe arrays";
            return false;
        }
    }
    return true;
}
}  // namespace

// one pair's edge layout, fixed by the sequential pass of build_arap_graph
struct PairEmit {
    int a = 0, b = 0, q = 0, ns12 = 0;
    int32_t c1 = 0, c2 = 0, s1 = 0, s2 = 0, rot_base = 0;
    int64_t w_off = 0, n_obs = 0, n_arap = 0, obs_off = 0, arap_off = 0;
    std::vector<int32_t> slot_pt;          // per slot: the graph points of (keyframe 1, keyframe 2)
    std::vector<int64_t> chunk_obs, chunk_arap;   // the counts before each kEmitChunk-slot chunk
    std::vector<int32_t> enc;              // the slots in the order the pair meets them
};
constexpr int kEmitChunk = 1 << 14;

// one pair's slot walk (:765-953's loop): the observation checks, the edge counts per slot chunk and
// the first-encounter order of the slots (a slot with both MapPoints, then its ARAP neighbours)
void scan_pair(const deftri_map &map, PairEmit &pe, const GraphResult::MeshData &MD, std::string &err) {
    const deftri_keyframe &kf1 = map.keyframes[pe.b], &kf2 = map.keyframes[pe.a];
    const int ns12 = pe.ns12;
    std::vector<uint8_t> seen((size_t)ns12, 0);
    pe.enc.reserve((size_t)ns12);
    auto meet = [&](int slot) {
        if (!seen[slot]) { seen[slot] = 1; pe.enc.push_back(slot); }
    };
    for (int mp = 0; mp < ns12; mp++) {
        if (mp % kEmitChunk == 0) { pe.chunk_obs.push_back(pe.n_obs); pe.chunk_arap.push_back(pe.n_arap); }
        if (kf1.point_id[mp] < 0 || kf2.point_id[mp] < 0) continue;
        meet(mp);
        const int32_t o1 = kf1.obs_index[mp], o2 = kf2.obs_index[mp];
        if (o1 < 0 || o2 < 0) continue;
        if (o1 >= kf1.n_obs || o2 >= kf2.n_obs) { err = "observation index out of range"; return; }
        const int32_t oc1 = kf1.kp_octave[o1], oc2 = kf2.kp_octave[o2];
        if (oc1 < 0 || oc1 >= kf1.n_scales || oc2 < 0 || oc2 >= kf2.n_scales) { err = "keypoint octave out of range"; return; }
        pe.n_obs++;
        if (mp >= MD.n1) continue;
        const int i = MD.inv[mp];
        if (i < 0) continue;
        for (int32_t k = MD.off[i]; k < MD.off[i + 1]; k++) {
            const int slot = MD.pos_idx[MD.adj[k]];
            if (slot >= ns12 || kf1.point_id[slot] < 0 || kf2.point_id[slot] < 0) continue;
            meet(slot);
            pe.n_arap++;
        }
    }
}

// the reprojection (:765-812), depth (:816-856) and ARAP (:871-953) edges of one pair, written
// into the pair's ranges; the same filters as the counting pass, so the counts agree
void emit_pair_edges(const deftri_map &map, const PairEmit &pe, int chunk, const GraphResult::MeshData &MD, double rep_weight,
                     double info_dep, GraphResult &g) {
    const deftri_keyframe &kf1 = map.keyframes[pe.b], &kf2 = map.keyframes[pe.a];
    const int32_t *sp = pe.slot_pt.data();
    const double *w = g.wcat.data() + pe.w_off;
    int64_t r = 2 * (pe.obs_off + pe.chunk_obs[chunk]), e = pe.arap_off + pe.chunk_arap[chunk];
    const int mp1 = std::min(pe.ns12, (chunk + 1) * kEmitChunk);
    for (int mp = chunk * kEmitChunk; mp < mp1; mp++) {
        if (kf1.point_id[mp] < 0 || kf2.point_id[mp] < 0) continue;
        const int32_t o1 = kf1.obs_index[mp], o2 = kf2.obs_index[mp];
        if (o1 < 0 || o2 < 0) continue;
        const int32_t p1 = sp[2 * (size_t)mp], p2 = sp[2 * (size_t)mp + 1];
        const double base1 = (double)kf1.inv_sigma2[kf1.kp_octave[o1]], base2 = (double)kf2.inv_sigma2[kf2.kp_octave[o2]];
        g.rep_point[r] = p1; g.rep_cam[r] = pe.c1;
        g.rep_obs[2 * r] = (double)kf1.kp_uv[2 * o1]; g.rep_obs[2 * r + 1] = (double)kf1.kp_uv[2 * o1 + 1];
        g.rep_base[r] = base1; g.rep_info[r] = base1 * rep_weight;
        g.rep_point[r + 1] = p2; g.rep_cam[r + 1] = pe.c2;
        g.rep_obs[2 * r + 2] = (double)kf2.kp_uv[2 * o2]; g.rep_obs[2 * r + 3] = (double)kf2.kp_uv[2 * o2 + 1];
        g.rep_base[r + 1] = base2; g.rep_info[r + 1] = base2 * rep_weight;
        g.dep_point[r] = p1; g.dep_scale[r] = pe.s1; g.dep_cam[r] = pe.c1;
        g.dep_meas[r] = (double)kf1.depth[o1]; g.dep_info[r] = info_dep;
        g.dep_point[r + 1] = p2; g.dep_scale[r + 1] = pe.s2; g.dep_cam[r + 1] = pe.c2;
        g.dep_meas[r + 1] = (double)kf2.depth[o2]; g.dep_info[r + 1] = info_dep;
        r += 2;
        if (mp >= MD.n1) continue;
        const int i = MD.inv[mp];
        if (i < 0) continue;
        for (int32_t k = MD.off[i]; k < MD.off[i + 1]; k++) {
            const int j = MD.adj[k];
            const int slot = MD.pos_idx[j];
            if (slot >= pe.ns12 || kf1.point_id[slot] < 0 || kf2.point_id[slot] < 0) continue;
            g.arap_pts[4 * e] = p1; g.arap_pts[4 * e + 1] = p2;
            g.arap_pts[4 * e + 2] = sp[2 * (size_t)slot]; g.arap_pts[4 * e + 3] = sp[2 * (size_t)slot + 1];
            g.arap_pair[e] = pe.q;
            g.arap_rot[2 * e] = pe.rot_base + i; g.arap_rot[2 * e + 1] = pe.rot_base + j;
            g.arap_w[e] = w[k];
            g.arap_wk[e] = pe.w_off + k;
            e++;
        }
    }
}

bool build_arap_graph(const deftri_map &map, double rep_weight, double arap_weight, float depth_error,
                      GraphResult &g, std::string &err, int pair_window, GraphDevice *gdev) {
    if (!map_ok(map, err)) return false;
    const double info_dep = 1.0 / ((double)depth_error * (double)depth_error);
    static const bool no_memo = std::getenv("DEFTRI_NO_GRAPH_MEMO") != nullptr;
    const auto t_build = std::chrono::steady_clock::now();
    std::vector<unsigned char> key = graph_key(map, pair_window);
    if (!no_memo && g.memo_valid && key == g.memo_key) {
        // the same map: only the weights can differ; recompute the information entries they scale
        for (size_t e = 0; e < g.rep_info.size(); e++) g.rep_info[e] = g.rep_base[e] * rep_weight;
        for (size_t q = 0; q < g.pair_info.size(); q++) g.pair_info[q] = arap_weight * std::pow((double)g.pair_T[q], 2);
        std::fill(g.dep_info.begin(), g.dep_info.end(), info_dep);
        g.memo_hits++;
        g.ms_last = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build).count();
        return true;
    }
    std::vector<unsigned char> skey = graph_key(map, pair_window, false);
    static const bool no_struct = std::getenv("DEFTRI_NO_STRUCT_MEMO") != nullptr;
    if (!no_memo && !no_struct && g.struct_valid && skey == g.struct_key) {
        // refresh_graph writes the values pair by pair: until it succeeds neither memo describes g
        // (a failure half-way must not leave a memo hit on the previous map's mixed values)
        g.memo_valid = g.struct_valid = false;
        int rc = refresh_graph(map, rep_weight, arap_weight, info_dep, g, gdev, err);
        if (rc < 0) return false;
        if (rc == 0) {
            g.memo_key = std::move(key);
            g.memo_valid = true;
            g.struct_valid = true;
            g.struct_hits++;
            g.ms_last = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build).count();
            return true;
        }
        // rc 1: a pair's triangulation or vector map changed — the full build below
    }
    const int64_t hits = g.memo_hits, shits = g.struct_hits, reps = g.mesh_repairs, nflips = g.mesh_flips;
    // the previous round's meshes by keyframe 1 (deformationOptimization's next round: the same
    // vertices moved), the hint for a flip repair of each keyframe's triangulation
    std::vector<std::shared_ptr<const GraphResult::MeshData>> prev_mesh(map.n_keyframes);
    for (const GraphResult::PairMesh &pm : g.meshes)
        if (pm.kf1 >= 0 && pm.kf1 < map.n_keyframes && pm.mesh && pm.mesh->skipped == 0) prev_mesh[pm.kf1] = pm.mesh;
    // the edge arrays keep their storage across rebuilds (deformationOptimization's rounds): the
    // pages are already mapped, so refilling them costs no page faults
    auto keep = [](auto &dst, auto &src) { dst.swap(src); dst.clear(); };
    GraphResult old;
    keep(old.rep_point, g.rep_point); keep(old.rep_cam, g.rep_cam); keep(old.rep_obs, g.rep_obs);
    keep(old.rep_info, g.rep_info); keep(old.rep_base, g.rep_base); keep(old.dep_point, g.dep_point);
    keep(old.dep_scale, g.dep_scale); keep(old.dep_cam, g.dep_cam); keep(old.dep_meas, g.dep_meas);
    keep(old.dep_info, g.dep_info); keep(old.arap_pts, g.arap_pts); keep(old.arap_pair, g.arap_pair);
    keep(old.arap_rot, g.arap_rot); keep(old.arap_w, g.arap_w); keep(old.arap_wk, g.arap_wk);
    g = GraphResult();
    keep(g.rep_point, old.rep_point); keep(g.rep_cam, old.rep_cam); keep(g.rep_obs, old.rep_obs);
    keep(g.rep_info, old.rep_info); keep(g.rep_base, old.rep_base); keep(g.dep_point, old.dep_point);
    keep(g.dep_scale, old.dep_scale); keep(g.dep_cam, old.dep_cam); keep(g.dep_meas, old.dep_meas);
    keep(g.dep_info, old.dep_info); keep(g.arap_pts, old.arap_pts); keep(g.arap_pair, old.arap_pair);
    keep(g.arap_rot, old.arap_rot); keep(g.arap_w, old.arap_w); keep(g.arap_wk, old.arap_wk);
    g.memo_hits = hits;
    g.struct_hits = shits;
    g.mesh_repairs = reps;
    g.mesh_flips = nflips;
    const int K = map.n_keyframes;
    std::vector<int32_t> cam_of(K, -1);
    IdIndex pidx;
    {
        int64_t slots = 0, npairs = 0;
        for (int a = 0; a < K; a++)
            for (int b = a + 1; b < K; b++) {
                if (pair_window > 0 && b - a > pair_window) continue;
                slots += std::min(map.keyframes[a].n_slots, map.keyframes[b].n_slots);
                npairs++;
            }
        // the range of the MapPoint ids the pairs can meet, and how many distinct ones at most
        int64_t id_lo = INT64_MAX, id_hi = -1, nid = 0;
        for (int a = 0; a < K; a++) {
            const deftri_keyframe &f = map.keyframes[a];
            for (int s = 0; s < f.n_slots; s++)
                if (f.point_id[s] >= 0) {
                    id_lo = std::min(id_lo, f.point_id[s]);
                    id_hi = std::max(id_hi, f.point_id[s]);
                    nid++;
                }
        }
        pidx.init_range(id_lo, id_hi, std::min<int64_t>(nid, 2 * slots));
        g.rot.reserve(9 * slots);
        g.point_mpid.reserve(2 * slots); g.points.reserve(6 * slots); g.point_orig.reserve(6 * slots);
        g.order_xy.reserve(4 * slots);
        (void)npairs;
    }
    auto cam_index = [&](int k) {
        if (cam_of[k] < 0) {
            cam_of[k] = (int32_t)(g.cam_pose.size() / 7);
            const deftri_keyframe &kf = map.keyframes[k];
            for (int i = 0; i < 7; i++) g.cam_pose.push_back(kf.pose[i]);
            for (int i = 0; i < 8; i++) g.cam_kb8.push_back(kf.kb8[i]);
        }
        return cam_of[k];
    };
    g.kf_scale.assign(K, -1);
    int32_t rot_base = 0;
    static const bool timing = std::getenv("DEFTRI_GRAPH_TIMING") != nullptr;
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    // the mesh of keyframe 1's positions (Delaunay, adjacency, area, cot weights, vector map), built
    // once per keyframe: every pair with that keyframe 1 has the same v1Positions
    std::vector<std::shared_ptr<GraphResult::MeshData>> kf1_mesh(K);
    auto make_mesh = [&](int b, std::string &e) -> std::shared_ptr<GraphResult::MeshData> {
        const deftri_keyframe &kf1 = map.keyframes[b];
        auto md = std::make_shared<GraphResult::MeshData>();
        for (int s = 0; s < kf1.n_slots; s++)
            if (kf1.point_id[s] >= 0)
                for (int k = 0; k < 3; k++) md->pos1.push_back((double)kf1.point_pos[3 * s + k]);
        md->n1 = (int)md->pos1.size() / 3;
        Mesh M;
        const std::vector<int32_t> *hint =
            prev_mesh[b] && prev_mesh[b]->n1 == md->n1 ? &prev_mesh[b]->tris : nullptr;
        if (!build_mesh(md->pos1, md->n1, M, e, gdev == nullptr, hint)) return nullptr;   // device: weights in the device pass
        md->tris = std::move(M.tris); md->off = std::move(M.off); md->adj = std::move(M.adj);
        md->w = std::move(M.w);
        md->T = M.T; md->hull = M.hull; md->area = M.area;
        md->skipped = M.skipped; md->flips = M.flips;
        md->pos_idx = vector_map(md->pos1, md->n1);
        md->inv.assign(md->n1, -1);          // invertedPosIndexes: the last vertex wins
        for (int v = 0; v < md->n1; v++) md->inv[md->pos_idx[v]] = v;
        md->identity_map = M.skipped == 0;
        for (int v = 0; v < md->n1 && md->identity_map; v++) md->identity_map = md->pos_idx[v] == v;
        return md;
    };
    {
        // every keyframe 1's mesh up front, the keyframes on parallel host threads (each mesh is a
        // function of its keyframe's positions alone)
        std::vector<int> need;
        for (int b = 1; b < K; b++)
            for (int a = 0; a < b; a++)
                if (!(pair_window > 0 && b - a > pair_window)) { need.push_back(b); break; }
        std::vector<std::string> errs(need.size());
        parallel_for((int)need.size(), 1, [&](int lo, int hi) {
            for (int i = lo; i < hi; i++) kf1_mesh[need[i]] = make_mesh(need[i], errs[i]);
        });
        for (size_t i = 0; i < need.size(); i++)
            if (!kf1_mesh[need[i]]) { err = errs[i]; return false; }
        for (int b : need)
            if (kf1_mesh[b]->flips >= 0) { g.mesh_repairs++; g.mesh_flips += kf1_mesh[b]->flips; }
    }
    std::vector<PairEmit> emits;
    for (int a = 0; a < K; a++) {
        for (int b = a + 1; b < K; b++) {
            if (pair_window > 0 && b - a > pair_window) continue;
            const deftri_keyframe &kf1 = map.keyframes[b];   // pKF1 = k2->second
            const deftri_keyframe &kf2 = map.keyframes[a];   // pKF2 = k1->second
            const int32_t q = (int32_t)g.pair_area.size();
            // extractPositions
            std::vector<double> pos2;
            pos2.reserve(3 * (size_t)kf2.n_slots);
            for (int s = 0; s < kf2.n_slots; s++)
                if (kf2.point_id[s] >= 0)
                    for (int k = 0; k < 3; k++) pos2.push_back((double)kf2.point_pos[3 * s + k]);
            auto t0 = tnow();
            if (!kf1_mesh[b] && !(kf1_mesh[b] = make_mesh(b, err))) return false;
            const GraphResult::MeshData &MD = *kf1_mesh[b];
            const std::vector<double> &pos1 = MD.pos1;
            const std::vector<int32_t> &posIdx = MD.pos_idx, &inv = MD.inv;
            const int n1 = MD.n1, n2 = (int)pos2.size() / 3;
            Mesh M;                                         // this pair's weights over the shared structure
            M.off = MD.off; M.adj = MD.adj; M.w = MD.w; M.T = MD.T; M.hull = MD.hull; M.area = MD.area;
            auto t1 = tnow();
            double Tg[7];
            pair_tg(map, a, b, Tg);
            auto t2 = tnow();
            // computeR: one Procrustes rotation per vertex, identity where no position maps to it
            const size_t rbase = g.rot.size();
            g.rot.resize(rbase + 9 * (size_t)n1);
            double *Rs = g.rot.data() + rbase;
            int dev_rc = 1;
            if (gdev) {
                M.w.resize(M.adj.size());
                dev_rc = gdev->mesh_pass(n1, n2, MD.tris.data(), (int)MD.tris.size() / 3, M.off.data(), M.adj.data(),
                                         (int64_t)M.adj.size(), posIdx.data(), inv.data(), pos1.data(), pos2.data(), M.w.data(),
                                         Rs, err);
                if (dev_rc < 0) return false;
                if (dev_rc == 1) { M.tris = MD.tris; mesh_cot_weights(pos1, M); }   // non-manifold edge: the host loops
            }
            if (dev_rc != 0) {
                parallel_for(n1, 2048, [&](int lo, int hi) {
                    for (int i = lo; i < hi; i++)
                        compute_r_vertex(i, n2, M.off.data(), M.adj.data(), M.w.data(), posIdx.data(), inv.data(), pos1.data(),
                                         pos2.data(), Rs + 9 * (size_t)i);
                });
            }
            auto t3 = tnow();
            {
                GraphResult::PairMesh pm;
                pm.mesh = kf1_mesh[b];
                pm.n2 = n2; pm.kf1 = b; pm.kf2 = a;
                pm.w_off = (int64_t)g.wcat.size();
                g.wcat.insert(g.wcat.end(), M.w.begin(), M.w.end());
                g.meshes.push_back(std::move(pm));
            }
            const int64_t w_off = g.meshes.back().w_off;
            for (int i = 0; i < 7; i++) g.tg.push_back(Tg[i]);
            const int32_t s1 = (int32_t)g.scales.size();
            g.scales.push_back(kf1.depth_scale); g.kf_scale[b] = s1;
            const int32_t s2 = (int32_t)g.scales.size();
            g.scales.push_back(kf2.depth_scale); g.kf_scale[a] = s2;
            const int32_t c1 = cam_index(b), c2 = cam_index(a);
            g.pair_area.push_back(M.area);
            g.pair_info.push_back(arap_weight * std::pow((double)M.T, 2));
            g.pair_kf1.push_back(b); g.pair_kf2.push_back(a);
            g.pair_T.push_back(M.T); g.pair_hull.push_back(M.hull);
            // the pair's slots are scanned after this loop, the pairs in parallel
            emits.emplace_back();
            PairEmit &pe = emits.back();
            pe.a = a; pe.b = b; pe.q = q; pe.c1 = c1; pe.c2 = c2; pe.s1 = s1; pe.s2 = s2;
            pe.rot_base = rot_base; pe.w_off = w_off; pe.ns12 = std::min(kf1.n_slots, kf2.n_slots);
            rot_base += n1;
            if (timing)
                std::fprintf(stderr, "[deftri graph] pair %d: mesh %.1f ms (delaunay %.1f), vector map %.1f, computeR %.1f%s (kernel %.3f), edges %.1f\n", q,
                             ms(t0, t1), M.ms_delaunay, ms(t1, t2), ms(t2, t3), gdev ? " device" : " host", gdev ? gdev->ms_last : 0.0,
                             ms(t3, tnow()));
        }
    }
    {
        // (i) every pair's slot scan on its own host thread: the observation checks, the pair's edge
        //     counts per slot chunk and the order in which it meets its slots (its ARAP neighbours
        //     included) — the order the reference creates their points in
        auto ts = tnow();
        std::vector<std::string> perr(emits.size());
        parallel_for((int)emits.size(), 1, [&](int lo, int hi) {
            for (int e = lo; e < hi; e++) scan_pair(map, emits[e], *g.meshes[e].mesh, perr[e]);
        });
        for (size_t e = 0; e < emits.size(); e++)
            if (!perr[e].empty()) { err = perr[e]; return false; }   // the first pair's first error
        const auto ts_scan = tnow();
        // (ii) the points, created in the pairs' order, each at its first encounter; a slot's two
        //      MapPoints are fixed within the pair, so their graph indices are looked up once
        auto add_point = [&](int64_t id, int kf, int slot, int ord_kf, int ord_slot) {
            int32_t *v = pidx.slot(id);
            if (*v >= 0) return *v;
            const int32_t k = (int32_t)g.point_mpid.size();
            *v = k;
            g.point_mpid.push_back(id);
            const float *p = map.keyframes[kf].point_pos + 3 * (size_t)slot;
            for (int c = 0; c < 3; c++) { g.points.push_back((double)p[c]); g.point_orig.push_back(p[c]); }
            const float *o = map.keyframes[ord_kf].point_pos + 3 * (size_t)ord_slot;
            g.order_xy.push_back((double)o[0]);
            g.order_xy.push_back((double)o[1]);
            g.point_kf.push_back(kf); g.point_slot.push_back(slot);
            g.order_kf.push_back(ord_kf); g.order_slot.push_back(ord_slot);
            return k;
        };
        // With the direct id table (every id in one dense range) and no point yet, on host threads: the
        //  occurrences j = 2 (the pair's encounter index) + side, pairs concatenated, each id's first
        //  occurrence by an atomic minimum, the first occurrences flagged and prefix-summed into the
        //  point numbers — the numbering of the sequential loop below
        std::vector<int64_t> pbase(emits.size() + 1, 0);
        for (size_t e = 0; e < emits.size(); e++) pbase[e + 1] = pbase[e] + 2 * (int64_t)emits[e].enc.size();
        const int64_t nocc = pbase[emits.size()];
        const bool par_points = pidx.span >= 0 && g.point_mpid.empty() && nocc >= (1 << 16) && nocc < (1LL << 31);
        if (par_points) {
            auto occ = [&](int64_t j, int64_t &id, int &kf, int &slot, int &okf) {
                const size_t e = (size_t)(std::upper_bound(pbase.begin(), pbase.end(), j) - pbase.begin()) - 1;
                const PairEmit &pe = emits[e];
                const int64_t x = j - pbase[e];
                slot = pe.enc[(size_t)(x >> 1)];
                kf = (x & 1) ? pe.a : pe.b;
                okf = pe.b;
                id = map.keyframes[kf].point_id[slot];
            };
            std::vector<int32_t> first((size_t)pidx.span, INT32_MAX);
            parallel_for((int)nocc, 1 << 15, [&](int j0, int j1) {
                for (int j = j0; j < j1; j++) {
                    int64_t id; int kf, slot, okf;
                    occ(j, id, kf, slot, okf);
                    int32_t *f = &first[(size_t)(id - pidx.lo)];
                    int32_t cur = __atomic_load_n(f, __ATOMIC_RELAXED);
                    while (j < cur && !__atomic_compare_exchange_n(f, &cur, j, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
                }
            });
            const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(64, nocc >> 15));
            std::vector<int64_t> cb(nch + 1, 0);
            auto lo_of = [&](int c) { return (int)(nocc * c / nch); };
            parallel_for(nch, 1, [&](int c0, int c1) {
                for (int c = c0; c < c1; c++)
                    for (int j = lo_of(c); j < lo_of(c + 1); j++) {
                        int64_t id; int kf, slot, okf;
                        occ(j, id, kf, slot, okf);
                        cb[c + 1] += first[(size_t)(id - pidx.lo)] == j;
                    }
            });
            for (int c = 0; c < nch; c++) cb[c + 1] += cb[c];
            const size_t np = (size_t)cb[nch];
            g.point_mpid.resize(np); g.points.resize(3 * np); g.point_orig.resize(3 * np); g.order_xy.resize(2 * np);
            g.point_kf.resize(np); g.point_slot.resize(np); g.order_kf.resize(np); g.order_slot.resize(np);
            parallel_for(nch, 1, [&](int c0, int c1) {
                for (int c = c0; c < c1; c++) {
                    int64_t k = cb[c];
                    for (int j = lo_of(c); j < lo_of(c + 1); j++) {
                        int64_t id; int kf, slot, okf;
                        occ(j, id, kf, slot, okf);
                        if (first[(size_t)(id - pidx.lo)] != j) continue;
                        pidx.val[(size_t)(id - pidx.lo)] = (int32_t)k;
                        g.point_mpid[k] = id;
                        const float *p = map.keyframes[kf].point_pos + 3 * (size_t)slot;
                        for (int cc = 0; cc < 3; cc++) { g.points[3 * k + cc] = (double)p[cc]; g.point_orig[3 * k + cc] = p[cc]; }
                        const float *o = map.keyframes[okf].point_pos + 3 * (size_t)slot;
                        g.order_xy[2 * k] = (double)o[0];
                        g.order_xy[2 * k + 1] = (double)o[1];
                        g.point_kf[k] = kf; g.point_slot[k] = slot;
                        g.order_kf[k] = okf; g.order_slot[k] = slot;
                        k++;
                    }
                }
            });
            for (PairEmit &pe : emits) pe.slot_pt.assign(2 * (size_t)pe.ns12, -1);
            parallel_for((int)nocc, 1 << 15, [&](int j0, int j1) {
                for (int j = j0; j < j1; j++) {
                    int64_t id; int kf, slot, okf;
                    occ(j, id, kf, slot, okf);
                    const size_t e = (size_t)(std::upper_bound(pbase.begin(), pbase.end(), (int64_t)j) - pbase.begin()) - 1;
                    emits[e].slot_pt[2 * (size_t)slot + ((j - pbase[e]) & 1)] = pidx.val[(size_t)(id - pidx.lo)];
                }
            });
            for (PairEmit &pe : emits) { pe.enc.clear(); pe.enc.shrink_to_fit(); }
        }
        for (PairEmit &pe : emits) {
            if (par_points) break;
            const deftri_keyframe &kf1 = map.keyframes[pe.b], &kf2 = map.keyframes[pe.a];
            pe.slot_pt.assign(2 * (size_t)pe.ns12, -1);
            for (int32_t slot : pe.enc) {
                pe.slot_pt[2 * (size_t)slot] = add_point(kf1.point_id[slot], pe.b, slot, pe.b, slot);
                pe.slot_pt[2 * (size_t)slot + 1] = add_point(kf2.point_id[slot], pe.a, slot, pe.b, slot);
            }
            pe.enc.clear();
            pe.enc.shrink_to_fit();
        }
        if (timing) std::fprintf(stderr, "[deftri graph] slot scan %.1f + points %.1f ms (%s)\n", ms(ts, ts_scan), ms(ts_scan, tnow()), par_points ? "threads" : "one thread");
    }
    {
        // the edges, each pair into its own range (the reference's order: pairs, then slots)
        auto t0 = tnow();
        int64_t nobs = 0, narap = 0;
        for (PairEmit &pe : emits) {
            pe.obs_off = nobs; pe.arap_off = narap;
            nobs += pe.n_obs; narap += pe.n_arap;
        }
        g.rep_point.resize(2 * nobs); g.rep_cam.resize(2 * nobs); g.rep_obs.resize(4 * nobs);
        g.rep_info.resize(2 * nobs); g.rep_base.resize(2 * nobs);
        g.dep_point.resize(2 * nobs); g.dep_scale.resize(2 * nobs); g.dep_cam.resize(2 * nobs);
        g.dep_meas.resize(2 * nobs); g.dep_info.resize(2 * nobs);
        g.arap_pts.resize(4 * narap); g.arap_pair.resize(narap); g.arap_rot.resize(2 * narap);
        g.arap_w.resize(narap); g.arap_wk.resize(narap);
        auto t1 = tnow();
        std::vector<std::pair<int, int>> tasks;       // (pair, slot chunk)
        for (size_t e = 0; e < emits.size(); e++)
            for (int c = 0; c < (int)emits[e].chunk_obs.size(); c++) tasks.emplace_back((int)e, c);
        parallel_for((int)tasks.size(), 1, [&](int lo, int hi) {
            for (int t = lo; t < hi; t++) {
                const int e = tasks[t].first;
                emit_pair_edges(map, emits[e], tasks[t].second, *g.meshes[e].mesh, rep_weight, info_dep, g);
            }
        });
        if (timing) std::fprintf(stderr, "[deftri graph] edges written: %.1f ms (arrays %.1f)\n", ms(t0, tnow()), ms(t0, t1));
    }
    deftri_problem_desc &d = g.desc;
    d = deftri_problem_desc{};
    d.n_points = (int32_t)g.point_mpid.size();
    d.n_pairs = (int32_t)g.pair_area.size();
    d.n_scales = (int32_t)g.scales.size();
    d.n_cams = (int32_t)(g.cam_pose.size() / 7);
    d.n_rep = (int32_t)g.rep_point.size();
    d.n_depth = (int32_t)g.dep_point.size();
    d.n_arap = (int32_t)g.arap_pair.size();
    d.n_rot = (int32_t)(g.rot.size() / 9);
    d.points = g.points.data(); d.tg = g.tg.data(); d.scales = g.scales.data();
    d.cam_kb8 = g.cam_kb8.data(); d.cam_pose = g.cam_pose.data();
    d.rep_point = g.rep_point.data(); d.rep_cam = g.rep_cam.data(); d.rep_obs = g.rep_obs.data();
    d.rep_info = g.rep_info.data();
    d.huber_delta = (double)(float)std::sqrt(100.991);          // const float deltaMono = sqrt(100.991)
    d.dep_point = g.dep_point.data(); d.dep_scale = g.dep_scale.data(); d.dep_cam = g.dep_cam.data();
    d.dep_meas = g.dep_meas.data(); d.dep_info = g.dep_info.data();
    d.arap_pts = g.arap_pts.data(); d.arap_pair = g.arap_pair.data(); d.arap_rot = g.arap_rot.data();
    d.arap_w = g.arap_w.data(); d.rot = g.rot.data(); d.pair_area = g.pair_area.data(); d.pair_info = g.pair_info.data();
    d.order_xy = g.order_xy.data();
    g.memo_key = std::move(key);
    g.memo_valid = true;
    g.struct_key = std::move(skey);
    g.struct_valid = true;
    g.ms_last = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build).count();
    return true;
}

void writeback_arap(deftri_map &map, const GraphResult &g, const std::vector<double> &points,
                    const std::vector<double> &scales, const std::vector<double> &tg, double *optimization_update) {
    // scales: the last vertex created for each KeyFrame (mKeyFrameId overwrite, :967-972)
    for (int k = 0; k < map.n_keyframes; k++)
        if (g.kf_scale[k] >= 0) map.keyframes[k].depth_scale = scales[g.kf_scale[k]];
    // points: fp32 writeback + sum ||p_old - p_new|| (:974-990)
    IdIndex pidx;
    {
        int64_t id_lo = INT64_MAX, id_hi = -1;
        for (int64_t id : g.point_mpid) { id_lo = std::min(id_lo, id); id_hi = std::max(id_hi, id); }
        pidx.init_range(id_lo, id_hi, (int64_t)g.point_mpid.size());
    }
    for (size_t i = 0; i < g.point_mpid.size(); i++) *pidx.slot(g.point_mpid[i]) = (int32_t)i;
    double upd = 0;
    for (size_t i = 0; i < g.point_mpid.size(); i++) {
        float nf[3] = {(float)points[3 * i], (float)points[3 * i + 1], (float)points[3 * i + 2]};
        float dx = g.point_orig[3 * i] - nf[0], dy = g.point_orig[3 * i + 1] - nf[1], dz = g.point_orig[3 * i + 2] - nf[2];
        upd += (double)std::sqrt(dx * dx + dy * dy + dz * dz);
    }
    for (int k = 0; k < map.n_keyframes; k++) {
        deftri_keyframe &kf = map.keyframes[k];
        for (int s = 0; s < kf.n_slots; s++) {
            if (kf.point_id[s] < 0) continue;
            const int32_t i = pidx.get(kf.point_id[s]);
            if (i < 0) continue;
            for (int c = 0; c < 3; c++) kf.point_pos[3 * s + c] = (float)points[3 * (size_t)i + c];
        }
    }
    if (optimization_update) *optimization_update = upd;
    // global transformation of the last pair (insertGlobalKeyFramesTransformation(0, 1, T), :999-1007)
    if (!g.pair_area.empty()) {
        size_t q = g.pair_area.size() - 1;
        for (int i = 0; i < 7; i++) map.global_t[i] = tg[7 * q + i];
    }
}

}  // namespace deftri
