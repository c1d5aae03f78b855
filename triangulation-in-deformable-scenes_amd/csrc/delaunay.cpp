// delaunay.cpp — 2-D Delaunay triangulation (replaces the reference's qhull "d Qbb Qt" call in
// ComputeDelaunayTriangulation3D, Modules/Utils/Geometry.cc:317-368).
//
// Algorithm: radial sweep-hull with incremental Lawson legalization (points sorted by distance
// from the seed triangle's circumcentre; each new point lies outside the current hull, is joined to
// every visible hull edge, and the new edges are flipped until locally Delaunay).  Predicates
// orient2d / incircle use a floating-point filter and fall back to exact expansion arithmetic
// (two-sum / FMA two-product), so the output is THE Delaunay triangulation for points in general
// position — which is what qhull's lower hull of the lifted points is.  O(n log n).
#include "delaunay.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <vector>

namespace deftri {

namespace {

// ---------------- exact arithmetic (expansions, increasing magnitude, non-overlapping) -------
inline void two_sum(double a, double b, double &s, double &e) {
    s = a + b;
    double bv = s - a, av = s - bv;
    e = (a - av) + (b - bv);
}
inline void two_prod(double a, double b, double &p, double &e) {
    p = a * b;
    e = std::fma(a, b, -p);
}
using Exp = std::vector<double>;
void grow(Exp &e, double b) {
    Exp out;
    out.reserve(e.size() + 1);
    double q = b;
    for (double x : e) {
        double s, h;
        two_sum(q, x, s, h);
        if (h != 0.0) out.push_back(h);
        q = s;
    }
    if (q != 0.0 || out.empty()) out.push_back(q);
    e.swap(out);
}
Exp add(const Exp &a, const Exp &b) {
    Exp r = a;
    for (double x : b) grow(r, x);
    return r;
}
Exp neg(Exp a) { for (double &x : a) x = -x; return a; }
Exp scale(const Exp &e, double b) {
    Exp r;
    for (double x : e) {
        double p, q;
        two_prod(x, b, p, q);
        grow(r, q);
        grow(r, p);
    }
    return r;
}
Exp mul(const Exp &a, const Exp &b) {
    Exp r;
    for (double x : b) r = add(r, scale(a, x));
    return r;
}
Exp diff(double a, double b) {
    double s, e;
    two_sum(a, -b, s, e);
    Exp r;
    if (e != 0.0) r.push_back(e);
    r.push_back(s);
    return r;
}
int sign(const Exp &e) {
    for (size_t i = e.size(); i-- > 0;)
        if (e[i] != 0.0) return e[i] > 0 ? 1 : -1;
    return 0;
}

int orient_exact(const double *a, const double *b, const double *c) {
    Exp acx = diff(a[0], c[0]), bcx = diff(b[0], c[0]), acy = diff(a[1], c[1]), bcy = diff(b[1], c[1]);
    return sign(add(mul(acx, bcy), neg(mul(acy, bcx))));
}

int incircle_exact(const double *a, const double *b, const double *c, const double *d) {
    Exp adx = diff(a[0], d[0]), ady = diff(a[1], d[1]);
    Exp bdx = diff(b[0], d[0]), bdy = diff(b[1], d[1]);
    Exp cdx = diff(c[0], d[0]), cdy = diff(c[1], d[1]);
    Exp alift = add(mul(adx, adx), mul(ady, ady));
    Exp blift = add(mul(bdx, bdx), mul(bdy, bdy));
    Exp clift = add(mul(cdx, cdx), mul(cdy, cdy));
    Exp bc = add(mul(bdx, cdy), neg(mul(bdy, cdx)));
    Exp ca = add(mul(cdx, ady), neg(mul(cdy, adx)));
    Exp ab = add(mul(adx, bdy), neg(mul(ady, bdx)));
    return sign(add(add(mul(alift, bc), mul(blift, ca)), mul(clift, ab)));
}

// > 0 : a, b, c counter-clockwise
int orient2d(const double *a, const double *b, const double *c) {
    double detl = (a[0] - c[0]) * (b[1] - c[1]);
    double detr = (a[1] - c[1]) * (b[0] - c[0]);
    double det = detl - detr;
    double bound = 3.3306690738754716e-16 * (std::fabs(detl) + std::fabs(detr));
    if (det > bound) return 1;
    if (-det > bound) return -1;
    return orient_exact(a, b, c);
}

// > 0 : d inside the circumcircle of counter-clockwise (a, b, c)
int incircle(const double *a, const double *b, const double *c, const double *d) {
    double adx = a[0] - d[0], ady = a[1] - d[1], bdx = b[0] - d[0], bdy = b[1] - d[1];
    double cdx = c[0] - d[0], cdy = c[1] - d[1];
    double bdxcdy = bdx * cdy, cdxbdy = cdx * bdy, cdxady = cdx * ady, adxcdy = adx * cdy;
    double adxbdy = adx * bdy, bdxady = bdx * ady;
    double alift = adx * adx + ady * ady, blift = bdx * bdx + bdy * bdy, clift = cdx * cdx + cdy * cdy;
    double det = alift * (bdxcdy - cdxbdy) + blift * (cdxady - adxcdy) + clift * (adxbdy - bdxady);
    double perm = (std::fabs(bdxcdy) + std::fabs(cdxbdy)) * alift + (std::fabs(cdxady) + std::fabs(adxcdy)) * blift +
                  (std::fabs(adxbdy) + std::fabs(bdxady)) * clift;
    double bound = 1.2e-15 * perm;
    if (det > bound) return 1;
    if (-det > bound) return -1;
    return incircle_exact(a, b, c, d);
}

struct Sweep {
    const double *xy;
    int n;
    std::vector<int> tri, half;
    std::vector<int> hprev, hnext, htri, hhash;
    int hsize = 0, hstart = 0;
    double cx = 0, cy = 0;
    std::vector<int> stack;
    std::vector<int> ids;                                // sweep position -> point id
    std::vector<double> sorted_xy;

    const double *P(int i) const { return xy + 2 * (size_t)i; }

    int key(double x, double y) const {
        double dx = x - cx, dy = y - cy;
        double p = dx / (std::fabs(dx) + std::fabs(dy));
        double a = (dy > 0 ? 3 - p : 1 + p) / 4;        // pseudo-angle in [0, 1]
        int k = (int)std::floor(a * hsize);
        return ((k % hsize) + hsize) % hsize;
    }
    void link(int a, int b) {
        half[a] = b;
        if (b != -1) half[b] = a;
    }
    int add_tri(int i0, int i1, int i2, int a, int b, int c) {
        int t = (int)tri.size();
        tri.push_back(i0); tri.push_back(i1); tri.push_back(i2);
        half.push_back(-1); half.push_back(-1); half.push_back(-1);
        link(t, a); link(t + 1, b); link(t + 2, c);
        return t;
    }
    int legalize(int a) {
        size_t i = 0;
        int ar = 0;
        stack.clear();
        while (true) {
            int b = half[a];
            int a0 = a - a % 3;
            ar = a0 + (a + 2) % 3;
            if (b == -1) {
                if (stack.empty()) break;
                a = stack.back(); stack.pop_back();
                continue;
            }
            int b0 = b - b % 3;
            int al = a0 + (a + 1) % 3;
            int bl = b0 + (b + 2) % 3;
            int p0 = tri[ar], pr = tri[a], pl = tri[al], p1 = tri[bl];
            bool illegal = incircle(P(pr), P(pl), P(p0), P(p1)) > 0;
            if (illegal) {
                tri[a] = p1;
                tri[b] = p0;
                int hbl = half[bl];
                if (hbl == -1) {
                    int e = hstart;
                    do {
                        if (htri[e] == bl) { htri[e] = a; break; }
                        e = hprev[e];
                    } while (e != hstart);
                }
                link(a, hbl);
                link(b, half[ar]);
                link(ar, bl);
                int br = b0 + (b + 1) % 3;
                stack.push_back(br);
            } else {
                if (stack.empty()) break;
                a = stack.back(); stack.pop_back();
            }
            (void)i;
        }
        return ar;
    }

    bool run(int &skipped) {
        skipped = 0;
        double minx = 1e300, miny = 1e300, maxx = -1e300, maxy = -1e300;
        for (int i = 0; i < n; i++) {
            minx = std::min(minx, P(i)[0]); maxx = std::max(maxx, P(i)[0]);
            miny = std::min(miny, P(i)[1]); maxy = std::max(maxy, P(i)[1]);
        }
        double mx = (minx + maxx) / 2, my = (miny + maxy) / 2;
        auto d2 = [&](int i, double x, double y) { double dx = P(i)[0] - x, dy = P(i)[1] - y; return dx * dx + dy * dy; };
        int i0 = 0;
        double best = 1e300;
        for (int i = 0; i < n; i++) { double v = d2(i, mx, my); if (v < best) { best = v; i0 = i; } }
        int i1 = -1;
        best = 1e300;
        for (int i = 0; i < n; i++) {
            if (i == i0) continue;
            double v = d2(i, P(i0)[0], P(i0)[1]);
            if (v < best && v > 0) { best = v; i1 = i; }
        }
        if (i1 < 0) return false;
        auto circumr2 = [&](int a, int b, int c, double &ox, double &oy) {
            double dx = P(b)[0] - P(a)[0], dy = P(b)[1] - P(a)[1];
            double ex = P(c)[0] - P(a)[0], ey = P(c)[1] - P(a)[1];
            double bl = dx * dx + dy * dy, cl = ex * ex + ey * ey;
            double dd = 0.5 / (dx * ey - dy * ex);
            double x = (ey * bl - dy * cl) * dd, y = (dx * cl - ex * bl) * dd;
            ox = P(a)[0] + x; oy = P(a)[1] + y;
            return x * x + y * y;
        };
        int i2 = -1;
        double minr = 1e300, ox, oy;
        for (int i = 0; i < n; i++) {
            if (i == i0 || i == i1) continue;
            if (orient2d(P(i0), P(i1), P(i)) == 0) continue;
            double r = circumr2(i0, i1, i, ox, oy);
            if (std::isfinite(r) && r < minr) { minr = r; i2 = i; }
        }
        if (i2 < 0) return false;                        // all collinear
        if (orient2d(P(i0), P(i1), P(i2)) < 0) std::swap(i1, i2);
        circumr2(i0, i1, i2, cx, cy);
        // the sweep order (distance from the seed circumcentre, then index); the points are copied into
        // that order and the sweep runs on positions, so its hull walks and in-circle tests read
        // neighbouring memory (the triangles are mapped back to point ids at the end)
        std::vector<std::pair<double, int>> di(n);
        for (int i = 0; i < n; i++) di[i] = {d2(i, cx, cy), i};
        std::sort(di.begin(), di.end());
        ids.resize(n);
        std::vector<int> pos(n);
        sorted_xy.resize(2 * (size_t)n);
        for (int k = 0; k < n; k++) {
            ids[k] = di[k].second;
            pos[ids[k]] = k;
            sorted_xy[2 * (size_t)k] = P(ids[k])[0];
            sorted_xy[2 * (size_t)k + 1] = P(ids[k])[1];
        }
        std::vector<std::pair<double, int>>().swap(di);
        xy = sorted_xy.data();
        i0 = pos[i0]; i1 = pos[i1]; i2 = pos[i2];
        hsize = std::max(1, (int)std::ceil(std::sqrt((double)n)));
        hprev.assign(n, -1); hnext.assign(n, -1); htri.assign(n, -1); hhash.assign(hsize, -1);
        hstart = i0;
        hnext[i0] = i1; hprev[i2] = i1;
        hnext[i1] = i2; hprev[i0] = i2;
        hnext[i2] = i0; hprev[i1] = i0;
        htri[i0] = 0; htri[i1] = 1; htri[i2] = 2;
        hhash[key(P(i0)[0], P(i0)[1])] = i0;
        hhash[key(P(i1)[0], P(i1)[1])] = i1;
        hhash[key(P(i2)[0], P(i2)[1])] = i2;
        tri.reserve(6 * (size_t)n); half.reserve(6 * (size_t)n);
        add_tri(i0, i1, i2, -1, -1, -1);
        double px = 0, py = 0;
        for (int k = 0; k < n; k++) {
            int i = k;
            double x = P(i)[0], y = P(i)[1];
            if (k > 0 && x == px && y == py) { skipped++; continue; }      // exact duplicate
            px = x; py = y;
            if (i == i0 || i == i1 || i == i2) continue;
            int start = 0, kk = key(x, y);
            for (int j = 0; j < hsize; j++) {
                start = hhash[(kk + j) % hsize];
                if (start != -1 && start != hnext[start]) break;
            }
            start = hprev[start];
            int e = start, q;
            while (q = hnext[e], orient2d(P(e), P(q), P(i)) >= 0) {
                e = q;
                if (e == start) { e = -1; break; }
            }
            if (e == -1) { skipped++; continue; }
            int t = add_tri(e, i, hnext[e], -1, -1, htri[e]);
            htri[i] = legalize(t + 2);
            htri[e] = t;
            int nn = hnext[e];
            while (q = hnext[nn], orient2d(P(nn), P(q), P(i)) < 0) {
                t = add_tri(nn, i, q, htri[i], -1, htri[nn]);
                htri[i] = legalize(t + 2);
                hnext[nn] = nn;
                nn = q;
            }
            if (e == start) {
                while (q = hprev[e], orient2d(P(q), P(e), P(i)) < 0) {
                    t = add_tri(q, i, e, -1, htri[e], htri[q]);
                    legalize(t + 2);
                    htri[q] = t;
                    hnext[e] = e;
                    e = q;
                }
            }
            hstart = hprev[i] = e;
            hnext[e] = hprev[nn] = i;
            hnext[i] = nn;
            hhash[key(x, y)] = i;
            hhash[key(P(e)[0], P(e)[1])] = e;
        }
        for (int &v : tri) v = ids[v];                  // positions -> point ids
        return true;
    }
};

}  // namespace

// canonical order: each triangle rotated to start at its smallest vertex (orientation kept), the
// triangles sorted by (first, second, third) — the output then depends only on the triangle set,
// so the mesh area (a sum in this order) is the same whoever built the set (a full sweep, the graph
// builder's re-validated previous mesh or a flip-repaired one, graph_builder.cpp)
static void canonical_tris(const std::vector<int32_t> &in, int n, std::vector<int32_t> &tris) {
    // bucketed by first vertex (a counting sort), each bucket's (second, third) packed in one 64-bit
    // key and insertion-sorted in place (a vertex starts ~2 triangles)
    const int nt = (int)in.size() / 3;
    auto rot = [&](int t, int32_t &a, int32_t &b, int32_t &c) {
        const int32_t x = in[3 * (size_t)t], y = in[3 * (size_t)t + 1], z = in[3 * (size_t)t + 2];
        if (x < y && x < z) { a = x; b = y; c = z; }
        else if (y < z) { a = y; b = z; c = x; }
        else { a = z; b = x; c = y; }
    };
    std::vector<int32_t> cnt(n + 1, 0);
    for (int t = 0; t < nt; t++) {
        int32_t a, b, c;
        rot(t, a, b, c);
        cnt[a + 1]++;
    }
    for (int i = 0; i < n; i++) cnt[i + 1] += cnt[i];
    std::vector<uint64_t> key(nt);
    {
        std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
        for (int t = 0; t < nt; t++) {
            int32_t a, b, c;
            rot(t, a, b, c);
            key[fill[a]++] = (uint64_t)(uint32_t)b << 32 | (uint32_t)c;
        }
    }
    tris.resize(in.size());
    for (int i = 0; i < n; i++) {
        uint64_t *k0 = key.data() + cnt[i], *k1 = key.data() + cnt[i + 1];
        for (uint64_t *p = k0 + 1; p < k1; p++)
            for (uint64_t *q = p; q > k0 && q[-1] > q[0]; q--) std::swap(q[-1], q[0]);
        for (int32_t k = cnt[i]; k < cnt[i + 1]; k++) {
            tris[3 * (size_t)k] = i;
            tris[3 * (size_t)k + 1] = (int32_t)(key[k] >> 32);
            tris[3 * (size_t)k + 2] = (int32_t)(key[k] & 0xffffffffu);
        }
    }
}

bool delaunay2d(const double *xy, int n, std::vector<int32_t> &tris, int &hull_size, int &skipped) {
    tris.clear();
    hull_size = 0;
    skipped = 0;
    if (n < 3) return false;
    Sweep s{xy, n, {}, {}, {}, {}, {}, {}, 0, 0, 0, 0, {}, {}, {}};
    if (!s.run(skipped)) return false;
    canonical_tris(s.tri, n, tris);
    int h = 0, e = s.hstart;
    do { h++; e = s.hnext[e]; } while (e != s.hstart && h <= n);
    hull_size = h;
    return true;
}

// the boundary cycle bnext (nb half-edges u -> bnext[u]) is one strictly convex polygon winding once:
// with every turn in (0, pi), the edge direction passes angle 0 exactly when it moves from the lower
// half-plane [pi, 2 pi) to the upper [0, pi) — sign tests on coordinate comparisons, exact — and a
// simple convex polygon does that once (a strict left turn everywhere still admits a pentagram)
static bool boundary_convex_once(const double *xy, int n, const std::vector<int32_t> &bnext, int nb) {
    auto P = [&](int i) { return xy + 2 * (size_t)i; };
    auto upper = [&](int a, int b) {           // direction a -> b in [0, pi)
        const double *pa = P(a), *pb = P(b);
        return pb[1] > pa[1] || (pb[1] == pa[1] && pb[0] > pa[0]);
    };
    int start = -1;
    for (int i = 0; i < n && start < 0; i++) if (bnext[i] >= 0) start = i;
    if (start < 0) return false;
    int u = start, len = 0, wraps = 0;
    do {
        const int v = bnext[u];
        if (v < 0 || bnext[v] < 0) return false;
        if (orient2d(P(u), P(v), P(bnext[v])) <= 0) return false;
        if (!upper(u, v) && upper(v, bnext[v])) wraps++;
        u = v;
        if (++len > nb) return false;
    } while (u != start);
    return len == nb && wraps == 1;
}

bool delaunay_still_valid(const double *xy, int n, const std::vector<int32_t> &tris) {
    const int nt = (int)tris.size() / 3;
    if (n < 3 || nt == 0) return false;
    auto P = [&](int i) { return xy + 2 * (size_t)i; };
    // vertex -> incident triangles (CSR)
    std::vector<int32_t> off(n + 1, 0), inc(3 * (size_t)nt);
    for (int32_t v : tris) {
        if (v < 0 || v >= n) return false;
        off[v + 1]++;
    }
    for (int i = 0; i < n; i++) {
        if (off[i + 1] == 0) return false;                // a vertex on no triangle (a skipped point)
        off[i + 1] += off[i];
    }
    {
        std::vector<int32_t> fill(off.begin(), off.end() - 1);
        for (int t = 0; t < nt; t++)
            for (int k = 0; k < 3; k++) inc[fill[tris[3 * (size_t)t + k]]++] = t;
    }
    std::vector<int32_t> bnext(n, -1);                   // boundary half-edge u -> v (counter-clockwise)
    int nb = 0;
    for (int t = 0; t < nt; t++) {
        const int32_t *T = &tris[3 * (size_t)t];
        if (orient2d(P(T[0]), P(T[1]), P(T[2])) <= 0) return false;
        for (int k = 0; k < 3; k++) {
            const int32_t u = T[k], v = T[(k + 1) % 3], w = T[(k + 2) % 3];
            // the twin half-edge v -> u in a triangle around v
            int32_t x = -1;
            int twins = 0;
            for (int32_t m = off[v]; m < off[v + 1]; m++) {
                const int32_t t2 = inc[m];
                if (t2 == t) continue;
                const int32_t *S = &tris[3 * (size_t)t2];
                for (int c = 0; c < 3; c++)
                    if (S[c] == v && S[(c + 1) % 3] == u) { x = S[(c + 2) % 3]; twins++; }
            }
            if (twins > 1) return false;
            if (twins == 0) {                            // boundary
                if (bnext[u] >= 0) return false;         // not a simple boundary polygon
                bnext[u] = v;
                nb++;
            } else if (u < v && incircle(P(u), P(v), P(w), P(x)) >= 0) {
                return false;                            // not strictly locally Delaunay
            }
        }
    }
    // the boundary: one cycle, strictly convex, winding once (the convex hull)
    return boundary_convex_once(xy, n, bnext, nb);
}

bool delaunay_repair(const double *xy, int n, const std::vector<int32_t> &prev, std::vector<int32_t> &tris, int &hull_size,
                     int &flips) {
    flips = 0;
    hull_size = 0;
    const int nt = (int)prev.size() / 3;
    if (n < 3 || nt == 0 || n >= (1 << 30)) return false;
    auto P = [&](int i) { return xy + 2 * (size_t)i; };
    std::vector<int32_t> T(prev);
    std::vector<uint8_t> seen(n, 0);
    for (int32_t v : T) {
        if (v < 0 || v >= n) return false;
        seen[v] = 1;
    }
    for (int i = 0; i < n; i++)
        if (!seen[i]) return false;                      // a vertex on no triangle (a skipped point)
    // a triangle the motion folded (a sliver's vertex crossed its opposite edge): the flips cannot
    // untangle it — fail before any other work
    for (int t = 0; t < nt; t++)
        if (orient2d(P(T[3 * t]), P(T[3 * t + 1]), P(T[3 * t + 2])) <= 0) return false;
    // half-edge h = 3 t + k runs T[h] -> T[3 t + (k + 1) % 3]; twin[h] its opposite (-1: boundary),
    // paired by an LSD radix sort of the undirected keys (min << 32 | max; sequential passes)
    auto nx = [](int h) { return h - h % 3 + (h % 3 + 1) % 3; };
    const int nh = 3 * nt;
    std::vector<uint64_t> key(nh), key2(nh);
    std::vector<int32_t> idx(nh), idx2(nh);
    for (int h = 0; h < nh; h++) {
        const uint64_t u = (uint64_t)T[h], v = (uint64_t)T[nx(h)];
        key[h] = u < v ? (u << 32 | v) : (v << 32 | u);
        idx[h] = h;
    }
    {
        int bits = 1;
        while ((1 << bits) < n) bits++;
        std::vector<int> shifts;                         // 11-bit digits of the low, then the high word
        for (int sh = 0; sh < bits; sh += 11) shifts.push_back(sh);
        for (int sh = 0; sh < bits; sh += 11) shifts.push_back(32 + sh);
        for (int shift : shifts) {
            std::vector<int32_t> cnt(2049, 0);
            for (int h = 0; h < nh; h++) cnt[((key[h] >> shift) & 2047) + 1]++;
            for (int d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
            for (int h = 0; h < nh; h++) {
                const int d = (int)((key[h] >> shift) & 2047);
                key2[cnt[d]] = key[h];
                idx2[cnt[d]++] = idx[h];
            }
            key.swap(key2);
            idx.swap(idx2);
        }
    }
    std::vector<int32_t> twin(nh, -1);
    for (int i = 0; i < nh;) {
        int j = i + 1;
        while (j < nh && key[j] == key[i]) j++;
        if (j - i > 2) return false;                      // a non-manifold edge
        if (j - i == 2) {
            const int a = idx[i], b = idx[i + 1];
            if (T[a] == T[b]) return false;              // the same direction twice: not oriented
            twin[a] = b;
            twin[b] = a;
        }
        i = j;
    }
    // Lawson's flips: an interior edge whose opposite vertex lies strictly inside the circumcircle is
    // replaced by the other diagonal of its quadrilateral; the four outer edges are checked again.
    // Each flip lowers the lifted surface, so the flips end; a cap guards the loop
    std::vector<int32_t> stack;
    stack.reserve(nh);
    for (int h = 0; h < nh; h++)
        if (twin[h] > h) stack.push_back(h);
    const int64_t cap = 16 * (int64_t)nt + 64;
    while (!stack.empty()) {
        const int h = stack.back();
        stack.pop_back();
        const int g = twin[h];
        if (g < 0) continue;
        const int h1 = nx(h), h2 = nx(h1), g1 = nx(g), g2 = nx(g1);
        const int32_t u = T[h], v = T[h1], w = T[h2], x = T[g2];      // t = (u, v, w), t2 = (v, u, x)
        if (incircle(P(u), P(v), P(w), P(x)) <= 0) continue;
        if (++flips > cap) return false;
        // the new triangles (u, x, w) and (x, v, w): strictly counter-clockwise (a convex quadrilateral)
        if (orient2d(P(u), P(x), P(w)) <= 0 || orient2d(P(x), P(v), P(w)) <= 0) return false;
        const int t = h / 3, t2 = g / 3;
        // outer half-edges before the flip: v -> w (h1), w -> u (h2), u -> x (g1), x -> v (g2)
        const int o_vw = twin[h1], o_wu = twin[h2], o_ux = twin[g1], o_xv = twin[g2];
        T[3 * t] = u; T[3 * t + 1] = x; T[3 * t + 2] = w;
        T[3 * t2] = x; T[3 * t2 + 1] = v; T[3 * t2 + 2] = w;
        auto link = [&](int a, int b) { twin[a] = b; if (b >= 0) twin[b] = a; };
        link(3 * t, o_ux);             // u -> x
        link(3 * t + 1, 3 * t2 + 2);   // x -> w  |  w -> x
        link(3 * t + 2, o_wu);         // w -> u
        link(3 * t2, o_xv);            // x -> v
        link(3 * t2 + 1, o_vw);        // v -> w
        for (int e : {3 * t, 3 * t + 2, 3 * t2, 3 * t2 + 1})
            if (twin[e] >= 0) stack.push_back(e);
    }
    // THE Delaunay triangulation — delaunay_still_valid's conditions on this structure: every vertex on
    // a triangle (above), every triangle strictly counter-clockwise (above and at every flip), every
    // interior edge strictly locally Delaunay (no cocircular ambiguity), the boundary one strictly
    // convex polygon winding once (the convex hull).  Then tris is triangle for triangle delaunay2d's
    std::vector<int32_t> bnext(n, -1);
    int nb = 0;
    for (int h = 0; h < nh; h++) {
        const int g = twin[h];
        if (g < 0) {
            const int32_t u = T[h], v = T[nx(h)];
            if (bnext[u] >= 0) return false;             // not a simple boundary polygon
            bnext[u] = v;
            nb++;
        } else if (g > h && incircle(P(T[h]), P(T[nx(h)]), P(T[nx(nx(h))]), P(T[nx(nx(g))])) >= 0) {
            return false;
        }
    }
    if (!boundary_convex_once(xy, n, bnext, nb)) return false;
    hull_size = nb;
    canonical_tris(T, n, tris);
    return true;
}

int orient2d_sign(const double *a, const double *b, const double *c) { return orient2d(a, b, c); }
int incircle_sign(const double *a, const double *b, const double *c, const double *d) { return incircle(a, b, c, d); }

}  // namespace deftri
