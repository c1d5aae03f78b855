// delaunay.h — robust 2-D Delaunay triangulation (see delaunay.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace deftri {

// xy: n points (x, y interleaved).  tris: 3 vertex indices per triangle, counter-clockwise, in the
// canonical order (each starting at its smallest vertex; sorted).  hull_size: number of convex-hull
// vertices; skipped: duplicate points that were not inserted.
bool delaunay2d(const double *xy, int n, std::vector<int32_t> &tris, int &hull_size, int &skipped);

int orient2d_sign(const double *a, const double *b, const double *c);
int incircle_sign(const double *a, const double *b, const double *c, const double *d);

// Is the triangle list `tris` (canonical, counter-clockwise) still THE Delaunay triangulation of the
// n points xy — the one delaunay2d would return, triangle for triangle?  True when every triangle is
// strictly counter-clockwise, every interior edge strictly locally Delaunay (its opposite vertex
// strictly outside the circumcircle: no cocircular ambiguity), every vertex is on a triangle and
// the boundary is a strictly convex polygon winding once (so it is the convex hull): then the
// triangulation is the unique Delaunay triangulation.  Exact predicates; one sequential pass over the
// triangles' half-edges, then the boundary cycle.
bool delaunay_still_valid(const double *xy, int n, const std::vector<int32_t> &tris);

// The Delaunay triangulation of the moved points from a previous triangulation `prev` of the same
// vertices (canonical, counter-clockwise): Lawson's edge flips with exact predicates, then the canonical
// order and delaunay_still_valid — true only when the result is THE Delaunay triangulation, so `tris`
// is then triangle for triangle delaunay2d's.  False (tris unspecified) when a triangle folded, the
// hull changed, a cocircular tie remains or the flips ran past their cap: the caller triangulates anew.
bool delaunay_repair(const double *xy, int n, const std::vector<int32_t> &prev, std::vector<int32_t> &tris, int &hull_size,
                     int &flips);

}  // namespace deftri
