// delaunay.h — robust 2-D Delaunay triangulation (see delaunay.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace deftri {

// xy: n points (x, y interleaved).  tris: 3 vertex indices per triangle, counter-clockwise.
// hull_size: number of convex-hull vertices; skipped: duplicate points that were not inserted.
bool delaunay2d(const double *xy, int n, std::vector<int32_t> &tris, int &hull_size, int &skipped);

int orient2d_sign(const double *a, const double *b, const double *c);
int incircle_sign(const double *a, const double *b, const double *c, const double *d);

}  // namespace deftri
